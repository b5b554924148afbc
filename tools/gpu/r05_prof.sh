# Round 5: rocprofv3 evidence of the shipped bench (MCraftBenchXL), its per-level
# times (the cost model's T1), and the sharded kernel's rate at one rank (k_dist).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/prof; mkdir -p $O
OUT=$O/pmc_xl bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summary.py $O/pmc_xl $O/summary MCraftBenchXL || exit 1
ls $O/summary
timeout -k 10 300 python -u tools/level_times.py specs/MCraftBenchXL.cfg 0 0 spill > $O/levels_MCraftBenchXL.jsonl 2> $O/levels.err || exit 1
tail -1 $O/levels_MCraftBenchXL.jsonl
