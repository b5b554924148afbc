# Round 5: rocprofv3 evidence of the shipped bench (MCraftBenchXL), its per-level
# times (the cost model's T1), and the sharded kernel's rate at one rank (k_dist).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05/prof}; mkdir -p $O
OUT=$O/pmc_xl bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summary.py $O/pmc_xl $O/summary MCraftBenchXL || exit 1
ls $O/summary
timeout -k 10 300 python -u tools/level_times.py specs/MCraftBenchXL.cfg 0 0 spill > $O/levels_MCraftBenchXL.jsonl 2> $O/levels.err || exit 1
tail -1 $O/levels_MCraftBenchXL.jsonl
timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --steps 5 --warmup 1 > $O/bench_MCraftBench.json 2> $O/bench_MCraftBench.err || exit 1
python -c "import json; d=json.load(open('$O/bench_MCraftBench.json')); print('MCraftBench', round(d['ms_per_step'],2), d['roofline']['frac'])"
