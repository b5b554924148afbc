# Round 5: PMC passes of the S=5 model on the sorted 128-lane walk (rmc-tlc,
# depth 20) and of the sharded expansion kernel at one rank (MCraftBench).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/prof2; mkdir -p $O
OUT=$O/pmc_s5 CMD="raft.tla_amd/bin/rmc-tlc -builtin-raft -nospill -depth 20 specs/MCraft5.tla" bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summary.py $O/pmc_s5 $O/summary MCraft5_depth20 || exit 1
OUT=$O/pmc_dist BENCH_ARGS="--config specs/MCraftBench.cfg --force-dist" bash tools/gpu/pmc.sh || exit 1
python3 tools/pmc_summary.py $O/pmc_dist $O/summary MCraftBench_dist1 || exit 1
ls $O/summary
