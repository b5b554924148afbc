# rocprofv3 kernel trace (--stats, CSV) of the bench command: per-kernel
# average durations to set beside bench.py's HIP-event kernel time.
#   OUT=gpurun_out/<tag> [BENCH_ARGS=...] bash tools/gpu/kt.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=${OUT:-gpurun_out/kt}
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-probe-ceiling --v2-config= ${BENCH_ARGS} > $P/kt_bench.json 2> $P/kt.err || exit 1
find $P/kt -name "*kernel_trace.csv" -delete
find $P/kt -name "*stats.csv" | head -5
