# The GPU suite, smoke and bench lines in one call (each step under its own limit):
#   OUT=gpurun_out/<tag> BENCH_ARGS="..." bash tools/gpu/suite.sh
# SKIP_TESTS=1 skips pytest; DIST_BENCH=1 adds the one-rank sharded bench (RCCL).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/suite}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    ${TESTS:+-k "$TESTS"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ -n "$DIST_BENCH" ]; then
  timeout -k 10 300 python -u bench.py --force-dist --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --v2-config= --steps 5 > $O/bench_dist1.json 2> $O/bench_dist1.err || { tail -20 $O/bench_dist1.err; exit 1; }
  cat $O/bench_dist1.json
fi
