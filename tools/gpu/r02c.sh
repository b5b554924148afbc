# GPU suite with the in-library sharded BFS; bench single vs forced-sharded (RCCL, world 1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/dist_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/bench_single.json 2> $O/bench_single.err || exit 1
timeout -k 10 300 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/bench_forcedist.json 2> $O/bench_forcedist.err || exit 1
