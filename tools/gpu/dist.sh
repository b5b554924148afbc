set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -k verification -x -v --timeout 240 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 2 > gpurun_out/bench_forcedist.json 2> gpurun_out/bench_forcedist.err || exit 1
