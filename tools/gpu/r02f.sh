# Config 3 at full size (MCraft5 depth 20, MCraft5Wide depth 14), then the whole GPU suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k config3 -x -v --timeout 300 --timeout-method thread > $O/config3.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
