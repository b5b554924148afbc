# Frontier spill: spill tests, checkpoint/recover and CLI tests, then the whole GPU suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k "spill or checkpoint or recover or cli" -x -v --timeout 240 --timeout-method thread > $O/spill.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
