# Link-only spill: spill tests, then spill at MCraftBench scale.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -k "spill or checkpoint or recover or cli or bug_variant" -x -v --timeout 240 --timeout-method thread > $O/spill.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/spill_demo.py > $O/spill_demo.jsonl 2> $O/spill_demo.err || exit 1
