# SYMMETRY rework: sym parity tests first, then the sym bench, then the whole suite.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -k "sym or kat" -x -v --timeout 240 --timeout-method thread > $O/sym_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/sym_bench.py > $O/sym_bench.jsonl 2> $O/sym_bench.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
