# SYMMETRY: parity of the incremental-key kernel, then same-box A/B of the
# three expansion variants (RMC_SYM_VARIANT 0 = whole successor, 1 = incremental
# at 5 waves/SIMD, 2 = incremental at 4 waves/SIMD), two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "sym or kat" > $O/tests.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1 2; do
  RMC_SYM_VARIANT=$v timeout -k 10 120 python -u tools/sym_bench.py default 300000000 > $O/sym_v${v}_r$r.jsonl 2> $O/sym_v${v}_r$r.err || exit 1
done; done
