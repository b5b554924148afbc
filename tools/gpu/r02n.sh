# SYMMETRY with the lane-superset walk over class-sorted windows
# (RMC_SYM_VARIANT 3: 3 waves/SIMD, 4: 4 waves) vs 0: parity, then A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n
mkdir -p $O
for v in 3 4; do
  RMC_SYM_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "sym or kat" > $O/tests_sym$v.log 2>&1 || exit 1
done
for r in 1 2; do for v in 0 3 4; do
  RMC_SYM_VARIANT=$v timeout -k 10 120 python -u tools/sym_bench.py default 300000000 > $O/sym_v${v}_r$r.jsonl 2> $O/sym_v${v}_r$r.err || exit 1
done; done
