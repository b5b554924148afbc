# Same-box A/B of k_expand variants (RMC_EXPAND_VARIANT) on the bench model,
# after parity of each variant on the BFS fixtures.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
VARS=${VARS:-"0 1 2"}
for v in $VARS; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "bfs_matches_oracle or salt" -x -q --timeout 240 --timeout-method thread > $O/parity_$v.log 2>&1 || exit 1
done
for r in 1 2; do
  for v in $VARS; do
    RMC_EXPAND_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('variant $v run $r', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['fp_salt_crosscheck']['agrees'])" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
