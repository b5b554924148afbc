# Same-box A/B of the sharded expansion kernel on S = 5 (specs/MCraft5.cfg to depth 20)
# at one rank (gloo host transport): wall seconds per RMC_DIST_KVARIANT value,
# after the S = 4/5 sharded parity tests of each value.
#   VARS="3 5" [ROUNDS=2] [OUT=gpurun_out/s5d] bash tools/gpu/s5_dist_ab.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/s5d}
mkdir -p $O
for v in $VARS; do
  RMC_DIST_KVARIANT=$v timeout -k 10 400 python -u -m pytest tests/test_dist.py -m gpu -x -q --timeout 240 --timeout-method thread -k "s5 or s4" > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "RMC_DIST_KVARIANT=$v parity: $(tail -1 $O/parity_$v.log)" >> $O/ab.txt
done
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARS; do
    RMC_DIST_KVARIANT=$v timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
      --master-addr 127.0.0.1 --master-port 2981$v tests/dist_worker.py --cfg specs/MCraft5.cfg --out $O/d_${v}_$r.json \
      --device 0 --backend gloo --capacity 1500000000 --rerun 0 --max-depth 20 > $O/d_${v}_$r.out 2> $O/d_${v}_$r.err || { tail -5 $O/d_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/d_${v}_$r.json')); print('RMC_DIST_KVARIANT=$v run $r', d['distinct'], round(d['wall_s'], 4))" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
