# Same-box A/B of bench.py command lines: each variant is a label whose extra
# arguments are in X_<label>:
#   VARS="auto big" X_big="--capacity 4140000000 --set-bytes 137438953472"
#   [BENCH_EXTRA="--config specs/MCraftBench.cfg"] [ROUNDS=2] [STEPS=5] [OUT=gpurun_out/abb]
#   bash tools/gpu/ab_bench_args.sh
# Each round runs every variant once, the order rotated by one per round.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/abb}
mkdir -p $O
read -r -a VA <<< "$VARS"
NV=${#VA[@]}
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in $(seq 0 $((NV - 1))); do
    v=${VA[$(( (i + r - 1) % NV ))]}
    xv="X_$v"
    timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling --v2-config= --steps ${STEPS:-5} --warmup 1 $BENCH_EXTRA ${!xv} > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$v run $r', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], (d['config']['fp_salt_crosscheck'] or {}).get('agrees'))" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
