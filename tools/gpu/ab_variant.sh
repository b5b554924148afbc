# Same-box A/B of a kernel knob on the bench model, after parity of each value
# on the BFS fixtures:
#   VARS="6 7" [KNOB=RMC_EXPAND_VARIANT] [PARITY="tests/test_gpu.py -k 'bfs_matches_oracle or salt'"]
#   [BENCH_EXTRA="--force-dist"] [ROUNDS=2] [OUT=gpurun_out/ab] bash tools/gpu/ab_variant.sh
# Each round runs every value once, the order rotated by one per round (a
# value's place in the round does not favour it).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/ab}
mkdir -p $O
KNOB=${KNOB:-RMC_EXPAND_VARIANT}
VARS=${VARS:-"6 7"}
PARITY=${PARITY:-"tests/test_gpu.py -k 'bfs_matches_oracle or salt'"}
for v in $VARS; do
  env $KNOB=$v timeout -k 10 400 bash -c "python -u -m pytest $PARITY -x -q --timeout 240 --timeout-method thread" > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  tail -1 $O/parity_$v.log
done
read -r -a VA <<< "$VARS"
NV=${#VA[@]}
for r in $(seq 1 ${ROUNDS:-2}); do
  for i in $(seq 0 $((NV - 1))); do
    v=${VA[$(( (i + r - 1) % NV ))]}
    env $KNOB=$v timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --v2-config= --steps ${STEPS:-5} --warmup 1 $BENCH_EXTRA > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -20 $O/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$KNOB=$v run $r', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], (d['config']['fp_salt_crosscheck'] or {}).get('agrees'))" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
