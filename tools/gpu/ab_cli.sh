# Same-box A/B of a knob on an rmc-tlc run (its "Finished in" line), after
# the knob's GPU parity tests:
#   KNOB=RMC_SYM_VARIANT VARS="0 1" ARGS="-builtin-raft specs/MCraftBenchSym.tla"
#   [PARITY="tests/test_gpu.py -k sym"] [ROUNDS=3] [OUT=gpurun_out/abc] bash tools/gpu/ab_cli.sh
# Each round runs every value once, the order rotated by one per round.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/abc}
mkdir -p $O
read -r -a VA <<< "$VARS"
NV=${#VA[@]}
if [ -n "$PARITY" ]; then
  for v in $VARS; do
    env $KNOB=$v timeout -k 10 400 bash -c "python -u -m pytest $PARITY -m gpu -x -q --timeout 240 --timeout-method thread" > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
    echo "$KNOB=$v parity: $(tail -1 $O/parity_$v.log)" >> $O/ab.txt
  done
fi
for r in $(seq 1 ${ROUNDS:-3}); do
  for i in $(seq 0 $((NV - 1))); do
    v=${VA[$(( (i + r - 1) % NV ))]}
    env $KNOB=$v timeout -k 10 200 ./raft.tla_amd/bin/rmc-tlc $ARGS > $O/c_${v}_$r.txt 2>&1 || { tail -20 $O/c_${v}_$r.txt; exit 1; }
    echo "$KNOB=$v run $r: $(grep -h 'distinct states found' $O/c_${v}_$r.txt) $(grep -h '^Finished' $O/c_${v}_$r.txt)" >> $O/ab.txt
  done
done
cat $O/ab.txt
