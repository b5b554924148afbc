# Same-box A/B of rmc-tlc command lines (their "Finished in" lines): each
# variant is a label whose extra arguments are in X_<label>:
#   VARS="auto fp4g" X_auto="" X_fp4g="-fpmem 4G" ARGS="-builtin-raft specs/MCraftBenchSym.tla"
#   [ROUNDS=3] [OUT=gpurun_out/aba] bash tools/gpu/ab_args.sh
# Each round runs every variant once, the order rotated by one per round.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/aba}
mkdir -p $O
read -r -a VA <<< "$VARS"
NV=${#VA[@]}
for r in $(seq 1 ${ROUNDS:-3}); do
  for i in $(seq 0 $((NV - 1))); do
    v=${VA[$(( (i + r - 1) % NV ))]}
    xv="X_$v"
    timeout -k 10 300 ./raft.tla_amd/bin/rmc-tlc ${!xv} $ARGS > $O/c_${v}_$r.txt 2>&1 || { tail -20 $O/c_${v}_$r.txt; exit 1; }
    echo "$v (${!xv}) run $r: $(grep -h '^[0-9]* states generated' $O/c_${v}_$r.txt | tail -1)" >> $O/ab.txt
  done
done
cat $O/ab.txt
