# Round 5: config 3 (MCraft5 -depth 20) per expansion variant — 19 (fixed shares)
# against 20 (dynamic units), before / after the Drop-first order's build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/s5; mkdir -p $O
B="raft.tla_amd/bin/rmc-tlc -builtin-raft -nospill -depth 20 specs/MCraft5.tla"
for r in 1 2; do
  for v in 19 20; do
    RMC_EXPAND_VARIANT=$v timeout -k 10 120 $B > $O/s5_v${v}_$r.txt 2>&1 || exit 1
  done
  RMC_EXPAND_VARIANT=20 timeout -k 10 120 raft.tla_amd/bin/rmc-tlc -builtin-raft specs/MCraftBenchSym.tla > $O/sym_$r.txt 2>&1 || exit 1
done
for f in $O/*.txt; do echo "$f $(grep -E 'Finished' $f)"; done
