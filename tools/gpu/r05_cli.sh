# Round 5: TLC-format CLI runs of every BASELINE config with the final build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/cli; mkdir -p $O
B="raft.tla_amd/bin/rmc-tlc -builtin-raft"
timeout -k 10 120 $B specs/MCraftBenchXL.tla > $O/cli_config1_xl.txt 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBench.tla > $O/cli_config1.txt 2>&1 || exit 1
timeout -k 10 120 $B -depth 13 tests/golden/models/MCunbounded.tla > $O/cli_config1_mcraft_as_shipped_depth13.txt 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBenchSym.tla > $O/cli_config2.txt 2>&1 || exit 1
timeout -k 10 120 $B -depth 20 specs/MCraft5.tla > $O/cli_config3.txt 2>&1 || exit 1
timeout -k 10 120 $B -simulate num=16777216 -seed 1 specs/MCraftSmoke.tla > $O/cli_config4.txt 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBug.tla > $O/cli_config5.txt 2>&1; test $? -eq 12 || exit 1
for f in $O/*.txt; do echo "== $f"; grep -E "distinct states|depth of|Finished|steps|violated|Invariant" $f | head -4; done
