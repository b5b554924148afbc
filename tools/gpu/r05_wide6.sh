# Round 5: wide records sized from the run + the faster wave simulator —
# wide tests; Smokeraft's 16.8 M walks in each draw mode; MCraft.cfg as shipped
# to depth 13 (compact) and 12 (full); the CLI at depth 13.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/wide6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wide.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/sim_wide.py > $O/sim_wide.jsonl 2> $O/sim_wide.err || { tail -5 $O/sim_wide.err; exit 1; }
cut -c1-220 $O/sim_wide.jsonl
timeout -k 10 200 python -u tools/mcraft_shipped.py 13 auto > $O/shipped_d13_auto.jsonl 2> $O/s13.err || { tail -5 $O/s13.err; exit 1; }
tail -1 $O/shipped_d13_auto.jsonl
timeout -k 10 200 python -u tools/mcraft_shipped.py 12 full > $O/shipped_d12_full.jsonl 2> $O/s12.err || { tail -5 $O/s12.err; exit 1; }
tail -1 $O/shipped_d12_full.jsonl
timeout -k 10 200 raft.tla_amd/bin/rmc-tlc -builtin-raft -depth 13 tests/golden/models/MCunbounded.tla > $O/cli_mcraft_shipped_depth13.txt 2>&1; echo "cli rc $?"
tail -6 $O/cli_mcraft_shipped_depth13.txt
