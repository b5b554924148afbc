# Round 5: the wave simulator with the wave-cooperative apply / invariants —
# wide tests (incl. wave == thread behaviours) and Smokeraft's walks timed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/wsim; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/sim_wide.py 4194304 > $O/sim_wide.jsonl 2> $O/sim_wide.err || { tail -20 $O/sim_wide.err; exit 1; }
cat $O/sim_wide.jsonl
