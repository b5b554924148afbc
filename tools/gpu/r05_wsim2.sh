# Round 5: wide simulator after the wave apply — wide tests, then the three draw modes timed.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/wsim2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for m in 2 1 0; do timeout -k 10 300 python tools/sim_ab.py 4194304 $m 1 RMC_WSIM_INPLACE=1 >> $O/modes.jsonl || exit 1; done
cat $O/modes.jsonl
