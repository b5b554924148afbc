# Round 5: compact wide records and the simulator's faster
# TLC draw — wide + ABI tests, then MCraft.cfg as shipped under growing depth
# bounds (compact and full records), then the simulator's three draw modes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/wide5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_wide.py tests/test_abi.py -k "not without_gpu" -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/mcraft_shipped.py 11 full > $O/shipped_d11_full.jsonl 2> $O/shipped_full.err || { tail -5 $O/shipped_full.err; exit 1; }
tail -1 $O/shipped_d11_full.jsonl
timeout -k 10 400 python -u tools/mcraft_shipped.py 17 compact > $O/shipped_d17_compact.jsonl 2> $O/shipped_compact.err || { tail -5 $O/shipped_compact.err; exit 1; }
tail -3 $O/shipped_d17_compact.jsonl
for m in 2 1 0; do timeout -k 10 300 python tools/sim_ab.py 4194304 $m 1 RMC_WSIM_INPLACE=1 >> $O/modes.jsonl || exit 1; done
cat $O/modes.jsonl
