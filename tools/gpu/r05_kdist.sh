# Round 5: one-rank sharded bench against the unsharded one on MCraftBench (k_dist,
# loop overhead), plus the sharded parity tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=gpurun_out/r05/kdist2; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/dist_tests.log 2>&1 || { tail -30 $P/dist_tests.log; exit 1; }
tail -1 $P/dist_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $P/b_plain_$r.json 2> $P/b_plain_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $P/b_dist_$r.json 2> $P/b_dist_$r.err || exit 1
done
for f in $P/b_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
