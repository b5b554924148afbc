# Round 5: the sharded pool kernel with dynamic per-wave units (RMC_DIST_KVARIANT=4)
# against 3, one rank on MCraftBench, with the unsharded line; a 2-rank parity check.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/kv4; mkdir -p $O
RMC_DIST_KVARIANT=4 timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -k "oracle or parity or level" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/plain_$r.json 2> $O/plain_$r.err || exit 1
  for v in 3 4; do
    RMC_DIST_KVARIANT=$v timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $O/kv${v}_$r.json 2> $O/kv${v}_$r.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
