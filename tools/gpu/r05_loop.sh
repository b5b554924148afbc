# Round 5: the sharded level loop's host wait polls without sleeping for the
# first 100 ms — one-rank sharded vs unsharded on MCraftBench, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/loop; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/plain_$r.json 2> $O/plain_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $O/dist_$r.json 2> $O/dist_$r.err || exit 1
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
