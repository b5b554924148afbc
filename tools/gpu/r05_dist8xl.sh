# Round 5: the 8-rank rehearsal (gloo, ranks sharing the GPU) of the XL bench model's
# first 36 levels (1.4 G states) — the sharded cost model's per-rank keys and states —
# and the one-rank sharded bench against the unsharded one on MCraftBench (k_dist).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/dist8_xl
OUT=$O CFG=specs/MCraftBenchXL.cfg DEPTH=36 CAP=200000000 CAP1=1600000000 REP=1048576 bash tools/gpu/dist8.sh || { tail -30 $O/dist8.err; exit 1; }
P=gpurun_out/r05/kdist; mkdir -p $P
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $P/b_plain_$r.json 2> $P/b_plain_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $P/b_dist_$r.json 2> $P/b_dist_$r.err || exit 1
done
for f in $P/b_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
