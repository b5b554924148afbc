# Round 5: the pool flush (sharded kernel at the single-GPU shape) — parity, then
# same-box A/B of the one-rank sharded bench (kvariant 2 = round 4's, 3 = pool) and the
# unsharded bench; then the size of the V=1 MaxLogLen 2 model (spill, 8 G capacity).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/pool; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/b_plain_$r.json 2> $O/b_plain_$r.err || exit 1
  for v in 2 3; do
    RMC_DIST_KVARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $O/b_dist${v}_$r.json 2> $O/b_dist${v}_$r.err || exit 1
  done
done
for f in $O/b_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
timeout -k 10 400 python -u tools/sizing.py 3:1:2:2:3:1:spill:c8000000000 --budget 300 > gpurun_out/r05/sizing2.jsonl 2> gpurun_out/r05/sizing2.err
cat gpurun_out/r05/sizing2.jsonl
# S = 5 (config 3) on the sorted kernel: 19 (default, 6 waves) / 15 (5 waves, mixes held) / 1 (every lane)
for v in 19 15 1; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 ./raft.tla_amd/bin/rmc-tlc -depth 20 -nospill specs/MCraft5.cfg > $O/s5_v$v.txt 2>&1 || { tail $O/s5_v$v.txt; exit 1; }
  grep -E "distinct|Finished|states/s" $O/s5_v$v.txt | head -5
done
