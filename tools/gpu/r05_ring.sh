# Round 5: the ring window (spill with the trace links in HBM) — spill / bench-model
# tests, the XL bench, the one-rank sharded bench on MCraftBench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/ring; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k 'spill or bench_model_prefix or checkpoint or recover' > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/bench_xl.json 2> $O/bench_xl.err || { tail -20 $O/bench_xl.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_xl.json')); print('XL', round(d['ms_per_step'],1), round(d['value']/1e9,3), 'G/s kernel', round(d['roofline']['kernel_ms_per_step'],1), d['roofline']['launches_per_step'], d['roofline']['frac_of_probe_ceiling'], d['config']['fp_salt_crosscheck']['agrees'], d['config']['spill'])"
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/b_plain_$r.json 2> $O/b_plain_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $O/b_dist_$r.json 2> $O/b_dist_$r.err || exit 1
done
for f in $O/b_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
