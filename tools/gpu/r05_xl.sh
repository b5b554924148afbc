# Round 5: the XL bench model (spill, trace links in HBM) — tests, bench, level times,
# and config 3 (S = 5) on the sorted kernel (A/B of expansion variants).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/xl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k 'spill or bench_model_prefix' > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/bench_xl.json 2> $O/bench_xl.err || { tail -20 $O/bench_xl.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_xl.json')); print('XL', round(d['ms_per_step'],1), round(d['value']/1e9,3), 'G/s kernel', round(d['roofline']['kernel_ms_per_step'],1), d['config']['spill'], d['roofline']['frac_of_probe_ceiling'], d['config']['fp_salt_crosscheck'])"
timeout -k 10 300 python -u tools/level_times.py specs/MCraftBenchXL.cfg 0 0 spill > $O/levels_MCraftBenchXL.jsonl 2> $O/levels.err || exit 1
tail -1 $O/levels_MCraftBenchXL.jsonl
for v in 19 15 1; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 ./raft.tla_amd/bin/rmc-tlc -nospill -depth 20 specs/MCraft5.tla > $O/s5_v$v.txt 2>&1 || { tail $O/s5_v$v.txt; exit 1; }
  echo "variant $v"; grep -E "distinct states found|Finished in|states/s" $O/s5_v$v.txt | head -3
done
