# Round 5: 96-bit fingerprints (k + the folded second sum) — the XL model under three
# salts, the whole GPU suite, the bench lines of both bench models, config 3 A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/fp; mkdir -p $O
timeout -k 10 200 python -u tools/xl_salts.py > $O/xl_salts.jsonl 2> $O/xl_salts.err || { tail -20 $O/xl_salts.err; exit 1; }
cat $O/xl_salts.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect "tests/test_gpu.py::test_bench_model_prefix_equals_oracle[MCraftBenchXL.cfg-benchxl_prefix22]" --deselect "tests/test_gpu.py::test_bench_model_prefix_equals_oracle[MCraftBenchXL.cfg-benchxl_prefix24]" > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/bench_xl.json 2> $O/bench_xl.err || { tail -20 $O/bench_xl.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 1 --config specs/MCraftBench.cfg > $O/bench_mc.json 2> $O/bench_mc.err || { tail -20 $O/bench_mc.err; exit 1; }
for f in bench_xl bench_mc; do python -c "import json; d=json.load(open('$O/$f.json')); print('$f', round(d['ms_per_step'],1), round(d['value']/1e9,3), 'G/s kernel', round(d['roofline']['kernel_ms_per_step'],1), d['roofline']['frac_of_probe_ceiling'], d['config']['fp_salt_crosscheck'], d['config'].get('spill'))"; done
for v in 19 15 1; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 ./raft.tla_amd/bin/rmc-tlc -builtin-raft -nospill -depth 20 specs/MCraft5.tla > $O/s5_v$v.txt 2>&1 || { tail $O/s5_v$v.txt; exit 1; }
  echo "variant $v"; grep -E "distinct states found|Finished in|states/s" $O/s5_v$v.txt | head -3
done
