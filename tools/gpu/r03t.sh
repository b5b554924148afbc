#!/bin/bash
# Round 3: lane-code variants with the per-family dispatch chain (abtest/):
# c1 = per-lane descriptors only, c2 = + branch-light Receive, c3 = + branch-
# light family bodies (the default build).  Parity suite on the default, then
# the bench model, config 3 (S = 5, depth 20) and config 4 (simulation) on each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_sim.py -m gpu > gpurun_out/r03t_gpu.log 2>&1 || exit $?
for v in c1 c2 c3 c1 c2 c3; do
  timeout -k 10 200 python tools/ab_bench.py librmc_$v.so > gpurun_out/r03t_ab_$v.json 2> gpurun_out/r03t_ab_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r03t_ab_$v.json')); r=d['roofline']; print(json.dumps({'ab':'$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/r03t_ab.jsonl
  timeout -k 10 200 python tools/ab_model.py abtest/librmc_$v.so specs/MCraft5.cfg 20 >> gpurun_out/r03t_s5.jsonl 2>> gpurun_out/r03t_s5.err || exit $?
  timeout -k 10 200 python tools/ab_model.py abtest/librmc_$v.so specs/MCraftSmoke.cfg 0 sim >> gpurun_out/r03t_sim.jsonl 2>> gpurun_out/r03t_sim.err || exit $?
done
