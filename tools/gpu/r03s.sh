#!/bin/bash
# Round 3: branch-light lane code (default build): single-GPU parity suite,
# then same-box A/B of the builds under abtest/ (desc = per-lane descriptors; r = + branch-light Receive; rf = + branch-light family bodies
# only, bl = descriptors + branch-light delta/diamond code), then the CLI
# transcripts of configs 1-5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_sim.py -m gpu > gpurun_out/r03s_gpu.log 2>&1 || exit $?
for v in desc r rf desc r rf; do
  timeout -k 10 200 python tools/ab_bench.py librmc_$v.so > gpurun_out/r03s_ab_$v.json 2> gpurun_out/r03s_ab_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r03s_ab_$v.json')); r=d['roofline']; print(json.dumps({'ab':'$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/r03s_ab.jsonl
done
