#!/bin/bash
# Round 3: window-sort classes A/B: roles (default, variant 6) vs roles x
# message count (variant 10), bench model, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for v in 6 10 6 10 6 10; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 python bench.py $A > gpurun_out/ab2_v$v.json 2> gpurun_out/ab2_v$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab2_v$v.json')); r=d['roofline']; print(json.dumps({'ab':'v$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/ab2.jsonl
done
