#!/bin/bash
# Round 3: probe loads issued during the lane code (variants 11: per lane, 13: 11 + next-state prefetch,
# 12: per half batch) against the default 6, bench model, alternating; then
# the same on config 3's shape is not needed (bench shape only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for v in 6 11 13 6 11 13 6 11 13; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 python bench.py $A > gpurun_out/pipe2_v$v.json 2> gpurun_out/pipe2_v$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pipe2_v$v.json')); r=d['roofline']; print(json.dumps({'ab':'v$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/pipe2.jsonl
done
