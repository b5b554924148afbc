#!/bin/bash
# Round 3: the per-lane probe issue (PIPE) now default (expand variant 6) vs
# the same kernel issuing after the batch (14); sharded at one rank: markers
# + diamonds (6) vs the same with PIPE (8).  Bench model, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for v in 6 14 6 14; do
  RMC_EXPAND_VARIANT=$v timeout -k 10 200 python bench.py $A > gpurun_out/pipe3_v$v.json 2> gpurun_out/pipe3_v$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pipe3_v$v.json')); r=d['roofline']; print(json.dumps({'ab':'expand v$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/pipe3.jsonl
done
for v in 6 8 6 8; do
  RMC_DIST_VARIANT=$v timeout -k 10 300 python bench.py $A --force-dist > gpurun_out/pipe3_d$v.json 2> gpurun_out/pipe3_d$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/pipe3_d$v.json')); print(json.dumps({'ab':'dist v$v','ms':d['ms_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/pipe3.jsonl
done
