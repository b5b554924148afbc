#!/bin/bash
# Round 3: sharded suite after the idle-round skip and the priority stream,
# then A/B: unsharded default vs 16-tile windows (variant 8), one-rank sharded.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -m gpu -k "not full" > gpurun_out/r03n_dist.log 2>&1 || exit $?
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
run() {  # name, extra bench args, env...
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py $A $extra > gpurun_out/r03n_$name.json 2> gpurun_out/r03n_$name.err || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03n_$name.json')); r=d['roofline']; s=d.get('sharded') or {}; print(json.dumps({'ab':'$name','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated'],'depth':d['config']['depth'],'rounds':s.get('chunks_rank0'),'xfer_s':s.get('exchange_s_rank0')}))" >> gpurun_out/r03n_ab.jsonl
}
run single "" && run wt16 "" RMC_EXPAND_VARIANT=8 && run dist1 --force-dist && run single_b "" && run wt16_b "" RMC_EXPAND_VARIANT=8 && run dist1_b --force-dist
