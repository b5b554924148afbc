#!/bin/bash
# Round 3: the send-marker sharded kernel (RMC_DIST_VARIANT 6/7): sharded
# parity at 2-4 ranks (gloo, ranks share the GPU), then the one-rank RCCL A/B
# against variants 4/5 and the unsharded default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
RMC_DIST_VARIANT=6 timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -m gpu -k "not full and not verification" > gpurun_out/r03k_dist6.log 2>&1 || exit $?
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
run() {  # name, extra bench args, env...
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py $A $extra > gpurun_out/r03k_$name.json 2> gpurun_out/r03k_$name.err || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03k_$name.json')); r=d['roofline']; s=d.get('sharded') or {}; print(json.dumps({'ab':'$name','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated'],'depth':d['config']['depth'],'rounds':s.get('chunks_rank0'),'xfer_s':s.get('exchange_s_rank0')}))" >> gpurun_out/r03k_ab.jsonl
}
run single "" && run d6 --force-dist RMC_DIST_VARIANT=6 && run d7 --force-dist RMC_DIST_VARIANT=7 \
  && run d4 --force-dist RMC_DIST_VARIANT=4 && run d5 --force-dist RMC_DIST_VARIANT=5 && run d6b --force-dist RMC_DIST_VARIANT=6 \
  && run single2 ""
