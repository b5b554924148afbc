#!/bin/bash
# Round 3: same-box A/B of the sharded expansion kernel at one rank on RCCL
# (RMC_DIST_VARIANT 1..5) against the unsharded default (variant 6, grid
# 1024), SYMMETRY with full-size launches, then PC sampling (r03g.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
run() {  # name, extra bench args, env...
  local name=$1 extra=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py $A $extra > gpurun_out/r03h_$name.json 2> gpurun_out/r03h_$name.err || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03h_$name.json')); r=d['roofline']; s=d.get('sharded') or {}; print(json.dumps({'ab':'$name','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated'],'depth':d['config']['depth'],'rounds':s.get('chunks_rank0'),'xfer_s':s.get('exchange_s_rank0')}))" >> gpurun_out/r03h_ab.jsonl
}
run single "" && run d1 --force-dist RMC_DIST_VARIANT=1 && run d5 --force-dist RMC_DIST_VARIANT=5 \
  && run d2 --force-dist RMC_DIST_VARIANT=2 && run d3 --force-dist RMC_DIST_VARIANT=3 && run d4 --force-dist RMC_DIST_VARIANT=4 \
  && run single2 "" && run d1b --force-dist RMC_DIST_VARIANT=1 || exit $?
timeout -k 10 200 python -u tools/sym_bench.py default 300000000 > gpurun_out/r03h_sym.jsonl 2> gpurun_out/r03h_sym.err || exit $?
RMC_EXPAND_GRID=2048 timeout -k 10 200 python -u tools/sym_bench.py default 300000000 > gpurun_out/r03h_sym2048.jsonl 2> gpurun_out/r03h_sym2048.err || exit $?
# (PC sampling is not available on this pool)
