#!/bin/bash
# Round 3: same-box A/B of the expansion kernel (diamond skipping on/off,
# variants 6/7, grid 1024 = the resident blocks vs 2048), then the sizing of the
# next MCraft bounds up (is MCraftBench the largest single-GPU model?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py $A > gpurun_out/r03f_$name.json 2> gpurun_out/r03f_$name.err || return $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03f_$name.json')); r=d['roofline']; print(json.dumps({'ab':'$name','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated'],'depth':d['config']['depth']}))" >> gpurun_out/r03f_ab.jsonl
}
run v6 RMC_EXPAND_VARIANT=6 && run v6_nodia RMC_EXPAND_VARIANT=6 RMC_DIAMOND=0 && run v7 RMC_EXPAND_VARIANT=7 \
  && run v7_g1024 RMC_EXPAND_VARIANT=7 RMC_EXPAND_GRID=1024 && run v6_g1024 RMC_EXPAND_VARIANT=6 RMC_EXPAND_GRID=1024 \
  && run v6_nodia2 RMC_EXPAND_VARIANT=6 RMC_DIAMOND=0 && run v6b RMC_EXPAND_VARIANT=6 || exit $?
timeout -k 10 200 python -u tools/sym_bench.py default 300000000 > gpurun_out/r03f_sym.jsonl 2> gpurun_out/r03f_sym.err || exit $?
timeout -k 10 600 python tools/sizing.py 3:2:3:2:3:1:spill 3:2:2:1:4:1:spill --budget 200 > gpurun_out/r03f_sizing.jsonl 2> gpurun_out/r03f_sizing.err
