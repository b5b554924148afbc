#!/bin/bash
# Round 3: grid A/B for the every-lane kernel (S = 5 depth 20: resident 1280
# vs 2048 vs 4096 blocks), the sorted kernel (resident 1024 vs 2048), the
# unconditional-probe variant 9, and the sharded kernels at 2048.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp raft.tla_amd/lib/librmc.so /tmp/librmc_cur.so
mkdir -p abtest && cp raft.tla_amd/lib/librmc.so abtest/librmc_cur.so
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for i in 1 2; do
  for g in 0 2048 4096; do
    if [ $g = 0 ]; then E=""; else E="RMC_EXPAND_GRID=$g"; fi
    env $E timeout -k 10 200 python tools/ab_model.py abtest/librmc_cur.so specs/MCraft5.cfg 20 | sed "s/^{/{\"grid\": $g, /" >> gpurun_out/r03v_s5.jsonl || exit $?
  done
  for v in base v9 g2048 d6 d6g2048; do
    case $v in base) E=""; X="";; v9) E="RMC_EXPAND_VARIANT=9"; X="";; g2048) E="RMC_EXPAND_GRID=2048"; X="";;
      d6) E="RMC_DIST_VARIANT=6"; X="--force-dist";; d6g2048) E="RMC_DIST_VARIANT=6 RMC_EXPAND_GRID=2048"; X="--force-dist";; esac
    env $E timeout -k 10 200 python bench.py $A $X > gpurun_out/r03v_$v.json 2> gpurun_out/r03v_$v.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/r03v_$v.json')); r=d['roofline']; print(json.dumps({'ab':'$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'distinct':d['config']['distinct']}))" >> gpurun_out/r03v_ab.jsonl
  done
done
