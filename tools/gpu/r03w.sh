#!/bin/bash
# Round 3: the final lane code (per-lane descriptors, branchy family bodies)
# with expansion grids from occupancy, the capacity pass out of the hot
# kernels, footprints only for the sorted shapes: the whole GPU suite, the bench model,
# config 3 (S = 5, depth 20) and config 4 timing, and the sharded kernel with
# and without diamond skipping at one rank.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/r03w_tests.log 2>&1 || exit $?
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for i in 1 2; do
  timeout -k 10 200 python bench.py $A > gpurun_out/r03w_single$i.json 2> gpurun_out/r03w_single$i.err || exit $?
  timeout -k 10 200 python tools/ab_model.py abtest/librmc_final.so specs/MCraft5.cfg 20 >> gpurun_out/r03w_s5.jsonl 2>> gpurun_out/r03w_s5.err || exit $?
  timeout -k 10 200 python tools/ab_model.py abtest/librmc_final.so specs/MCraftSmoke.cfg 0 sim >> gpurun_out/r03w_sim.jsonl 2>> gpurun_out/r03w_sim.err || exit $?
  timeout -k 10 200 python tools/sym_bench.py default 300000000 >> gpurun_out/r03w_sym.jsonl 2>> gpurun_out/r03w_sym.err || exit $?
  timeout -k 10 200 python bench.py $A --force-dist > gpurun_out/r03w_d6_$i.json 2> gpurun_out/r03w_d6_$i.err || exit $?
  RMC_DIST_VARIANT=7 timeout -k 10 200 python bench.py $A --force-dist > gpurun_out/r03w_d7b_$i.json 2> gpurun_out/r03w_d7b_$i.err || exit $?
done
