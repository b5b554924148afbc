#!/bin/bash
# Round 3: per-level latency of the sharded loop at one rank (RCCL loopback)
# against the unsharded loop, on small models whose levels are latency-bound.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 20 --warmup 3 --no-cpu --no-probe-ceiling --capacity 50000000 --cpu-fixpoint="
for cfg in MCraftTiny2 MCraftSmall MCraftBounded; do
  timeout -k 10 200 python bench.py $A --config specs/$cfg.cfg > gpurun_out/lat_${cfg}_single.json 2> gpurun_out/lat_${cfg}_single.err || exit $?
  timeout -k 10 200 python bench.py $A --config specs/$cfg.cfg --force-dist > gpurun_out/lat_${cfg}_dist1.json 2> gpurun_out/lat_${cfg}_dist1.err || exit $?
done
