#!/bin/bash
# Round 3: cost-model inputs for the final build: per-level times of the
# unsharded bench BFS, and the bench model sharded 8 ways over gloo on this one
# GPU with per-round exchange logs (RMC_DIST_DEBUG).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/level_times.py specs/MCraftBench.cfg > gpurun_out/r03y_levels.jsonl 2> gpurun_out/r03y_levels.err || exit $?
RMC_DIST_DEBUG=1 OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29818 tests/dist_worker.py --cfg specs/MCraftBench.cfg \
  --out gpurun_out/r03y_dist8.json --device 0 --backend gloo --capacity 180000000 \
  --keys-per-dest $((1 << 22)) --rerun 0 > gpurun_out/r03y_dist8.out 2> gpurun_out/r03y_dist8.err
