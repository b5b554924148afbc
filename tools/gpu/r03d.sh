#!/bin/bash
# Round 3: (1) bench.py --gpus 2 self-launching on the one-GPU box (host
# transport, ranks share the GPU): the full bench model's counts; (2) owner
# balance and exchange volume at 8 ranks (gloo, ranks sharing the GPU) on the
# 78 M-state model for the two owner functions; (3) the bench model on 8 ranks
# with per-round exchange logs (RMC_DIST_DEBUG): rounds per level and keys per
# round, the input of DESIGN.md's 8-GPU cost model.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/level_times.py specs/MCraftBench.cfg > gpurun_out/r03d_levels.jsonl 2> gpurun_out/r03d_levels.err || exit $?
timeout -k 10 600 python bench.py --gpus 2 --transport host --steps 1 --warmup 0 --no-cpu > gpurun_out/r03d_bench2.json 2> gpurun_out/r03d_bench2.err || exit $?
for om in 2 1; do
  RMC_OWNER=$om OMP_NUM_THREADS=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
    --master-addr 127.0.0.1 --master-port 2981$om tests/dist_worker.py --cfg specs/MCraftBounded.cfg \
    --out gpurun_out/r03d_own${om}_w8.json --device 0 --backend gloo --capacity 20000000 \
    --keys-per-dest $((1 << 22)) --rerun 0 > gpurun_out/r03d_own$om.out 2> gpurun_out/r03d_own$om.err || exit $?
done
RMC_DIST_DEBUG=1 OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29808 tests/dist_worker.py --cfg specs/MCraftBench.cfg \
  --out gpurun_out/r03d_dist8.json --device 0 --backend gloo --capacity 180000000 \
  --keys-per-dest $((1 << 22)) --rerun 0 > gpurun_out/r03d_dist8.out 2> gpurun_out/r03d_dist8.err
