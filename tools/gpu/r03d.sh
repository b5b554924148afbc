#!/bin/bash
# Round 3: (1) bench.py --gpus 2 self-launching on the one-GPU box (host
# transport, ranks share the GPU): the full bench model's counts; (2) the bench
# model on 4 and 8 ranks sharing the GPU over gloo, with per-round exchange
# logs (RMC_DIST_DEBUG): the keys/states each rank sends at 4 and 8 ranks, the
# input of DESIGN.md's 8-GPU cost model.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 2 --transport host --steps 1 --warmup 0 --no-cpu > gpurun_out/r03d_bench2.json 2> gpurun_out/r03d_bench2.err || exit $?
for n in 4 8; do
  RMC_DIST_DEBUG=1 OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
    --master-addr 127.0.0.1 --master-port 2980$n tests/dist_worker.py --cfg specs/MCraftBench.cfg \
    --out gpurun_out/r03d_dist$n.json --device 0 --backend gloo --capacity $((1600000000 / n)) \
    --keys-per-dest $((1 << 22)) --rerun 0 --sent-cache $((1 << 27)) > gpurun_out/r03d_dist$n.out 2> gpurun_out/r03d_dist$n.err || exit $?
done
