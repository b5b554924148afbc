#!/bin/bash
# Round 3: owner hash over all server words (RMC_OWNER=3) vs servers 0+1 (2):
# sharded parity after the owner-code change, then the bench model sharded 8
# ways over gloo with RMC_OWNER=3 and per-round logs (cost-model input).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -m gpu -k "not full" > gpurun_out/r03z_dist.log 2>&1 || exit $?
RMC_OWNER=3 timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_dist.py -m gpu -k "matches_oracle" > gpurun_out/r03z_dist_own3.log 2>&1 || exit $?
RMC_OWNER=3 RMC_DIST_DEBUG=1 OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node=8 \
  --master-addr 127.0.0.1 --master-port 29828 tests/dist_worker.py --cfg specs/MCraftBench.cfg \
  --out gpurun_out/r03z_dist8_own3.json --device 0 --backend gloo --capacity 180000000 \
  --keys-per-dest $((1 << 22)) --rerun 0 > gpurun_out/r03z_dist8_own3.out 2> gpurun_out/r03z_dist8_own3.err
