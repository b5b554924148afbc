set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for om in 2; do
RMC_OWNER=$om timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 2957$om tests/dist_worker.py --cfg specs/MCraftBounded.cfg --out gpurun_out/balance8_owner$om.json --device 0 --backend gloo --chunk 2097152 --cap-per-dest 4194304 --capacity 30000000 --rerun 0 > gpurun_out/balance8_owner$om.log 2>&1 || exit 1
done
