# bench.py's multi-rank path end to end on the one-GPU box: 2 ranks sharing the
# GPU over gloo (host transport), the same JSON line the driver's scaling run prints.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29681 bench.py --gpus 2 --dist-backend gloo --device 0 --steps 1 --warmup 0 --capacity 800000000 --sent-cache 268435456 --keys-per-dest 16777216 > $O/bench2.json 2> $O/bench2.err || exit 1
