# Sharded path: the full bench model on 2 ranks (host transport) for both
# expansion variants with per-chunk logging, then the dist parity tests,
# then the bench model through the sharded path at one rank on RCCL.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02q
mkdir -p $O
for v in 0 1; do
  RMC_DIST_DEBUG=1 RMC_DIST_VARIANT=$v timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 2966$v tests/dist_worker.py --cfg specs/MCraftBench.cfg --out $O/full_v$v.json --device 0 --backend gloo --capacity 800000000 --keys-per-dest 16777216 --rerun 0 --sent-cache 268435456 > $O/full_v$v.out 2> $O/full_v$v.err
  echo "variant $v rc $?" >> $O/rc.txt
done
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests_dist.log 2>&1
echo "tests rc $?" >> $O/rc.txt
for v in 0 1; do
  RMC_DIST_VARIANT=$v timeout -k 10 200 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/fd_v$v.json 2> $O/fd_v$v.err || exit 1
done
