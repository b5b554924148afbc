# Checkpoint of the build with the sharded chunk sizing from the previous
# level's worst rho: the full-size 2-rank run with per-chunk logging, the full
# GPU suite, smoke, the bench line and the one-rank sharded bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
RMC_DIST_DEBUG=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29671 tests/dist_worker.py --cfg specs/MCraftBench.cfg --out $O/full.json --device 0 --backend gloo --capacity 800000000 --keys-per-dest 16777216 --rerun 0 --sent-cache 268435456 > $O/full.out 2> $O/full.err || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
timeout -k 10 200 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/bench_dist1.json 2> $O/bench_dist1.err || exit 1
