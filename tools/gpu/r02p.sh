# Sharded path: parity (tests/test_dist.py -m gpu, default RMC_DIST_VARIANT 1),
# then the bench model through the sharded path at one rank on RCCL
# (bench.py --force-dist) for variants 0 and 1, twice, and the plain path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests_dist.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1; do
  RMC_DIST_VARIANT=$v timeout -k 10 200 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/fd_v${v}_r$r.json 2> $O/fd_v${v}_r$r.err || exit 1
done; done
timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/plain.json 2> $O/plain.err || exit 1
