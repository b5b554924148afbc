# bench.py after the transport-label change: default line and one-rank sharded line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02x
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
timeout -k 10 200 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 2 --warmup 1 > $O/bench_dist1.json 2> $O/bench_dist1.err || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
