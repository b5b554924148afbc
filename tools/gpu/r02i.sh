# SYMMETRY orbit rate vs fingerprint-set size; bench-model rate vs set size.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 200 python -u tools/sym_bench.py default 0 > $O/sym_auto.jsonl 2> $O/sym_auto.err || exit 1
timeout -k 10 200 python -u tools/sym_bench.py default 300000000 > $O/sym_3e8.jsonl 2> $O/sym_3e8.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 --capacity 1600000000 > $O/b_16e8.json 2> $O/b_16e8.err || exit 1
timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 --capacity 3000000000 > $O/b_3e9.json 2> $O/b_3e9.err || exit 1
