#!/bin/bash
# Round 3 final check, third build (SYMMETRY 16-tile windows):
# the whole GPU suite, smoke(), the default bench line, SYMMETRY (default and
# 16-tile windows) and the one-rank sharded bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/fin3_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin3_smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/fin3_bench.json 2> gpurun_out/fin3_bench.err || exit $?
timeout -k 10 200 python tools/sym_bench.py default 300000000 > gpurun_out/fin3_sym.jsonl 2> gpurun_out/fin3_sym.err || exit $?

timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-probe-ceiling --force-dist > gpurun_out/fin3_dist1.json 2> gpurun_out/fin3_dist1.err || exit $?
