#!/bin/bash
# Round 3: the whole GPU suite with diamond skipping, then bench lines with and
# without it (same box), and the 1-rank sharded overhead.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu.py -m gpu -k diamond > gpurun_out/r03b_diamond.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || exit $?
RMC_DIAMOND=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-probe-ceiling > gpurun_out/r03b_bench_nodia.json 2> gpurun_out/r03b_bench_nodia.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-dist --no-cpu --no-probe-ceiling > gpurun_out/r03b_bench_dist1.json 2> gpurun_out/r03b_bench_dist1.err || exit $?
timeout -k 10 1200 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests -m gpu > gpurun_out/r03b_tests.log 2>&1
