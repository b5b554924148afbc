#!/bin/bash
# Round 3: sharded-path parity (gloo ranks sharing the GPU, 1-rank RCCL), the
# self-launching bench, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_dist.py tests/test_bench_launch.py -m gpu > gpurun_out/r03a_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-dist --no-cpu > gpurun_out/r03a_bench_dist1.json 2> gpurun_out/r03a_bench_dist1.err
