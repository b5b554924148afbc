set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof4
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit 1
timeout -k 10 120 python -u -c "
import sys; sys.path.insert(0,'raft.tla_amd'); import rmc
for tb in (2<<30, 64<<30):
  for mode in (0,1):
    print(tb>>30, 'GB', ['load','cas'][mode], rmc.probe_bench(0, tb, 1<<32, mode)/1e9, 'G/s', flush=True)
" > gpurun_out/probe_bench.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/kt -o kt --output-format csv -- $B > gpurun_out/prof4/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof4/fetch -o fetch --output-format csv -- $B > gpurun_out/prof4/fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof4/write -o write --output-format csv -- $B > gpurun_out/prof4/write.log 2>&1 || exit 1
