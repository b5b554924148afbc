set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_dist.py -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for kc in 1 0 1; do
RMC_KEY_CACHE=$kc timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling > gpurun_out/bench_kc$kc.json 2> gpurun_out/bench_kc$kc.err || exit 1
done
