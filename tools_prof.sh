set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof3
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --config specs/MCraftBounded.cfg --capacity 100000000"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
for bt in 8 4; do
RMC_BATCH=$bt timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu --capacity 100000000 > gpurun_out/bench_b$bt.json || exit 1
RMC_BATCH=$bt timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu --config specs/MCraftBench.cfg --capacity 1500000000 > gpurun_out/benchC_b$bt.json || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof3/sq -o sq --output-format csv -- $B > gpurun_out/prof3/sq.log 2>&1 || exit 1
