set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_sim.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 120 $B -depth 40 -checkpoint gpurun_out/bench.ckpt specs/MCraftBench.tla > gpurun_out/cli_ckpt1.txt 2>&1 || exit 1
timeout -k 10 120 $B -recover gpurun_out/bench.ckpt specs/MCraftBench.tla > gpurun_out/cli_ckpt2.txt 2>&1 || exit 1
rm -f gpurun_out/bench.ckpt
