set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B=raft.tla_amd/bin/rmc-tlc
export RMC_BUILTIN_RAFT=1  # the GPU box has no raft.tla: the compiled-in lemmy/raft.tla (said in the output)
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_sim.py -k "cli or sim" -x -v --timeout 240 --timeout-method thread > gpurun_out/cli_tests.log 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBench.tla > gpurun_out/cli_config1.txt 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBoundedSym.tla > gpurun_out/cli_config2.txt 2>&1 || exit 1
timeout -k 10 120 $B -depth 20 specs/MCraft5.tla > gpurun_out/cli_config3.txt 2>&1 || exit 1
timeout -k 10 200 $B -depth 20 -verify -fpmem 32G specs/MCraft5.tla > gpurun_out/cli_config3_verify.txt 2>&1 || exit 1
timeout -k 10 120 $B -simulate num=16777216 -seed 1 specs/MCraftSmoke.tla > gpurun_out/cli_config4.txt 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftBug.tla > gpurun_out/cli_config5.txt 2>&1; test $? -eq 12 || exit 1
