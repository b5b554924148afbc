set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 500 python -u -m pytest tests -m gpu -k "messages or bug or kat or bounded_full or elections or cand_term or cli" -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_msg_tests.log 2>&1 || exit 1
timeout -k 10 120 $B specs/MCraftMessages.tla > gpurun_out/cli_messages.txt 2>&1; test $? -eq 12 || exit 1
timeout -k 10 120 $B specs/MCraftElections.tla > gpurun_out/cli_elections.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_msg.json 2> gpurun_out/bench_msg.err || exit 1
