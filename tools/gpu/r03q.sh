#!/bin/bash
# Round 3 final: the whole GPU suite, smoke(), the default bench line (probe
# ceiling + CPU baseline), CLI transcripts of configs 1-5 (+ -gpus 1 -verify,
# the reference's MCraft layout under -depth), for profiles/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/r03q_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q_smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r03q_bench.json 2> gpurun_out/r03q_bench.err || exit $?
timeout -k 10 120 $B -builtin-raft specs/MCraftBench.tla > gpurun_out/r03q_cli_config1.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft specs/MCraftBenchSym.tla > gpurun_out/r03q_cli_config2_bench_bounds.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -depth 20 specs/MCraft5.tla > gpurun_out/r03q_cli_config3.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -simulate num=16777216 -seed 1 specs/MCraftSmoke.tla > gpurun_out/r03q_cli_config4.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft specs/MCraftBug.tla > gpurun_out/r03q_cli_config5.txt 2>&1; test $? -eq 12 || exit 1
timeout -k 10 200 $B -builtin-raft -verify specs/MCraftBench.tla > gpurun_out/r03q_cli_config1_verify.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -depth 3 tests/golden/models/MCunbounded.tla > gpurun_out/r03q_cli_mcraft_as_shipped_depth3.txt 2>&1 || exit $?
