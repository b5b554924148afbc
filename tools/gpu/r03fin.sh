#!/bin/bash
# Round 3 final check of the shipped build: the whole GPU suite, smoke(), the
# default bench line, the self-launched 2-rank bench (host transport), CLI
# -gpus 1 with -verify and a checkpoint/recover pair.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/fin_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || exit $?
timeout -k 10 120 $B -builtin-raft -gpus 1 -verify specs/MCraftBounded.tla > gpurun_out/fin_cli_gpus1_verify.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -depth 30 -checkpoint /tmp/ck_fin specs/MCraftBounded.tla > gpurun_out/fin_cli_ckpt.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -recover /tmp/ck_fin specs/MCraftBounded.tla > gpurun_out/fin_cli_recover.txt 2>&1 || exit $?
rm -f /tmp/ck_fin*
