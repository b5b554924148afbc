#!/bin/bash
# Round 3: branch-light lane code (default build): single-GPU parity suite,
# then same-box A/B of the builds under abtest/ (desc = per-lane descriptors
# only, bl = descriptors + branch-light delta/diamond code), then the CLI
# transcripts of configs 1-5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_sim.py -m gpu > gpurun_out/r03r_gpu.log 2>&1 || exit $?
for v in desc bl desc bl; do
  timeout -k 10 200 python tools/ab_bench.py librmc_$v.so > gpurun_out/r03r_ab_$v.json 2> gpurun_out/r03r_ab_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r03r_ab_$v.json')); r=d['roofline']; print(json.dumps({'ab':'$v','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated']}))" >> gpurun_out/r03r_ab.jsonl
done
timeout -k 10 120 $B -builtin-raft specs/MCraftBench.tla > gpurun_out/r03r_cli_config1.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft specs/MCraftBenchSym.tla > gpurun_out/r03r_cli_config2_bench_bounds.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -depth 20 specs/MCraft5.tla > gpurun_out/r03r_cli_config3.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -simulate num=16777216 -seed 1 specs/MCraftSmoke.tla > gpurun_out/r03r_cli_config4.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft specs/MCraftBug.tla > gpurun_out/r03r_cli_config5.txt 2>&1; test $? -eq 12 || exit 1
timeout -k 10 200 $B -builtin-raft -verify specs/MCraftBench.tla > gpurun_out/r03r_cli_config1_verify.txt 2>&1 || exit $?
timeout -k 10 120 $B -builtin-raft -depth 3 tests/golden/models/MCunbounded.tla > gpurun_out/r03r_cli_mcraft_as_shipped_depth3.txt 2>&1 || exit $?
