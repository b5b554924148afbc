#!/bin/bash
# Round 3 final check, fourth build (probe loads issued during the lane code):
# the whole GPU suite, smoke(), the default bench line, SYMMETRY, the one-rank
# sharded bench, then rocprofv3: kernel trace + FETCH/WRITE/instruction passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/fin4_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin4_smoke.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/fin4_bench.json 2> gpurun_out/fin4_bench.err || exit $?
timeout -k 10 200 python tools/sym_bench.py default 300000000 > gpurun_out/fin4_sym.jsonl 2> gpurun_out/fin4_sym.err || exit $?
timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu --no-probe-ceiling --force-dist > gpurun_out/fin4_dist1.json 2> gpurun_out/fin4_dist1.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
P=gpurun_out/prof4
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 bench.py $B > $P/kt.json 2> $P/kt.err || exit 1
find $P/kt -name "*.db" -delete
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch -- python3 bench.py $B > $P/fetch.json 2> $P/fetch.err || exit 1
python3 tools/pmc_totals.py $P/fetch fetch >> $P/totals.jsonl || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/write -o write -- python3 bench.py $B > $P/write.json 2> $P/write.err || exit 1
python3 tools/pmc_totals.py $P/write write >> $P/totals.jsonl || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES -d $P/insts -o insts -- python3 bench.py $B > $P/insts.json 2> $P/insts.err || exit 1
python3 tools/pmc_totals.py $P/insts insts >> $P/totals.jsonl || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d $P/stall -o stall -- python3 bench.py $B > $P/stall.json 2> $P/stall.err || exit 1
python3 tools/pmc_totals.py $P/stall waits >> $P/totals.jsonl || exit 1
