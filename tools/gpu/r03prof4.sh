#!/bin/bash
# Round 3, fourth build: rocprofv3 passes of the default expansion kernel kept
# as databases for tools/prof_summary.py (kernel trace, FETCH, WRITE,
# instruction mix, waits).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
P=gpurun_out/prof
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 bench.py $B > $P/kt.json 2> $P/kt.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch -- python3 bench.py $B > $P/fetch.json 2> $P/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/write -o write -- python3 bench.py $B > $P/write.json 2> $P/write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES -d $P/insts -o insts -- python3 bench.py $B > $P/insts.json 2> $P/insts.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d $P/stall -o stall -- python3 bench.py $B > $P/stall.json 2> $P/stall.err || exit 1
du -sh $P
