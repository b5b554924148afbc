#!/bin/bash
# Round 3 final build: the default bench line (probe ceiling + CPU baseline), then
# the rocprofv3 passes of the default expansion kernel (kernel trace, FETCH,
# WRITE, instruction mix, waits, TCC, LDS) for profiles/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
P=gpurun_out/prof
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 bench.py $B > $P/kt.json 2> $P/kt.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch -- python3 bench.py $B > $P/fetch.json 2> $P/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/write -o write -- python3 bench.py $B > $P/write.json 2> $P/write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES -d $P/insts -o insts -- python3 bench.py $B > $P/insts.json 2> $P/insts.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d $P/stall -o stall -- python3 bench.py $B > $P/stall.json 2> $P/stall.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum -d $P/tcc -o tcc -- python3 bench.py $B > $P/tcc.json 2> $P/tcc.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL -d $P/lds -o lds -- python3 bench.py $B > $P/lds.json 2> $P/lds.err || exit 1
