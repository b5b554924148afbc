# Round-2 profile of the bench command: kernel trace, HBM bytes (FETCH/WRITE,
# one counter per pass), instruction mix and stall split of k_expand, L2 hits.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
P=gpurun_out/prof2
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 bench.py $A > $P/kt.json 2> $P/kt.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch -- python3 bench.py $A > $P/fetch.json 2> $P/fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/write -o write -- python3 bench.py $A > $P/write.json 2> $P/write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES -d $P/insts -o insts -- python3 bench.py $A > $P/insts.json 2> $P/insts.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d $P/stall -o stall -- python3 bench.py $A > $P/stall.json 2> $P/stall.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_ATOMIC_sum -d $P/tcc -o tcc -- python3 bench.py $A > $P/tcc.json 2> $P/tcc.err || exit 1
