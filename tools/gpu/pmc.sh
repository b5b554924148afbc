# rocprofv3 evidence for the bench command (the build in the tree):
# a kernel trace with stats, then one PMC pass per counter group (separate
# runs: FETCH_SIZE and WRITE_SIZE alone, instruction mix, waits, LDS, atomics).
#   OUT=gpurun_out/<tag> [ENVS="RMC_EXPAND_VARIANT=7"] [CMD="raft.tla_amd/bin/rmc-tlc ..."] bash tools/gpu/pmc.sh
# (CMD replaces the bench command; it must be the program itself, no wrapper)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=${OUT:-gpurun_out/pmc}
mkdir -p $P
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling --v2-config= ${BENCH_ARGS}"
C=${CMD:-python3 bench.py $B}
for v in $ENVS; do export $v; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- $C > $P/kt.json 2> $P/kt.err || exit 1
find $P/kt -name "*.db" -delete
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d $P/$name -o $name -- $C > $P/$name.json 2> $P/$name.err || exit 1
  python3 tools/pmc_totals.py $P/$name $name >> $P/totals.jsonl || exit 1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass insts SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES
pass waits SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
# atomics: requests at L2 (all), those that go on to memory, and their in-flight sum (latency)
pass atomics TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_EA0_ATOMIC_LEVEL_sum
