#!/bin/bash
# Round 3: why the sharded kernel loses the diamond's gain — instruction and
# wait counters of the sharded kernel without (4) and with (5) diamond
# skipping, and of the unsharded kernel, one rank, MCraftBench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P=gpurun_out/pmc_i
mkdir -p $P
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
for v in single d4 d5 d6; do
  case $v in single) X="";; d4) X="--force-dist"; export RMC_DIST_VARIANT=4;; d5) X="--force-dist"; export RMC_DIST_VARIANT=5;; d6) X="--force-dist"; export RMC_DIST_VARIANT=6;; esac
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM -d $P/${v}_i -o i -- python3 bench.py $B $X > $P/${v}_i.json 2> $P/${v}_i.err || exit 1
  python3 tools/pmc_totals.py $P/${v}_i ${v}_insts >> $P/totals.jsonl || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES -d $P/${v}_w -o w -- python3 bench.py $B $X > $P/${v}_w.json 2> $P/${v}_w.err || exit 1
  python3 tools/pmc_totals.py $P/${v}_w ${v}_waits >> $P/totals.jsonl || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/${v}_f -o f -- python3 bench.py $B $X > $P/${v}_f.json 2> $P/${v}_f.err || exit 1
  python3 tools/pmc_totals.py $P/${v}_f ${v}_fetch >> $P/totals.jsonl || exit 1
done
