# The sharded kernel's cost at one rank (k_dist of DESIGN.md §e), by counters:
# rocprofv3 kernel traces and one SQ instruction/wait pass of bench.py on
# MCraftBench, unsharded and --force-dist.   OUT=gpurun_out/<tag> bash tools/gpu/kdist_prof.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=${OUT:-gpurun_out/kdist_prof}
mkdir -p $P
B="--config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --v2-config="
for m in plain dist; do
  X=""; [ $m = dist ] && X=--force-dist
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt_$m -o kt -- python3 bench.py $B --steps 2 --warmup 1 $X > $P/b_$m.json 2> $P/b_$m.err || exit 1
  find $P/kt_$m -name "*kernel_trace.csv" -delete
done
for m in plain dist; do
  X=""; [ $m = dist ] && X=--force-dist
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $P/pmc_$m -o pmc -- python3 bench.py $B --steps 1 --warmup 0 $X > $P/p_$m.json 2> $P/p_$m.err || exit 1
  python3 tools/pmc_totals.py $P/pmc_$m $m >> $P/totals.jsonl || exit 1
done
cat $P/totals.jsonl
