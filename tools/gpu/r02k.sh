# Wave-aggregated tie queue: symmetry parity + A/B (RMC_SYM_VARIANT 0/1), then
# the plain expansion with the delta loop rolled (RMC_EXPAND_VARIANT 3) vs 1,
# each after its own parity run; an instruction-cache counter pass for both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "sym or kat" > $O/tests_sym.log 2>&1 || exit 1
RMC_SYM_VARIANT=0 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "sym or kat" > $O/tests_sym0.log 2>&1 || exit 1
for r in 1 2; do for v in 0 1; do
  RMC_SYM_VARIANT=$v timeout -k 10 120 python -u tools/sym_bench.py default 300000000 > $O/sym_v${v}_r$r.jsonl 2> $O/sym_v${v}_r$r.err || exit 1
done; done
O=gpurun_out/r02k VARS="1 3" bash tools/gpu/ab_variant.sh > /dev/null || exit 1
cp gpurun_out/ab/* $O/ || exit 1
for v in 1 3; do
  RMC_EXPAND_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d $O/ic$v -o ic -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-probe-ceiling > $O/ic$v.json 2> $O/ic$v.err || exit 1
done
