# Round 5: DropMessage first in the commuting-diamond order — parity subset,
# then MCraftBench and the XL bench with the old build (RMC_LIB=librmc_prev.so) alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05/dropfirst}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "level or prefix or golden or config3 or symmetry or violation" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  RMC_LIB=librmc_prev.so timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --steps 5 --warmup 1 > $O/prev_$r.json 2> $O/prev_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --steps 5 --warmup 1 > $O/new_$r.json 2> $O/new_$r.err || exit 1
done
RMC_LIB=librmc_prev.so timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/xl_prev.json 2> $O/xl_prev.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/xl_new.json 2> $O/xl_new.err || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['ms_per_step'],2), round(r['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['generated'], d['config']['fp_salt_crosscheck']['agrees'], r['probes_per_step'], round(r['frac_of_probe_ceiling'],3))"; done
