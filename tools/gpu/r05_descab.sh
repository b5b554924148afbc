# Round 5: A/B of the batch-prefetched lane descriptors (this tree) against the
# previous build (RMC_LIB=librmc_base.so), alternated on one box; MCraftBench and XL.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/descab; mkdir -p $O
for r in 1 2; do
  RMC_LIB=librmc_base.so timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/base_$r.json 2> $O/base_$r.err || exit 1
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/new_$r.json 2> $O/new_$r.err || exit 1
done
RMC_LIB=librmc_base.so timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/xl_base.json 2> $O/xl_base.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/xl_new.json 2> $O/xl_new.err || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['fp_salt_crosscheck']['agrees'])"; done
