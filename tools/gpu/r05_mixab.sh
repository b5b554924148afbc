# Round 5: A/B of the fingerprint mix: the shipped mix64 vs a
# candidate build (RMC_LIB=librmc_cheapmix.so), alternated on one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/mixab; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/base_$r.json 2> $O/base_$r.err || exit 1
  RMC_LIB=librmc_cheapmix.so timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/cheap_$r.json 2> $O/cheap_$r.err || exit 1
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['generated'], d['config']['fp_salt_crosscheck']['agrees'])"; done
