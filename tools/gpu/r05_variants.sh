# Round 5: the expansion-kernel variants again after the Drop-first order (fewer
# probes, same instructions) — XL bench per RMC_EXPAND_VARIANT, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/variants; mkdir -p $O
for r in 1 2; do
  for v in 19 20 18 10 15; do
    RMC_EXPAND_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu --no-probe-ceiling --steps 2 --warmup 1 > $O/v${v}_$r.json 2> $O/v${v}_$r.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['fp_salt_crosscheck']['agrees'])"; done
