# Round 5: the same-parent undo / twin rules on top of Drop-first diamonds —
# parity subset (single GPU and sharded), then MCraftBench (plain, one-rank
# sharded) and XL against the previous build (RMC_LIB=librmc_prev.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/r05/samepar}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -k "level or prefix or golden or config3 or violation or parity or oracle" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in prev new; do
    L=""; [ $v = prev ] && L=librmc_prev.so
    RMC_LIB=$L timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --steps 5 --warmup 1 > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 1
    RMC_LIB=$L timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 --force-dist > $O/${v}_dist_$r.json 2> $O/${v}_dist_$r.err || exit 1
  done
done
RMC_LIB=librmc_prev.so timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/xl_prev.json 2> $O/xl_prev.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > $O/xl_new.json 2> $O/xl_new.err || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', round(d['ms_per_step'],2), round(r['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['generated'], (d['config'].get('fp_salt_crosscheck') or {}).get('agrees'), r['probes_per_step'])"; done
