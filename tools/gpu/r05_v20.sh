# Round 5: dynamic per-wave units (variant 20) as the default — parity subset,
# then MCraftBench alternated with variant 19.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05/v20; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -k "level or prefix or golden or config3 or violation or parity or oracle or spill or trace" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in 19 20; do
    RMC_EXPAND_VARIANT=$v timeout -k 10 200 python -u bench.py --config specs/MCraftBench.cfg --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/mcb_v${v}_$r.json 2> $O/mcb_v${v}_$r.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])"; done
