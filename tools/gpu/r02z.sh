# Grid size of the expansion kernels (RMC_EXPAND_GRID): 1024 (one resident
# round at 4 waves/SIMD), 2048 (default), 4096; bench runs, two rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02z
mkdir -p $O
RMC_EXPAND_GRID=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -k "bfs_matches_oracle or salt" -x -q --timeout 240 --timeout-method thread > $O/parity_1024.log 2>&1 || exit 1
for r in 1 2; do for gsz in 1024 2048 4096; do
  RMC_EXPAND_GRID=$gsz timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/b_${gsz}_$r.json 2> $O/b_${gsz}_$r.err || exit 1
  python -c "import json; d=json.load(open('$O/b_${gsz}_$r.json')); print('grid $gsz run $r', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'])" >> $O/ab.txt || exit 1
done; done
