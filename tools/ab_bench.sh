set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in old inl noinl old inl noinl; do
  timeout -k 10 200 python -u tools/ab_bench.py librmc_$v.so > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'], d['roofline']['kernel_ms_per_step'])" >> gpurun_out/ab.txt || exit 1
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_noinl.log 2>&1 || exit 1
