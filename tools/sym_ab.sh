set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in wpe0 wpe3 wpe0 wpe3; do
  timeout -k 10 200 python -u tools/sym_bench.py abtest/librmc_$v.so >> gpurun_out/sym_ab.jsonl 2> gpurun_out/sym_ab_$v.err || exit 1
done
timeout -k 10 300 python -u -m pytest tests -m gpu -k "sym" -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_sym.log 2>&1 || exit 1
