# Round 5: size candidate bench models (no spill: a model that fails with CAPACITY does
# not fit one GPU resident) and run the wide-layout tests.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r05
timeout -k 10 200 python -u -m pytest tests/test_wide.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r05/wide_tests.log 2>&1
echo "wide tests rc=$?"
timeout -k 10 500 python -u tools/sizing.py ${MODELS:-3:2:3:1:3:1 3:2:2:1:3:2 3:1:2:2:3:1 3:1:3:1:3:1 3:1:2:1:4:1 3:2:2:2:3:1 3:1:3:2:3:1} --budget 30 > gpurun_out/r05/sizing.jsonl 2> gpurun_out/r05/sizing.err
