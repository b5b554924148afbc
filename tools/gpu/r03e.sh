#!/bin/bash
# Round 3: the whole GPU suite (sharded verification, checkpoints, the
# unconstrained depth-bounded model, diamonds), then r03c.sh's A/B and profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/r03e_tests.log 2>&1 || exit $?
bash tools/gpu/r03c.sh
