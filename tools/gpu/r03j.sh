#!/bin/bash
# Round 3: sharded parity after the owner-routing change (owner from the
# fingerprint's own word mixes), then r03i's counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py -m gpu -k "not full" > gpurun_out/r03j_dist.log 2>&1 || exit $?
bash tools/gpu/r03i.sh
