# Class-sorted flushes + lane-superset walk (RMC_EXPAND_VARIANT 4 uncapped, 5 at
# 5 waves/SIMD) vs 1: parity of each on the BFS fixtures, then same-box A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VARS="1 4 5" bash tools/gpu/ab_variant.sh > /dev/null || exit 1
mkdir -p gpurun_out/r02l && cp gpurun_out/ab/* gpurun_out/r02l/ || exit 1
