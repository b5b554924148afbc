# k_expand_sort at 5 waves/SIMD (384-entry lists, 48 B spills; RMC_EXPAND_VARIANT 8) vs 6.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VARS="6 8" bash tools/gpu/ab_variant.sh > /dev/null || exit 1
mkdir -p gpurun_out/r02s && cp gpurun_out/ab/* gpurun_out/r02s/ || exit 1
