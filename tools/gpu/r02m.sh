# Lane-superset walk variants (RMC_EXPAND_VARIANT): 1 baseline, 4 class-sorted
# flushes, 6 class-sorted windows, 7 both: parity of each, then same-box A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VARS="1 4 6 7" bash tools/gpu/ab_variant.sh > /dev/null || exit 1
mkdir -p gpurun_out/r02m && cp gpurun_out/ab/* gpurun_out/r02m/ || exit 1
