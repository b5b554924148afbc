# Targeted GPU tests: TESTS (pytest -k expression) over FILES, one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${LIMIT:-500} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -k "${TESTS}" > gpurun_out/quick.log 2>&1
rc=$?
tail -5 gpurun_out/quick.log
exit $rc
