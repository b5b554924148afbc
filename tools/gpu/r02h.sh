# Spill at MCraftBench scale, then a kernel-trace profile of the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 300 python -u tools/spill_demo.py > $O/spill_demo.jsonl 2> $O/spill_demo.err || exit 1
