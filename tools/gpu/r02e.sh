# Config 3 sizing: per-level sizes of wider 5-server models.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 300 python -u tools/size_s5.py 3 2 4 1 > $O/s5_3241.jsonl 2> $O/s5_3241.err || exit 1
timeout -k 10 300 python -u tools/size_s5.py 3 2 3 2 > $O/s5_3232.jsonl 2> $O/s5_3232.err || exit 1
