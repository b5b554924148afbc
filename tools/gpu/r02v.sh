# SYMMETRY kernel evidence: rocprofv3 kernel trace and FETCH/WRITE passes of the
# MCraftBench-bounds symmetry search (tools/sym_bench.py runs it 3 times, plus
# the MaxMsgs-2 model 3 times).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P=gpurun_out/prof_sym
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 tools/sym_bench.py default 300000000 > $P/kt.jsonl 2> $P/kt.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $P/fetch -o fetch -- python3 tools/sym_bench.py default 300000000 > $P/fetch.jsonl 2> $P/fetch.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $P/write -o write -- python3 tools/sym_bench.py default 300000000 > $P/write.jsonl 2> $P/write.err || exit 1
