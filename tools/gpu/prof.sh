set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt -- python3 bench.py $A > gpurun_out/prof/kt.json 2> gpurun_out/prof/kt.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o fetch -- python3 bench.py $A > gpurun_out/prof/fetch.json 2> gpurun_out/prof/fetch.err || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o write -- python3 bench.py $A > gpurun_out/prof/write.json 2> gpurun_out/prof/write.err || exit 1
