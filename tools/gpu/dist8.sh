# The 8-rank rehearsal of the sharded search on the one-GPU box (gloo host
# transport, ranks sharing the GPU): counts, and per-round exchange logs
# (RMC_DIST_DEBUG) — the input of tools/dist_cost_model.py.
#   OUT=gpurun_out/<tag> REP=<RMC_DIST_REP> [CFG=specs/X.cfg DEPTH=d CAP=<per rank> CAP1=<1 GPU>] bash tools/gpu/dist8.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/dist8}
CFG=${CFG:-specs/MCraftBench.cfg}
mkdir -p $O
timeout -k 10 180 python tools/level_times.py $CFG ${CAP1:-1500000000} ${DEPTH:-0} > $O/levels.jsonl 2> $O/levels.err || exit 1
RMC_DIST_REP=${REP:-1048576} RMC_DIST_DEBUG=1 OMP_NUM_THREADS=1 timeout -k 10 900 python -m torch.distributed.run \
  --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 --master-port 29808 tests/dist_worker.py \
  --cfg $CFG --out $O/dist8.json --device 0 --backend gloo --capacity ${CAP:-180000000} \
  --keys-per-dest $((1 << 22)) --rerun ${RERUN:-0} --max-depth ${DEPTH:-0} > $O/dist8.out 2> $O/dist8.err || exit 1
grep -h "\[rmc rank" $O/dist8.err > $O/rounds.txt
python3 -c "import json; d=json.load(open('$O/dist8.json')); print(d['distinct'], d['generated'], d['depth'], d['keys_sent'], d['states_sent'], d['rerun'])"
