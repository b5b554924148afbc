# Round 2, first box: GPU suite on the current build, counter list, probe-rate
# calibration over table sizes, FETCH_SIZE per random probe, k_expand counters.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_cal.py > $O/probe_cal.jsonl 2> $O/probe_cal.err || exit 1
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
P="python3 tools/probe_cal.py --modes 0 --accesses 1073741824"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pcal_f64g -o f -- $P --sizes-mb 65536 > $O/pcal_f64g.out 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pcal_rq64g -o r -- $P --sizes-mb 65536 > $O/pcal_rq64g.out 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pcal_f256m -o f -- $P --sizes-mb 256 > $O/pcal_f256m.out 2>&1 || exit 1
A="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o sq -- python3 bench.py $A > $O/sq.json 2> $O/sq.err || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum --output-format csv -d $O/tcc -o tcc -- python3 bench.py $A > $O/tcc.json 2> $O/tcc.err || exit 1
