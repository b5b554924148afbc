#!/bin/bash
# Round 3: PC sampling of the default expansion kernel (rocprofv3 stochastic
# sampling, cycles) over one MCraftBench BFS, then host-trap sampling if the
# stochastic method is unavailable.  Output: gpurun_out/pcs/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pcs
B="--steps 1 --warmup 0 --no-cpu --no-probe-ceiling"
timeout -k 10 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || true
grep -i -A12 "pc.sampl" gpurun_out/pcs/list.txt | head -60 > gpurun_out/pcs/pcs_configs.txt || true
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 65536 -d gpurun_out/pcs/st -o st --output-format csv -- python3 bench.py $B \
  > gpurun_out/pcs/st.json 2> gpurun_out/pcs/st.err
rc=$?
echo "stochastic rc=$rc" > gpurun_out/pcs/rc.txt
if [ $rc -eq 1 ] || [ $rc -eq 2 ]; then  # unsupported (not a fault, abort or time limit)
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 100 -d gpurun_out/pcs/ht -o ht --output-format csv -- python3 bench.py $B \
    > gpurun_out/pcs/ht.json 2> gpurun_out/pcs/ht.err
  echo "host_trap rc=$?" >> gpurun_out/pcs/rc.txt
fi
ls -laR gpurun_out/pcs | head -40
