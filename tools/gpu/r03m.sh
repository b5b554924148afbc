#!/bin/bash
# Round 3: the default sharded kernel is now send markers (RMC_DIST_VARIANT 7,
# fingerprint set doubled at world > 1): the whole sharded GPU suite (incl. the
# 2-rank full bench model and sharded verification), then one-rank overhead.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_dist.py tests/test_bench_launch.py -m gpu > gpurun_out/r03m_dist.log 2>&1 || exit $?
A="--steps 5 --warmup 2 --no-cpu --no-probe-ceiling"
for name in single dist1 single_b dist1_b; do
  case $name in single*) X="";; dist1*) X="--force-dist";; esac
  timeout -k 10 200 python bench.py $A $X > gpurun_out/r03m_$name.json 2> gpurun_out/r03m_$name.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r03m_$name.json')); r=d['roofline']; s=d.get('sharded') or {}; print(json.dumps({'ab':'$name','ms':d['ms_per_step'],'kernel_ms':r['kernel_ms_per_step'],'probes':r['probes_per_step'],'distinct':d['config']['distinct'],'generated':d['config']['generated'],'depth':d['config']['depth'],'rounds':s.get('chunks_rank0'),'xfer_s':s.get('exchange_s_rank0')}))" >> gpurun_out/r03m_ab.jsonl
done
