# Full GPU suite on the current build, the config-5 CLI transcript, and a
# same-box A/B of k_expand variants 0/1 (RMC_EXPAND_VARIANT).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 120 $B -builtin-raft specs/MCraftBug.tla > $O/cli_config5.txt 2>&1; test $? -eq 12 || exit 1
for r in 1 2 3; do
  for v in 0 1; do
    RMC_EXPAND_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-probe-ceiling --steps 5 --warmup 1 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('variant $v run $r', round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_step'],2), d['config']['distinct'], d['config']['fp_salt_crosscheck']['agrees'])" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
