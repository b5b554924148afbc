# Check of the pruned build (variants 0/2/3/5/7/8 and sym 2/3 removed): full GPU suite, smoke, bench line,
# one-rank sharded bench, SYMMETRY bench, CLI transcripts of configs 1-5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r02u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_full.json 2> $O/bench_full.err || exit 1
timeout -k 10 200 python -u bench.py --force-dist --no-cpu --no-probe-ceiling --steps 3 --warmup 1 > $O/bench_dist1.json 2> $O/bench_dist1.err || exit 1
timeout -k 10 120 python -u tools/sym_bench.py default 300000000 > $O/sym.jsonl 2> $O/sym.err || exit 1
B=raft.tla_amd/bin/rmc-tlc
timeout -k 10 120 $B -builtin-raft -config specs/MCraftBench.cfg specs/MCraftBench.tla > $O/cli_config1.txt 2>&1 || exit 1
timeout -k 10 120 $B -builtin-raft -config specs/MCraftBoundedSym.cfg specs/MCraftBoundedSym.tla > $O/cli_config2.txt 2>&1 || exit 1
timeout -k 10 120 $B -builtin-raft -config specs/MCraftBenchSym.cfg specs/MCraftBenchSym.tla > $O/cli_config2_bench_bounds.txt 2>&1 || exit 1
timeout -k 10 120 $B -builtin-raft -depth 20 -config specs/MCraft5.cfg specs/MCraft5.tla > $O/cli_config3.txt 2>&1 || exit 1
timeout -k 10 120 $B -builtin-raft -simulate num=16777216 -config specs/MCraftSmoke.cfg specs/MCraftSmoke.tla > $O/cli_config4.txt 2>&1 || exit 1
timeout -k 10 120 $B -builtin-raft -config specs/MCraftBug.cfg specs/MCraftBug.tla > $O/cli_config5.txt 2>&1; test $? -eq 12 || exit 1
VARS="1 4" bash tools/gpu/ab_variant.sh > /dev/null || exit 1
cp gpurun_out/ab/* $O/ || exit 1
RMC_SYM_VARIANT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "sym or kat" > $O/tests_sym1.log 2>&1 || exit 1
