set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
for c in A B C F G E D; do
  timeout -k 10 150 ./raft.tla_amd/bin/rmc-tlc -config specs/sizing/$c.cfg specs/sizing/$c.tla > gpurun_out/size_$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; tail -3 gpurun_out/size_$c.log
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ]; then exit 1; fi
done
