cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
nproc > gpurun_out/nproc.txt
for c in 4 8 12; do
  RAYDP_BENCH_CPUS=$c timeout -k 10 300 python bench.py > gpurun_out/bench_cpus$c.log 2>&1 || exit $?
  echo "cpus=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_cpus$c.log) $(grep -o '"rank0_breakdown_s": {[^}]*}' gpurun_out/bench_cpus$c.log)"
done
