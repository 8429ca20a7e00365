#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/bench_$i.log 2>&1 || exit $?
  echo "$(grep -o '"value": [0-9.]*' gpurun_out/bench_$i.log) $(grep -o '"rank0_breakdown_s": {[^}]*}' gpurun_out/bench_$i.log)"
done
