#!/bin/bash
# rocprofv3 kernel times of the Linear GEMM microbench at forced split-K factors.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
for s in 1 2 4 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o sp$s -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 --splits $s > $R/gpurun_out/prof_sp$s.log 2>&1 || exit 1
done
