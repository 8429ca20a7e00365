#!/bin/bash
# rocprofv3 kernel stats of the Linear GEMM microbench per tile config (true kernel times).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
for t in 64 128; do
  RAYDP_LIN_TILE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o lin$t -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 > $R/gpurun_out/prof_lin$t.log 2>&1 || exit 1
done
ls -R $R/gpurun_out/prof | head -20
