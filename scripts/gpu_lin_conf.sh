#!/bin/bash
# GEMM kernel times (rocprofv3 kernel trace) and LDS bank-conflict counters of the microbench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o lin -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 > $R/gpurun_out/prof_lin.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "lin_gemm" --output-format csv -d $R/gpurun_out/pmc -o lin_p1 -- python3 $R/benchmarks/linear_gemm_bench.py --reps 3 > $R/gpurun_out/pmc/lin_p1.log 2>&1
echo "pmc rc=$?"
