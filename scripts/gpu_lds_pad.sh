#!/bin/bash
# After the LDS row-pad changes: all GPU tests, kernel times of the fused epoch and the GEMMs,
# LDS bank-conflict counters of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_tests.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
RAYDP_MLP_COOPERATIVE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1000 --warmup 100 --no-reference-config > $R/gpurun_out/prof_bench.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' $R/gpurun_out/prof_bench.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o lin -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 > $R/gpurun_out/prof_lin.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-include-regex "lin_gemm" --output-format csv -d $R/gpurun_out/pmc -o lin_p1 -- python3 $R/benchmarks/linear_gemm_bench.py --reps 3 > $R/gpurun_out/pmc/lin_p1.log 2>&1
echo "pmc rc=$?"
