#!/bin/bash
# Linear GEMM: fused-tower / DLRM GPU tests, kernel times at the default split heuristic, DLRM bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_dlrm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_linear.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_linear.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
for mode in "" "--fused-sgd"; do
  timeout -k 10 200 python benchmarks/dlrm_bench.py $mode >> gpurun_out/dlrm_bench.jsonl 2>gpurun_out/dlrm_err.log || { tail -5 gpurun_out/dlrm_err.log; exit 1; }
done
cut -c1-200 gpurun_out/dlrm_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o auto -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 > $R/gpurun_out/prof_auto.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o dlrm -- python3 $R/benchmarks/dlrm_bench.py --steps 50 --warmup 10 > $R/gpurun_out/prof_dlrm.log 2>&1
