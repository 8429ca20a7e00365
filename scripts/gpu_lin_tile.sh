#!/bin/bash
# Linear GEMM tiles: GPU tests of the fused towers, GEMM microbench per tile config, DLRM bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_dlrm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_linear.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_linear.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
for t in auto 64 128; do
  if [ $t = auto ]; then unset RAYDP_LIN_TILE; else export RAYDP_LIN_TILE=$t; fi
  timeout -k 10 120 python benchmarks/linear_gemm_bench.py > gpurun_out/lin_$t.jsonl 2>gpurun_out/lin_err.log || { tail -5 gpurun_out/lin_err.log; exit 1; }
  echo "== tile $t"; cat gpurun_out/lin_$t.jsonl
done
unset RAYDP_LIN_TILE
for mode in "" "--fused-sgd"; do
  timeout -k 10 200 python benchmarks/dlrm_bench.py $mode >> gpurun_out/dlrm_bench.jsonl 2>gpurun_out/dlrm_err.log || { tail -5 gpurun_out/dlrm_err.log; exit 1; }
done
cut -c1-200 gpurun_out/dlrm_bench.jsonl
