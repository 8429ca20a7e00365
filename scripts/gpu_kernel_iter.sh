#!/bin/bash
# Kernel iteration: fused-MLP numerics tests, per-phase stamps, then the 1-GPU bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_xgmi.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/kernel_tests.log 2>&1; rc=$?
tail -3 gpurun_out/kernel_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/stamp_kernel.py > gpurun_out/stamps.log 2>&1 || exit $?
tail -17 gpurun_out/stamps.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*\|"rank0_breakdown_s": {[^}]*}' gpurun_out/bench.log
