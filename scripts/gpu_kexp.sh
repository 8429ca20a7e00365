#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/kernel_tests.log 2>&1; rc=$?
tail -2 gpurun_out/kernel_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_stamp_exp.sh
