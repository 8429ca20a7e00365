#!/bin/bash
# Persistent-epoch kernel: numerics vs the launch-per-step loop, epoch timing, then the 1-GPU bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_kernels.py \
  -k "persistent or rccl or converges or one_step" > gpurun_out/persist_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error" gpurun_out/persist_tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/dev/persist_time.py > gpurun_out/persist_time.log 2>&1 || exit $?
cat gpurun_out/persist_time.log
bash scripts/gpu_bench3.sh
