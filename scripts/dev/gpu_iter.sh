#!/bin/bash
# one iteration of kernel work: per-phase stamps, kernel numerics tests, persistent epoch timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 180 python scripts/stamp_kernel.py 2>&1 | grep -v amdgpu.ids || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_kernels.py \
  -k "persistent or converges or one_step or bn_before" > gpurun_out/iter_tests.log 2>&1
rc=$?; tail -3 gpurun_out/iter_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/dev/persist_time.py 2>&1 | grep -v amdgpu.ids
