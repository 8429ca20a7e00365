#!/bin/bash
# quick GPU iteration: kernel tests, stamp breakdown, short bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_tests.log | head -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/stamp_kernel.py > gpurun_out/stamps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/stamps.log | tail -17
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 3000 --warmup 300 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
exit $rc
