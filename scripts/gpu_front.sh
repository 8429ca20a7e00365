#!/bin/bash
# Embedding-front fused trainer: GPU tests + the fused-kernel regression tests + stroke bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_front.py tests/test_gpu_kernels.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/front_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/front_tests.log | tail -25
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python benchmarks/stroke_bench.py > gpurun_out/stroke_bench.log 2>&1
rc=$?; echo "stroke rc=$rc"; grep metric gpurun_out/stroke_bench.log | cut -c1-900
exit $rc
