#!/bin/bash
# Quick fused-MLP iteration: GPU numerics tests of the fused engine, then the persistent NYC epoch
# timing (plain and with intra-layer stamps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_kernels.py tests/test_gpu_mw.py tests/test_gpu_front.py tests/test_gpu_fused_losses.py \
  > gpurun_out/r5_kernel_tests.log 2>&1
rc=$?; grep -E "passed|failed|^E  |FAIL" gpurun_out/r5_kernel_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u scripts/dev/persist_ab.py . >> gpurun_out/r5_persist.jsonl 2>> gpurun_out/r5_persist.err || exit 3
RAYDP_MLP_LAYER_STAMPS=1 timeout -k 10 150 python -u scripts/dev/persist_ab.py . >> gpurun_out/r5_persist.jsonl 2>> gpurun_out/r5_persist.err || exit 4
tail -2 gpurun_out/r5_persist.jsonl | cut -c1-400
