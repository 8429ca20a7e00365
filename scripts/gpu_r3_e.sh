#!/bin/bash
# Round 3, batch E: 2-worker DLRM e2e after the warm-worker graph fix; GPU tests touching graphs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_dlrm.py tests/test_gpu_spawned.py tests/test_gpu_xgmi.py \
  > gpurun_out/re_tests.log 2>&1 || { grep -E "passed|failed|Error" gpurun_out/re_tests.log | tail -20; exit 21; }
grep -E "passed|failed" gpurun_out/re_tests.log | tail -2
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 --workers 2 \
  > gpurun_out/re_dlrm2w.jsonl 2> gpurun_out/re_dlrm2w.err || exit 22
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 \
  >> gpurun_out/re_dlrm2w.jsonl 2>> gpurun_out/re_dlrm2w.err || exit 23
cut -c1-600 gpurun_out/re_dlrm2w.jsonl
