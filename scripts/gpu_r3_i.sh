#!/bin/bash
# Round 3, batch I: sharded-embedding exchanges over the xGMI all-to-all; estimator-topology trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_xgmi.py -k "sharded or replicated or ddp" > gpurun_out/ri_tests.log 2>&1 || { grep -E "passed|failed|Error|^E " gpurun_out/ri_tests.log | tail -25; exit 21; }
grep -E "passed|failed" gpurun_out/ri_tests.log | tail -2
rm -f gpurun_out/tr/est.*
RAYDP_TRACE=gpurun_out/tr/est timeout -k 10 300 python bench.py --gpus 2 --gpu-share 0.5 --topology estimator \
  --steps 20 --warmup 5 --no-reference-config > gpurun_out/ri_est.jsonl 2> gpurun_out/ri_est.err || exit 22
python scripts/trace_summary.py gpurun_out/tr/est > gpurun_out/ri_est_timeline.txt 2>&1
head -90 gpurun_out/ri_est_timeline.txt
