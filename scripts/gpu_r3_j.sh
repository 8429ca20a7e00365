#!/bin/bash
# Round 3, batch J: estimator-topology timeline after the single-pickle payload; spawned tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_spawned.py tests/test_gpu_hvd.py > gpurun_out/rj_tests.log 2>&1 || { grep -E "passed|failed|Error|^E " gpurun_out/rj_tests.log | tail -25; exit 21; }
grep -E "passed|failed" gpurun_out/rj_tests.log | tail -2
rm -f gpurun_out/tr/est.*
RAYDP_TRACE=gpurun_out/tr/est timeout -k 10 300 python bench.py --gpus 2 --gpu-share 0.5 --topology estimator \
  --steps 20 --warmup 5 --no-reference-config > gpurun_out/rj_est.jsonl 2> gpurun_out/rj_est.err || exit 22
python scripts/trace_summary.py gpurun_out/tr/est > gpurun_out/rj_est_timeline.txt 2>&1
head -60 gpurun_out/rj_est_timeline.txt
