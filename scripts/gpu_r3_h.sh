#!/bin/bash
# Round 3, batch H: span timeline of the estimator topology (one driver, 2 spawned workers).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/tr/est.*
RAYDP_TRACE=gpurun_out/tr/est timeout -k 10 300 python bench.py --gpus 2 --gpu-share 0.5 --topology estimator \
  --steps 20 --warmup 5 --no-reference-config > gpurun_out/rh_est.jsonl 2> gpurun_out/rh_est.err || exit 21
python scripts/trace_summary.py gpurun_out/tr/est > gpurun_out/rh_est_timeline.txt 2>&1
cat gpurun_out/rh_est_timeline.txt | head -90
