#!/bin/bash
# Round 3, batch B: DLRM graph capture without per-step memset+add, the 2-worker DLRM e2e
# timeline, headline bench with the native executor.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_dlrm.py > gpurun_out/rb_dlrm_tests.log 2>&1 || { tail -30 gpurun_out/rb_dlrm_tests.log; exit 21; }
grep -E "passed|failed" gpurun_out/rb_dlrm_tests.log | tail -2
bash scripts/gpu.sh dlrm 2048 128 || exit 22
bash scripts/gpu.sh prof dlrm2048_v2 python3 $(pwd)/benchmarks/dlrm_bench.py --batch 2048 --steps 64 --warmup 16 --graph || exit 23
RAYDP_TRACE=gpurun_out/tr/dlrm2w timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 \
  --warmup-rows 5000 --workers 2 > gpurun_out/rb_dlrm2w.jsonl 2> gpurun_out/rb_dlrm2w.err || exit 24
cat gpurun_out/rb_dlrm2w.jsonl
python scripts/trace_summary.py gpurun_out/tr/dlrm2w > gpurun_out/rb_dlrm2w_timeline.txt 2>&1 || true
bash scripts/gpu.sh bench 1 20 5 4 || exit 25
