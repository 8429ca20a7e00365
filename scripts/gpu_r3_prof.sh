#!/bin/bash
# Round 3 measurements: kernel profiles (bench, DLRM fused tail, xGMI buckets), B4 on the GPU,
# DLRM end to end at the notebook's batch 128 and at 2048.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
timeout -k 10 300 python benchmarks/xgmi_bench.py --world 4 > gpurun_out/r3_xgmi_w4.json 2> gpurun_out/r3_xgmi.err || exit 21
timeout -k 10 300 python benchmarks/xgmi_bench.py --world 8 --reps 100 > gpurun_out/r3_xgmi_w8.json 2>> gpurun_out/r3_xgmi.err || exit 22
cat gpurun_out/r3_xgmi_w4.json gpurun_out/r3_xgmi_w8.json
bash scripts/gpu.sh prof bench20 python3 $R/bench.py --steps 20 --warmup 5 --no-reference-config || exit 23
bash scripts/gpu.sh prof dlrm2048 python3 $R/benchmarks/dlrm_bench.py --batch 2048 --steps 64 --warmup 16 --graph || exit 24
bash scripts/gpu.sh prof dlrm2048_eager python3 $R/benchmarks/dlrm_bench.py --batch 2048 --steps 64 --warmup 16 || exit 25
bash scripts/gpu.sh prof xgmi_w4 python3 $R/benchmarks/xgmi_bench.py --world 4 --reps 50 || exit 26
RAYTRAIN_DEVICE=cuda timeout -k 10 300 python benchmarks/raytrain_bench.py > gpurun_out/r3_b4_cuda.json 2> gpurun_out/r3_b4.err || exit 27
timeout -k 10 300 python benchmarks/raytrain_bench.py > gpurun_out/r3_b4_cpu.json 2>> gpurun_out/r3_b4.err || exit 28
cat gpurun_out/r3_b4_cuda.json gpurun_out/r3_b4_cpu.json
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 2048 > gpurun_out/r3_dlrm_e2e.jsonl 2> gpurun_out/r3_dlrm_e2e.err || exit 29
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 >> gpurun_out/r3_dlrm_e2e.jsonl 2>> gpurun_out/r3_dlrm_e2e.err || exit 30
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 --workers 2 >> gpurun_out/r3_dlrm_e2e.jsonl 2>> gpurun_out/r3_dlrm_e2e.err || exit 31
cat gpurun_out/r3_dlrm_e2e.jsonl
