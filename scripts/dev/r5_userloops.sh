#!/bin/bash
# User-written loops on the GPU: the bench's Horovod extra (and DLRM / word count extras) and the
# Ray Train stroke tutorial (B4) on cuda vs its CPU run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_bench_extras.jsonl 2> gpurun_out/r5_bench_extras.err || { echo "bench rc=$?"; tail -5 gpurun_out/r5_bench_extras.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r5_bench_extras.jsonl').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['config'].get('other_workloads'))[:1500])"
RAYTRAIN_DEVICE=cuda timeout -k 10 300 python benchmarks/raytrain_bench.py > gpurun_out/r5_b4_gpu.jsonl 2> gpurun_out/r5_b4_gpu.err || { echo "b4 gpu rc=$?"; tail -5 gpurun_out/r5_b4_gpu.err; exit 2; }
timeout -k 10 300 python benchmarks/raytrain_bench.py > gpurun_out/r5_b4_cpu.jsonl 2> gpurun_out/r5_b4_cpu.err || { echo "b4 cpu rc=$?"; exit 3; }
tail -1 gpurun_out/r5_b4_gpu.jsonl | cut -c1-400; tail -1 gpurun_out/r5_b4_cpu.jsonl | cut -c1-400
