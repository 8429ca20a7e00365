#!/bin/bash
# DLRM throughput: replicated fused embeddings (1 GPU) and the sharded/all-to-all path at world 1 (RCCL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/dlrm_bench.py --fused-sgd --amp > gpurun_out/dlrm_1gpu.log 2>&1 || exit $?
tail -1 gpurun_out/dlrm_1gpu.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 benchmarks/dlrm_bench.py --amp --model-parallel > gpurun_out/dlrm_mp1.log 2>&1 || exit $?
tail -1 gpurun_out/dlrm_mp1.log
RAYDP_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 benchmarks/dlrm_bench.py --amp --steps 50 --warmup 5 > gpurun_out/dlrm_mp2_gloo.log 2>&1
echo "2-rank gloo rehearsal rc=$?"; grep metric gpurun_out/dlrm_mp2_gloo.log | tail -1; grep -m3 -i error gpurun_out/dlrm_mp2_gloo.log
exit 0
