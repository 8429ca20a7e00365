#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 300 python benchmarks/nyctaxi_paths_bench.py --path fused > gpurun_out/nyc_fused.log 2>&1; rc=$?
echo "nyc_fused rc=$rc $(grep metric gpurun_out/nyc_fused.log)"; [ $rc -eq 0 ] || exit $rc
RAYDP_BENCH_BACKEND=gloo timeout -k 10 300 $TR --nproc-per-node 2 --master-port 29571 benchmarks/nyctaxi_paths_bench.py --path fused --steps 1000 --warmup 100 > gpurun_out/nyc_fused_2r.log 2>&1; rc=$?
echo "nyc_fused_2r rc=$rc $(grep metric gpurun_out/nyc_fused_2r.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/stamp_kernel.py > gpurun_out/stamps.log 2>&1; rc=$?
cat gpurun_out/stamps.log | tail -30; exit $rc
