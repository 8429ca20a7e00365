#!/bin/bash
# DLRM end to end through Spark + the model-parallel path at world 1 (async id exchange).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 > gpurun_out/dlrm_e2e.log 2>&1
rc=$?; echo "e2e rc=$rc"; tail -2 gpurun_out/dlrm_e2e.log | cut -c1-1500
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048 --fused-sgd > gpurun_out/dlrm_e2e_fsgd.log 2>&1
rc=$?; echo "e2e fused-sgd rc=$rc"; tail -1 gpurun_out/dlrm_e2e_fsgd.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 benchmarks/dlrm_bench.py --model-parallel --fused-sgd >> gpurun_out/dlrm_mp.log 2>&1
rc=$?; echo "mp rc=$rc"; tail -1 gpurun_out/dlrm_mp.log | cut -c1-300
exit $rc
