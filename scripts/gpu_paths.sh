#!/bin/bash
# DLRM + NYC alternative-path benches (1 GPU, plus 2-rank gloo rehearsals on the same GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dlrm.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dlrm_tests.log 2>&1 || { tail -20 gpurun_out/dlrm_tests.log; exit 1; }
tail -1 gpurun_out/dlrm_tests.log
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; rc=$?; echo "$name rc=$rc $(grep -h '"metric"' gpurun_out/$name.log | tail -1)"; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run dlrm_1gpu python benchmarks/dlrm_bench.py --fused-sgd --amp || exit 1
run dlrm_mp1 $TR --nproc-per-node 1 --master-port 29551 benchmarks/dlrm_bench.py --amp --fused-sgd --model-parallel || exit 1
RAYDP_BENCH_BACKEND=gloo run dlrm_mp2_gloo $TR --nproc-per-node 2 --master-port 29552 benchmarks/dlrm_bench.py --amp --fused-sgd --steps 50 --warmup 5 || exit 1
for p in fused ddp horovod; do
  run nyc_$p python benchmarks/nyctaxi_paths_bench.py --path $p || exit 1
  RAYDP_BENCH_BACKEND=gloo run nyc_${p}_2r $TR --nproc-per-node 2 --master-port 2956${#p} benchmarks/nyctaxi_paths_bench.py --path $p --steps 1000 --warmup 100 || exit 1
done
