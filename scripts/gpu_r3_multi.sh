#!/bin/bash
# Round 3: multi-rank paths on the one GPU (xGMI world 2/4/8, spawned estimator workers,
# Horovod), the GPU suite, then 1-GPU and 2-rank rehearsal benches (SPMD self-launch and the
# estimator topology).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 700 $T tests/test_gpu_hvd.py tests/test_gpu_xgmi.py -k "hvd or embedding_rows" -m gpu > gpurun_out/r3_multi_tests.log 2>&1
rc=$?; echo "targeted rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r3_multi_tests.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 $T tests/ -m gpu > gpurun_out/r3_gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r3_gpu_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_b1.jsonl 2> gpurun_out/r3_b1.err || exit 11
tail -c 600 gpurun_out/r3_b1.jsonl
RAYDP_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r3_b2_spmd.jsonl 2> gpurun_out/r3_b2_spmd.err || exit 12
tail -c 900 gpurun_out/r3_b2_spmd.jsonl
timeout -k 10 300 python bench.py --gpus 2 --gpu-share 0.5 --topology estimator --steps 20 --warmup 5 > gpurun_out/r3_b2_est.jsonl 2> gpurun_out/r3_b2_est.err || exit 13
tail -c 900 gpurun_out/r3_b2_est.jsonl
for B in 2048 128; do
  timeout -k 10 200 python benchmarks/dlrm_bench.py --batch $B --steps 400 --warmup 40 --graph >> gpurun_out/r3_dlrm.jsonl 2>> gpurun_out/r3_dlrm.err || exit 14
  timeout -k 10 200 python benchmarks/dlrm_bench.py --batch $B --steps 400 --warmup 40 >> gpurun_out/r3_dlrm.jsonl 2>> gpurun_out/r3_dlrm.err || exit 15
done
cat gpurun_out/r3_dlrm.jsonl
