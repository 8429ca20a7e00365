#!/bin/bash
# xGMI one-shot all-reduce checks on a 1-GPU box: 2-rank tests, then a 2-rank bench rehearsal
# (gloo bootstrap, both ranks on cuda:0). Each GPU step has its own limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_xgmi.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/xgmi_tests.log 2>&1
rc=$?; echo "xgmi tests rc=$rc"; tail -5 gpurun_out/xgmi_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
RAYDP_BENCH_BACKEND=gloo RAYDP_BENCH_CPUS=2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1000 --warmup 100 > gpurun_out/bench2_gloo.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -3 gpurun_out/bench2_gloo.log
exit $rc
