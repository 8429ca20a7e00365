#!/bin/bash
# DLRM: fused-tower tests, bench (fused vs eager), rocprof kernel stats of the fused step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_dlrm.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_linear.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|^E  " gpurun_out/gpu_linear.log | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
for mode in "" "--eager-mlp" "--eager-mlp --amp" "--fused-sgd"; do
  timeout -k 10 200 python benchmarks/dlrm_bench.py $mode >> gpurun_out/dlrm_bench.jsonl 2>gpurun_out/dlrm_err.log
  rc=$?; if [ $rc -ne 0 ]; then echo "dlrm bench '$mode' rc=$rc"; tail -5 gpurun_out/dlrm_err.log; exit $rc; fi
done
cat gpurun_out/dlrm_bench.jsonl | cut -c1-220
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o dlrm -- python3 $R/benchmarks/dlrm_bench.py --steps 50 --warmup 10 > $R/gpurun_out/prof_dlrm.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
