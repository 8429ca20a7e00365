#!/bin/bash
# GEMM pipeline change: linear/DLRM GPU tests, kernel times of the microbench, DLRM graph bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_gpu_linear.py tests/test_gpu_dlrm.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/lin_tests.log; if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" gpurun_out/lin_tests.log | head; exit $rc; fi
for m in "--graph" "--graph --fused-sgd"; do
  timeout -k 10 200 python benchmarks/dlrm_bench.py $m >> gpurun_out/dlrm_graph.jsonl 2>>gpurun_out/dlrm.err || exit 1
done
cut -c1-150 gpurun_out/dlrm_graph.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o lin -- python3 $R/benchmarks/linear_gemm_bench.py --reps 20 > $R/gpurun_out/prof_lin.log 2>&1
echo "prof rc=$?"
