#!/bin/bash
# GBDT histogram kernel: numerics tests -> HIP-vs-torch boosting bench -> rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof_gbdt
timeout -k 10 300 python -u -m pytest tests/test_gpu_gbdt.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gbdt_tests.log 2>&1
rc=$?; echo "gbdt tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/gbdt_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u benchmarks/gbdt_bench.py --rows 1000000 --rounds 20 > gpurun_out/gbdt_bench.log 2>&1
rc=$?; echo "gbdt bench rc=$rc"; cat gpurun_out/gbdt_bench.log | grep -v "^W2"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_gbdt -o gbdt -- python3 $R/benchmarks/gbdt_bench.py --rows 1000000 --rounds 10 --paths hip > $R/gpurun_out/prof_gbdt.log 2>&1
rc=$?; echo "prof rc=$rc"
find $R/gpurun_out/prof_gbdt -name "*kernel_stats*"
exit $rc
