#!/bin/bash
# GBDT kernels: GPU tests (exact parity / determinism) + boosting bench + kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_gbdt.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gbdt_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gbdt_tests.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/gbdt_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python benchmarks/gbdt_bench.py --rows 1000000 --rounds 20 > gpurun_out/gbdt_bench.jsonl 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/gbdt_bench.jsonl | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o gbdt -- python3 $R/benchmarks/gbdt_bench.py --rows 1000000 --rounds 10 --paths hip > $R/gpurun_out/prof_gbdt.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
