#!/bin/bash
# Fused-MLP publish-store change: full GPU tests, then the 1,000-step epoch kernel time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" gpurun_out/gpu_tests.log | head; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
RAYDP_MLP_COOPERATIVE=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1000 --warmup 100 --no-reference-config > $R/gpurun_out/prof_bench.log 2>&1
echo "prof rc=$?"
