#!/bin/bash
# Persistent-kernel launch mode: cooperative vs plain (occupancy-checked). GPU kernel tests in
# plain mode, driver-config bench A/B, and a profiled run in plain mode (exit status).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
RAYDP_MLP_COOPERATIVE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_front.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/coop0_tests.log 2>&1
rc=$?; echo "plain-launch tests rc=$rc"; tail -1 gpurun_out/coop0_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for k in 1 2 3; do
  for c in 1 0; do
    RAYDP_MLP_COOPERATIVE=$c timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config > gpurun_out/ab_c${c}_$k.log 2>&1 || exit 1
    echo "coop=$c $(grep -o '"value": [0-9.]*' gpurun_out/ab_c${c}_$k.log) $(grep -o '"train": [0-9.]*' gpurun_out/ab_c${c}_$k.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
RAYDP_MLP_COOPERATIVE=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof -o p -- python3 $R/bench.py --steps 20 --warmup 5 --no-reference-config > $R/gpurun_out/prof.log 2>&1
echo "profiled plain-launch rc=$?"
