#!/bin/bash
# Final check: all GPU tests, smoke, driver-config bench, and a default-settings rocprofv3 run
# of the bench (clean exit expected with the plain persistent launch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -1 gpurun_out/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" gpurun_out/gpu_tests.log | head; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$i.log 2>&1 || exit 1
  echo "bench20 #$i $(grep -o '"value": [0-9.]*' gpurun_out/bench20_$i.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 20 --warmup 5 --no-reference-config > $R/gpurun_out/prof.log 2>&1
echo "profiled bench rc=$?"
