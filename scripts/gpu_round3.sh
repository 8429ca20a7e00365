#!/bin/bash
# GPU tests -> smoke -> 4 runs of the driver-config bench -> the no-flag default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/gpu_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$i.log 2>&1
  rc=$?; echo "bench20 #$i rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench20_$i.log) $(grep -o '"rank0_breakdown_s": {[^}]*}' gpurun_out/bench20_$i.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
grep -o '"reference_config_e2e": {[^}]*}' gpurun_out/bench20_1.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bench.log)"
exit $rc
