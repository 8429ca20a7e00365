#!/bin/bash
# Round-end style check: all GPU tests -> smoke -> bench at the driver's short config (x3) and the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/gpu_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$i.log 2>&1
  rc=$?; echo "bench20 #$i rc=$rc"; grep metric gpurun_out/bench20_$i.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/bench.log | cut -c1-400
exit $rc
