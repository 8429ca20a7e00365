#!/bin/bash
# Round-2 first GPU check: gpu tests -> smoke -> bench at the driver's config -> cProfile of the
# short pipeline -> rocprof kernel trace of the short bench. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|^E  |Error" gpurun_out/gpu_tests.log | tail -15
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; tail -1 gpurun_out/bench20.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/prof_small.py --steps 20 --warmup 5 > gpurun_out/prof_small.log 2>&1
rc=$?; echo "prof_small rc=$rc"; head -4 gpurun_out/prof_small_20.txt
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench20 -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof20.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 $R/gpurun_out/prof20.log
exit $rc
