#!/bin/bash
# MW iteration: multi-workgroup tests, step times at batch 4096 / 1000, kernel stats at 4096.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_mw.py > gpurun_out/r5_mw_tests.log 2>&1; rc=$?; grep -E "passed|failed" gpurun_out/r5_mw_tests.log | tail -2; [ $rc -ne 0 ] && { grep -E "^E  |FAILED" gpurun_out/r5_mw_tests.log | head; exit $rc; }
timeout -k 10 200 python -u scripts/dev/mw_time.py 4096 1000 || exit 2
timeout -k 10 200 python -u scripts/dev/mw_stamps.py 4096 > gpurun_out/r5_mw_stamps.json 2> gpurun_out/r5_mw_stamps.err || exit 3
bash scripts/dev/mw_prof.sh || exit 4
