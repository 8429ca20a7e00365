# MW determinism / numerics after the global-qualified sc1 hand-offs
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_mw.py -m gpu \
  > gpurun_out/mw_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|^E " gpurun_out/mw_tests.log | tail -30
timeout -k 10 300 python scripts/dev/mw_err.py > gpurun_out/mw_err.txt 2>&1; cut -c1-330 gpurun_out/mw_err.txt
exit $rc
