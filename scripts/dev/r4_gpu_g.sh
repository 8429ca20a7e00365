cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_mw.py -m gpu \
  > gpurun_out/mw_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|^E " gpurun_out/mw_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
bash scripts/dev/r4_gpu_f.sh
