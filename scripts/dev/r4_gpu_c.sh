# DLRM persistent step after the phase rework: tests, phase profile; MW error diag
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dlrm_step.py \
  > gpurun_out/dlrm_step_tests.txt 2>&1; rc=$?
grep -E "PASS|FAIL|passed|failed|^E " gpurun_out/dlrm_step_tests.txt | head -20; [ $rc -ne 0 ] && exit $rc
bash scripts/dev/r4_dlrm_phase.sh || exit 1
timeout -k 10 300 python scripts/dev/mw_err.py > gpurun_out/mw_err.txt 2>&1; tail -16 gpurun_out/mw_err.txt
