# Persistent NYC epoch phase stamps after the LDS swizzles (compare profiles/r4_persist_step_timeline.txt)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/persist_time.py 1 > gpurun_out/persist_time_swz.txt 2>&1 || exit 1
cat gpurun_out/persist_time_swz.txt
