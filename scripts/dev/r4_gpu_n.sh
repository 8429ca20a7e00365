# Final check: GPU suite + smoke, headline x2
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
bash scripts/gpu.sh tests || exit 1
bash scripts/gpu.sh bench 1 20 5 2 || exit 2
