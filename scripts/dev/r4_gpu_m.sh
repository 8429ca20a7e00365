# Round-end style check: GPU suite + smoke, headline x3, DLRM end to end (1/2 workers, batch 128 / 2048)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
bash scripts/gpu.sh tests || exit 1
bash scripts/gpu.sh bench 1 20 5 3 || exit 2
bash scripts/gpu.sh e2e || exit 3
