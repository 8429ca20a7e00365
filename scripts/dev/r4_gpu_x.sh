# Final-code headline distribution: 10 back-to-back driver-config runs
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/bench.jsonl gpurun_out/bench.err
bash scripts/gpu.sh bench 1 20 5 10 || exit 2
