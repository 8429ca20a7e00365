# Headline distribution (10 runs) after the pickler / actor transport changes + 1-worker span timeline
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/bench.jsonl gpurun_out/bench.err
bash scripts/gpu.sh bench 1 20 5 10 || exit 2
bash scripts/gpu.sh trace 1 || exit 3
