# Headline distribution (10 runs) + 1-worker span timeline after the executor inline-run change
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/bench.jsonl gpurun_out/bench.err
bash scripts/gpu.sh bench 1 20 5 10 || exit 2
bash scripts/gpu.sh trace 1 || exit 3
python scripts/trace_summary.py gpurun_out/tr/est nyc > gpurun_out/trace_nyc_timeline.txt 2>&1
