cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 200 python scripts/dev/mw_diag.py && \
timeout -k 10 120 python benchmarks/grid_barrier_bench.py | tee gpurun_out/grid_barrier.jsonl
