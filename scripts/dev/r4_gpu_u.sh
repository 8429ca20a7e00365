# R-image chunk swizzle: GPU suite + smoke, PMC pass 1 (LDS conflicts) on the 200-step headline
# epoch and the batch-4096 MW step, headline x3
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/bench.jsonl gpurun_out/bench.err gpurun_out/pmc/bench_p1* gpurun_out/pmc/mw_p1*
bash scripts/gpu.sh tests || exit 1
bash scripts/gpu.sh pmc 1 bench || exit 4
bash scripts/gpu.sh pmc 1 mw || exit 5
bash scripts/gpu.sh bench 1 20 5 3 || exit 2
