# Hoisted swizzle in the publish step: phase stamps first (quick), then GPU suite + smoke, PMC pass 1, headline x3
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/bench.jsonl gpurun_out/bench.err gpurun_out/pmc/bench_p1* gpurun_out/pmc/mw_p1*
timeout -k 10 200 python scripts/dev/persist_time.py 1 > gpurun_out/persist_time_swz2.txt 2>&1 || exit 6
cat gpurun_out/persist_time_swz2.txt
bash scripts/gpu.sh tests || exit 1
bash scripts/gpu.sh pmc 1 bench || exit 4
bash scripts/gpu.sh pmc 1 mw || exit 5
bash scripts/gpu.sh bench 1 20 5 3 || exit 2
