# PMC passes on the current kernels (round 4): fused Linear GEMMs (DLRM tower shapes) and the
# headline pipeline's persistent epoch; each pass its own rocprofv3 run under a hard time limit
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out/pmc
for p in 1 3; do bash scripts/gpu.sh pmc $p lin || exit 1; done
for p in 1 3; do bash scripts/gpu.sh pmc $p bench || exit 2; done
for p in 1 2 3; do bash scripts/gpu.sh pmc $p mw || exit 3; done
python scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.md 2>&1; head -40 gpurun_out/pmc_summary.md
