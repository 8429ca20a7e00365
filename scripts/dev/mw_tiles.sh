#!/bin/bash
# Multi-workgroup step time at batch 4096 by row tile (workgroups = 4096 / 16 MT).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for mt in 8 4 2; do
  RAYDP_MLP_MW_MT=$mt timeout -k 10 200 python -u scripts/dev/mw_time.py 4096 >> gpurun_out/r5_mw_tiles.jsonl 2>> gpurun_out/r5_mw_tiles.err || { echo "mt $mt rc=$?"; tail -5 gpurun_out/r5_mw_tiles.err; exit 1; }
  tail -1 gpurun_out/r5_mw_tiles.jsonl
done
