#!/bin/bash
# Fused-optimizer A/B at batch 4096 / 1000: RAYDP_MLP_MW_FUSED_OPT (0 separate launch, N cap,
# 1 all), optionally x the optimizer workgroups' poll sleep (SLEEPS: RX_MWOPT_SLEEP via
# RAYDP_MLP_DEFINES), then workgroup 0's timeline of the fused default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
for cap in ${CAPS:-0 1}; do
  echo "cap=$cap"
  RAYDP_MLP_MW_FUSED_OPT=$cap timeout -k 10 200 python -u scripts/dev/mw_time.py 4096 1000 || exit 2
done
for sl in ${SLEEPS:-}; do
  echo "sleep=$sl"
  RAYDP_MLP_DEFINES="RX_MWOPT_SLEEP=$sl" timeout -k 10 200 python -u scripts/dev/mw_time.py 4096 1000 || exit 3
done
timeout -k 10 200 python -u scripts/dev/mw_stamps.py 4096 > gpurun_out/r5_mw_stamps_fused.json 2>&1 || exit 4
