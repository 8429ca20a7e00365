#!/bin/bash
# Per-phase stamps of the fused step under timing experiments (numerics intentionally wrong).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for e in "" PLAINSTORE SCRATCHWT; do
  RAYDP_MLP_EXPERIMENT=$e timeout -k 10 180 python scripts/stamp_kernel.py > gpurun_out/stamps_$e.log 2>&1 || exit $?
  echo "== exp '$e'"; grep -E "^(fwd|bwd|load|total)" gpurun_out/stamps_$e.log | tr '\n' ' ' | sed 's/  */ /g'; echo
done
