#!/bin/bash
# A/B of bench variants selected by environment (each run: train time of rank 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "X=1" "RAYDP_OPT_XCD_AFFINE=0" "X=1" "RAYDP_OPT_XCD_AFFINE=0" "RAYDP_MLP_WGRAD=step"; do
  env $v timeout -k 10 300 python bench.py > gpurun_out/ab.log 2>&1 || exit $?
  echo "$v $(grep -o '"value": [0-9.]*' gpurun_out/ab.log) $(grep -o '"train": [0-9.]*' gpurun_out/ab.log)"
done
