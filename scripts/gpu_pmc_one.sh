#!/bin/bash
# ONE PMC counter pass (scripts/gpu_pmc.sh lists the passes): $1 = pass (1..3), $2 = bench|lin
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
case $1 in
  1) P="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE";;
  2) P="FETCH_SIZE TCC_HIT_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES";;
  3) P="WRITE_SIZE TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU";;
esac
REGEX="rx_jit_persist|mlp_persist|lin_gemm|arrow_ingest"
if [ "$2" = bench ]; then
  CMD="python3 $R/bench.py --steps 200 --warmup 5 --no-reference-config"
else
  CMD="python3 $R/benchmarks/linear_gemm_bench.py --reps 3"
fi
RAYDP_MLP_COOPERATIVE=0 timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$REGEX" --output-format csv -d $R/gpurun_out/pmc -o $2_p$1 -- $CMD > $R/gpurun_out/pmc/$2_p$1.log 2>&1
rc=$?
echo "rc=$rc rows=$(wc -l < $R/gpurun_out/pmc/$2_p$1_counter_collection.csv)"
