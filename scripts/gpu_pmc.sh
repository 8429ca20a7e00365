#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, counter/block limits respected) over the hot
# kernels: the persistent fused-MLP epoch (bench.py, 200 steps), the fused Linear GEMMs
# (DLRM tower shapes) and the Arrow ingest kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
P3="WRITE_SIZE TCC_MISS_sum SQ_INSTS_VALU SQ_INSTS_SALU"
REGEX="rx_jit_persist|mlp_persist|lin_gemm|arrow_ingest|ingest"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  RAYDP_MLP_COOPERATIVE=0 timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$REGEX" --output-format csv -d $R/gpurun_out/pmc -o bench_p$i -- python3 $R/bench.py --steps 200 --warmup 5 --no-reference-config > $R/gpurun_out/pmc/bench_p$i.log 2>&1 || { echo "bench pass $i failed"; tail -5 $R/gpurun_out/pmc/bench_p$i.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$REGEX" --output-format csv -d $R/gpurun_out/pmc -o lin_p$i -- python3 $R/benchmarks/linear_gemm_bench.py --reps 3 > $R/gpurun_out/pmc/lin_p$i.log 2>&1 || { echo "lin pass $i failed"; tail -5 $R/gpurun_out/pmc/lin_p$i.log; exit 1; }
  echo "pass $i ok"
done
ls $R/gpurun_out/pmc | head -40
