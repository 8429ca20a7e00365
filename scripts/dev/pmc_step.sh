#!/bin/bash
# PMC passes over the fused NYC step kernel (launch-per-step epoch: step body only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd); mkdir -p gpurun_out/pmc5
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=1
for P in "$P1" "$P2"; do
  STEPS=300 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "rx_jit_step$|opt_tiled" --output-format csv \
    -d $R/gpurun_out/pmc5 -o step_p$i -- python3 $R/scripts/dev/step_loop.py > $R/gpurun_out/pmc5/step_p$i.log 2>&1 || { echo "pmc pass $i rc=$?"; exit 7; }
  i=$((i+1))
done
echo pmc ok
