#!/bin/bash
# Kernel statistics of the multi-workgroup NYC step at batch 4096 (rocprofv3 --kernel-trace --stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd); mkdir -p gpurun_out/mwprof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mwprof -o mw \
  -- python3 $R/scripts/dev/mw_time.py 4096 > $R/gpurun_out/mwprof/mw.log 2>&1 || { echo "rc=$?"; tail -20 $R/gpurun_out/mwprof/mw.log; exit 1; }
cat $R/gpurun_out/mwprof/mw.log | tail -2
head -8 $R/gpurun_out/mwprof/mw_kernel_stats.csv
