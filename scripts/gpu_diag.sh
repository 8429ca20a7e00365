#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
timeout -k 10 300 python scripts/diag_fused_grads.py > gpurun_out/diag.log 2>&1
rc=$?; echo "diag rc=$rc"; cat gpurun_out/diag.log | grep -v amdgpu.ids
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 3000 --warmup 300 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 $R/gpurun_out/prof.log
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
