#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/stamp_kernel.py > gpurun_out/stamps.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/stamps.log | tail -16
exit $rc
