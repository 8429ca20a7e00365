#!/bin/bash
# Quick iteration on both fused paths: kernel + MW tests, persistent NYC timing, MW timing/timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/dev/r5_quick.sh || exit $?
timeout -k 10 200 python -u scripts/dev/mw_time.py 4096 1000 || exit 12
timeout -k 10 200 python -u scripts/dev/mw_stamps.py 4096 > gpurun_out/r5_mw_stamps.json 2> gpurun_out/r5_mw_stamps.err || exit 13
