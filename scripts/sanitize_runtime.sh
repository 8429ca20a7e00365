#!/bin/bash
# Host C++ runtime under sanitizers (CPU only; no GPU sanitizers on this pool):
#   1. ASan+UBSan and TSan builds of the object-store / frame stress test, run multi-threaded
#      and multi-process;
#   2. ASan builds of the supervisor, app master and shuffle service, driven through their
#      protocol tests (tests/test_sanitizers.py) with RAYDP_NATIVE_BIN_DIR pointing at them.
set -e
cd "$(dirname "$0")/.."
OUT=${1:-/tmp/raydp_sanitize}
python -m raydp_amd.native.build --sanitize asan "$OUT/asan"
python -m raydp_amd.native.build --sanitize tsan "$OUT/tsan"
"$OUT/asan/runtime_stress" 4 3 3000
"$OUT/tsan/runtime_stress" 4 1 2000
"$OUT/asan/expr_vm_fuzz" 1000 1
"$OUT/asan/executor_stress" 4 8 5000
"$OUT/tsan/executor_stress" 4 40 5000 sync
python -m pytest tests/test_sanitizers.py -q -p no:cacheprovider
