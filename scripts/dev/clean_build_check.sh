#!/bin/bash
# Clean build ON THE GPU BOX: copy the tree, delete every prebuilt native library, executable and
# JIT code object, run __graft_entry__.build() (hipcc for gfx950, cmake for the C++ runtime),
# then smoke() and the kernel tests from that copy -- nothing compiled in the container is used.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/dev/clean_build_check.sh
set -o pipefail
SRC="${GRAFT_REPO_ROOT:-$(pwd)}"; DST=/tmp/raydp_clean_build; OUT="$SRC/gpurun_out/clean_build"
mkdir -p "$OUT"; rm -rf "$DST"; cp -r "$SRC" "$DST"; cd "$DST" || exit 1
rm -rf build gpurun_out raydp_amd/native/jit
find raydp_amd/native -maxdepth 1 -type f \( -name "*.so" -o -name "raydp_supervisor" -o -name "raydp_appmaster" \
  -o -name "raydp_shuffle_service" \) -delete
echo "prebuilt binaries left: $(find . -name '*.so' -o -name '*.hsaco' | wc -l)" | tee "$OUT/summary.txt"
( while sleep 45; do echo "building: $(ls raydp_amd/native/jit 2>/dev/null | wc -l) jit files, $(ls raydp_amd/native/*.so 2>/dev/null | wc -l) libraries"; done ) &
HB=$!
t0=$(date +%s)
timeout -k 10 1000 python -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1
rc=$?
kill $HB
echo "build rc=$rc in $(( $(date +%s) - t0 )) s on $(nproc) visible CPUs" | tee -a "$OUT/summary.txt"
[ $rc -ne 0 ] && { tail -30 "$OUT/build.log"; exit $rc; }
(ls -la raydp_amd/native/*.so raydp_amd/native/raydp_* ; echo "jit code objects: $(ls raydp_amd/native/jit/*.hsaco | wc -l)") | tee -a "$OUT/summary.txt"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 | tee -a "$OUT/summary.txt" || exit 5
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_xgmi.py -x -q --timeout 120 \
  --timeout-method thread -m gpu 2>&1 | tail -2 | tee -a "$OUT/summary.txt"
