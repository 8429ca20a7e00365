#!/bin/bash
# Build every native library + the JIT cache (__graft_entry__.build), plus the layer-stamp
# variant of the NYC batch-64 kernel, then drop JIT objects this build did not produce.
cd "$(dirname "$0")/../.."
touch /tmp/.build_mark
timeout 1500 python -c "import __graft_entry__ as g; g.build()" > /tmp/build.log 2>&1 || { grep -B2 -A8 " error" /tmp/build.log | head -40; exit 1; }
RAYDP_MLP_LAYER_STAMPS=1 timeout 900 python scripts/dev/jit_one.py 64 > /dev/null 2>&1 || exit 2
find raydp_amd/native/jit -maxdepth 1 -name "*.hsaco" ! -newer /tmp/.build_mark -delete
for f in raydp_amd/native/jit/*.hip; do [ -e "${f%.hip}.hsaco" ] || rm -f "$f"; done
echo "built; jit objects: $(ls raydp_amd/native/jit | wc -l)"
