#!/bin/bash
# Static ISA statistics of one kernel of a hipcc --genco code object (bundled or not):
#   scripts/dev/isa_stats.sh <code object> [kernel name substring] [dump.s]
f=$1; k=${2:-rx_jit_persist}; out=${3:-/tmp/isa_$$.s}
L=/opt/rocm/lib/llvm/bin
co=/tmp/isa_$$.co
$L/clang-offload-bundler --unbundle --type=o --input=$f --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$co 2>/dev/null || cp $f $co
$L/llvm-readelf --notes $co | grep -E "\.name:|vgpr_count|sgpr_count|spill_count" | paste - - - - - | grep "$k" | tr -s ' \t' ' '
$L/llvm-objdump -d --no-show-raw-insn $co | awk -v k="<$k>:" '$0 ~ k {p=1; next} p && /^[0-9a-f]+ <.*>:/ {p=0} p' > $out
c() { grep -cE "$1" $out; }
echo "insts $(grep -cE '^\s+[a-z]' $out) valu $(c '^\s+v_') salu $(c '^\s+s_') mfma $(c v_mfma) lds $(c '^\s+ds_') vmem $(c '^\s+(global|buffer)_') spill_lanes $(c 'v_writelane|v_readlane') cndmask $(c v_cndmask) pk $(c v_pk_) dsw16 $(c ds_write_b16) waitcnt $(c s_waitcnt) nop $(c s_nop)"
rm -f $co
