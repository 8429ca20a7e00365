#!/bin/bash
# Round-3 code vs this tree, interleaved on one box: the driver's headline command 5 + 5 times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=$R/gpurun_out/r5_headline_ab.jsonl
for i in 1 2 3 4 5; do
  for t in r3 head; do
    if [ $t = r3 ]; then d=$R/bisect/r3full; else d=$R; fi
    line=$(cd $d && timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 2>> $R/gpurun_out/r5_headline_ab.err | tail -1) || { echo "fail $t"; exit 3; }
    echo "{\"tree\": \"$t\", \"run\": $i, \"bench\": $line}" >> $out
    echo "$t $i $(echo $line | cut -c1-160)"
  done
done
