#!/bin/bash
# A/B of the overlapped conversion (RAYDP_OVERLAP_CONVERSION) at the driver's 20-step config,
# alternating runs, then one traced run (span timeline of the timed region).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
for k in 1 2 3 4; do
  for ov in 1 0; do
    RAYDP_OVERLAP_CONVERSION=$ov timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config > gpurun_out/ab_${ov}_$k.log 2>&1 || exit 1
    echo "overlap=$ov $(grep -o '"value": [0-9.]*' gpurun_out/ab_${ov}_$k.log) $(grep -o '"rank0_breakdown_s": {[^}]*}' gpurun_out/ab_${ov}_$k.log)"
  done
done
RAYDP_TRACE=gpurun_out/tr/nyc timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config > gpurun_out/ab_traced.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/tr/nyc > gpurun_out/ab_timeline.txt || exit 1
cat gpurun_out/ab_timeline.txt
