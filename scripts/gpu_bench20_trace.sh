#!/bin/bash
# Driver-config bench: 5 runs, then one traced run (span timeline) and a cProfile of the timed region.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tr
for k in 1 2 3 4 5; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config > gpurun_out/b20_$k.log 2>&1 || exit 1
  echo "$(grep -o '"value": [0-9.]*' gpurun_out/b20_$k.log) $(grep -o '"rank0_breakdown_s": {[^}]*}' gpurun_out/b20_$k.log)"
done
RAYDP_TRACE=gpurun_out/tr/nyc timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config > gpurun_out/b20_traced.log 2>&1 || exit 1
python scripts/trace_summary.py gpurun_out/tr/nyc > gpurun_out/b20_timeline.txt || exit 1
cat gpurun_out/b20_timeline.txt
timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-reference-config --profile-timed gpurun_out/b20_cprofile.txt > gpurun_out/b20_prof.log 2>&1 || exit 1
