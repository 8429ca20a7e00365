#!/bin/bash
# rocprofv3 kernel stats of a short bench run (summary copied to profiles/ afterwards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python3 $R/bench.py --steps 1000 --warmup 100 > $R/gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; head -6 $R/gpurun_out/prof/bench_kernel_stats.csv | cut -c1-160; exit $rc
