#!/bin/bash
# Ingest throughput (10M x 20 f64) + a kernel/copy trace of a smaller run (copy/decode overlap).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out/prof
df -h /dev/shm | tail -1
timeout -k 10 300 python benchmarks/ingest_bench.py --rows 10000000 --cols 20 --blocks 16 > gpurun_out/ingest_bench.log 2>&1
rc=$?; echo "ingest rc=$rc"; tail -1 gpurun_out/ingest_bench.log | cut -c1-1200
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/prof -o ingest -- python3 $R/benchmarks/ingest_bench.py --rows 2000000 --cols 20 --blocks 8 --repeat 2 > $R/gpurun_out/prof_ingest.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
