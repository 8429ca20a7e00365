#!/bin/bash
# Round 3, batch D: worker logs of the 2-worker DLRM e2e; headline cProfile + span timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sess gpurun_out/tr /tmp/rs
export HSA_ENABLE_IPC_MODE_LEGACY=0
RAYDP_KEEP_SESSION_DIR=1 TMPDIR=/tmp/rs timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 \
  --rows 20000 --warmup-rows 5000 --workers 2 > gpurun_out/rd_dlrm2w.jsonl 2> gpurun_out/rd_dlrm2w.err
rc=$?
echo "rc=$rc"; cut -c1-300 gpurun_out/rd_dlrm2w.jsonl
for f in $(find /tmp/rs -name "actor-*.log" -size +0); do cp $f gpurun_out/sess/; done
for f in gpurun_out/sess/actor-*.log; do echo "== $f"; grep -v amdgpu.ids $f | grep -v "^\[Gloo\]" | tail -25; done
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-reference-config --profile-timed gpurun_out/rd_cprof.txt \
  > gpurun_out/rd_bench_prof.jsonl 2> gpurun_out/rd_bench_prof.err || exit 26
RAYDP_TRACE=gpurun_out/tr/nyc timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-reference-config \
  > gpurun_out/rd_bench_tr.jsonl 2> gpurun_out/rd_bench_tr.err || exit 27
python scripts/trace_summary.py gpurun_out/tr/nyc > gpurun_out/rd_nyc_timeline.txt 2>&1
head -70 gpurun_out/rd_nyc_timeline.txt
