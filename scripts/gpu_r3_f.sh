#!/bin/bash
# Round 3, batch F: full GPU suite (trainer arena + single readback, warm-worker graphs), the
# 2-worker DLRM e2e, a repeated-run profile of the headline, then the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $T tests/ -m gpu > gpurun_out/rf_tests.log 2>&1 || { grep -E "passed|failed|Error|^E " gpurun_out/rf_tests.log | tail -25; exit 21; }
grep -E "passed|failed" gpurun_out/rf_tests.log | tail -2
rm -f gpurun_out/bench.jsonl
bash scripts/gpu.sh bench 1 20 5 4 || exit 25
python - <<'PY'
import json
for l in open("gpurun_out/bench.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["config"]["rank0_breakdown_s"])
PY
timeout -k 10 300 python scripts/profile_headline.py --runs 30 > gpurun_out/rf_headline_profile.txt 2> gpurun_out/rf_headline_profile.err || exit 26
head -30 gpurun_out/rf_headline_profile.txt
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 --workers 2 \
  > gpurun_out/rf_dlrm2w.jsonl 2> gpurun_out/rf_dlrm2w.err || exit 22
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 \
  >> gpurun_out/rf_dlrm2w.jsonl 2>> gpurun_out/rf_dlrm2w.err || exit 23
cut -c1-700 gpurun_out/rf_dlrm2w.jsonl
