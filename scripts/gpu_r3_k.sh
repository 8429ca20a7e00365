#!/bin/bash
# Round 3, batch K: full GPU suite + smoke, headline x6, 2-rank rehearsals (both topologies),
# DLRM graph bench, DLRM e2e 1/2 workers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu.sh tests || exit 20
rm -f gpurun_out/bench.jsonl gpurun_out/rehearse_spmd.jsonl gpurun_out/rehearse_estimator.jsonl gpurun_out/dlrm.jsonl
bash scripts/gpu.sh bench 1 20 5 6 > /dev/null || exit 25
bash scripts/gpu.sh rehearse 2 20 5 > /dev/null || exit 27
python - <<'PY'
import json
for f in ("gpurun_out/bench.jsonl", "gpurun_out/rehearse_spmd.jsonl", "gpurun_out/rehearse_estimator.jsonl"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["config"]
            print(f.split("/")[-1], d["value"], c.get("topology"), c.get("allreduce"), c.get("rank0_breakdown_s"))
PY
bash scripts/gpu.sh dlrm 2048 128 > /dev/null || exit 28
cut -c1-200 gpurun_out/dlrm.jsonl
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 50000 --warmup-rows 5000 --workers 2 \
  > gpurun_out/rk_dlrm_e2e.jsonl 2> gpurun_out/rk_dlrm_e2e.err || exit 22
timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 2048 >> gpurun_out/rk_dlrm_e2e.jsonl 2>> gpurun_out/rk_dlrm_e2e.err || exit 23
cut -c1-400 gpurun_out/rk_dlrm_e2e.jsonl
