#!/bin/bash
# Round 3, batch G: headline after the host-path trims (6 runs), profile, 2-rank rehearsals.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f gpurun_out/bench.jsonl gpurun_out/rehearse_spmd.jsonl gpurun_out/rehearse_estimator.jsonl
bash scripts/gpu.sh bench 1 20 5 6 || exit 25
python - <<'PY'
import json
for l in open("gpurun_out/bench.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["config"]["rank0_breakdown_s"])
PY
timeout -k 10 300 python scripts/profile_headline.py --runs 30 > gpurun_out/rg_headline_profile.txt 2> gpurun_out/rg_headline_profile.err || exit 26
head -14 gpurun_out/rg_headline_profile.txt
bash scripts/gpu.sh rehearse 2 20 5 > /dev/null || exit 27
python - <<'PY'
import json
for f in ("gpurun_out/rehearse_spmd.jsonl", "gpurun_out/rehearse_estimator.jsonl"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l); c = d["config"]
            print(f, d["value"], c.get("topology"), c.get("allreduce"), c.get("rank0_breakdown_s"))
PY
