#!/bin/bash
# Round 3, batch C: why the warm 2-worker DLRM group aborts in its second fit (actor logs kept).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sess /tmp/rs
export HSA_ENABLE_IPC_MODE_LEGACY=0
TMPDIR=/tmp/rs timeout -k 10 400 python benchmarks/dlrm_e2e_bench.py --batch 128 --rows 20000 \
  --warmup-rows 5000 --workers 2 > gpurun_out/rc_dlrm2w.jsonl 2> gpurun_out/rc_dlrm2w.err
rc=$?
echo "rc=$rc"; cut -c1-400 gpurun_out/rc_dlrm2w.jsonl
for f in $(find /tmp/rs -name "actor-*.log" -size +0); do cp $f gpurun_out/sess/; done
for f in gpurun_out/sess/actor-*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -40; done
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/bench.jsonl
bash scripts/gpu.sh bench 1 20 5 5 || exit 25
python - <<'PY'
import json
for l in open("gpurun_out/bench.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["value"], d["config"]["rank0_breakdown_s"])
PY
