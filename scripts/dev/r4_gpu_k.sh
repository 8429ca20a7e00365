# Data scale with 8 executors (10 M rows: batch 64 x 1 epoch, batch 4096 x 1 epoch), then the
# 2-worker estimator topology (span timeline: workers start while the conversion runs)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 500 python bench.py --rows 10000000 --epochs 1 --batch 64 --steps 20 --warmup 5 > gpurun_out/k_ds.jsonl 2> gpurun_out/k_ds.err || exit 1
timeout -k 10 400 python bench.py --rows 10000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 >> gpurun_out/k_ds.jsonl 2>> gpurun_out/k_ds.err || exit 2
python - <<'PY'
import json
for l in open("gpurun_out/k_ds.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["value"], d["steps"], c.get("global_batch"), c.get("engine"), c.get("rank0_breakdown_s"))
PY
bash scripts/gpu.sh trace 2 || exit 3
bash scripts/gpu.sh rehearse 2 20 5 || exit 4
