# Headline x3, its kernel stats, then the fused engine at batch 4096 / 1000 at data scale (+ rocprof at 4096)
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out/prof
R=$(pwd)
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/h_bench.jsonl 2>> gpurun_out/h_bench.err || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/h_bench.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["value"], d["ms_per_step"], c.get("engine"), {k: v.get("value") for k, v in c.get("other_workloads", {}).items()})
PY
timeout -k 10 400 python bench.py --rows 10000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 > gpurun_out/h_ds4096.jsonl 2> gpurun_out/h_ds.err || exit 2
timeout -k 10 400 python bench.py --rows 2000000 --epochs 1 --batch 1000 --steps 20 --warmup 5 >> gpurun_out/h_ds4096.jsonl 2>> gpurun_out/h_ds.err || exit 3
python - <<'PY'
import json
for l in open("gpurun_out/h_ds4096.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["value"], d["steps"], c.get("global_batch"), c.get("engine"), c.get("train_rows_per_gpu"), c.get("rank0_breakdown_s"), c.get("step_time_us"))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/mw4096 -o run -- \
  python3 $R/bench.py --rows 2000000 --epochs 1 --batch 4096 --steps 20 --warmup 5 --extra-workloads none \
  > $R/gpurun_out/prof/mw4096.log 2>&1 || { echo prof failed; tail -5 $R/gpurun_out/prof/mw4096.log; exit 4; }
head -8 $R/gpurun_out/prof/mw4096/run_kernel_stats.csv | cut -c1-200
