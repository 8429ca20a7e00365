# DLRM persistent step: per-phase profile at G = 64 / 128 / 256 and the grid-barrier price
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
for G in 64 128 256; do
  RAYDP_DLRM_STEP_G=$G timeout -k 10 120 python benchmarks/dlrm_bench.py --persistent --batch 128 --steps 80 --warmup 16 \
    >> gpurun_out/dlrm_phase.jsonl 2>> gpurun_out/dlrm_phase.err || exit 1
done
timeout -k 10 120 python benchmarks/grid_barrier_bench.py > gpurun_out/grid_barrier.json 2>> gpurun_out/dlrm_phase.err
python - <<'PY'
import json
for l in open("gpurun_out/dlrm_phase.jsonl"):
    d = json.loads(l); print(d["workgroups"], d["ms_per_step"], d["phase_us"])
PY
cat gpurun_out/grid_barrier.json
