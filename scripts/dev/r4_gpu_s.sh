# Actor wake-up latency on the box (CPU only) and a headline A/B of the busy-poll window
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
rm -f gpurun_out/actor_rtt.jsonl gpurun_out/bench_spin.jsonl gpurun_out/bench_spin.err
for v in 0 2000 10000; do
  RAYDP_ACTOR_SPIN_US=$v timeout -k 10 120 python scripts/dev/actor_rtt.py | sed "s/^/{\"spin_us\": $v, \"rtt\": /; s/\$/}/" >> gpurun_out/actor_rtt.jsonl || exit 3
done
cat gpurun_out/actor_rtt.jsonl
for i in 1 2 3 4; do
  for v in 0 5000; do
    RAYDP_ACTOR_SPIN_US=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
      | sed "s/^/{\"spin_us\": $v, \"bench\": /; s/\$/}/" >> gpurun_out/bench_spin.jsonl 2>> gpurun_out/bench_spin.err || exit 4
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/bench_spin.jsonl"):
    d = json.loads(l); print(d["spin_us"], d["bench"]["value"])
PY
