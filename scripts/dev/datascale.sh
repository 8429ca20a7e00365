# Data-scale end-to-end runs: 10M rows, 1 epoch, at each batch in $BATCHES (default "64 4096").
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
ROWS=${ROWS:-10000000}
for b in ${BATCHES:-64 4096}; do
  echo "rows=$ROWS batch=$b start $(date +%T)"
  RAYDP_TRACE=gpurun_out/ds_b$b timeout -k 10 400 python bench.py --rows $ROWS --epochs 1 --batch $b --steps 20 --warmup 5 \
    --extra-workloads none >> gpurun_out/datascale.jsonl 2> gpurun_out/datascale_b$b.err || { echo "failed rc=$?"; tail -20 gpurun_out/datascale_b$b.err; exit 1; }
  tail -1 gpurun_out/datascale.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print(d['value'], c.get('rank0_breakdown_s'), c.get('step_time_us') and {k: c['step_time_us'][k] for k in ('p50','p90')}, c.get('host_resources'))"
done
