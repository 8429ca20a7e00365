# Data-scale end-to-end runs: 10M rows x 1 and x 5 epochs at batch 64.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
ROWS=${ROWS:-10000000}
for cfg in "1 64" "5 64"; do
  set -- $cfg
  echo "rows=$ROWS epochs=$1 batch=$2 start $(date +%T)"
  RAYDP_TRACE=gpurun_out/ds_e$1 timeout -k 10 500 python bench.py --rows $ROWS --epochs $1 --batch $2 --steps 20 --warmup 5 \
    >> gpurun_out/datascale.jsonl 2> gpurun_out/datascale_e$1.err || { echo "failed rc=$?"; tail -20 gpurun_out/datascale_e$1.err; exit 1; }
  tail -c 2500 gpurun_out/datascale.jsonl
done
