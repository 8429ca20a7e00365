# DDP bucket size x comm stream sweep on the DLRM dense gradients (8.7 MB), ranks sharing the one
# GPU (gloo bootstrap, buckets over the xGMI kernels); then a kernel trace of one configuration
# for the overlap check (scripts/trace_overlap.py --kernel lin_ --with xg_allreduce).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof; export HSA_ENABLE_IPC_MODE_LEGACY=0
export RAYDP_BENCH_BACKEND=gloo
for W in 2 4; do
  for MB in 1 2 4 8 32; do
    for CS in 1 0; do
      RAYDP_DDP_BUCKET_MB=$MB RAYDP_DDP_COMM_STREAM=$CS timeout -k 10 200 python -m torch.distributed.run \
        --nnodes=1 --nproc-per-node $W --master-addr 127.0.0.1 --master-port 29611 \
        benchmarks/dlrm_bench.py --batch 128 --steps 160 --warmup 16 --rows-per-table 20000 --graph \
        >> gpurun_out/ddp_sweep.jsonl 2>> gpurun_out/ddp_sweep.err || { echo "W=$W MB=$MB CS=$CS failed"; tail -5 gpurun_out/ddp_sweep.err; exit 1; }
    done
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/ddp_sweep.jsonl"):
    d = json.loads(l)
    print(d["n_gpus"], d["ddp"]["bucket_mb"], d["ddp"]["buckets"], d["ddp"]["allreduce"][:60], d["ms_per_step"], d["value"], d["hip_graph"])
PY
cd /tmp && export TMPDIR=/tmp
RAYDP_DDP_BUCKET_MB=2 RAYDP_DDP_COMM_STREAM=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
  -d $GRAFT_REPO_ROOT/gpurun_out/prof/ddp_overlap -o run -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 $GRAFT_REPO_ROOT/benchmarks/dlrm_bench.py --batch 128 --steps 64 \
  --warmup 8 --rows-per-table 20000 > $GRAFT_REPO_ROOT/gpurun_out/prof/ddp_overlap.log 2>&1 || { echo prof failed; tail -5 $GRAFT_REPO_ROOT/gpurun_out/prof/ddp_overlap.log; exit 1; }
echo prof ok
