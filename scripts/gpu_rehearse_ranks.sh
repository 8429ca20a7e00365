# Multi-rank rehearsal of the headline bench on the one-GPU box: ranks share the device, the
# process group is gloo (RCCL refuses two ranks on one GPU), the fused trainer's gradient
# exchange is the xGMI one-shot protocol over same-device IPC (with the RCCL rollback path).
set -o pipefail
for n in 2 4; do
  RAYDP_BENCH_BACKEND=gloo RAYDP_BENCH_CPUS=2 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 20 --warmup 5 --no-reference-config \
    > gpurun_out/rehearse_$n.log 2>&1 || exit 1
done
