"""NYC-taxi training throughput through the reference's alternative training paths, N GPUs.

* ``--path ddp``     : a user-written torch loop with ``train.torch.prepare_model`` semantics
  (examples/raytrain_nyctaxi.py:140-177) -> raydp_amd.parallel.ddp.DistributedDataParallel
  (bucketed gradient all-reduce; the 194 KB bucket takes the one-shot xGMI exchange).
* ``--path horovod`` : ``hvd.DistributedOptimizer(op=Average)`` + ``broadcast_parameters``
  (examples/horovod_nyctaxi.py:119-162) -> raydp_amd.hvd tensor fusion over the same exchange.
* ``--path fused``   : the TorchEstimator engine (fused HIP step + fused xGMI reduce) on the same
  data, for comparison.

Model NYC_Model (5 Linear + 4 BatchNorm1d, 48,513 params), SmoothL1, Adam 1e-3, 64 rows per GPU
per step, synthetic features resident in HBM (the ETL is not part of this measurement: see
bench.py for the end-to-end metric). Weak scaling. Launch with ``torchrun --nproc-per-node N``.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
import torch.nn as nn

from __graft_entry__ import _nyc_model


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", choices=["ddp", "horovod", "fused"], default="ddp")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_i = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_i)
    dev = torch.device("cuda", dev_i)
    backend = os.environ.get("RAYDP_BENCH_BACKEND", "nccl")
    if world > 1:
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    torch.manual_seed(0)
    model = _nyc_model().to(dev)
    n = args.batch * 256
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    x = torch.randn(n, 20, device=dev, generator=g)
    y = torch.randn(n, 1, device=dev, generator=g) * 10 + 12
    lossf = nn.SmoothL1Loss()
    step_fn = None
    if args.path == "fused":
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
        from raydp_amd.torch.engine import _xgmi_for
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(lossf), args.batch, dev)
        if world > 1:
            dist.broadcast(tr.params, 0)
            tr.refresh_images()
        feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16, device=dev)
        feats[:, :20] = x.to(torch.bfloat16)
        xg = _xgmi_for(tr) if world > 1 else None

        def run(k):
            # epochs over the resident 256 batches (the kernel reads rows [0, nr) only)
            while k > 0:
                nb = min(k, n // args.batch)
                nr = nb * args.batch
                tr.train_epoch(feats, y, nr, None, world_size=world, xg=xg,
                               allreduce=(lambda gr: dist.all_reduce(gr)) if world > 1 and xg is None else None)
                k -= nb
        run(args.warmup)
        kind = "fused step + " + ("xgmi_oneshot" if xg is not None else "allreduce" if world > 1 else "none")
    else:
        if args.path == "ddp":
            from raydp_amd.parallel.ddp import DistributedDataParallel
            net = DistributedDataParallel(model) if world > 1 else model
            opt = torch.optim.Adam(net.parameters(), lr=1e-3)
            kind = "DDP"
        else:
            import raydp_amd.hvd as hvd
            hvd.init()
            opt = torch.optim.Adam(model.parameters(), lr=1e-3 * hvd.size())
            opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), op=hvd.Average)
            hvd.broadcast_parameters(model.state_dict(), root_rank=0)
            hvd.broadcast_optimizer_state(opt, root_rank=0)
            net = model
            kind = "horovod"

        def step_fn(i):
            s = (i % 256) * args.batch
            opt.zero_grad(set_to_none=True)
            loss = lossf(net(x[s:s + args.batch]), y[s:s + args.batch])
            loss.backward()
            opt.step()
            return loss

        def run(k):
            for i in range(k):
                step_fn(i)
        run(args.warmup)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    run(args.steps)
    barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank == 0:
        print(json.dumps({"metric": f"NYCTaxi train samples/sec ({args.path} path)",
                          "value": round(world * args.steps * args.batch / dt, 1), "unit": "samples/s",
                          "n_gpus": world, "steps": args.steps, "ms_per_step": round(dt * 1e3 / args.steps, 4),
                          "per_gpu_batch": args.batch, "path": kind, "scaling": "weak",
                          "data": "synthetic NYCTaxi-shaped features resident in HBM"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
