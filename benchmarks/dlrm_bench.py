"""DLRM training throughput on N MI355X (synthetic Criteo-shaped batches, random init).

Model: the reference notebook's configuration (examples/pytorch_dlrm.ipynb cell 9: 13 dense
features, 26 tables, bottom MLP 512-128-32, top MLP 1024-1024-512-256-1, embedding dim 32),
``--rows-per-table`` rows per table. One GPU: fused multi-table embedding kernels (optionally
with the sparse SGD fused into backward). N GPUs (``torchrun --nproc-per-node N``): tables
sharded table-wise over the ranks with all-to-all of ids and rows (RCCL over xGMI), dense MLPs
data parallel (bucketed all-reduce); weak scaling, ``--batch`` rows per GPU.
Timed region: K full steps (forward, BCE loss, backward, all collectives, SGD incl. the sparse
embedding update) bracketed by barrier + synchronize; the max over ranks. One JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

from raydp_amd.models.dlrm import Dlrm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048, help="rows per GPU per step")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rows-per-table", type=int, default=100000)
    ap.add_argument("--fused-sgd", action="store_true", help="apply the embedding SGD inside backward")
    ap.add_argument("--amp", action="store_true", help="bf16 autocast for the MLP towers")
    ap.add_argument("--model-parallel", action="store_true", help="sharded tables even on 1 GPU")
    ap.add_argument("--graph", action="store_true",
                    help="one GPU: replay the 8 steps of a data cycle from one captured HIP graph")
    ap.add_argument("--eager-tail", action="store_true",
                    help="torch SGD + nn.BCEWithLogitsLoss + sparse embedding gradients instead of the fused "
                         "step tail (multi-tensor SGD writing the tower images, fused BCE, embedding SGD in "
                         "backward: raydp_amd/ops/fused_optim.py)")
    ap.add_argument("--eager-mlp", action="store_true",
                    help="run the MLP towers as eager nn.Linear/ReLU instead of the fused MFMA kernels")
    args = ap.parse_args()
    if args.eager_mlp:
        os.environ["RAYDP_FUSED_LINEAR"] = "0"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev_i = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_i)
    dev = torch.device("cuda", dev_i)
    mp = world > 1 or args.model_parallel
    if mp:
        dist.init_process_group(os.environ.get("RAYDP_BENCH_BACKEND", "nccl"), device_id=dev
                                if os.environ.get("RAYDP_BENCH_BACKEND", "nccl") == "nccl" else None)
    torch.manual_seed(0)
    sizes = [args.rows_per_table] * 26
    lr = 0.01
    fused_tail = not args.eager_tail
    model = Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32,
                 fused_embedding_sgd_lr=lr if (args.fused_sgd or fused_tail) else None, model_parallel=mp,
                 static_batch=True).to(dev)
    net = model
    if mp:
        from raydp_amd.parallel.ddp import DistributedDataParallel
        net = DistributedDataParallel(model)
    from raydp_amd.ops.fused_optim import FusedBCEWithLogits, FusedSGD
    opt_cls = FusedSGD if fused_tail else torch.optim.SGD
    opt = opt_cls([p for p in model.parameters() if p.requires_grad], lr=lr)
    lossf = FusedBCEWithLogits() if fused_tail else torch.nn.BCEWithLogitsLoss()
    n = args.batch * 8
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    dense = torch.randn(n, 13, device=dev, generator=g)
    cats = torch.randint(0, args.rows_per_table, (n, 26), device=dev, generator=g)
    y = torch.randint(0, 2, (n, 1), device=dev, generator=g).float()

    def step(i):
        s = (i % 8) * args.batch
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp):
            out = net(dense[s:s + args.batch], cats[s:s + args.batch])
        loss = lossf(out.float(), y[s:s + args.batch])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    def barrier():
        torch.cuda.synchronize()
        if mp:
            dist.barrier()
            torch.cuda.synchronize()

    for i in range(args.warmup):
        step(i)
    graph, graph_err = None, None
    # model parallel: capturable when the DDP buckets and the sharded tables' exchanges all ride
    # the one-shot xGMI kernels (no torch.distributed call inside a step)
    mp_capturable = mp and net.capturable() and all(
        getattr(m, "_xg", None) is not None for m in model.modules() if hasattr(m, "_xg_plan"))
    if args.graph and (not mp or mp_capturable):
        graph, graph_err = _capture_cycle(_graph_step(net, lossf, opt, dense, cats, y, args), opt, dev)
    barrier()
    t = time.perf_counter()
    if graph is not None:
        g, static_loss = graph
        assert args.steps % 8 == 0, "--graph replays whole 8-step data cycles"
        for _ in range(args.steps // 8):
            g.replay()
        loss = static_loss
    else:
        for i in range(args.steps):
            loss = step(i)
    barrier()
    dt = time.perf_counter() - t
    if mp:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    if rank == 0:
        print(json.dumps({"metric": "DLRM training samples/sec (synthetic Criteo-shaped)",
                          "value": round(world * args.steps * args.batch / dt, 1), "unit": "samples/s",
                          "n_gpus": world, "ms_per_step": round(dt * 1e3 / args.steps, 3),
                          "per_gpu_batch": args.batch, "steps": args.steps, "warmup": args.warmup,
                          "embeddings": "table-wise sharded + all-to-all" if mp else "replicated fused",
                          "fused_sgd": args.fused_sgd or fused_tail, "fused_tail": fused_tail,
                          "amp": args.amp, "loss": float(loss),
                          "mlp": "eager torch" if args.eager_mlp else "fused MFMA towers (csrc/hip/linear_act.hip)",
                          "tables": 26, "rows_per_table": args.rows_per_table, "scaling": "weak",
                          "hip_graph": graph is not None, "graph_error": graph_err,
                          "mp_capturable": bool(mp_capturable),
                          "ddp": {"buckets": len(net.buckets), "bucket_mb": os.environ.get("RAYDP_DDP_BUCKET_MB"),
                                  "allreduce": net._allreduce.kind,
                                  "launched": dict(net._allreduce.launched)} if mp else None}), flush=True)
    if mp:
        dist.destroy_process_group()


def _graph_step(net, lossf, opt, dense, cats, y, args):
    """The training step of data slice k for capture. Every step drops the gradients before its
    backward, so autograd ASSIGNS each parameter's gradient (from the graph's private pool; the
    captured optimizer kernel reads that step's buffers) instead of a captured memset followed
    by an accumulate-add per parameter. ``first`` is kept for callers that zero eagerly."""
    def run(k, first):
        s = k * args.batch
        out = net(dense[s:s + args.batch], cats[s:s + args.batch])
        loss = lossf(out.float(), y[s:s + args.batch])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss
    return run


def _capture_cycle(run, opt, dev):
    """Capture the 8 steps of one data cycle into one graph; (graph, last loss) or the error."""
    try:
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):       # eager steps on a side stream first, as capture requires
            for k in range(2):
                run(k, False)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            loss = None
            for k in range(8):
                loss = run(k, k == 0)
        g.replay()
        torch.cuda.synchronize(dev)
        return (g, loss), None
    except Exception as e:  # noqa: BLE001 - report and run eagerly
        torch.cuda.synchronize(dev)
        return None, repr(e)[:300]


if __name__ == "__main__":
    main()
