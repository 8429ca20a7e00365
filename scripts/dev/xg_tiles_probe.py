"""Probe the in-launch xGMI gradient exchange with W ranks sharing the one GPU: per rank, the
time of each epoch (persistent batch 64 or multi-workgroup batch > 128), the path taken, and
any error, printed as it happens (a hang shows which rank stopped where).

  python scripts/dev/xg_tiles_probe.py --world 8 --batch 64 --steps 4 --epochs 2
"""
import argparse
import multiprocessing as mp
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main_rank(rank, world, port, args):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import torch.nn as nn
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from test_gpu_xgmi import _nyc_full
        from raydp_amd.models.mlp_spec import extract_mlp_spec
        from raydp_amd.ops.comm import XgmiComm
        from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
        dev = torch.device("cuda", 0)
        torch.manual_seed(0)
        model = _nyc_full()
        opt = torch.optim.SGD(model.parameters(), lr=1e-2, momentum=0.9)
        tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(opt), loss_code(nn.SmoothL1Loss()),
                             args.batch, dev, world=world)
        tr.record_steps = True
        n = args.batch * args.steps
        g = torch.Generator().manual_seed(7 + rank)
        feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
        feats[:, :20] = torch.randn(n, 20, generator=g).to(torch.bfloat16)
        feats, labels = feats.to(dev), torch.randn(n, 1, generator=g).to(dev)
        xg = XgmiComm.create(tr.total if tr.G > 1 else tr.grads.numel(), timeout_s=args.timeout, host_seq=True)
        if xg is not None:       # (world 1: no communicator, the plain one-GPU kernels)
            tr.share = xg.share
            if tr._mw_args is not None:
                tr._mw_args.share = xg.share
        print(f"rank {rank}: share {getattr(xg, 'share', 1)} G {tr.G}", flush=True)
        for ep in range(args.epochs):
            t0 = time.perf_counter()
            try:
                tr.train_epoch(feats, labels, n, None, world_size=world, xg=xg)
                raw = getattr(tr, "_step_stamps", None)
                st = tr.step_times_us()
                if args.timeline and raw is not None and ep == args.epochs - 1 and tr.last_path.startswith("persistent"):
                    s = [int(x) for x in raw[:32]]
                    us = lambda k: round((s[k] - s[0]) * 0.01, 2) if s[k] else None   # noqa: E731
                    print(f"rank {rank} middle step (us from its start): fwd {us(3)} bwd {us(4)} vec {us(5)} | "
                          f"L0 opt: flag {us(16)} wgrad {us(28)} pushed {us(29)} lane0 summed {us(31)} "
                          f"wg summed {us(30)} updated {us(26)} images {us(27)} counted {us(17)}", flush=True)
                    if st is not None:
                        print(f"rank {rank} step_us p50 {float(np.median(st)):.2f} min {float(st.min()):.2f}", flush=True)
                print(f"rank {rank} epoch {ep}: {time.perf_counter() - t0:.4f} s path {tr.last_path} "
                      f"step_us {None if st is None else [round(float(x), 1) for x in st[:8]]}", flush=True)
            except Exception:  # noqa: BLE001
                print(f"rank {rank} epoch {ep}: FAILED after {time.perf_counter() - t0:.2f} s\n"
                      + traceback.format_exc()[-800:], flush=True)
                break
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=10.0)
    ap.add_argument("--timeline", action="store_true", help="print the middle step's layer-0 exchange stamps")
    ap.add_argument("--dry-run", action="store_true",
                    help="RAYDP_XG_DRYRUN=1: the world > 1 kernels without the exchange (its cost = the difference)")
    a = ap.parse_args()
    if a.dry_run:
        os.environ["RAYDP_XG_DRYRUN"] = "1"
    sys.path.insert(0, ROOT)
    from raydp_amd.train.trainer import _free_port
    port = _free_port()
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=main_rank, args=(r, a.world, port, a)) for r in range(a.world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join()
    sys.exit(max((p.exitcode or 0) for p in ps))
