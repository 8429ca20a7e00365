"""DLRM training throughput on one MI355X (synthetic Criteo-shaped batches, random init).

Model: the reference notebook's configuration (13 dense features, 26 tables, bottom MLP
512-128-32, top MLP 1024-1024-512-256-1, embedding dim 32), table sizes from the synthetic
preprocessing vocabulary (or --rows-per-table). Timed region: K full steps (forward, BCE loss,
backward, SGD incl. sparse embedding update) bracketed by synchronize. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from raydp_amd.models.dlrm import Dlrm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rows-per-table", type=int, default=100000)
    ap.add_argument("--fused-sgd", action="store_true", help="apply the embedding SGD inside backward")
    ap.add_argument("--amp", action="store_true", help="bf16 autocast for the MLP towers")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    sizes = [args.rows_per_table] * 26
    lr = 0.01
    model = Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32,
                 fused_embedding_sgd_lr=lr if args.fused_sgd else None).to(dev)
    opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=lr)
    lossf = torch.nn.BCEWithLogitsLoss()
    n = args.batch * 8
    dense = torch.randn(n, 13, device=dev)
    cats = torch.randint(0, args.rows_per_table, (n, 26), device=dev)
    y = torch.randint(0, 2, (n, 1), device=dev).float()

    def step(i):
        s = (i % 8) * args.batch
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=args.amp):
            out = model(dense[s:s + args.batch], cats[s:s + args.batch])
        loss = lossf(out.float(), y[s:s + args.batch])
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(json.dumps({"metric": "DLRM training samples/sec (synthetic Criteo-shaped)", "value": round(args.steps * args.batch / dt, 1),
                      "unit": "samples/s", "ms_per_step": round(dt * 1e3 / args.steps, 3), "batch": args.batch,
                      "steps": args.steps, "fused_sgd": args.fused_sgd, "amp": args.amp,
                      "loss": float(loss), "tables": 26, "rows_per_table": args.rows_per_table}))


if __name__ == "__main__":
    main()
