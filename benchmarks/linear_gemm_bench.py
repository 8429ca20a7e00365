#!/usr/bin/env python
"""Fused Linear GEMM (csrc/hip/linear_act.hip) at the DLRM tower shapes: time per launch and
TFLOP/s of each epilogue (forward with bias+ReLU, dgrad with the ReLU mask, wgrad with the bias
row sums), next to a plain bf16 ``torch.matmul`` (hipBLASLt) of the same shape without any
epilogue. Batch 2048 (benchmarks/dlrm_bench.py), towers of examples/pytorch_dlrm.ipynb cell 9.

Launches are timed as GPU time: ``--reps`` launches are captured into one HIP graph and the
graph is replayed (the ctypes launch path costs more host time than the small kernels take).

``--sweep`` times every tile shape x split-K factor per GEMM (the table rx_lin_plan's
heuristic is fitted to); ``--splits`` / ``--tile`` force one configuration. Prints one JSON line
per shape."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

TILE_NAMES = {1: "64x64", 2: "128x128", 3: "128x64", 4: "64x128"}


def timed(fn, reps, rounds=5):
    """Median GPU us per call over ``rounds`` replays of a graph of ``reps`` calls."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--splits", type=int, default=None)
    ap.add_argument("--tile", type=int, default=0, help="0 auto, 1 64x64, 2 128x128, 3 128x64, 4 64x128")
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--no-torch", action="store_true")
    args = ap.parse_args()
    from raydp_amd.ops import linear_ops as L
    B = args.batch
    layers = [(13, 512), (512, 128), (128, 32), (384, 1024), (1024, 1024), (1024, 512), (512, 256)]
    g = torch.Generator(device="cuda").manual_seed(0)
    tot = {"ours_us": 0.0, "torch_us": 0.0, "best_sweep_us": 0.0}
    for K, N in layers:
        X = torch.randn(B, K, device="cuda", generator=g).to(torch.bfloat16)
        W = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda", generator=g)
        Y = torch.empty(B, N, device="cuda", dtype=torch.bfloat16)
        G = torch.randn(B, N, device="cuda", generator=g).to(torch.bfloat16)
        dX = torch.empty(B, K, device="cuda", dtype=torch.bfloat16)
        dW = torch.empty(N, K, device="cuda")
        db = torch.empty(N, device="cuda")

        def runs(sp, tl):
            return {
                "fwd": (B, N, K, lambda: L.gemm(L.FWD, B, N, K, X, L.ROW, W, L.ROW, Y, bias=bias, relu=True,
                                                splits=sp, tile=tl), lambda: X @ W.T),
                "dgrad": (B, K, N, lambda: L.gemm(L.DGRAD, B, K, N, G, L.ROW, W, L.RED, dX, mask=X, splits=sp,
                                                  tile=tl), lambda: G @ W),
                "wgrad": (N, K, B, lambda: L.gemm(L.WGRAD, N, K, B, G, L.RED, X, L.RED, dW, dbias=db, splits=sp,
                                                  tile=tl), lambda: G.T @ X),
            }
        out = {"K": K, "N": N, "M": B}
        flop = 2.0 * B * N * K
        for name, (m, n, k, ours, ref) in runs(args.splits, args.tile).items():
            t_o = timed(ours, args.reps)
            tl, sp = L.plan(m, n, k, torch.cuda.get_device_properties(0).multi_processor_count, args.tile)
            rec = {"us": round(t_o, 2), "tflops": round(flop / t_o / 1e6, 1),
                   "tile": TILE_NAMES.get(tl, tl), "splits": args.splits or sp}
            tot["ours_us"] += t_o
            if not args.no_torch:
                t_r = timed(ref, args.reps)
                rec.update(torch_us=round(t_r, 2), torch_tflops=round(flop / t_r / 1e6, 1))
                tot["torch_us"] += t_r
            if args.sweep:
                grid = {}
                nk = (k + 63) // 64
                for tl_ in (1, 2, 3, 4):
                    for sp_ in (1, 2, 3, 4, 6, 8, 12, 16):
                        if sp_ > 1 and sp_ > nk // 2:
                            continue
                        fn = runs(sp_, tl_)[name][3]
                        grid[f"{TILE_NAMES[tl_]}/s{sp_}"] = round(timed(fn, args.reps, rounds=3), 2)
                best = min(grid, key=grid.get)
                rec["sweep"] = grid
                rec["best"] = [best, grid[best]]
                tot["best_sweep_us"] += grid[best]
            out[name] = rec
        print(json.dumps(out), flush=True)
    print(json.dumps({"total_per_step_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
