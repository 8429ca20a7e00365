#!/usr/bin/env python
"""Fused Linear GEMM (csrc/hip/linear_act.hip) at the DLRM tower shapes: time per launch and
TFLOP/s of each epilogue (forward with bias+ReLU, dgrad with the ReLU mask, wgrad with the bias
row sums), next to a plain bf16 ``torch.matmul`` (hipBLASLt) of the same shape without any
epilogue. Batch 2048 (benchmarks/dlrm_bench.py), towers of examples/pytorch_dlrm.ipynb cell 9.

``--splits`` forces the split-K factor. Prints one JSON line per shape. The launch loop is
host-bound for the small shapes: take kernel times from ``rocprofv3 --kernel-trace`` of this
script (profiles/r2_linear_gemm_kernel_times.txt)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--splits", type=int, default=None)
    args = ap.parse_args()
    from raydp_amd.ops import linear_ops as L
    B = args.batch
    layers = [(13, 512), (512, 128), (128, 32), (384, 1024), (1024, 1024), (1024, 512), (512, 256)]
    g = torch.Generator(device="cuda").manual_seed(0)
    tot = {"ours_us": 0.0, "torch_us": 0.0}
    for K, N in layers:
        X = torch.randn(B, K, device="cuda", generator=g).to(torch.bfloat16)
        W = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda", generator=g)
        Y = torch.empty(B, N, device="cuda", dtype=torch.bfloat16)
        G = torch.randn(B, N, device="cuda", generator=g).to(torch.bfloat16)
        dX = torch.empty(B, K, device="cuda", dtype=torch.bfloat16)
        dW = torch.empty(N, K, device="cuda")
        db = torch.empty(N, device="cuda")
        sp = args.splits
        runs = {
            "fwd": (lambda: L.gemm(L.FWD, B, N, K, X, L.ROW, W, L.ROW, Y, bias=bias, relu=True, splits=sp),
                    lambda: X @ W.T),
            "dgrad": (lambda: L.gemm(L.DGRAD, B, K, N, G, L.ROW, W, L.RED, dX, mask=X, splits=sp),
                      lambda: G @ W),
            "wgrad": (lambda: L.gemm(L.WGRAD, N, K, B, G, L.RED, X, L.RED, dW, dbias=db, splits=sp),
                      lambda: G.T @ X),
        }
        out = {"K": K, "N": N, "M": B, "splits": sp}
        flop = 2.0 * B * N * K
        for name, (ours, ref) in runs.items():
            t_o, t_r = timed(ours, args.reps), timed(ref, args.reps)
            out[name] = {"us": round(t_o, 2), "tflops": round(flop / t_o / 1e6, 1),
                         "torch_us": round(t_r, 2), "torch_tflops": round(flop / t_r / 1e6, 1)}
            tot["ours_us"] += t_o
            tot["torch_us"] += t_r
        print(json.dumps(out), flush=True)
    print(json.dumps({"total_per_step_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
