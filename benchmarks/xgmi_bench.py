"""One-shot xGMI all-reduce (csrc/comm/xgmi_allreduce.hip) latency per bucket size, W ranks.

On the one-GPU box the W ranks share the device (the peer mapping is the same IPC path as
across 8 GPUs, but the "links" are local HBM and the ranks' kernels time-share CUs), so the
numbers are an upper bound of the protocol's cost, not a link measurement. Device time per call
from HIP events over R calls after a warm-up, median over ranks; plus the same through
torch.distributed (gloo here) for the host-bounce reference. One JSON line.

  python benchmarks/xgmi_bench.py --world 4 --sizes 194052,1048576
"""
import argparse
import json
import multiprocessing as mp
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, sizes, reps, q, kernel="oneshot"):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from raydp_amd.ops.comm import XgmiComm
        comm = XgmiComm.create(max(sizes) // 4 + 64, timeout_s=20.0)
        out = {}
        for nbytes in sizes:
            n = nbytes // 4
            t = torch.randn(n, device="cuda")
            op = comm.allreduce2_ if kernel == "twoshot" else comm.allreduce_
            for _ in range(10):
                op(t, 1.0 / world)
            torch.cuda.synchronize()
            dist.barrier()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(reps):
                op(t, 1.0 / world)
            ev[1].record()
            ev[1].synchronize()
            out[nbytes] = ev[0].elapsed_time(ev[1]) * 1000.0 / reps
        q.put((rank, out, comm.error()))
        dist.barrier()
        comm.close()
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--sizes", default="194052,1048576,8708740")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--kernel", choices=["oneshot", "twoshot"], default="oneshot",
                    help="oneshot: every rank pulls the whole bucket from every peer; twoshot: all-pairs "
                         "reduce-scatter + all-gather (2S/N bytes per link)")
    args = ap.parse_args()
    sizes = [int(x) for x in args.sizes.split(",")]
    sys.path.insert(0, ROOT)
    from raydp_amd.train.trainer import _free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, args.world, port, sizes, args.reps, q, args.kernel)) for r in range(args.world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    per = {s: statistics.median(r[1][s] for r in res) for s in sizes}
    print(json.dumps({"metric": f"xGMI {args.kernel} all-reduce device time per call (us), ranks sharing one GPU",
                      "kernel": args.kernel, "world": args.world, "reps": args.reps,
                      "us_per_call": {str(s): round(v, 2) for s, v in per.items()},
                      "errors": [r[2] for r in res]}), flush=True)


if __name__ == "__main__":
    main()
