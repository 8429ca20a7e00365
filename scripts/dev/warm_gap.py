"""Why the headline's timed pipeline (the 3rd of a process) is slower than the steady state:
runs bench.py's pipeline after warm-up pipelines of the given sizes, then the timed size R
times, and prints each run's wall and phase breakdown (ms). Works on CPU (torch loop) and GPU.

  python scripts/dev/warm_gap.py --warm 3,2 --steps 20 --runs 6
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warm", default="3,2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--pin", type=int, default=0, help="confine the process tree to this many CPUs")
    ap.add_argument("--gc", choices=["collect_freeze", "freeze", "none"], default="freeze",
                    help="what runs between the warm-up and the measured runs")
    args = ap.parse_args()
    if args.pin:
        cpus = sorted(os.sched_getaffinity(0))[:args.pin]
        os.sched_setaffinity(0, cpus)
        print("pinned to", cpus, file=sys.stderr)
    import torch
    import bench
    import raydp  # noqa: F401
    from raydp_amd import context, runtime
    from raydp_amd.torch.estimator import LAST_TIMINGS
    cuda = torch.cuda.is_available()
    if cuda:
        torch.cuda.set_device(0)
    tmp = tempfile.mkdtemp(prefix="raydp_warm_")
    warm = [int(x) for x in args.warm.split(",") if x]
    paths = []
    for k, s in enumerate(warm + [args.steps] * args.runs):
        p = os.path.join(tmp, f"d{k}.csv")
        bench.make_csv(p, s * bench.BATCH, 5000 + k)
        paths.append((p, s))
    runtime.init(num_cpus=4)
    spark = context.init_spark("nyc-warm", 4, 1, "1G")
    spark.conf.set("spark.sql.session.timeZone", "UTC")
    storage = os.path.join(tmp, "results")
    for p, s in paths[:len(warm)]:
        bench.run_pipeline(spark, p, s, 1, storage, fused=cuda)
    import gc
    if args.gc == "collect_freeze":
        gc.collect()
    if args.gc != "none":
        gc.freeze()
    gcs = []   # (phase, generation, t) of every collection during the measured runs

    def on_gc(phase, info):
        gcs.append((phase, info["generation"], time.perf_counter()))
    gc.callbacks.append(on_gc)
    for i, (p, s) in enumerate(paths[len(warm):]):
        gcs.clear()
        if cuda:
            torch.cuda.synchronize()
        bench.DRIVER_TIMINGS.clear()
        t0 = time.perf_counter()
        bench.run_pipeline(spark, p, s, 1, storage, fused=cuda)
        if cuda:
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        gc_ms, gen_n, t_start = 0.0, [0, 0, 0], {}
        for phase, g, t in gcs:
            if phase == "start":
                t_start[g] = t
            elif g in t_start:
                gc_ms += t - t_start.pop(g)
                gen_n[g] += 1
        ph = {k: round(v * 1e3, 2) for k, v in list(LAST_TIMINGS.items()) + list(bench.DRIVER_TIMINGS.items())}
        print(json.dumps({"run": i, "warm": args.warm, "pin": args.pin, "gc": args.gc, "wall_ms": round(wall * 1e3, 2), "gc_ms": round(gc_ms * 1e3, 2), "gc_collections": gen_n, "phases_ms": ph}), flush=True)
    context.stop_spark()
    runtime.shutdown()


if __name__ == "__main__":
    main()
