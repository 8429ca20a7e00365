"""Where the headline's timed region goes, with enough repetitions to resolve 0.1 ms items:
runs bench.py's pipeline (CSV -> NYC ETL -> fit_on_spark, 20 steps) R times under cProfile after
a warm-up and prints per-function cumulative / own time per pipeline run (ms), plus the
estimator's phase timings averaged over the runs.

  python scripts/profile_headline.py --runs 30 > gpurun_out/headline_profile.txt
"""
import argparse
import cProfile
import io
import os
import pstats
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=30)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import bench
    import raydp  # noqa: F401
    from raydp_amd import context, runtime
    from raydp_amd.torch.estimator import LAST_TIMINGS
    torch.cuda.set_device(0)
    tmp = tempfile.mkdtemp(prefix="raydp_prof_")
    paths = []
    for k in range(args.runs + 3):
        p = os.path.join(tmp, f"d{k}.csv")
        bench.make_csv(p, args.steps * bench.BATCH, 3000 + k)
        paths.append(p)
    runtime.init(num_cpus=4)
    spark = context.init_spark("nyc-prof", 4, 1, "1G")
    spark.conf.set("spark.sql.session.timeZone", "UTC")
    storage = os.path.join(tmp, "results")
    for p in paths[:3]:
        bench.run_pipeline(spark, p, args.steps, 1, storage)
    import gc
    gc.freeze()
    phases, walls = {}, []
    prof = cProfile.Profile()
    for p in paths[3:]:
        torch.cuda.synchronize()
        prof.enable()
        t0 = time.perf_counter()
        bench.DRIVER_TIMINGS.clear()
        bench.run_pipeline(spark, p, args.steps, 1, storage)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        prof.disable()
        for k, v in list(LAST_TIMINGS.items()) + list(bench.DRIVER_TIMINGS.items()):
            phases.setdefault(k, []).append(v)
    n = len(walls)
    print(f"pipeline wall: median {statistics.median(walls) * 1e3:.3f} ms over {n} runs (profiled)")
    for k, v in sorted(phases.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"  {k:32s} {statistics.median(v) * 1e3:7.3f} ms")
    buf = io.StringIO()
    st = pstats.Stats(prof, stream=buf)
    st.sort_stats("cumulative").print_stats(90)
    st.sort_stats("tottime").print_stats(50)
    print(f"(cProfile totals below are for all {n} runs: divide by {n} for per-run ms)")
    print(buf.getvalue())
    context.stop_spark()
    runtime.shutdown()


if __name__ == "__main__":
    main()
