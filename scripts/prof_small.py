"""Where does a short bench run spend its time? Runs the bench pipeline at the driver's config
(warm-up pipeline of W steps, then a timed pipeline of K steps) and writes a cProfile of the
timed pipeline (cumulative and self time) plus the estimator's phase marks to
gpurun_out/prof_small_<K>.txt."""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "examples"))
import torch  # noqa: E402

import bench  # noqa: E402
from raydp_amd import context, runtime  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--repeat", type=int, default=3)
args = ap.parse_args()

torch.cuda.set_device(0)
tmp = tempfile.mkdtemp()
warm = os.path.join(tmp, "w.csv")
bench.make_csv(warm, max(1, args.warmup) * 64, 1)
mains = []
for r in range(args.repeat):
    p = os.path.join(tmp, f"m{r}.csv")
    bench.make_csv(p, args.steps * 64, 2 + r)
    mains.append(p)
runtime.init(num_cpus=4)
spark = context.init_spark("prof", 4, 1, "1G")
spark.conf.set("spark.sql.session.timeZone", "UTC")
bench.run_pipeline(spark, warm, args.warmup, 1, os.path.join(tmp, "r"))
torch.cuda.synchronize()
from raydp_amd.torch.estimator import LAST_TIMINGS  # noqa: E402
out = io.StringIO()
for r, p in enumerate(mains):
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if r == len(mains) - 1:
        pr.enable()
    bench.run_pipeline(spark, p, args.steps, 1, os.path.join(tmp, "r"))
    torch.cuda.synchronize()
    pr.disable()
    dt = time.perf_counter() - t0
    out.write(f"=== repeat {r}: {dt * 1e3:.2f} ms  phases(ms): "
              + ", ".join(f"{k}={v * 1e3:.2f}" for k, v in LAST_TIMINGS.items()) + "\n")
    if r == len(mains) - 1:
        for key in ("cumulative", "tottime"):
            s = io.StringIO()
            pstats.Stats(pr, stream=s).sort_stats(key).print_stats(60)
            out.write(f"--- sorted by {key}\n" + s.getvalue())
os.makedirs(os.path.join(HERE, "gpurun_out"), exist_ok=True)
open(os.path.join(HERE, "gpurun_out", f"prof_small_{args.steps}.txt"), "w").write(out.getvalue())
print(out.getvalue()[:3000])
context.stop_spark()
runtime.shutdown()
