"""cProfile of one bench pipeline (after a warm-up pipeline) -> gpurun_out/pipeline_prof.txt."""
import cProfile
import io
import os
import pstats
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "examples"))
import torch  # noqa: E402

import bench  # noqa: E402
from raydp_amd import context, runtime  # noqa: E402

torch.cuda.set_device(0)
tmp = tempfile.mkdtemp()
warm, main = os.path.join(tmp, "w.csv"), os.path.join(tmp, "m.csv")
bench.make_csv(warm, 300 * 64, 1)
bench.make_csv(main, 3000 * 64, 2)
runtime.init(num_cpus=4)
spark = context.init_spark("prof", 4, 1, "1G")
spark.conf.set("spark.sql.session.timeZone", "UTC")
bench.run_pipeline(spark, warm, 300, 1, os.path.join(tmp, "r"))
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
bench.run_pipeline(spark, main, 3000, 1, os.path.join(tmp, "r"))
torch.cuda.synchronize()
pr.disable()
out = io.StringIO()
pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(45)
os.makedirs(os.path.join(HERE, "gpurun_out"), exist_ok=True)
open(os.path.join(HERE, "gpurun_out", "pipeline_prof.txt"), "w").write(out.getvalue())
print(out.getvalue()[:6000])
context.stop_spark()
runtime.shutdown()
