"""Probe for a crash at interpreter exit under rocprofv3: runtime + Spark bring-up / tear-down
with one trivial GPU op (no fused kernels, no ingest)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
torch.zeros(1, device="cuda").add_(1)
torch.cuda.synchronize()
from raydp_amd import context, runtime  # noqa: E402
runtime.init(num_cpus=2)
spark = context.init_spark("exit-probe", 2, 1, "1G")
print("count", spark.range(0, 10).count(), flush=True)
context.stop_spark()
runtime.shutdown()
print("done", flush=True)
