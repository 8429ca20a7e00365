"""Where a Horovod-style user step spends its time on the GPU: the bench's hvd_train_fn loop body
(NYC_Model, batch 64, Adam, DistributedOptimizer at world 1, device-resident to_torch shard, a
loss.item() every 10 steps) timed per variant, then a cProfile of the default variant.
  python scripts/dev/hvd_profile.py"""
import cProfile, io, json, os, pstats, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import pyarrow as pa
import torch
import torch.nn.functional as F
import raydp_amd.hvd as hvd
from raydp_amd.data.dataset import Dataset
from raydp_amd.train.gpu_policy import native_batchnorm
from __graft_entry__ import _nyc_model

dev = torch.device("cuda")
n, B = 64 * 600, 64
rng = np.random.default_rng(0)
cols = {f"f{i}": rng.standard_normal(n).astype(np.float32) for i in range(20)}
cols["y"] = rng.standard_normal(n).astype(np.float32)
t = pa.table(cols)
ds = Dataset([t], t.schema)
feats = [f"f{i}" for i in range(20)]


def run(variant, steps=500, prof=None):
    torch.manual_seed(0)
    model = _nyc_model(20).to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, **({"fused": True} if variant == "torch_fused" else {}))
    hvd.init()
    if variant != "no_hvd":
        opt = hvd.DistributedOptimizer(opt, named_parameters=model.named_parameters(), op=hvd.Average)
    if variant == "presliced":
        X = torch.randn(n, 20, device=dev)
        Y = torch.randn(n, 1, device=dev)
        batches = [(X[i * B:(i + 1) * B], Y[i * B:(i + 1) * B]) for i in range(n // B)]
    else:
        batches = ds.to_torch(feature_columns=feats, label_column="y", label_column_dtype=torch.float,
                              feature_column_dtypes=torch.float, batch_size=B, drop_last=True, device=dev)
    ctx = native_batchnorm(variant != "miopen_bn")
    with ctx:
        def loop(k):
            i = 0
            while i < k:
                for bi, (x, y) in enumerate(batches):
                    opt.zero_grad()
                    loss = F.smooth_l1_loss(model(x), y)
                    loss.backward()
                    opt.step()
                    if bi % 10 == 0:
                        loss.item()
                    i += 1
                    if i >= k:
                        break
        loop(50)
        torch.cuda.synchronize()
        if prof:
            prof.enable()
        t0 = time.perf_counter()
        loop(steps)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / steps
        if prof:
            prof.disable()
    hvd.shutdown()
    return dt


for v in ("default", "presliced", "no_hvd", "torch_fused", "miopen_bn"):
    print(json.dumps({"variant": v, "ms_per_step": round(run(v) * 1e3, 4)}), flush=True)
p = cProfile.Profile()
run("default", 300, p)
s = io.StringIO()
pstats.Stats(p, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
