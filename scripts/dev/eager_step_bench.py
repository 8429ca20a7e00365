"""Host-bound eager torch step of a user-written loop (the Horovod NYCTaxi example's step:
NYC_Model, smooth-L1, Adam, batch 64, a loss.item() every 10 steps), under backend settings the
framework can choose for its GPU workers without touching user code. One JSON line per run:
  ES_VARIANT=base|fused_adam|native_bn|rocblas|all|rx python scripts/dev/eager_step_bench.py
rx: what the framework's GPU workers now do -- hvd.DistributedOptimizer's multi-tensor Adam
(csrc/hip/fused_optim.hip) under the native-BatchNorm worker policy."""
import json, os, sys, time
v = os.environ.get("ES_VARIANT", "base")
if v in ("rocblas", "all"):
    os.environ["TORCH_BLAS_PREFER_HIPBLASLT"] = "0"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch
import torch.nn.functional as F
from __graft_entry__ import _nyc_model
if v in ("native_bn", "all"):
    torch.backends.cudnn.enabled = False
dev = torch.device("cuda")
torch.manual_seed(0)
model = _nyc_model(20).to(dev)
opt = torch.optim.Adam(model.parameters(), lr=1e-3, **({"fused": True} if v in ("fused_adam", "all") else {}))
if v == "rx":
    import raydp_amd.hvd as hvd
    from raydp_amd.train.gpu_policy import native_batchnorm
    hvd.init()
    opt = hvd.DistributedOptimizer(opt)
    native_batchnorm(True).__enter__()
X = torch.randn(64 * 600, 20, device=dev)
Y = torch.randn(64 * 600, 1, device=dev)
def run(steps):
    for i in range(steps):
        xb, yb = X[i * 64:(i + 1) * 64], Y[i * 64:(i + 1) * 64]
        opt.zero_grad()
        loss = F.smooth_l1_loss(model(xb), yb)
        loss.backward()
        opt.step()
        if i % 10 == 0:
            loss.item()
run(50)
torch.cuda.synchronize()
t = time.perf_counter()
run(500)
torch.cuda.synchronize()
dt = (time.perf_counter() - t) / 500
print(json.dumps({"variant": v, "ms_per_step": round(dt * 1e3, 4), "samples_per_s": round(64 / dt, 1)}), flush=True)
