"""Launch-per-step NYC epoch (RAYDP_MLP_PERSISTENT=0): one step workgroup per launch, the kernel
whose PMC counters give the step body's instruction mix without the persistent launch's spinning
optimizer workgroups. Also prints the launch-per-step device time."""
import json, os, sys
os.environ["RAYDP_MLP_PERSISTENT"] = "0"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch, torch.nn as nn
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
dev = torch.device("cuda")
torch.manual_seed(0)
n = 64 * int(os.environ.get("STEPS", "1000"))
m2 = NYC()
tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(torch.optim.Adam(m2.parameters(), lr=1e-3)),
                     loss_code(nn.SmoothL1Loss()), 64, dev)
feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
feats[:, :20] = torch.randn(n, 20).to(torch.bfloat16)
feats, Yd = feats.to(dev), torch.randn(n, 1).to(dev)
perm = torch.randperm(n).to(torch.int32).to(dev)
ts = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    met = tr.train_epoch(feats, Yd, n, perm)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"launch_per_step_us": round(min(ts) * 1000 / (n // 64), 2), "loss": round(met["loss"], 5)}))
