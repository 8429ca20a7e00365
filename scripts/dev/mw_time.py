"""Device time per step of the fused engine at wide batches (multi-workgroup step + split-K
optimizer): one epoch of N rows at batch B, best of 3 (events)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch, torch.nn as nn
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
dev = torch.device("cuda")
for batch in [int(b) for b in (sys.argv[1:] or ["4096", "1000"])]:
    torch.manual_seed(0)
    n = batch * 200
    m2 = NYC()
    tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(torch.optim.Adam(m2.parameters(), lr=1e-3)),
                         loss_code(nn.SmoothL1Loss()), batch, dev)
    feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
    feats[:, :20] = torch.randn(n, 20).to(torch.bfloat16)
    feats, Yd = feats.to(dev), torch.randn(n, 1).to(dev)
    perm = torch.randperm(n).to(torch.int32).to(dev)
    tr.train_epoch(feats, Yd, n, perm)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        met = tr.train_epoch(feats, Yd, n, perm)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(json.dumps({"batch": batch, "G": tr.G, "mt": tr.mt, "steps": n // batch,
                      "us_per_step": round(min(ts) * 1000 / (n // batch), 2), "loss": round(met["loss"], 5)}),
          flush=True)
