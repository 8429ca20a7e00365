"""Workgroup 0's intra-layer timeline of the multi-workgroup step at batch B (diagnostic build:
RAYDP_MLP_LAYER_STAMPS=1 is set here), middle step of one epoch: shader-clock cycles per phase.
  python scripts/dev/mw_stamps.py [batch]"""
import json, os, sys
os.environ["RAYDP_MLP_LAYER_STAMPS"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import torch, torch.nn as nn
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
dev = torch.device("cuda")
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = batch * 40
torch.manual_seed(0)
m2 = NYC()
tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(torch.optim.Adam(m2.parameters(), lr=1e-3)),
                     loss_code(nn.SmoothL1Loss()), batch, dev)
feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
feats[:, :20] = torch.randn(n, 20).to(torch.bfloat16)
feats, Yd = feats.to(dev), torch.randn(n, 1).to(dev)
tr.train_epoch(feats, Yd, n, None)
tr.record_steps = True
tr.train_epoch(feats, Yd, n, None)
L = [int(x) for x in tr._mw_layer_stamps]
seq = []
for l in range(5):
    for k, nm in enumerate(("export", "gemm", "epi", "sync1", "publish")):
        seq.append((f"f{l}.{nm}", L[40 + 5 * l + k]))
for l in range(4, -1, -1):
    for k, nm in enumerate(("wgrad", "dgrad", "sync", "post")):
        if l == 0 and k > 0:
            break
        seq.append((f"b{l}.{nm}", L[20 + 4 * l + k]))
seq += [("end.bwd_done", L[0]), ("end.barrier", L[1])]
seq = [(a, b) for a, b in seq if b]
out = [(a, b - seq[i - 1][1]) for i, (a, b) in enumerate(seq) if i > 0]
print(json.dumps({"batch": batch, "G": tr.G, "mt": tr.mt, "cycles": out, "total": sum(v for _, v in out)}))
