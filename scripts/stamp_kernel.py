"""Per-phase cycle breakdown of the fused MLP train-step kernel (s_memtime stamps)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn

from __graft_entry__ import smoke  # noqa: F401
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_kernels import NYC

dev = torch.device("cuda")
model = NYC()
tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(torch.optim.Adam(model.parameters())),
                     loss_code(nn.SmoothL1Loss()), 64, dev)
stamps = torch.zeros(128, dtype=torch.int64, device=dev)
tr.bufs.stamps = stamps.data_ptr()
n = 64 * 200
feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16, device=dev)
feats[:, :20] = torch.randn(n, 20, device=dev).to(torch.bfloat16)
labels = torch.randn(n, 1, device=dev)
names = ["load_in"] + [f"fwd{i}" for i in range(1, 6)] + [f"bwd{i}" for i in range(5, 0, -1)]
acc = torch.zeros(11, dtype=torch.float64)
for it in range(60):
    tr.forward_backward(feats, labels, n, None, step=it % 200)
    if it >= 10:
        tr.opt_step(1e-3, 0.1, 0.001)
        s = stamps[:12].cpu().double()
        acc += (s[1:] - s[:-1])
torch.cuda.synchronize()
acc /= 50
tot = acc.sum().item()
for nm, v in zip(names, acc.tolist()):
    print(f"{nm:8s} {v:9.0f} cyc  {100 * v / tot:5.1f}%")
print(f"total {tot:.0f} cycles (~{tot / 2.1e3:.1f} us at 2.1 GHz)")
# within-backward breakdown: [start-of-layer .. wgrad done | dgrad done (wave0) | sync | epilogue (wave0)]
s = stamps.cpu().double()
ends = {l: s[11 - l] for l in range(5)}
for l in range(4, 0, -1):
    start = s[10 - l]
    w, dg, sy, ep = s[20 + 4 * l], s[21 + 4 * l], s[22 + 4 * l], s[23 + 4 * l]
    print(f"bwd{l + 1}: wgrad {w - start:7.0f}  dgrad {dg - w:7.0f}  sync {sy - dg:7.0f}  epi {ep - sy:7.0f}  tail {ends[l] - ep:7.0f}")
# within-forward breakdown (wave 0): export | GEMM | epilogue | barrier | publish (to the end of the layer)
s = stamps.cpu().double()
for l in range(5):
    b = s[40 + 5 * l: 45 + 5 * l].tolist()
    start, end = s[1 + l], s[2 + l]
    print(f"fwd{l + 1}: export {b[0] - start:7.0f}  gemm {b[1] - b[0]:7.0f}  epi {b[2] - b[1]:7.0f}  "
          f"sync {b[3] - b[2]:7.0f}  publish {b[4] - b[3]:7.0f}  tail {end - b[4]:7.0f}")
