"""Time the fused NYC train step in isolation: one epoch of N steps through the native step
loop (train kernel + optimizer kernel per step), no ETL. Prints us/step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import torch.nn as nn

from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
from test_gpu_kernels import NYC

dev = torch.device("cuda")
steps = int(os.environ.get("STEPS", "3000"))
torch.manual_seed(0)
model = NYC()
tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(torch.optim.Adam(model.parameters(), lr=1e-3)),
                     loss_code(nn.SmoothL1Loss()), 64, dev)
n = 64 * steps
feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16, device=dev)
feats[:, :20] = torch.randn(n, 20, device=dev).to(torch.bfloat16)
labels = torch.randn(n, 1, device=dev)
perm = torch.randperm(n, device=dev).to(torch.int32)
for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    m = tr.train_epoch(feats, labels, n, perm, drop_last=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"{os.environ.get('TAG', '')} rep {rep}: {dt * 1e6 / steps:.2f} us/step  loss {m['loss']:.4f}", flush=True)
