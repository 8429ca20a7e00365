"""Same-box A/B of the persistent NYC epoch across old trees: `python bisect/persist_ab.py <tree>`.
Prints one JSON line: best-of-3 device time of a 3000-step epoch (batch 64) and the middle step's
phase stamps when the tree's kernel writes them."""
import json, os, sys, time
tree = os.path.abspath(sys.argv[1])
sys.path.insert(0, tree)
sys.path.insert(0, os.path.join(tree, "tests"))
import torch, torch.nn as nn
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config
import raydp_amd.ops._hip as H
dev = torch.device("cuda")
torch.manual_seed(0)
n = 64 * 3000
X, Y = torch.randn(n, 20), torch.randn(n, 1)
os.environ["RAYDP_MLP_PERSISTENT"] = "1"
m2 = NYC()
tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(torch.optim.Adam(m2.parameters(), lr=1e-3)),
                     loss_code(nn.SmoothL1Loss()), 64, dev)
feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
feats[:, :20] = X.to(torch.bfloat16)
feats, Yd = feats.to(dev), Y.to(dev)
perm = torch.randperm(n).to(torch.int32).to(dev)
tr.train_epoch(feats, Yd, n, perm)
ts = []
for _ in range(int(os.environ.get("AB_REPS", "5"))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    met = tr.train_epoch(feats, Yd, n, perm)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
st = torch.zeros(32 + n // 64 + 1 + 96, dtype=torch.int64, device=dev)
tr.bufs.stamps = st.data_ptr()
tr.train_epoch(feats, Yd, n, perm)
torch.cuda.synchronize()
s = st.cpu().tolist()
tr.bufs.stamps = 0
us = lambda k: round((s[k] - s[0]) * 0.01, 2) if s[k] and s[0] else None
# intra-layer shader-clock stamps of the middle step (new kernels only)
L = s[32 + n // 64 + 1:]
seq = []
for l in range(5):
    for k, nm in enumerate(("export", "gemm", "epi", "sync1", "publish")):
        seq.append((f"f{l}.{nm}", L[40 + 5 * l + k]))
for l in range(4, -1, -1):
    for k, nm in enumerate(("wgrad", "dgrad", "sync", "post")):
        if l == 0 and k > 0:
            break
        seq.append((f"b{l}.{nm}", L[20 + 4 * l + k]))
seq = [(a, b) for a, b in seq if b]
layer = [(a, b - seq[i - 1][1]) for i, (a, b) in enumerate(seq) if i > 0]
print(json.dumps({"tree": os.path.basename(tree), "us_per_step_min": round(min(ts) * 1000 / 3000, 3),
                  "epoch_ms": [round(t, 2) for t in ts], "loss": round(float(met["loss"]), 6),
                  "grid": getattr(tr, "_ps_grid", None),
                  "phases_us": {"inputs": us(1), "weights": us(2), "fwd": us(3), "bwd": us(4), "vec": us(5)},
                  # first optimizer workgroup of each layer: flag seen -> counter raised
                  "opt_us": {f"L{l}": [us(16 + 2 * l), us(17 + 2 * l)] for l in range(5)},
                  "bwd_layer_done_us": {f"L{l}": us(8 + l) for l in range(5)},
                  "opt_L0_loaded_updated_drained_us": [us(28), us(26), us(27)],
                  "layer_cycles": layer}),
      flush=True)
