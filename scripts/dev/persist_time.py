"""Device time of one 3000-step NYC epoch: persistent launch vs launch-per-step loop."""
import copy, os, sys, time
import torch, torch.nn as nn
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config

dev = torch.device("cuda")
torch.manual_seed(0)
n = 64 * 3000
X = torch.randn(n, 20)
Y = torch.randn(n, 1)
for ps in sys.argv[1:] or ["1", "0"]:
    os.environ["RAYDP_MLP_PERSISTENT"] = ps
    m2 = NYC()
    tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(torch.optim.Adam(m2.parameters(), lr=1e-3)),
                         loss_code(nn.SmoothL1Loss()), 64, dev)
    feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
    feats[:, :20] = X.to(torch.bfloat16)
    feats, Yd = feats.to(dev), Y.to(dev)
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
    print(f"persistent={ps} epoch_ms={min(ts):.2f} ({', '.join(f'{t:.2f}' for t in ts)}) "
          f"us_per_step={min(ts) * 1000 / 3000:.2f} loss={met['loss']:.5f} grid={getattr(tr, '_ps_grid', None)}",
          flush=True)

# timeline of the middle step of a persistent epoch (wall clock ticks, 10 ns)
os.environ["RAYDP_MLP_PERSISTENT"] = "1"
# the kernel writes the middle step's phase stamps at [0, 32) AND every step's start time at
# [32 + s] (csrc/hip/mlp_persist.h RX_PS_STEP_STAMPS), so the buffer holds 32 + nsteps + 1 words
st = torch.zeros(32 + n // 64 + 1, dtype=torch.int64, device=dev)
tr.bufs.stamps = st.data_ptr()
tr.train_epoch(feats, Yd, n, perm)
torch.cuda.synchronize()
s = st.cpu().tolist()
t0 = s[0]
us = lambda k: (s[k] - t0) * 0.01 if s[k] else float("nan")
print("step WG: start 0 | inputs %.2f | weights ready %.2f | fwd done %.2f | bwd done %.2f | vec done %.2f us"
      % (us(1), us(2), us(3), us(4), us(5)))
print("  bwd layer done: " + " ".join(f"L{l}={us(8 + l):.2f}" for l in range(5)))
print("  opt (first wg per layer) flag seen -> counted: " +
      " ".join(f"L{l}={us(16 + 2 * l):.2f}->{us(17 + 2 * l):.2f}" for l in range(5)))
tr.bufs.stamps = 0
