"""Where does the persistent epoch first differ from the launch-per-step loop? (diagnostic)"""
import copy, os, sys
import torch, torch.nn as nn
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_kernels import NYC
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config

dev = torch.device("cuda")
torch.manual_seed(5)
model = NYC()
n = 64 * 8
X = torch.randn(n, 20) * 2.0
Y = torch.randn(n, 1) * 3.0
opt_name = sys.argv[1] if len(sys.argv) > 1 else "adam"
for k in (1, 2, 3, 5):
    res = []
    for ps in ("1", "0"):
        os.environ["RAYDP_MLP_PERSISTENT"] = ps
        m2 = copy.deepcopy(model)
        opt = torch.optim.Adam(m2.parameters(), lr=1e-3) if opt_name == "adam" else \
            torch.optim.SGD(m2.parameters(), lr=0.01, momentum=0.9)
        tr = FusedMLPTrainer(extract_mlp_spec(m2), optimizer_config(opt), loss_code(nn.SmoothL1Loss()), 64, dev)
        feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
        feats[:, :20] = X.to(torch.bfloat16)
        met = tr.train_epoch(feats.to(dev), Y.to(dev), n, None, max_steps=k)
        torch.cuda.synchronize()
        res.append((tr.params.clone(), tr.m.clone(), tr.img.clone(), met, tr))
    (p1, m1, i1, e1, tr), (p0, m0, i0, e0, _) = res
    print(f"k={k} loss ps={e1['loss']:.9f} loop={e0['loss']:.9f} img_equal={torch.equal(i1, i0)}")
    for kind, _, off, cnt in tr.layout:
        d = (p1[off:off + cnt] - p0[off:off + cnt]).abs()
        dm = (m1[off:off + cnt] - m0[off:off + cnt]).abs()
        if float(d.max()) > 0 or float(dm.max()) > 0:
            print(f"   {kind:6s} off={off:6d} n={cnt:6d} maxdiff p={float(d.max()):.3e} m={float(dm.max()):.3e} "
                  f"ndiff={int((d > 0).sum())}")
