"""Kernel vs bf16-GEMM-emulated torch over several optimizer steps (isolates real bugs from
bf16 rounding effects)."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import torch.nn as nn
import torch.nn.functional as F

from test_gpu_kernels import NYC, _relerr, emulate
from raydp_amd.models.mlp_spec import extract_mlp_spec
from raydp_amd.ops.fused_mlp import FusedMLPTrainer, loss_code, optimizer_config

dev = torch.device("cuda")
for lossfn in (nn.SmoothL1Loss(), nn.MSELoss(), nn.L1Loss()):
    torch.manual_seed(0)
    model = NYC()
    emu = copy.deepcopy(model).to(dev)
    eopt = torch.optim.Adam(emu.parameters(), lr=1e-3)
    tr = FusedMLPTrainer(extract_mlp_spec(model), optimizer_config(torch.optim.Adam(model.parameters(), lr=1e-3)),
                         loss_code(lossfn), 64, dev)
    n = 64 * 20
    X = torch.randn(n, 20) * 2
    Y = torch.randn(n, 1) * 3 + 1
    feats = torch.zeros(n, tr.feat_k, dtype=torch.bfloat16)
    feats[:, :20] = X.to(torch.bfloat16)
    feats, Yd, Xd = feats.to(dev), Y.to(dev), X.to(dev).to(torch.bfloat16).float()
    kl, el = [], []
    for s in range(20):
        tr.metrics.zero_()
        rc = tr.lib.rx_mlp_fwdbwd(__import__("ctypes").byref(tr.desc), tr._dd, tr.mt,
                                  *[__import__("ctypes").c_void_p(t.data_ptr()) for t in (tr.params, tr.grads, feats, Yd)],
                                  __import__("ctypes").c_void_p(0), n, 64, s,
                                  __import__("ctypes").c_void_p(tr.scratch.data_ptr()),
                                  __import__("ctypes").c_void_p(tr.metrics.data_ptr()),
                                  __import__("raydp_amd.ops._hip", fromlist=["x"]).stream_ptr())
        assert rc == 0
        kl.append(tr._read_metrics()["loss"])
        tr.opt_step(1e-3, 1 - 0.9 ** (s + 1), 1 - 0.999 ** (s + 1), 1.0, s == 0)
        emu.train()
        out = emulate(emu, Xd[s * 64:(s + 1) * 64])
        l = lossfn(out, Yd[s * 64:(s + 1) * 64])
        eopt.zero_grad()
        l.backward()
        eopt.step()
        el.append(l.item())
    pmap = tr.unflatten(tr.params)
    em = dict(emu.named_modules())
    worst = max(_relerr(pmap[(id(mod), a)], getattr(em[nm], a).data)
                for nm, mod in model.named_modules() for a in ("weight", "bias") if (id(mod), a) in pmap)
    rm_err = max(_relerr(rm, em[[n2 for n2, mm in model.named_modules() if mm is bn][0]].running_mean)
                 for bn, rm, rv in tr.run_bufs)
    print(type(lossfn).__name__, "kernel losses", [round(x, 4) for x in kl[:4]], "...", round(kl[-1], 4))
    print(type(lossfn).__name__, "emu    losses", [round(x, 4) for x in el[:4]], "...", round(el[-1], 4))
    print("  worst param relerr after 20 steps", round(worst, 5), "running_mean relerr", round(rm_err, 5))
    for nm, mod in model.named_modules():
        for a in ("weight", "bias"):
            if (id(mod), a) in pmap:
                e = _relerr(pmap[(id(mod), a)], getattr(em[nm], a).data)
                if e > 1e-2:
                    print("   ", nm, a, round(e, 4), pmap[(id(mod), a)].flatten()[:3].tolist(),
                          getattr(em[nm], a).data.flatten()[:3].tolist())
    m = tr._read_metrics()
    print("  last-step metrics", m)
