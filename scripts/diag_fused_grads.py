"""Diagnose fused-MLP gradient error: kernel vs fp32 torch vs a bf16-GEMM emulation."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import torch.nn as nn
import torch.nn.functional as F

from test_gpu_kernels import NYC, _relerr, _setup


class BfLin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        xb, wb = x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float()
        ctx.save_for_backward(xb, wb)
        return xb @ wb.t() + b

    @staticmethod
    def backward(ctx, g):
        xb, wb = ctx.saved_tensors
        gb = g.to(torch.bfloat16).float()
        return gb @ wb, gb.t() @ xb, g.sum(0)


def emu_forward(m, x):
    def lin(l, x):
        return BfLin.apply(x, l.weight, l.bias)
    x = m.bn1(F.relu(lin(m.fc1, x)))
    x = m.bn2(F.relu(lin(m.fc2, x)))
    x = m.bn3(F.relu(lin(m.fc3, x)))
    x = m.bn4(F.relu(lin(m.fc4, x)))
    return lin(m.fc5, x)


for nvalid in (64, 38):
    model = NYC()
    loss = nn.SmoothL1Loss()
    tr, ref, ropt, feats, Y, X = _setup(model, loss, torch.optim.Adam, 64, nvalid, 20, 1, lr=1e-3)
    g = tr.forward_backward(feats, Y, nvalid).clone()
    emu = copy.deepcopy(ref)
    ref.train()
    emu.train()
    xin = X.to(torch.bfloat16).float()
    loss(ref(xin), Y).backward()
    loss(emu_forward(emu, xin), Y).backward()
    gmap = tr.unflatten(g)
    rm = dict(ref.named_modules())
    em = dict(emu.named_modules())
    print("nvalid", nvalid, "loss kernel", tr._read_metrics()["loss"])
    for name, mod in model.named_modules():
        for attr in ("weight", "bias"):
            key = (id(mod), attr)
            if key in gmap:
                k = gmap[key]
                r = getattr(rm[name], attr).grad
                e = getattr(em[name], attr).grad
                print(f"{name:5s}.{attr:6s} kernel-vs-fp32 {_relerr(k, r):.4f}  kernel-vs-emu "
                      f"{_relerr(k, e):.4f}  emu-vs-fp32 {_relerr(e, r):.4f}")
