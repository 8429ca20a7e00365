"""Diagnose multi-workgroup fused-MLP gradients: the same rows through layouts with and without
trailing empty workgroups; dumps the per-workgroup partials of both."""
import copy
import sys

import torch
import torch.nn as nn

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_kernels import NYC, _relerr, _setup, emulate  # noqa: E402

nvalid = 3001
for batch in (3008, 3072, 4096):
    model = NYC()
    tr, ref, ropt, feats, Y, X = _setup(model, nn.SmoothL1Loss(), torch.optim.Adam, batch, nvalid, 20, 1, lr=1e-3)
    g = tr.forward_backward(feats, Y, nvalid).clone()
    emu = copy.deepcopy(ref)
    emu.train()
    nn.SmoothL1Loss()(emulate(emu, X.to(torch.bfloat16).float()), Y).backward()
    gmap = tr.unflatten(g)
    errs = {}
    for name, mod in model.named_modules():
        for attr in ("weight", "bias"):
            k = (id(mod), attr)
            if k in gmap:
                errs[f"{name}.{attr}"] = round(_relerr(gmap[k], getattr(dict(emu.named_modules())[name], attr).grad), 5)
    print(batch, tr.mt, tr.G, max(errs.values()), errs, flush=True)
