"""Per-parameter gradient error of the multi-workgroup fused step vs the bf16 emulation and fp32
torch, over a few seeds and (batch, valid rows) shapes: separates a masking bug (one shape off)
from the bf16 error class (every shape alike)."""
import copy
import sys

import torch
import torch.nn as nn

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_kernels import NYC, _relerr, _setup, emulate  # noqa: E402


def one(batch, nvalid, seed):
    loss = nn.SmoothL1Loss()
    torch.manual_seed(seed)
    model = NYC()
    tr, ref, ropt, feats, Y, X = _setup(model, loss, torch.optim.Adam, batch, nvalid, 20, 1, seed=seed, lr=1e-3)
    g = tr.forward_backward(feats, Y, nvalid).clone()
    emu = copy.deepcopy(ref)
    ref.train()
    emu.train()
    xin = X.to(torch.bfloat16).float()
    loss(ref(xin), Y).backward()
    loss(emulate(emu, xin), Y).backward()
    gmap = tr.unflatten(g)
    rmods, emods = dict(ref.named_modules()), dict(emu.named_modules())
    out = []
    for name, mod in model.named_modules():
        for attr in ("weight", "bias"):
            if (id(mod), attr) in gmap:
                k = gmap[(id(mod), attr)]
                ge, gr = getattr(emods[name], attr).grad, getattr(rmods[name], attr).grad
                out.append(f"{name}.{attr[0]} emu {_relerr(k, ge):.4f} fp32 {_relerr(k, gr):.4f} "
                           f"emu-vs-fp32 {_relerr(ge, gr):.4f}")
    print(f"batch {batch} valid {nvalid} seed {seed} G {tr.G}: " + " | ".join(out), flush=True)


if __name__ == "__main__":
    for batch, nvalid in ((4096, 4096), (4096, 3001), (4096, 4000), (1000, 1000), (256, 200)):
        for seed in (0, 1, 2):
            one(batch, nvalid, seed)
