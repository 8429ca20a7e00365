"""Dump what an EMPTY trailing workgroup of the multi-workgroup step leaves behind (partials and
its columns of the batch-wide X^T / G^T export), batch 3072 with 3001 valid rows (G = 48)."""
import sys

import torch
import torch.nn as nn

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_kernels import NYC, _setup  # noqa: E402

nvalid = 3001
batch = 3072
model = NYC()
tr, ref, ropt, feats, Y, X = _setup(model, nn.SmoothL1Loss(), torch.optim.Adam, batch, nvalid, 20, 1, lr=1e-3)
for trial in range(2):
    tr.mw_part.fill_(float("nan")) if trial == 1 else None
    g = tr.forward_backward(feats, Y, nvalid).clone()
    torch.cuda.synchronize()
    G, BP = tr.G, tr.bp
    part = tr.mw_part.view(G, -1)
    print("trial", trial, "G", G, "BP", BP, "stride", tr._mw_stride, flush=True)
    for li in range(tr.desc.L):
        x = tr.desc.layer[li]
        o = x.mw_off
        on = x.out_n
        r32 = lambda n: (n + 31) // 32 * 32  # noqa: E731
        fwd = part[:, o:o + 2 * on]
        bwd = part[:, o + r32(2 * on):o + r32(2 * on) + 2 * on]
        bia = part[:, o + 2 * r32(2 * on):o + 2 * r32(2 * on) + on]
        print(f"layer {li}: WG47 fwd max {fwd[G - 1].abs().max().item():.3e} bwd {bwd[G - 1].abs().max().item():.3e} "
              f"bias {bia[G - 1].abs().max().item():.3e} | WG46 bias {bia[G - 2].abs().max().item():.3e} "
              f"nan? {bool(torch.isnan(part[G - 1, o:o + 2 * r32(2 * on) + on]).any())}", flush=True)
        act = g.new_tensor([])
        a16 = tr.grads.view(torch.int16)  # exported bf16 area after the flat gradient
        base = tr.desc.act_off * 2
        xg = a16[base + x.xg_off: base + x.xg_off + x.in_n * G * BP].view(x.in_n, G * BP)
        gg = a16[base + x.gg_off: base + x.gg_off + on * G * BP].view(on, G * BP)
        print(f"   export X^T cols[{nvalid}:] nonzero {int((xg[:, nvalid:] != 0).sum())}, "
              f"G^T cols[{nvalid}:] nonzero {int((gg[:, nvalid:] != 0).sum())}", flush=True)
