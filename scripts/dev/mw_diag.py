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
parts = {}
for batch in (3008, 3072):
    model = NYC()
    tr, ref, ropt, feats, Y, X = _setup(model, nn.SmoothL1Loss(), torch.optim.Adam, batch, nvalid, 20, 1, lr=1e-3)
    g = tr.forward_backward(feats, Y, nvalid).clone()
    torch.cuda.synchronize()
    P = tr.mw_part.view(tr.G, -1).cpu()
    parts[batch] = P
    d = tr.desc
    for li in range(d.L):
        ly = d.layer[li]
        o, n = ly.pr_off, ly.out_n
        print(batch, "layer", li, "pr_off", o, "out_n", n,
              "lastWG fwd", float(P[-1, o:o + 2 * n].abs().max()),
              "bwd", float(P[-1, o + 2 * n:o + 4 * n].abs().max()),
              "bias", float(P[-1, o + 4 * n:o + 5 * n].abs().max()), flush=True)
    print(batch, "ctl", tr.mw_ctl.cpu().tolist(), "pr_total", d.pr_total, flush=True)
a, b = parts[3008], parts[3072]
for w in range(47):
    diff = float((a[w] - b[w]).abs().max())
    if diff:
        print("WG", w, "partials differ by", diff)
print("done")
