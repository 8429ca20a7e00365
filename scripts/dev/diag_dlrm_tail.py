"""Per-step losses of tests/test_gpu_fused_optim.py::test_dlrm_step_with_fused_tail_matches_eager
with the paired tower backward on and off (diagnostic)."""
import copy
import sys

import torch
import torch.nn as nn

sys.path.insert(0, ".")
from raydp_amd.models.dlrm import Dlrm  # noqa: E402
from raydp_amd.ops import linear_ops  # noqa: E402
from raydp_amd.ops.fused_optim import FusedBCEWithLogits, sgd_step  # noqa: E402

for pair in (False, True):
    linear_ops.PAIR_BACKWARD = pair
    torch.manual_seed(0)
    base = Dlrm(13, [1000] * 26, [512, 128, 32], [1024, 1024, 512, 256, 1], 32).cuda()
    ref = copy.deepcopy(base)
    fused = copy.deepcopy(base)
    fused.embeddings.fused_sgd_lr = 0.05
    g = torch.Generator(device="cuda").manual_seed(3)
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.05)
    o_f = torch.optim.SGD(fused.parameters(), lr=0.05)
    for step in range(4):
        dense = torch.randn(256, 13, device="cuda", generator=g)
        cats = torch.randint(0, 1000, (256, 26), device="cuda", generator=g)
        y = torch.randint(0, 2, (256, 1), device="cuda", generator=g).float()
        o_ref.zero_grad(set_to_none=True)
        out_a = ref(dense, cats)
        la = nn.BCEWithLogitsLoss()(out_a, y)
        la.backward()
        o_f.zero_grad(set_to_none=True)
        out_b = fused(dense, cats)
        lb = FusedBCEWithLogits()(out_b, y)
        lb.backward()
        gd = {n: (p.grad.float() if p.grad is not None and not p.grad.is_sparse else None)
              for n, p in ref.named_parameters()}
        worst = []
        for n, p in fused.named_parameters():
            if p.grad is not None and gd.get(n) is not None:
                r = float((p.grad - gd[n]).norm() / (gd[n].norm() + 1e-12))
                worst.append((r, n))
        worst.sort(reverse=True)
        print(f"pair={pair} step={step} la={float(la):.7f} lb={float(lb):.7f} out_diff="
              f"{float((out_a - out_b).abs().max()):.3g} worst_grad={worst[:3]}", flush=True)
        o_ref.step()
        sgd_step(o_f)
