"""Which models crash torch.cuda.make_graphed_callables' backward capture on this image: one
variant per process (a crash ends the caller's chain), printed before and after the capture.

  python -X faulthandler scripts/dev/graph_bisect.py --variant nyc
variants: net (the GPU test's BatchNorm MLP), nyc_out2 (NYC_Model with a 2-wide head),
nyc_nobn (NYC_Model without BatchNorm), nyc (NYC_Model as in examples/horovod_nyctaxi.py),
gm* (nyc through raydp_amd.train.gpu_policy.graph_model in a user loop, see main).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def build(variant):
    import torch.nn as nn
    import torch.nn.functional as F

    class NYC(nn.Module):
        def __init__(self, cols=20, out=1, bn=True):
            super().__init__()
            self.fc = nn.ModuleList([nn.Linear(a, b) for a, b in ((cols, 256), (256, 128), (128, 64), (64, 16))])
            self.bn = nn.ModuleList([nn.BatchNorm1d(n) if bn else nn.Identity() for n in (256, 128, 64, 16)])
            self.head = nn.Linear(16, out)

        def forward(self, x):
            for fc, bn in zip(self.fc, self.bn):
                x = bn(F.relu(fc(x)))
            return self.head(x)

    if variant == "net":
        return nn.Sequential(nn.Linear(20, 32), nn.ReLU(), nn.BatchNorm1d(32), nn.Linear(32, 2))
    if variant == "nyc_out2":
        return NYC(out=2)
    if variant == "nyc_nobn":
        return NYC(bn=False)
    return NYC()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="nyc")
    a = ap.parse_args()
    import torch
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = build(a.variant).to(dev).train()
    x = torch.randn(64, 20, device=dev)
    print(f"{a.variant}: capturing", flush=True)
    if a.variant.startswith("gm"):
        # graph_model in a user loop: gm (as examples/horovod_nyctaxi.py), gm_first (captured on
        # the first call), gm_delloss (no earlier autograd graph alive at the capture), gm_noopt
        # (no optimizer step), gm_eager_only (eager steps, then a plain make_graphed_callables)
        from raydp_amd.train import gpu_policy
        if a.variant == "gm_first":
            gpu_policy._STEADY = 1
        if a.variant != "gm_eager_only":
            gpu_policy.graph_model(model)
        opt = torch.optim.Adam(model.parameters(), lr=1e-2)
        y = torch.randn(64, 1, device=dev)
        for i in range(6):
            opt.zero_grad()
            loss = torch.nn.functional.smooth_l1_loss(model(x), y)
            loss.backward()
            if a.variant != "gm_noopt":
                opt.step()
            print(f"{a.variant}: step {i} done", flush=True)
            if a.variant == "gm_delloss":
                del loss
                loss = torch.zeros(())
        if a.variant == "gm_eager_only":
            g = torch.cuda.make_graphed_callables(model, (x,), num_warmup_iters=3)
            g(x).sum().backward()
        torch.cuda.synchronize()
        print(f"{a.variant}: ok", flush=True)
        return
    g = torch.cuda.make_graphed_callables(model, (x,), num_warmup_iters=3)
    out = g(x)
    out.sum().backward()
    torch.cuda.synchronize()
    print(f"{a.variant}: ok {float(out.sum()):.4f}", flush=True)


if __name__ == "__main__":
    main()
