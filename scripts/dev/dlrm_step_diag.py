"""Per-parameter update error vs an fp32 CPU step: the persistent DLRM step, and the launch-per-op
GPU step (fused towers + torch SGD) of the same model, so the persistent step's error is judged
against what the bf16 tower path already gives."""
import copy
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from test_gpu_dlrm_step import _data, _model, _params, _ref_steps  # noqa: E402


def errs(before, ours, ref):
    out = {}
    for k in before:
        du, dr = ours[k] - before[k], ref[k] - before[k]
        n = float(dr.norm())
        out[k] = float((du - dr).norm()) / n if n else float(du.norm())
    return out


def main():
    from raydp_amd.ops.dlrm_step import DlrmStep
    dev = torch.device("cuda", 0)
    B, lr = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 0.05
    ref = _model()
    before = _params(ref)
    dense, cats, y = _data(B + 7)
    perm = torch.randperm(B + 7, generator=torch.Generator().manual_seed(3))
    gpu = copy.deepcopy(ref).to(dev)
    eager = copy.deepcopy(ref).to(dev)
    st = DlrmStep(gpu, lr, B, dev)
    st.bind_data(dense.to(dev), cats.to(dev), y.to(dev))
    st.steps(perm.to(dev), 0, 1)
    torch.cuda.synchronize()
    st.check()
    rl = _ref_steps(ref, dense, cats, y, perm, B, 1, lr)
    # launch-per-op GPU step
    opt = torch.optim.SGD(eager.parameters(), lr=lr)
    idx = perm[:B].to(dev)
    out = eager(dense.to(dev)[idx], cats.to(dev)[idx])
    loss = torch.nn.BCEWithLogitsLoss()(out.view(-1), y.to(dev)[idx])
    opt.zero_grad()
    loss.backward()
    opt.step()
    print("loss persistent", float(st.step_loss.item()), "eager", float(loss), "fp32", rl[0])
    ep, ee = errs(before, _params(gpu), _params(ref)), errs(before, _params(eager), _params(ref))
    for k in before:
        print(f"{k:34s} persistent {ep[k]:.4f}  launch-per-op {ee[k]:.4f}")


if __name__ == "__main__":
    main()
