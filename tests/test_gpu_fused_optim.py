"""Multi-tensor SGD (+ fused-tower bf16 images), multi-tensor Adam / AdamW and fused BCE-with-logits
(csrc/hip/fused_optim.hip) against fp32 PyTorch references of the same ops."""
import copy

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(512, 13), (512,), (128, 512), (128,), (7,), (1, 256), (3, 5, 9)] + [(33,)] * 24  # > 24 tensors
    ps = [torch.randn(s, generator=g).cuda().requires_grad_() for s in shapes]
    return ps


@pytest.mark.parametrize("cls,cfg", [(torch.optim.Adam, dict(lr=1e-3)),
                                     (torch.optim.Adam, dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6, weight_decay=1e-2)),
                                     (torch.optim.Adam, dict(lr=1e-3, maximize=True)),
                                     (torch.optim.AdamW, dict(lr=1e-3, weight_decay=0.05)),
                                     (torch.optim.Adam, dict(lr=1e-3, weight_decay=0.05, decoupled_weight_decay=True))])
def test_multi_tensor_adam_matches_torch_adam(cls, cfg):
    """rx_mt_adam (one launch per 24 tensors, >24 tensors here, odd lengths for the scalar tail)
    against torch's own single-tensor Adam / AdamW over 5 steps; the state stays torch's."""
    from raydp_amd.ops.fused_optim import adam_step, adam_supported
    ref = _params()
    mine = [p.detach().clone().requires_grad_() for p in ref]
    o_ref = cls(ref, foreach=False, **cfg)
    o_mine = cls(mine, **cfg)
    g = torch.Generator().manual_seed(1)
    for _ in range(5):
        grads = [torch.randn(p.shape, generator=g).cuda() for p in ref]
        for a, b, gr in zip(ref, mine, grads):
            a.grad, b.grad = gr.clone(), gr.clone()
        assert adam_supported(o_mine) is None
        o_ref.step()
        adam_step(o_mine)
    torch.cuda.synchronize()
    for a, b in zip(ref, mine):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
        for k in ("exp_avg", "exp_avg_sq"):
            torch.testing.assert_close(o_mine.state[b][k], o_ref.state[a][k], rtol=1e-5, atol=1e-7)
        assert float(o_mine.state[b]["step"]) == float(o_ref.state[a]["step"]) == 5.0
    # the state dict is torch's: it loads into a plain optimizer, whose next step matches
    o_again = cls(copy.deepcopy(mine), **cfg)
    o_again.load_state_dict(o_mine.state_dict())


def test_hvd_distributed_optimizer_takes_the_multi_tensor_step(monkeypatch):
    """hvd.DistributedOptimizer (world 1) runs a wrapped Adam on rx_mt_adam: parameters match
    torch's own Adam after a few steps of a BatchNorm MLP, under the native-BatchNorm worker policy."""
    import raydp_amd.hvd as hvd
    from raydp_amd.ops import fused_optim
    from raydp_amd.train.gpu_policy import native_batchnorm
    calls = []
    real = fused_optim.adam_step
    monkeypatch.setattr(fused_optim, "adam_step", lambda o: (calls.append(1), real(o)))
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.BatchNorm1d(64), nn.Linear(64, 1)).cuda()
    ref = copy.deepcopy(net)
    hvd.init()
    try:
        opt = hvd.DistributedOptimizer(torch.optim.Adam(net.parameters(), lr=1e-2))
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-2, foreach=False)
        x, y = torch.randn(64, 20, device="cuda"), torch.randn(64, 1, device="cuda")
        with native_batchnorm(True):
            for _ in range(4):
                for m, o in ((net, opt), (ref, ropt)):
                    o.zero_grad()
                    nn.functional.smooth_l1_loss(m(x), y).backward()
                    o.step()
    finally:
        hvd.shutdown()
    assert len(calls) == 4
    for a, b in zip(net.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("cfg", [dict(lr=0.05), dict(lr=0.05, momentum=0.9), dict(lr=0.02, momentum=0.9, nesterov=True),
                                 dict(lr=0.01, momentum=0.8, dampening=0.1, weight_decay=1e-3),
                                 dict(lr=0.01, weight_decay=1e-2, maximize=True)])
def test_multi_tensor_sgd_matches_torch_sgd(cfg):
    from raydp_amd.ops.fused_optim import FusedSGD, sgd_supported
    ref = _params()
    mine = [p.detach().clone().requires_grad_() for p in ref]
    o_ref = torch.optim.SGD(ref, foreach=False, **cfg)
    o_mine = FusedSGD(mine, **cfg)
    g = torch.Generator().manual_seed(1)
    for _ in range(4):
        grads = [torch.randn(p.shape, generator=g).cuda() for p in ref]
        for a, b, gr in zip(ref, mine, grads):
            a.grad, b.grad = gr.clone(), gr.clone()
        assert sgd_supported(o_mine) is None
        o_ref.step()
        o_mine.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, mine):
        torch.testing.assert_close(b, a, rtol=2e-6, atol=1e-6)
    if cfg.get("momentum"):
        for a, b in zip(ref, mine):
            torch.testing.assert_close(o_mine.state[b]["momentum_buffer"], o_ref.state[a]["momentum_buffer"],
                                       rtol=2e-6, atol=1e-6)
    # the state dict is torch's (a fused optimizer checkpoint loads into torch.optim.SGD)
    torch.optim.SGD(copy.deepcopy(ref), **cfg).load_state_dict(o_mine.state_dict())


def test_sgd_writes_fused_tower_images():
    from raydp_amd.ops.fused_optim import sgd_step
    from raydp_amd.ops.linear_ops import FusedLinearTower
    torch.manual_seed(0)
    lins = [nn.Linear(64, 128).cuda(), nn.Linear(128, 32).cuda()]
    tower = FusedLinearTower(lins, [True, False])
    x = torch.randn(256, 64, device="cuda")
    tower(x).sum().backward()
    opt = torch.optim.SGD([p for l in lins for p in l.parameters()], lr=0.1)
    sgd_step(opt)
    torch.cuda.synchronize()
    for li, lin in enumerate(lins):
        assert torch.equal(tower.images[li], lin.weight.detach().to(torch.bfloat16)), li
        assert tower._managed[li]
    # the next forward must not rebuild them (no stale check fires): same output as a fresh tower
    out = tower(x)
    fresh = FusedLinearTower(lins, [True, False])(x)
    torch.testing.assert_close(out, fresh, rtol=0, atol=0)


@pytest.mark.parametrize("n", [1, 127, 2048, 70000])
def test_fused_bce_with_logits_matches_torch(n):
    from raydp_amd.ops.fused_optim import FusedBCEWithLogits
    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, 1, generator=g) * 6).cuda()
    y = torch.randint(0, 2, (n, 1), generator=g).float().cuda()
    xa = x.clone().requires_grad_()
    xb = x.clone().requires_grad_()
    la = nn.BCEWithLogitsLoss()(xa.double(), y.double())       # fp64 reference
    lb = FusedBCEWithLogits()(xb, y)
    (la * 3.0).backward()
    (lb * 3.0).backward()
    assert abs(float(lb) - float(la)) <= 1e-5 * max(1.0, abs(float(la))), (float(lb), float(la))
    torch.testing.assert_close(xb.grad.double(), xa.grad.double(), rtol=1e-5, atol=1e-8)


def test_dlrm_step_with_fused_tail_matches_eager():
    """The DLRM step with every fusion (fused BCE, multi-tensor SGD writing the tower images,
    embedding SGD inside the backward, head copy inside the gather) against the same model
    trained with torch's SGD, BCEWithLogitsLoss and sparse embedding gradients."""
    from raydp_amd.models.dlrm import Dlrm
    from raydp_amd.ops.fused_optim import FusedBCEWithLogits, sgd_step
    torch.manual_seed(0)
    base = Dlrm(13, [1000] * 26, [512, 128, 32], [1024, 1024, 512, 256, 1], 32).cuda()
    ref = copy.deepcopy(base)
    fused = copy.deepcopy(base)
    fused.embeddings.fused_sgd_lr = 0.05
    g = torch.Generator(device="cuda").manual_seed(3)
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.05)
    o_f = torch.optim.SGD(fused.parameters(), lr=0.05)
    for _ in range(4):
        dense = torch.randn(256, 13, device="cuda", generator=g)
        cats = torch.randint(0, 1000, (256, 26), device="cuda", generator=g)
        y = torch.randint(0, 2, (256, 1), device="cuda", generator=g).float()
        o_ref.zero_grad(set_to_none=True)
        la = nn.BCEWithLogitsLoss()(ref(dense, cats), y)
        la.backward()
        o_ref.step()
        o_f.zero_grad(set_to_none=True)
        lb = FusedBCEWithLogits()(fused(dense, cats), y)
        lb.backward()
        sgd_step(o_f)
        assert abs(float(la) - float(lb)) < 1e-4, (float(la), float(lb))
    torch.cuda.synchronize()
    for (n, a), (_, b) in zip(ref.state_dict().items(), fused.state_dict().items()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5, msg=n)


def test_prepare_model_graphs_the_training_step_like_eager():
    """graph_model (train.torch.prepare_model on one GPU worker): a BatchNorm MLP with a
    multi-input forward trained for 12 steps, graphed after 3 same-shape calls, with a ragged last
    batch and an eval pass in between, ends with the same parameters, BatchNorm running statistics
    and losses as the eager model (the same kernels replayed)."""
    from raydp_amd.train.gpu_policy import graph_model

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc1, self.bn1, self.fc2 = nn.Linear(6, 32), nn.BatchNorm1d(32), nn.Linear(32, 2)

        def forward(self, *cols):
            x = torch.cat(cols, dim=1)
            return self.fc2(self.bn1(torch.relu(self.fc1(x))))

    torch.manual_seed(0)
    ref = Net().cuda()
    mine = copy.deepcopy(ref)
    graph_model(mine)
    ro = torch.optim.Adam(ref.parameters(), lr=1e-2)
    mo = torch.optim.Adam(mine.parameters(), lr=1e-2)
    g = torch.Generator().manual_seed(3)
    data = [(torch.randn(64 if i < 11 else 37, 6, generator=g).cuda(), torch.randint(0, 2, (64 if i < 11 else 37,),
                                                                                      generator=g).cuda())
            for i in range(12)]
    losses = []
    for i, (x, y) in enumerate(data):
        for m, o in ((ref, ro), (mine, mo)):
            m.train()
            cols = [x[:, k].unsqueeze(1) for k in range(6)]
            loss = nn.functional.cross_entropy(m(*cols), y)
            o.zero_grad()
            loss.backward()
            o.step()
            losses.append(loss.item())
        if i == 5:
            for m in (ref, mine):
                m.eval()
                with torch.no_grad():
                    m(*[x[:, k].unsqueeze(1) for k in range(6)])
    for a, b in zip(ref.state_dict().values(), mine.state_dict().values()):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(torch.tensor(losses[1::2]), torch.tensor(losses[0::2]), rtol=1e-5, atol=1e-6)
    assert getattr(mine, "_raydp_graphed", False)


def test_graph_model_captures_while_the_previous_steps_loss_is_alive():
    """A user loop that keeps last step's ``loss`` (and so its autograd graph and the parameters'
    gradient accumulators) alive into the step that triggers the capture -- the Horovod NYC loop
    -- must capture (the capture differentiates w.r.t. parameter aliases; capturing against the
    live accumulators crashed at capture end) and train like the eager model."""
    import torch.nn.functional as F
    from raydp_amd.train.gpu_policy import graph_model

    class NYC(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.ModuleList([nn.Linear(a, b) for a, b in ((20, 256), (256, 128), (128, 64), (64, 16))])
            self.bn = nn.ModuleList([nn.BatchNorm1d(n) for n in (256, 128, 64, 16)])
            self.head = nn.Linear(16, 1)

        def forward(self, x):
            for fc, bn in zip(self.fc, self.bn):
                x = bn(F.relu(fc(x)))
            return self.head(x)

    torch.manual_seed(0)
    ref = NYC().cuda()
    mine = copy.deepcopy(ref)
    graph_model(mine)
    g = torch.Generator().manual_seed(4)
    data = [(torch.randn(64, 20, generator=g).cuda(), torch.randn(64, 1, generator=g).cuda()) for _ in range(8)]
    losses = {}
    for m in (ref, mine):
        opt = torch.optim.Adam(m.parameters(), lr=1e-2)
        out, loss = [], None
        for x, y in data:          # `loss` of the previous step is alive at every forward
            opt.zero_grad()
            loss = F.smooth_l1_loss(m(x), y)
            loss.backward()
            opt.step()
            out.append(loss.item())
        losses[id(m)] = out
    assert len(mine._raydp_graphs) == 1      # captured (not fallen back to eager)
    torch.testing.assert_close(torch.tensor(losses[id(mine)]), torch.tensor(losses[id(ref)]), rtol=1e-4, atol=1e-5)
    for a, b in zip(ref.state_dict().values(), mine.state_dict().values()):
        torch.testing.assert_close(b, a, rtol=1e-4, atol=1e-5)


def test_graph_model_captures_a_forward_that_indexes_with_a_list():
    """The stroke tutorial's NET_Model indexes columns with a Python list (an H2D copy of the list
    per call, which a capture refuses) and owns layers its forward never uses: graph_model still
    captures it (cached device indices; unused parameters get no gradient) and trains exactly
    like the eager model."""
    from raydp_amd.train.gpu_policy import graph_model

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.emb = nn.Embedding(5, 3)
            self.fc_dense, self.fc = nn.Linear(3, 8), nn.Linear(11, 2)
            self.unused = nn.Linear(4, 4)      # (as the tutorial model's unused layers)

        def forward(self, *cols):
            x = torch.cat(cols, dim=1)
            dense = x[:, [1, 2, 3]]
            return self.fc(torch.cat([self.fc_dense(dense), self.emb(x[:, 0].long())], dim=1))

    torch.manual_seed(0)
    ref = Net().cuda()
    mine = copy.deepcopy(ref)
    graph_model(mine)
    g = torch.Generator().manual_seed(6)
    losses = {}
    for m in (ref, mine):
        opt = torch.optim.Adam(m.parameters(), lr=1e-2)
        crit = nn.CrossEntropyLoss(weight=torch.tensor([0.35, 0.65], device="cuda"))
        out = []
        g.manual_seed(6)
        for _ in range(8):
            x = torch.cat([torch.randint(0, 5, (64, 1), generator=g).float(), torch.randn(64, 3, generator=g)], 1).cuda()
            y = torch.randint(0, 2, (64,), generator=g).cuda()
            loss = crit(m(*[x[:, i].unsqueeze(1) for i in range(4)]), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            out.append(loss.item())
        losses[id(m)] = out
    assert len(mine._raydp_graphs) == 1
    torch.testing.assert_close(torch.tensor(losses[id(mine)]), torch.tensor(losses[id(ref)]), rtol=1e-5, atol=1e-6)


def test_worker_policy_runs_torch_optimizers_on_the_fused_kernels(monkeypatch):
    """Under the GPU worker's policies a user loop's plain torch.optim.Adam / SGD step runs on the
    multi-tensor kernels (fused_step), and trains like torch's own step; outside the policies (and
    for an optimizer with a step hook) torch's step runs."""
    from raydp_amd.ops import fused_optim
    from raydp_amd.train.gpu_policy import fused_optimizers
    calls = {"n": 0}
    real = fused_optim.fused_step

    def counting(opt):
        ok = real(opt)
        calls["n"] += int(ok)
        return ok
    monkeypatch.setattr(fused_optim, "fused_step", counting)
    for make in (lambda ps: torch.optim.Adam(ps, lr=1e-2, weight_decay=0.01),
                 lambda ps: torch.optim.SGD(ps, lr=1e-2, momentum=0.9)):
        torch.manual_seed(0)
        ref = nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 1)).cuda()
        mine = copy.deepcopy(ref)
        g = torch.Generator().manual_seed(2)
        data = [(torch.randn(64, 16, generator=g).cuda(), torch.randn(64, 1, generator=g).cuda()) for _ in range(6)]
        o_ref = make(ref.parameters())
        for x, y in data:
            o_ref.zero_grad()
            nn.functional.mse_loss(ref(x), y).backward()
            o_ref.step()
        before = calls["n"]
        with fused_optimizers(True):
            o = make(mine.parameters())
            for x, y in data:
                o.zero_grad()
                nn.functional.mse_loss(mine(x), y).backward()
                o.step()
        assert calls["n"] - before == len(data)
        for a, b in zip(ref.parameters(), mine.parameters()):
            torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    with fused_optimizers(True):   # a step hook keeps torch's step
        p = nn.Parameter(torch.randn(8, device="cuda"))
        o = torch.optim.Adam([p], lr=0.1)
        seen = []
        o.register_step_post_hook(lambda *a: seen.append(1))
        p.grad = torch.randn(8, device="cuda")
        n0 = calls["n"]
        o.step()
        assert seen == [1] and calls["n"] == n0


def test_graph_model_twin_forwards_before_one_backward_and_copies():
    """Two same-shape forwards before ONE backward (a twin network, two losses summed): the
    second call must not overwrite the first replay's saved activations, so the gradients equal
    the eager model's. deepcopy / torch.save of a graphed module give the plain module."""
    import io
    from raydp_amd.train.gpu_policy import graph_model
    torch.manual_seed(0)
    ref = nn.Sequential(nn.Linear(8, 32), nn.ReLU(), nn.Linear(32, 1)).cuda()
    mine = copy.deepcopy(ref)
    graph_model(mine)
    g = torch.Generator().manual_seed(5)
    for i in range(8):
        a = torch.randn(64, 8, generator=g).cuda()
        b = torch.randn(64, 8, generator=g).cuda()
        grads = []
        for m in (ref, mine):
            m.zero_grad()
            loss = (m(a) - m(b)).pow(2).mean() + m(a).mean()
            loss.backward()
            grads.append([p.grad.clone() for p in m.parameters()])
        for ga, gb in zip(*grads):
            torch.testing.assert_close(gb, ga, rtol=1e-5, atol=1e-6)
    twin = copy.deepcopy(mine)
    assert not getattr(twin, "_raydp_graphed", False) and "forward" not in twin.__dict__
    x = torch.randn(64, 8).cuda()
    torch.testing.assert_close(twin(x), ref(x))
    buf = io.BytesIO()
    torch.save(mine, buf)
    buf.seek(0)
    back = torch.load(buf, weights_only=False)      # (a file this test wrote itself)
    torch.testing.assert_close(back(x), ref(x))


def test_fused_step_declines_optimizers_with_step_hooks():
    """Step pre/post hooks run only inside torch's own step(): fused_step leaves such optimizers alone."""
    from raydp_amd.ops.fused_optim import fused_step
    ps = _params()
    o = torch.optim.Adam(ps, lr=1e-3)
    for p in ps:
        p.grad = torch.ones_like(p)
    seen = []
    h = o.register_step_post_hook(lambda *a: seen.append(1))
    assert fused_step(o) is False
    h.remove()
    assert fused_step(o) is True
