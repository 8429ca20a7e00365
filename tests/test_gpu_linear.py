"""Fused Linear+bias+ReLU towers (csrc/hip/linear_act.hip) against PyTorch references:
a bf16-emulating fp32 reference (same rounding points: tight) and plain fp32 torch (loose),
forward and backward, at the reference DLRM shapes (examples/pytorch_dlrm.ipynb cell 9) and at
ragged shapes that exercise every edge path."""
import numpy as np
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _bf(t):
    return t.to(torch.bfloat16).float()


def _emulated(x, lins, relus):
    """Forward/backward with the kernels' rounding points, in fp32 torch."""
    hs = [x.float() if x.dtype == torch.float32 else x.float()]
    h = hs[0]
    for lin, r in zip(lins, relus):
        y = _bf(h) @ _bf(lin.weight.detach()).T + (lin.bias.detach() if lin.bias is not None else 0)
        if r:
            y = torch.relu(y)
        h = _bf(y)
        hs.append(h)
    return hs


def _emulated_bwd(hs, lins, relus, gout, x_f32):
    G = gout.float() * (hs[-1] > 0).float() if relus[-1] else gout.float()
    G = _bf(G)
    grads, dx = [], None
    for li in range(len(lins) - 1, -1, -1):
        X = _bf(hs[li])
        dW = G.T @ X
        db = G.sum(0)
        grads.append((li, dW, db))
        d = G @ _bf(lins[li].weight.detach())
        if li > 0:
            if relus[li - 1]:
                d = d * (hs[li] > 0).float()
            G = _bf(d)
        else:
            dx = d if x_f32 else _bf(d)
    return dict((li, (dW, db)) for li, dW, db in grads), dx


def _tower(dims, relus, seed=0):
    torch.manual_seed(seed)
    return [nn.Linear(a, b).cuda() for a, b in zip(dims[:-1], dims[1:])], relus


def _rel(a, b):
    return float((a - b).norm() / max(b.norm(), 1e-12))


@pytest.mark.parametrize("case", ["top", "bottom", "ragged", "tiny"])
def test_fused_tower_matches_references(case):
    from raydp_amd.ops.linear_ops import FusedLinearTower
    if case == "top":      # interaction output -> 1024 -> 1024 -> 512 -> 256 -> 1 (logit)
        M, dims, relus, x_dtype = 2048, [384, 1024, 1024, 512, 256, 1], [True] * 4 + [False], torch.float32
    elif case == "bottom":  # dense features -> 512 -> 128 -> 32
        M, dims, relus, x_dtype = 2048, [13, 512, 128, 32], [True] * 3, torch.float32
    elif case == "ragged":
        M, dims, relus, x_dtype = 333, [72, 65, 130, 7], [True, False, True], torch.bfloat16
    else:
        M, dims, relus, x_dtype = 5, [3, 2, 1], [True, False], torch.float32
    lins, relus = _tower(dims, relus)
    tower = FusedLinearTower(lins, relus, out_f32=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(M, dims[0], device="cuda", generator=g).to(x_dtype).requires_grad_(True)
    y = tower(x)
    gout = torch.randn(M, dims[-1], device="cuda", generator=g)
    y.backward(gout)
    # bf16-emulating reference: same rounding points -> only fp32 summation order differs
    hs = _emulated(x.detach(), lins, relus)
    out_ref = hs[-1]
    y_exact = _bf(hs[-2]) @ _bf(lins[-1].weight.detach()).T + lins[-1].bias.detach()
    if relus[-1]:
        y_exact = torch.relu(y_exact)
    assert _rel(y.detach(), y_exact) < 2e-3, _rel(y.detach(), y_exact)
    gref, dxref = _emulated_bwd(hs, lins, relus, gout, x_dtype == torch.float32)
    for li, lin in enumerate(lins):
        dW, db = gref[li]
        assert _rel(lin.weight.grad, dW) < 5e-3, (li, _rel(lin.weight.grad, dW))
        assert _rel(lin.bias.grad, db) < 5e-3, (li, _rel(lin.bias.grad, db))
    assert _rel(x.grad.float(), dxref) < 5e-3
    # plain fp32 torch: bf16 operands cost ~1e-2
    xr = x.detach().float().clone().requires_grad_(True)
    h = xr
    for lin, r in zip(lins, relus):
        h = nn.functional.linear(h, lin.weight.detach().clone().requires_grad_(True), lin.bias.detach())
        h = torch.relu(h) if r else h
    assert _rel(y.detach(), h.detach()) < 3e-2
    del out_ref


def test_fused_tower_refreshes_images_after_optimizer_step():
    from raydp_amd.ops.linear_ops import FusedLinearTower
    lins, relus = _tower([64, 128, 16], [True, False], seed=3)
    tower = FusedLinearTower(lins, relus)
    opt = torch.optim.SGD([p for l in lins for p in l.parameters()], lr=0.5)
    x = torch.randn(256, 64, device="cuda")
    y0 = tower(x)
    y0.sum().backward()
    opt.step()
    y1 = tower(x)
    ref = torch.relu(x @ lins[0].weight.T + lins[0].bias) @ lins[1].weight.T + lins[1].bias
    assert _rel(y1.detach(), ref.detach()) < 2e-2
    assert _rel(y1.detach(), y0.detach()) > 1e-3          # the step was seen


def test_dlrm_fused_towers_match_eager_and_train(monkeypatch):
    """Same model, same batches: the fused-tower training trajectory follows the eager fp32 one
    (bf16 operands: loss within 2 %), and both learn."""
    import copy
    from raydp_amd.models.dlrm import Dlrm
    torch.manual_seed(0)
    sizes = [1000] * 26
    model = Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32).cuda()
    B = 512
    g = torch.Generator(device="cuda").manual_seed(2)
    dense = torch.randn(B, 13, device="cuda", generator=g)
    cats = torch.randint(0, 1000, (B, 26), device="cuda", generator=g)
    y = (dense[:, :1] + 0.5 * dense[:, 1:2] > 0).float()      # learnable from the dense features
    monkeypatch.setenv("RAYDP_FUSED_LINEAR", "0")
    eager_out = model(dense, cats).detach()
    monkeypatch.setenv("RAYDP_FUSED_LINEAR", "1")
    fused_out = model(dense, cats)
    assert _rel(fused_out.detach(), eager_out) < 3e-2
    lossf = nn.BCEWithLogitsLoss()
    traj = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("RAYDP_FUSED_LINEAR", mode)
        m = copy.deepcopy(model)
        opt = torch.optim.SGD([p for p in m.parameters() if p.requires_grad], lr=0.1)
        losses = []
        for _ in range(25):
            loss = lossf(m(dense, cats), y)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(float(loss))
        traj[mode] = np.array(losses)
    assert np.isfinite(traj["1"]).all()
    assert traj["1"][-1] < traj["1"][0] and traj["0"][-1] < traj["0"][0]
    np.testing.assert_allclose(traj["1"], traj["0"], rtol=2e-2)


@pytest.mark.parametrize("tile", [1, 2, 3, 4])
@pytest.mark.parametrize("splits", [1, 3, 8])
def test_split_k_is_deterministic_and_exact(splits, tile):
    """The split-K fix-up sums the partial tiles in split order: bitwise identical across runs,
    and equal (to fp32 reassociation) to the unsplit kernel, bias gradient included."""
    from raydp_amd.ops import linear_ops as L
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, K = 200, 96, 1000
    G = torch.randn(K, M, device="cuda", generator=g).to(torch.bfloat16)     # stored [K][rows]
    X = torch.randn(K, N, device="cuda", generator=g).to(torch.bfloat16)
    outs = []
    for _ in range(2):
        dW = torch.empty(M, N, device="cuda")
        db = torch.empty(M, device="cuda")
        L.gemm(L.WGRAD, M, N, K, G, L.RED, X, L.RED, dW, dbias=db, splits=splits, tile=tile)
        outs.append((dW, db))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = G.float().T @ X.float()
    assert _rel(outs[0][0], ref) < 1e-5
    assert _rel(outs[0][1], G.float().sum(0)) < 1e-5


@pytest.mark.parametrize("tile", [1, 2, 3, 4])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("shape", [(777, 333, 1000), (512, 384, 1024)])
def test_gemm_all_epilogues_ragged(splits, tile, shape):
    """Every epilogue on ragged edges in every dimension (M, N, K not multiples of the 64-wide
    tiles), bf16 and fp32 operands in both memory orientations, split and unsplit, every tile
    shape, against fp32 references of the bf16-rounded operands. The second shape is whole
    128-tiles with aligned rows (the unchecked-load fast path of every stage)."""
    from raydp_amd.ops import linear_ops as L
    g = torch.Generator(device="cuda").manual_seed(11)
    M, N, K = shape
    X = torch.randn(M, K, device="cuda", generator=g)                        # fp32, ROW
    W = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)     # bf16, ROW
    b = torch.randn(N, device="cuda", generator=g)
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y32 = torch.empty(M, N, device="cuda")
    L.gemm(L.FWD, M, N, K, X, L.ROW, W, L.ROW, y, bias=b, relu=True, out2=y32, splits=splits, tile=tile)
    ref = torch.relu(_bf(X) @ W.float().T + b)
    assert _rel(y32, ref) < 1e-5 and _rel(y.float(), ref) < 1e-2
    # dgrad: dX = (G W) * mask with W read transposed ([K][N] memory = RED)
    G = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    Wt = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)   # memory [N][K] = [red][rows]
    mask = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    dx = torch.empty(M, K, device="cuda")
    L.gemm(L.DGRAD, M, K, N, G, L.ROW, Wt, L.RED, dx, mask=mask, splits=splits, tile=tile)
    ref = (G.float() @ Wt.float()) * (mask.float() > 0).float()
    assert _rel(dx, ref) < 1e-5
    # wgrad: dW = G^T X over the batch (both stored [batch][rows] = RED), bias-gradient row sums
    Xb = torch.randn(M, K, device="cuda", generator=g)                       # fp32 RED operand
    dW = torch.empty(K, N, device="cuda")
    db = torch.empty(K, device="cuda")
    L.gemm(L.WGRAD, K, N, M, Xb, L.RED, G, L.RED, dW, dbias=db, splits=splits, tile=tile)
    assert _rel(dW, _bf(Xb).T @ G.float()) < 1e-5
    assert _rel(db, _bf(Xb).sum(0)) < 1e-5


@pytest.mark.parametrize("M", [128, 2048])
def test_paired_backward_is_bitwise_the_two_launch_backward(M, monkeypatch):
    """lin_pair_kernel (a layer's dgrad + wgrad in one launch) computes exactly what the two
    separate launches compute: same tiles, same split-K order (each problem has its own half
    of the workspace)."""
    from raydp_amd.ops import linear_ops
    from raydp_amd.ops.linear_ops import FusedLinearTower
    dims, relus = [384, 1024, 1024, 512, 256, 1], [True] * 4 + [False]
    out = {}
    for pair in (False, True):
        monkeypatch.setattr(linear_ops, "PAIR_BACKWARD", pair)
        lins, _ = _tower(dims, relus, seed=7)
        tower = FusedLinearTower(lins, relus, out_f32=True)
        g = torch.Generator(device="cuda").manual_seed(5)
        x = torch.randn(M, dims[0], device="cuda", generator=g).requires_grad_(True)
        tower(x).backward(torch.randn(M, 1, device="cuda", generator=g))
        out[pair] = [x.grad.clone()] + [t.grad.clone() for lin in lins for t in (lin.weight, lin.bias)]
    for a, b in zip(out[False], out[True]):
        assert torch.equal(a, b)
