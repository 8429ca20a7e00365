"""Table-wise sharded embeddings with all-to-all (raydp_amd.parallel.embedding_mp), gloo world 2:
forward equals a replicated lookup, backward gives every owner the summed gradient rows."""
import math
import multiprocessing as mp

import torch

from raydp_amd.train.trainer import _free_port

SIZES = [5, 9, 17, 40, 3]
D = 8


def _full_table(t, seed=0):
    s = SIZES[t]
    g = torch.Generator().manual_seed(seed * 1000003 + t)
    return (torch.rand(s, D, generator=g) * 2 - 1) * math.sqrt(1.0 / s)


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        B = 6 if rank == 0 else 4
        g = torch.Generator().manual_seed(100 + rank)
        idx = torch.stack([torch.randint(0, s, (B,), generator=g) for s in SIZES], 1)
        mlp = torch.randn(B, D, generator=g)
        coef = torch.randn(B, len(SIZES) + 1, D, generator=g)
        emb = ShardedEmbeddings(SIZES, D)
        X = emb(mlp, idx)
        (X * coef).sum().backward()
        # replicated reference
        tabs = [_full_table(t).requires_grad_(True) for t in range(len(SIZES))]
        Xr = torch.cat([mlp.unsqueeze(1)] + [tabs[t][idx[:, t]].unsqueeze(1) for t in range(len(SIZES))], 1)
        (Xr * coef).sum().backward()
        fwd_ok = torch.allclose(X, Xr.detach(), atol=1e-6)
        grads = [t.grad.clone() for t in tabs]
        for gr in grads:
            dist.all_reduce(gr)
        dense = emb.weight.grad.coalesce().to_dense() if emb.weight.grad is not None else None
        bwd_ok = True
        for t in emb.local_tables:
            i = emb.local_tables.index(t)
            o = int(emb.local_offsets[i])
            bwd_ok &= torch.allclose(dense[o:o + SIZES[t]], grads[t], atol=1e-5)
        q.put((rank, fwd_ok, bool(bwd_ok), emb.local_tables))
    finally:
        dist.destroy_process_group()


def test_sharded_embeddings_match_replicated():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
    owned = sorted(t for r in res for t in r[3])
    assert owned == list(range(len(SIZES)))


def test_place_tables_balances():
    from raydp_amd.parallel.embedding_mp import place_tables
    owner = place_tables([100, 90, 10, 10, 5], 2)
    load = [sum(s for s, o in zip([100, 90, 10, 10, 5], owner) if o == r) for r in range(2)]
    assert max(load) - min(load) <= 25


def _ddp_sparse_main(rank, world, port, q):
    import torch.distributed as dist
    import torch.nn as nn
    from raydp_amd.parallel.ddp import DistributedDataParallel
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        m = nn.Sequential(nn.Embedding(10, 4, sparse=True))
        ddp = DistributedDataParallel(m)
        ids = torch.tensor([rank, 3, 3])
        ddp(ids).sum().backward()
        g = m[0].weight.grad.to_dense()
        q.put((rank, g.tolist()))
    finally:
        dist.destroy_process_group()


def test_ddp_reduces_sparse_embedding_grads():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_sparse_main, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    exp = torch.zeros(10, 4)
    exp[0] += 0.5   # row 0 looked up once on rank 0, averaged over 2 ranks
    exp[1] += 0.5
    exp[3] += 2.0   # twice per rank: (2 + 2) / 2
    for r in (0, 1):
        assert torch.allclose(torch.tensor(res[r]), exp)


def _dlrm_rank(rank, world, port, q):
    import torch.distributed as dist
    from raydp_amd.models.dlrm import Dlrm
    from raydp_amd.parallel.ddp import DistributedDataParallel
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        torch.manual_seed(0)
        sizes = [7, 11, 5, 9]
        model = Dlrm(3, sizes, [16, 8], [32, 16, 1], 8, model_parallel=True)
        net = DistributedDataParallel(model)
        opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.1)
        g = torch.Generator().manual_seed(5 + rank)
        losses = []
        for _ in range(3):
            dense = torch.randn(6, 3, generator=g)
            cats = torch.stack([torch.randint(0, s, (6,), generator=g) for s in sizes], 1)
            y = torch.randint(0, 2, (6, 1), generator=g).float()
            loss = torch.nn.functional.binary_cross_entropy_with_logits(net(dense, cats), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(float(loss))
        dense_params = torch.cat([p.detach().reshape(-1) for n, p in model.named_parameters()
                                  if not n.startswith("embeddings")])
        gathered = [None] * world
        dist.all_gather_object(gathered, dense_params)
        q.put((rank, all(math.isfinite(x) for x in losses), all(torch.equal(gathered[0], t) for t in gathered),
               model.embeddings.local_tables))
    finally:
        dist.destroy_process_group()


def test_dlrm_model_parallel_trains_with_ddp():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dlrm_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] and r[2] for r in res), res
    assert sorted(t for r in res for t in r[3]) == [0, 1, 2, 3]


def _fused_rank(rank, world, port, q):
    import torch.distributed as dist
    from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        B = 5
        g = torch.Generator().manual_seed(300 + rank)
        idx = torch.stack([torch.randint(0, s, (B,), generator=g) for s in SIZES], 1)
        mlp = torch.randn(B, D, generator=g)
        coef = torch.randn(B, len(SIZES) + 1, D, generator=g)
        a = ShardedEmbeddings(SIZES, D, static_batch=True)
        b = ShardedEmbeddings(SIZES, D, fused_sgd_lr=0.5, static_batch=True)
        (a(mlp, idx) * coef).sum().backward()
        with torch.no_grad():
            if a.weight.grad is not None:
                a.weight.add_(a.weight.grad.coalesce().to_dense(), alpha=-0.5)
        (b(mlp, idx) * coef).sum().backward()
        q.put((rank, b.weight.grad is None, bool(torch.allclose(a.weight, b.weight, atol=1e-6))))
    finally:
        dist.destroy_process_group()


def test_sharded_fused_sgd_equals_sparse_sgd():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fused_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] and r[2] for r in res), res
