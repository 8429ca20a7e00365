"""Collectives at world sizes 4 and 8 on gloo (SURVEY.md §4.4 asks for 2-8 ranks): DDP buckets
and sparse embedding gradients, table-wise sharded embeddings with uneven tables (and ranks that
own no table), GBDT histogram all-reduce, the all-reduce routing threshold, and the spawned
TorchEstimator worker group."""
import math
import multiprocessing as mp

import numpy as np
import pytest
import torch
import torch.nn as nn

from raydp_amd.train.trainer import _free_port


def _spawn(target, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    try:
        res = sorted((q.get(timeout=timeout) for _ in ps), key=lambda r: r[0])
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return res


def _init(rank, world, port):
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    return dist


class _EmbMlp(nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(13, 4, sparse=True)
        self.l1 = nn.Linear(4 + 3, 32)
        self.l2 = nn.Linear(32, 16)
        self.l3 = nn.Linear(16, 1)

    def forward(self, ids, x):
        h = torch.cat([self.emb(ids), x], 1)
        return self.l3(torch.relu(self.l2(torch.relu(self.l1(h)))))


def _batch(seed, n=12):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 13, (n,), generator=g), torch.randn(n, 3, generator=g), torch.randn(n, 1, generator=g)


def _ddp_rank(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from raydp_amd.parallel.ddp import DistributedDataParallel
        torch.manual_seed(0)
        m = _EmbMlp()
        if rank:
            with torch.no_grad():      # different init: the wrap-time broadcast must fix it
                for p in m.parameters():
                    p.add_(0.5)
        # a bucket cap below one layer's size: several buckets, reduced as backward produces them
        ddp = DistributedDataParallel(m, bucket_cap_mb=0.0005)
        ids, x, y = _batch(100 + rank)
        nn.functional.mse_loss(ddp(ids, x), y).backward()
        grads = {n: (p.grad.to_dense() if p.grad.is_sparse else p.grad).clone() for n, p in m.named_parameters()}
        q.put((rank, len(ddp.buckets), {k: v.tolist() for k, v in grads.items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_ddp_buckets_and_sparse_grads_match_full_batch(world):
    res = _spawn(_ddp_rank, world)
    assert res[0][1] >= 3, "expected several buckets"
    torch.manual_seed(0)
    ref = _EmbMlp()
    # DDP averages per-rank mean-loss gradients: the reference is the mean of per-rank losses
    loss = sum(nn.functional.mse_loss(ref(*_batch(100 + r)[:2]), _batch(100 + r)[2]) for r in range(world)) / world
    loss.backward()
    for name, p in ref.named_parameters():
        want = p.grad.to_dense() if p.grad.is_sparse else p.grad
        for r in res:
            torch.testing.assert_close(torch.tensor(r[2][name]), want, atol=1e-5, rtol=1e-4)


SIZES = [5, 9, 17, 40, 3]
D = 8


def _full_table(t):
    g = torch.Generator().manual_seed(t)
    s = SIZES[t]
    return (torch.rand(s, D, generator=g) * 2 - 1) * math.sqrt(1.0 / s)


def _sharded_rank(rank, world, port, q, static):
    dist = _init(rank, world, port)
    try:
        from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
        B = 6 if static else 3 + rank           # uneven batches across ranks when not static
        g = torch.Generator().manual_seed(100 + rank)
        idx = torch.stack([torch.randint(0, s, (B,), generator=g) for s in SIZES], 1)
        mlp = torch.randn(B, D, generator=g)
        coef = torch.randn(B, len(SIZES) + 1, D, generator=g)
        emb = ShardedEmbeddings(SIZES, D, static_batch=static)
        X = emb(mlp, idx)
        (X * coef).sum().backward()
        tabs = [_full_table(t).requires_grad_(True) for t in range(len(SIZES))]
        Xr = torch.cat([mlp.unsqueeze(1)] + [tabs[t][idx[:, t]].unsqueeze(1) for t in range(len(SIZES))], 1)
        (Xr * coef).sum().backward()
        fwd_ok = torch.allclose(X, Xr.detach(), atol=1e-6)
        grads = [t.grad.clone() for t in tabs]
        for gr in grads:
            dist.all_reduce(gr)
        ok = True
        if emb.local_tables:
            dense = emb.weight.grad.coalesce().to_dense() if emb.weight.grad is not None else \
                torch.zeros(emb.weight.shape)
            for i, t in enumerate(emb.local_tables):
                o = int(emb.local_offsets[i])
                ok &= torch.allclose(dense[o:o + SIZES[t]], grads[t], atol=1e-5)
        q.put((rank, bool(fwd_ok), bool(ok), list(emb.local_tables)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,static", [(4, True), (8, True), (4, False)])
def test_sharded_embeddings_uneven_tables(world, static):
    res = _spawn(_sharded_rank, world, static)
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
    owned = sorted(t for r in res for t in r[3])
    assert owned == list(range(len(SIZES)))
    if world > len(SIZES):
        assert any(not r[3] for r in res), "some rank should own no table"


def _gbdt_rank(rank, world, port, q, x, y):
    dist = _init(rank, world, port)
    try:
        from raydp_amd.xgboost.gbdt import DMatrix, train
        n = x.shape[0] // world
        b = train({"objective": "reg:squarederror", "max_depth": 3, "eta": 0.3, "max_bin": 32},
                  DMatrix(x[rank * n:(rank + 1) * n].numpy(), y[rank * n:(rank + 1) * n].numpy()), 3)
        q.put((rank, np.asarray(b.inplace_predict(x[:50].numpy())).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4])
def test_gbdt_histograms_at_world_4(world):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((800, 5)).astype(np.float32)
    y = (x[:, 0] * 2 + x[:, 1] ** 2).astype(np.float32)
    res = _spawn(_gbdt_rank, world, torch.from_numpy(x), torch.from_numpy(y))
    preds = [np.array(r[1]) for r in res]
    for p in preds[1:]:
        np.testing.assert_allclose(p, preds[0], rtol=0, atol=0)   # every rank holds the same trees
    assert np.corrcoef(preds[0], y[:50])[0, 1] > 0.7


def _allgather_rank(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from raydp_amd.xgboost.gbdt import World
        w = World()
        rows = torch.full((rank + 1, 2), float(rank))
        got = w.allgather_rows(rows)
        t = torch.tensor([float(rank)], dtype=torch.float64)
        w.allreduce(t)
        q.put((rank, got.tolist(), float(t)))
    finally:
        dist.destroy_process_group()


def test_gbdt_world_allgather_uneven_rows():
    res = _spawn(_allgather_rank, 4)
    want = [[float(r)] * 2 for r in range(4) for _ in range(r + 1)]
    for r in res:
        assert r[1] == want and r[2] == 6.0


def test_gbdt_world_stages_cpu_tensors_through_gpu_for_rccl(monkeypatch):
    """RCCL (backend "nccl") takes device tensors only: CPU inputs are staged on the current GPU."""
    from raydp_amd.xgboost.gbdt import World

    class FakeDist:
        def get_backend(self):
            return "nccl"
    w = World.__new__(World)
    w.dist, w.size = FakeDist(), 2
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    assert w._comm_device(torch.zeros(1)) == torch.device("cuda", 3)

    class Gloo(FakeDist):
        def get_backend(self):
            return "gloo"
    w.dist = Gloo()
    assert w._comm_device(torch.zeros(1)) == torch.device("cpu")


def test_bucket_allreduce_routing_threshold():
    """One-shot xGMI for fp32 buckets up to spark.ray.mi355x.allreduce.oneshot_max_mb (16 MiB:
    the DLRM dense gradient, 8.7 MB, is one one-shot bucket); larger ones and other dtypes go
    to RCCL, and nothing routes to xGMI without a communicator."""
    from raydp_amd.ops import comm

    class FakeFlat:
        def __init__(self, n, dtype=torch.float32):
            self._n, self.dtype, self.is_cuda = n, dtype, True

        def numel(self):
            return self._n

        def is_contiguous(self):
            return True

    class FakeXg:
        max_floats = comm.XG_BUCKET_MAX_BYTES // 4
    b = comm.BucketAllreduce.__new__(comm.BucketAllreduce)
    b.group, b.xg, b.limit = None, FakeXg(), comm.oneshot_max_bytes()
    assert comm.oneshot_max_bytes() == 16 << 20
    limit = b.limit // 4
    assert b.routes_to_xgmi(FakeFlat(limit))
    assert not b.routes_to_xgmi(FakeFlat(limit + 1))
    assert b.routes_to_xgmi(FakeFlat(2_177_185))              # DLRM dense gradient (8.7 MB)
    assert not b.routes_to_xgmi(FakeFlat(1024, torch.bfloat16))
    b.limit = 1 << 20                                        # a lowered threshold is honoured
    assert not b.routes_to_xgmi(FakeFlat(2_177_185))
    b.xg = None
    assert not b.routes_to_xgmi(FakeFlat(16))


def test_torch_estimator_spawned_world_4(runtime_local, tmp_path):
    """TorchEstimator(num_workers=4) through the spawned worker group (gloo on CPU): every rank
    trains its shard, DDP keeps them identical, rank 0 checkpoints, the per-epoch report names
    the all-reduce path."""
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    rng = np.random.default_rng(0)
    x = rng.standard_normal((800, 3)).astype(np.float32)
    df = pd.DataFrame({"a": x[:, 0], "b": x[:, 1], "c": x[:, 2], "y": x @ np.array([1.0, -2.0, 0.5]) + 0.3})
    ds = from_pandas(df)
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(3, 16), nn.ReLU(), nn.Linear(16, 1))
    est = TorchEstimator(num_workers=4, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=0.02),
                         loss=nn.MSELoss(), feature_columns=["a", "b", "c"], label_column="y",
                         batch_size=50, num_epochs=4, use_gpu=False, storage_path=str(tmp_path))
    res = est.fit(ds)
    hist = [m for m in res.metrics_history if "train_loss" in m]
    assert len(hist) == 4 and hist[-1]["train_loss"] < hist[0]["train_loss"]
    assert hist[-1]["allreduce"].startswith("torch.distributed:gloo")
    trained = est.get_model()
    pred = trained(torch.from_numpy(x[:100])).detach().numpy()[:, 0]
    assert np.corrcoef(pred, df["y"].to_numpy()[:100])[0, 1] > 0.9


def _auto_batch_rank(rank, world, port, q):
    dist = _init(rank, world, port)
    try:
        from raydp_amd.parallel.embedding_mp import ShardedEmbeddings
        calls = {"n": 0}
        real = dist.all_gather

        def counting(*a, **k):
            calls["n"] += 1
            return real(*a, **k)
        dist.all_gather = counting
        emb = ShardedEmbeddings(SIZES, D)            # static_batch="auto"
        ok = True
        for B in (6, 6, 6, 4, 4):                    # every rank changes size at the same step
            g = torch.Generator().manual_seed(7 * B + rank)
            idx = torch.stack([torch.randint(0, s, (B,), generator=g) for s in SIZES], 1)
            X = emb(torch.zeros(B, D), idx)
            ref = torch.cat([torch.zeros(B, 1, D)] + [_full_table(t)[idx[:, t]].unsqueeze(1)
                                                      for t in range(len(SIZES))], 1)
            ok &= bool(torch.allclose(X, ref, atol=1e-6))
        dist.all_gather = real
        q.put((rank, ok, calls["n"]))
    finally:
        dist.destroy_process_group()


def test_sharded_embeddings_exchange_batch_sizes_only_on_change():
    res = _spawn(_auto_batch_rank, 2)
    for r in res:
        assert r[1], r
        assert r[2] == 2, r       # first step and the step where the size changed


def test_fused_engine_adds_no_host_sync_per_epoch_at_world_2(monkeypatch):
    """World > 1 costs of the fused engine's epoch: no collective and no host read of its own
    (the step count is agreed once at load -- and not at all for trainer-split equal shards;
    the xGMI vote rides in the metrics read inside the native epoch). Counted with the
    distributed API and Tensor.item instrumented around FusedMLPEngine.train_epoch / load."""
    import types

    import torch.distributed as dist
    from raydp_amd.torch import engine as E

    calls = []
    for name in ("all_reduce", "broadcast", "all_gather", "all_gather_object", "barrier", "broadcast_object_list"):
        monkeypatch.setattr(dist, name, lambda *a, _n=name, **k: calls.append(_n))
    real_item = torch.Tensor.item
    monkeypatch.setattr(torch.Tensor, "item", lambda self: (calls.append("item"), real_item(self))[1])
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "gloo")

    class FakeTrainer:
        batch, steps_in_epoch = 64, 4
        desc = types.SimpleNamespace(out_dim=1)

        def train_epoch(self, *a, **k):
            return {"loss": 0.5, "mae": 0.1, "mse": 0.2, "acc": 0.0, "xg_vote": 0.0}

        def note_steps(self, n):
            pass

        def step_times_us(self):
            return None
    shard = types.SimpleNamespace(feats_bf16=None, labels=None, n=256)
    eng = types.SimpleNamespace(trainer=FakeTrainer(), world=2, drop_last=True, xg=None, ar=None, comm=None,
                                max_steps=None, shuffle=False, epoch=0, metrics_names=["MeanAbsoluteError"],
                                train=shard, loss=None)
    eng._res = lambda m: E.FusedMLPEngine._res(eng, m)
    for _ in range(3):
        E.FusedMLPEngine.train_epoch(eng)
    assert calls == [], calls
    # load(): trainer-split shards are equal -> nothing; SPMD local shards -> one agreement
    monkeypatch.setattr(E, "_ShardTensors", lambda *a, **k: shard)
    eng.trainer.feat_k, eng.device = 24, torch.device("cpu")
    cfg = {"feature_columns": ["a"], "feature_types": None, "label_column": "y"}
    eng.equal_shards = True
    E.FusedMLPEngine.load(eng, None, None, cfg)
    assert calls == [], calls
    eng.equal_shards = False
    E.FusedMLPEngine.load(eng, None, None, cfg)
    assert calls == ["all_reduce", "item"], calls


def test_warm_worker_groups_are_reused_and_evicted_for_resources(runtime_local, tmp_path, monkeypatch):
    """Spawned worker groups stay warm between fits of the same shape (no new processes), a
    different shape that does not fit beside them evicts them, and runtime shutdown stops them."""
    import pandas as pd
    from raydp_amd.data import from_pandas
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.train import trainer as T
    df = pd.DataFrame({"a": np.arange(64.0), "y": np.arange(64.0) * 0.5})

    def fit(workers, cpus):
        torch.manual_seed(0)
        m = nn.Linear(1, 1)
        est = TorchEstimator(num_workers=workers, resources_per_worker={"CPU": cpus}, model=m,
                             optimizer=torch.optim.SGD(m.parameters(), lr=1e-3), loss=nn.MSELoss(),
                             feature_columns=["a"], label_column="y", batch_size=8, num_epochs=1, use_gpu=False,
                             storage_path=str(tmp_path), fused="off")
        return est.fit(from_pandas(df))
    fit(2, 1)
    g1 = next(iter(T._GROUPS._groups.values()))
    pids = [w._impl.pid for w in g1.workers]
    fit(2, 1)
    assert next(iter(T._GROUPS._groups.values())) is g1 and [w._impl.pid for w in g1.workers] == pids
    fit(2, 2.5)                 # 2 x 2.5 CPUs do not fit beside the warm group's 2 on 6 CPUs
    assert len(T._GROUPS) == 1 and next(iter(T._GROUPS._groups.values())) is not g1
    T.release_worker_groups()
    assert len(T._GROUPS) == 0
