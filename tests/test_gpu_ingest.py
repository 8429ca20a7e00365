"""Object store -> HBM ingest (csrc/hip/arrow_ingest.hip) against a numpy reference, and the
device epoch permutation."""
import os
import uuid

import numpy as np
import pyarrow as pa
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expected(tables, cols, stride, fill):
    n = sum(t.num_rows for t in tables)
    exp = np.zeros((n, stride), np.float32)
    r0 = 0
    for tab in tables:
        for j, c in enumerate(cols):
            v = tab.column(c).to_pandas().to_numpy(dtype=np.float64, na_value=fill)
            exp[r0:r0 + tab.num_rows, j] = v
        r0 += tab.num_rows
    return exp


def _table(n, seed=0):
    rng = np.random.default_rng(seed)
    return pa.table({
        "a": pa.array(rng.standard_normal(n)),
        "b": pa.array(rng.integers(-50, 50, n).astype(np.int32)),
        "c": pa.array([None if i % 7 == 0 else float(i % 1000) for i in range(n)], pa.float32()),
        "d": pa.array([None if i % 11 == 3 else bool(i % 3) for i in range(n)], pa.bool_()),
        "e": pa.array(rng.integers(-3, 3, n).astype(np.int64)),
        "f": pa.array(rng.integers(0, 200, n).astype(np.uint8)),
        "s": pa.array([f"x{i}" for i in range(n)]),   # unused column between the used ones
    })


@pytest.fixture
def store():
    from raydp_amd.runtime.store import SharedObjectStore
    path = f"/dev/shm/raydp_test_ingest_{uuid.uuid4().hex[:8]}"
    st = SharedObjectStore(path, "node-test", create=True, capacity=512 << 20)
    yield st
    st.destroy()


def test_ingest_sliced_nulls_bools_pageable():
    from raydp_amd.ops.ingest import ingest_columns
    t = _table(1000)
    parts = [t.slice(13, 700), t.slice(0, 5), t.slice(701, 299)]
    cols = ["a", "b", "c", "d", "e", "f"]
    for out_bf16 in (False, True):
        for stride in (6, 8, 32):
            got = ingest_columns(parts, cols, "cuda", out_bf16, stride=stride, fill=-1.0).float().cpu().numpy()
            exp = _expected(parts, cols, stride, -1.0)
            tol = 1e-2 if out_bf16 else 1e-6
            np.testing.assert_allclose(got, exp, rtol=tol, atol=tol)


def test_ingest_from_store_is_pinned_dma(store):
    from raydp_amd.ops import ingest
    t = _table(50_000, seed=1)
    tables = []
    for k in range(3):
        oid = uuid.uuid4().hex
        store.put(oid, t.slice(k * 10_000, 17_000))
        found, v = store.get(oid)
        assert found
        tables.append(v)
    cols = ["a", "c", "d", "e", "f"]
    ingest.reset_ingest_stats()
    got = ingest.ingest_columns(tables, cols, "cuda", True, stride=8, fill=0.5).float().cpu().numpy()
    st = ingest.ingest_stats()
    np.testing.assert_allclose(got, _expected(tables, cols, 8, 0.5), rtol=1e-2, atol=1e-2)
    assert st["host_copy_bytes"] == 0, st
    assert st["dma_pageable_bytes"] == 0, st
    assert st["dma_pinned_bytes"] > 0 and st["dma_copies"] >= 3, st
    assert st["pin_calls"] >= 1, st


def test_ingest_ring_wraps_many_chunks(store):
    """A staging ring far smaller than the data: chunks reuse ring space only after the decode
    that read it is done (event waits); results must be exact."""
    from raydp_amd.ops import ingest
    t = _table(300_000, seed=2)
    oid = uuid.uuid4().hex
    store.put(oid, t)
    _, v = store.get(oid)
    cols = ["a", "b", "c", "d", "e", "f"]
    ingest.reset_ingest_stats()
    got = ingest.ingest_columns([v, v.slice(123, 45_678)], cols, "cuda", False, stride=8, fill=-2.0,
                                stage_bytes=1 << 20).cpu().numpy()
    st = ingest.ingest_stats()
    assert st["chunks"] > 8, st
    np.testing.assert_allclose(got, _expected([v, v.slice(123, 45_678)], cols, 8, -2.0), rtol=1e-6, atol=1e-6)


def test_feistel_permutation():
    from raydp_amd.ops.ingest import random_permutation
    for n in (1, 2, 3, 17, 1000, 4096, (1 << 20) + 7):
        p = random_permutation(n, 42, "cuda").cpu().numpy()
        assert p.dtype == np.int32 and p.shape == (n,)
        np.testing.assert_array_equal(np.sort(p), np.arange(n))
    a = random_permutation(10_000, 1, "cuda").cpu().numpy()
    b = random_permutation(10_000, 1, "cuda").cpu().numpy()
    c = random_permutation(10_000, 2, "cuda").cpu().numpy()
    np.testing.assert_array_equal(a, b)
    assert (a != c).mean() > 0.99
    # a shuffle, not a rotation: positions are spread out (correlation with identity ~ 0)
    assert abs(np.corrcoef(a, np.arange(10_000))[0, 1]) < 0.05
    # every row is as likely to land in the first batch as any other (coarse uniformity)
    first = np.concatenate([random_permutation(1000, s, "cuda").cpu().numpy()[:64] for s in range(200)])
    counts = np.bincount(first // 100, minlength=10)
    assert counts.min() > 0.7 * counts.mean(), counts


def test_int64_ingest_is_exact_above_2_pow_24(store):
    """Category ids go to HBM as exact int64 (a float tile would round ids above 2^24)."""
    from raydp_amd.ops import ingest
    n = 10_000
    rng = np.random.default_rng(3)
    big = rng.integers(2 ** 24, 2 ** 40, n)
    t = pa.table({"a": pa.array(big, pa.int64()),
                  "b": pa.array([None if i % 5 == 0 else int(v) for i, v in enumerate(rng.integers(0, 2 ** 31 - 1, n))],
                                pa.int32()),
                  "c": pa.array(rng.integers(0, 200, n).astype(np.uint8))})
    oid = uuid.uuid4().hex
    store.put(oid, t)
    _, v = store.get(oid)
    got = ingest.ingest_columns([v.slice(7, 9000), v.slice(0, 7)], ["a", "b", "c"], "cuda", False,
                                out_i64=True, fill=-1).cpu().numpy()
    exp = np.zeros((9007, 3), np.int64)
    for r0, tab in ((0, v.slice(7, 9000)), (9000, v.slice(0, 7))):
        for j, c in enumerate("abc"):
            exp[r0:r0 + tab.num_rows, j] = tab.column(c).to_pandas().fillna(-1).to_numpy().astype(np.int64)
    np.testing.assert_array_equal(got, exp)


def test_multi_input_shard_batches():
    """DLRM-shaped shard: 13 float + 26 int columns become one float and one int64 matrix; a
    batch is one gather per matrix, the inputs are its column views."""
    import torch
    from raydp_amd.data import from_arrow
    from raydp_amd.torch.engine import _ShardTensors
    rng = np.random.default_rng(0)
    n = 3000
    cols = {f"_c{i}": rng.standard_normal(n) for i in range(1, 14)}
    cols.update({f"_c{i}": rng.integers(0, 10 ** 9, n) for i in range(14, 40)})
    cols["_c0"] = rng.integers(0, 2, n).astype(np.float64)
    ds = from_arrow(pa.table(cols))
    sh = _ShardTensors(ds, [f"_c{i}" for i in range(1, 40)], [torch.float32] * 13 + [torch.long] * 26, "_c0",
                       torch.float32, torch.device("cuda"))
    assert set(sh.mats) == {"f", "i"} and sh.mats["i"].dtype == torch.int64
    sel = torch.tensor([5, 0, 2999, 17], device="cuda")
    feats, lab = sh.batch(sel)
    assert len(feats) == 39 and feats[13].dtype == torch.int64 and feats[0].dtype == torch.float32
    for j, i in enumerate(range(1, 40)):
        want = torch.as_tensor(cols[f"_c{i}"][[5, 0, 2999, 17]])
        got = feats[j].reshape(-1).cpu()
        if i < 14:
            torch.testing.assert_close(got, want.float())
        else:
            assert torch.equal(got, want.long())
    torch.testing.assert_close(lab.reshape(-1).cpu(), torch.as_tensor(cols["_c0"][[5, 0, 2999, 17]]).float())
