"""gfx950 GBDT kernels (csrc/hip/gbdt_hist.hip): the histogram build against the fp64
``index_add_`` reference, and whole-booster parity (histograms + per-(node, feature) split
search on the GPU vs the tensor formulation on the CPU) over several parameter sets."""
import numpy as np
import pytest
import torch

from raydp_amd.ops.gbdt_ops import (level_histogram, partition_rows_, quant_scale, quantise, split_candidates,
                                    torch_level_histogram, torch_split_candidates)
from raydp_amd.xgboost import gbdt

pytestmark = pytest.mark.gpu


def _operands(n, F, B, K, seed=0, inactive=0.2):
    g = torch.Generator().manual_seed(seed)
    bins = torch.randint(0, B, (n, F), generator=g, dtype=torch.int16)
    pos = torch.randint(0, K, (n,), generator=g)
    pos[torch.rand(n, generator=g) < inactive] = -1
    gr = torch.randn(n, generator=g)
    hs = torch.rand(n, generator=g) + 0.1
    gq = quantise(gr, quant_scale(float(gr.abs().max())))
    hq = quantise(hs, quant_scale(float(hs.abs().max())))
    return bins, pos, gq, hq


@pytest.mark.parametrize("n,F,B,K", [(1, 1, 2, 1), (5000, 7, 258, 1), (100_003, 20, 258, 8), (70_000, 3, 66, 40),
                                     (20_000, 4, 3000, 5), (300_000, 28, 130, 32),
                                     (30_000, 2, 5000, 3), (10_000, 1, 32768, 2)])
def test_level_histogram_matches_index_add_exactly(n, F, B, K):
    """Fixed-point sums are exact: the kernel equals index_add_ bit for bit, including the
    global-atomic mode used when one node's bins exceed the LDS slice (B >= 4097)."""
    bins, pos, gq, hq = _operands(n, F, B, K)
    ref = torch_level_histogram(bins, pos, gq, hq, K, B)
    d = torch.device("cuda")
    out = level_histogram(bins.t().contiguous().to(d), pos.to(d), gq.to(d), hq.to(d), K, B)
    assert out.shape == ref.shape and out.dtype == torch.int64
    assert torch.equal(out.cpu(), ref)


def test_level_histogram_run_to_run_identical():
    bins, pos, gq, hq = _operands(400_000, 8, 258, 16, seed=3)
    d = torch.device("cuda")
    args = (bins.t().contiguous().to(d), pos.to(d), gq.to(d), hq.to(d), 16, 258)
    first = level_histogram(*args)
    for _ in range(3):
        assert torch.equal(level_histogram(*args), first)


def test_level_histogram_rejects_bins_beyond_int16():
    d = torch.device("cuda")
    bins_t = torch.zeros(1, 10, dtype=torch.int16, device=d)
    z = torch.zeros(10, dtype=torch.int32, device=d)
    with pytest.raises(ValueError):
        level_histogram(bins_t, torch.zeros(10, dtype=torch.long, device=d), z, z, 1, 40000)


def _split_operands(K, F, B, seed, empty_frac=0.0, zero_h=False):
    g = torch.Generator().manual_seed(seed)
    hist = torch.zeros(K, F, B, 2, dtype=torch.int64)
    hist[..., 0] = torch.randint(-(1 << 26), 1 << 26, (K, F, B), generator=g)
    hist[..., 1] = torch.randint(0, 1 << 26, (K, F, B), generator=g)
    if empty_frac:
        hist[torch.rand(K, F, B, generator=g) < empty_frac] = 0
    if zero_h:
        hist[..., 1] = 0
        hist[:, :, ::7, 1] = 1 << 20
    # every feature sees the same rows: make the per-node totals consistent across features
    tot = hist[:, 0].sum(1)
    for f in range(1, F):
        diff = tot - hist[:, f].sum(1)
        hist[:, f, B - 1] += diff
    return hist, tot


@pytest.mark.parametrize("K,F,B,empty,params", [
    (4, 6, 258, 0.0, (1.0, 0.0, 1.0)),
    (3, 5, 130, 0.9, (1.0, 0.0, 0.0)),           # many empty bins across 64-lane run boundaries
    (2, 4, 67, 0.5, (0.3, 0.5, 20.0)),
    (5, 3, 2, 0.0, (1.0, 0.0, 1.0)),             # a single threshold
    (2, 3, 300, 0.7, (0.0, 0.0, 0.0)),           # lambda = 0, min_child_weight = 0: no NaN gains
])
def test_split_kernel_matches_tensor_formulation(K, F, B, empty, params):
    lam, alpha, mcw = params
    hist, tot = _split_operands(K, F, B, seed=K * 100 + B, empty_frac=empty, zero_h=(lam == 0.0))
    g = torch.Generator().manual_seed(B)
    ncuts = torch.randint(0, B - 1, (F,), generator=g, dtype=torch.int32)
    ncuts[0] = B - 2
    fmask = (torch.rand(F, generator=g) < 0.7).to(torch.uint8)
    fmask[0] = 1
    inv_g, inv_h = 2.0 ** -24, 2.0 ** -26
    for fm in (None, fmask, torch.zeros(F, dtype=torch.uint8)):
        ref = torch_split_candidates(hist, tot, ncuts, fm, inv_g, inv_h, lam, alpha, mcw)
        out = split_candidates(hist.cuda(), tot.cuda(), ncuts, fm, inv_g, inv_h, lam, alpha, mcw).cpu()
        assert not torch.isnan(out).any()
        assert torch.equal(out, ref), (out - ref).abs().max()


def test_partition_kernel_matches_tensor_expression():
    g = torch.Generator().manual_seed(7)
    n, F, K = 50_000, 5, 6
    bins = torch.randint(0, 40, (n, F), generator=g, dtype=torch.int16)
    pos = torch.randint(-1, K + 2, (n,), generator=g)          # -1 inactive, >= K out of range
    leaf = torch.full((n,), 99, dtype=torch.long)
    remap = torch.tensor([0, -1, 2, -1, 4, 6])
    table = torch.stack([remap, torch.tensor([0, 1, 4, 2, 3, 1]), torch.tensor([5, 0, 39, 10, 1, 20]),
                         torch.tensor([1, 0, 0, 1, 1, 0]), torch.arange(K) + 10], 1)
    d = torch.device("cuda")
    bt, pd, ld = bins.t().contiguous().to(d), pos.to(d).clone(), leaf.to(d).clone()
    partition_rows_(bt, table, pd, ld)
    # tensor expression
    inr = (pos >= 0) & (pos < K)
    cur = pos.clamp(0, K - 1)
    t = table[cur]
    b = bins.long().gather(1, t[:, 1:2])[:, 0]
    left = torch.where(b == 0, t[:, 3] != 0, b <= t[:, 2])
    to_leaf = inr & (t[:, 0] < 0)
    exp_pos = torch.where(inr, torch.where(to_leaf, torch.full_like(pos, -1), t[:, 0] + (~left).long()), pos)
    exp_leaf = torch.where(to_leaf, t[:, 4], leaf)
    assert torch.equal(pd.cpu(), exp_pos)
    assert torch.equal(ld.cpu(), exp_leaf)


def _data(n=20_000, F=10, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, F)).astype(np.float32)
    x[rng.random((n, F)) < 0.05] = np.nan
    y = (np.nan_to_num(x[:, 0]) * 2 - np.nan_to_num(x[:, 1]) ** 2 + 0.5 * np.nan_to_num(x[:, 2] > 0)
         + 0.1 * rng.normal(size=n)).astype(np.float32)
    return x, y


def _assert_same_trees(a, b, exact_gain=True):
    assert len(a.trees) == len(b.trees)
    for ra, rb in zip(a.trees, b.trees):
        assert len(ra) == len(rb)
        for ta, tb in zip(ra, rb):
            assert ta.feature == tb.feature
            assert ta.default_left == tb.default_left
            assert ta.cond == tb.cond
            if exact_gain:
                assert ta.gain == tb.gain
            else:
                np.testing.assert_allclose(ta.gain, tb.gain, rtol=1e-4, atol=1e-6)
            np.testing.assert_allclose(ta.value, tb.value, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("extra", [{}, {"alpha": 0.5, "min_child_weight": 20.0, "lambda": 0.3},
                                   {"colsample_bytree": 0.6, "max_bin": 256, "gamma": 0.1},
                                   {"objective": "binary:logistic"},
                                   {"subsample": 0.5, "lambda": 0.0, "min_child_weight": 0.0},
                                   {"objective": "multi:softprob", "num_class": 3, "max_depth": 4},
                                   {"max_depth": 8, "weights": True}])
def test_booster_gpu_matches_cpu(extra):
    """Same trees on both devices: features, thresholds, default directions and gains exactly."""
    extra = dict(extra)
    weights = extra.pop("weights", False)
    x, y = _data()
    params = {"objective": "reg:squarederror", "max_depth": 5, "eta": 0.3, "max_bin": 64, **extra}
    if params["objective"] == "binary:logistic":
        y = (y > 0).astype(np.float32)
    if params["objective"].startswith("multi:"):
        y = np.digitize(y, [-1.0, 1.0]).astype(np.float32)
    w = np.random.default_rng(5).uniform(0.2, 3.0, len(y)).astype(np.float32) if weights else None
    cpu = gbdt.train(params, gbdt.DMatrix(x, y, weight=w), 8, device="cpu")
    gpu = gbdt.train(params, gbdt.DMatrix(x, y, weight=w), 8, device="cuda")
    # squared error: g = margin - y is the same fp32 value on both devices, so the fixed-point
    # histograms and every gain are identical; sigmoid/softmax gradients may differ by an ulp
    # between the CPU and GPU math libraries, which the 2^-30 quantum can see
    _assert_same_trees(cpu, gpu, exact_gain=params["objective"] == "reg:squarederror")
    for t in gpu.trees:
        assert not any(np.isnan(v) for v in t[0].value)
    pc = cpu.predict(gbdt.DMatrix(x))
    pg = gpu.predict(gbdt.DMatrix(x))
    np.testing.assert_allclose(np.asarray(pg), np.asarray(pc), rtol=1e-5, atol=1e-5)


def test_booster_gpu_run_to_run_identical():
    x, y = _data(n=200_000, F=12, seed=4)
    params = {"objective": "reg:squarederror", "max_depth": 6, "eta": 0.3, "max_bin": 256}
    dm = gbdt.DMatrix(x, y)
    a = gbdt.train(params, dm, 5, device="cuda")
    b = gbdt.train(params, dm, 5, device="cuda")
    _assert_same_trees(a, b)
    for ra, rb in zip(a.trees, b.trees):
        assert ra[0].value == rb[0].value


def test_xgboost_estimator_trains_on_gpu():
    import raydp_amd
    from raydp_amd import runtime
    from raydp_amd.spark.functions import rand
    from raydp_amd.utils import random_split
    from raydp_amd.xgboost import XGBoostEstimator
    runtime.shutdown()
    runtime.init(num_cpus=4, num_gpus=1)
    try:
        spark = raydp_amd.init_spark("gpu-xgb", 1, 2, "500M")
        df = spark.range(0, 20000)
        df = df.withColumn("x", rand() * 100)
        df = df.withColumn("y", rand() * 1000)
        df = df.withColumn("z", df.x * 3 + df.y * 4 + rand() + 5)
        train_df, test_df = random_split(df.select(df.x, df.y, df.z), [0.7, 0.3])
        est = XGBoostEstimator({"max_depth": 8, "eta": 0.3, "num_boost_round": 30}, "z",
                               resources_per_worker={"CPU": 1, "GPU": 1})
        est.fit_on_spark(train_df, test_df)
        hist = est.results.metrics_history
        assert hist[-1]["device"] == "cuda"
        assert hist[-1]["evaluate-rmse"] < 0.1 * hist[0]["evaluate-rmse"]
        pred = est.get_model().inplace_predict(np.asarray([[50, 500]]))
        assert abs(pred[0] - (150 + 2000 + 5.5)) < 0.05 * 2155
    finally:
        raydp_amd.stop_spark()
        runtime.shutdown()
