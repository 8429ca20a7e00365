"""gfx950 GBDT kernels (csrc/hip/gbdt_hist.hip): the histogram build against the fp64
``index_add_`` reference, and whole-booster parity (histograms + per-(node, feature) split
search on the GPU vs the tensor formulation on the CPU) over several parameter sets."""
import numpy as np
import pytest
import torch

from raydp_amd.ops.gbdt_ops import level_histogram, torch_level_histogram
from raydp_amd.xgboost import gbdt

pytestmark = pytest.mark.gpu


def _operands(n, F, B, K, seed=0, inactive=0.2):
    g = torch.Generator().manual_seed(seed)
    bins = torch.randint(0, B, (n, F), generator=g, dtype=torch.int16)
    pos = torch.randint(0, K, (n,), generator=g)
    pos[torch.rand(n, generator=g) < inactive] = -1
    gr = torch.randn(n, generator=g)
    hs = torch.rand(n, generator=g) + 0.1
    return bins, pos, gr, hs


@pytest.mark.parametrize("n,F,B,K", [(1, 1, 2, 1), (5000, 7, 258, 1), (100_003, 20, 258, 8), (70_000, 3, 66, 40),
                                     (20_000, 4, 3000, 5), (300_000, 28, 130, 32)])
def test_level_histogram_matches_index_add(n, F, B, K):
    bins, pos, gr, hs = _operands(n, F, B, K)
    ref = torch_level_histogram(bins, pos, gr, hs, K, B)
    d = torch.device("cuda")
    out = level_histogram(bins.t().contiguous().to(d), pos.to(d), gr.to(d), hs.to(d), K, B)
    assert out.shape == ref.shape and out.dtype == torch.float64
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-12, atol=1e-9)


def test_level_histogram_rejects_oversized_bins():
    d = torch.device("cuda")
    bins_t = torch.zeros(1, 10, dtype=torch.int16, device=d)
    z = torch.zeros(10, device=d)
    with pytest.raises(ValueError):
        level_histogram(bins_t, torch.zeros(10, dtype=torch.long, device=d), z, z, 1, 5000)


def _data(n=20_000, F=10, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, F)).astype(np.float32)
    x[rng.random((n, F)) < 0.05] = np.nan
    y = (np.nan_to_num(x[:, 0]) * 2 - np.nan_to_num(x[:, 1]) ** 2 + 0.5 * np.nan_to_num(x[:, 2] > 0)
         + 0.1 * rng.normal(size=n)).astype(np.float32)
    return x, y


@pytest.mark.parametrize("extra", [{}, {"alpha": 0.5, "min_child_weight": 20.0, "lambda": 0.3},
                                   {"colsample_bytree": 0.6, "max_bin": 256, "gamma": 0.1},
                                   {"objective": "binary:logistic"}])
def test_booster_gpu_matches_cpu(extra):
    x, y = _data()
    params = {"objective": "reg:squarederror", "max_depth": 5, "eta": 0.3, "max_bin": 64, **extra}
    if params["objective"] == "binary:logistic":
        y = (y > 0).astype(np.float32)
    cpu = gbdt.train(params, gbdt.DMatrix(x, y), 8, device="cpu")
    gpu = gbdt.train(params, gbdt.DMatrix(x, y), 8, device="cuda")
    for tc, tg in zip(cpu.trees, gpu.trees):
        assert tc[0].feature == tg[0].feature
        np.testing.assert_allclose(tc[0].cond, tg[0].cond, rtol=0, atol=0)
        np.testing.assert_allclose(tc[0].value, tg[0].value, rtol=1e-6, atol=1e-7)
    pc = cpu.predict(gbdt.DMatrix(x))
    pg = gpu.predict(gbdt.DMatrix(x))
    np.testing.assert_allclose(np.asarray(pg), np.asarray(pc), rtol=1e-5, atol=1e-5)


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
