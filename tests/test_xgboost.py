"""XGBoostEstimator (port of the reference's python/raydp/tests/test_xgboost.py) plus checks of
the native histogram GBDT it runs on. xgboost itself is not installed: parity with xgboost's
numbers is unpinned; the tests check learning quality and distributed == single-process."""
import os
import shutil

import numpy as np
import pytest

from raydp_amd.xgboost import Booster, DMatrix, XGBoostEstimator, train


@pytest.mark.parametrize("use_fs_directory", [True, False])
def test_xgb_estimator(spark_on_ray_small, use_fs_directory, tmp_path):
    from raydp_amd.spark.functions import rand
    from raydp_amd.utils import random_split
    spark = spark_on_ray_small
    df = spark.range(0, 20000)
    df = df.withColumn("x", rand() * 100)
    df = df.withColumn("y", rand() * 1000)
    df = df.withColumn("z", df.x * 3 + df.y * 4 + rand() + 5)
    df = df.select(df.x, df.y, df.z)
    train_df, test_df = random_split(df, [0.7, 0.3])
    est = XGBoostEstimator({"max_depth": 8, "eta": 0.3, "num_boost_round": 30}, "z",
                           resources_per_worker={"CPU": 1})
    if use_fs_directory:
        d = str(tmp_path / "test_xgboost")
        est.fit_on_spark(train_df, test_df, fs_directory="file://" + d)
    else:
        est.fit_on_spark(train_df, test_df)
    model = est.get_model()
    pred = model.inplace_predict(np.asarray([[1, 2], [50, 500]]))
    assert pred.shape == (2,)
    assert abs(pred[1] - (150 + 2000 + 5.5)) < 0.05 * 2155
    hist = est.results.metrics_history
    assert hist[-1]["evaluate-rmse"] < 0.1 * hist[0]["evaluate-rmse"]


def test_gbdt_objectives_and_missing_values():
    rng = np.random.default_rng(0)
    n = 8000
    x = rng.standard_normal((n, 4))
    x[rng.random((n, 4)) < 0.1] = np.nan
    y = ((np.nan_to_num(x[:, 0]) + np.nan_to_num(x[:, 1]) ** 2) > 1).astype(np.float32)
    res = {}
    bst = train({"objective": "binary:logistic", "eval_metric": ["logloss", "error"]},
                DMatrix(x[:6000], y[:6000]), 15, evals=[(DMatrix(x[6000:], y[6000:]), "t")], evals_result=res)
    assert res["t"]["error"][-1] < 0.05
    p = bst.predict(DMatrix(x[6000:]))
    assert ((p >= 0) & (p <= 1)).all()
    ym = (np.nan_to_num(x[:, 0]) > 0).astype(int) + (np.nan_to_num(x[:, 2]) > 0.5).astype(int)
    bst = train({"objective": "multi:softmax", "num_class": 3}, DMatrix(x[:6000], ym[:6000]), 10)
    assert (bst.predict(DMatrix(x[6000:])) == ym[6000:]).mean() > 0.97
    assert len(bst.get_dump()) == 30 and bst.num_boosted_rounds() == 10


def test_gbdt_save_load_roundtrip(tmp_path):
    rng = np.random.default_rng(1)
    x = rng.random((2000, 3))
    y = x @ [1.0, -2.0, 3.0]
    bst = train({"max_depth": 4}, DMatrix(x, y, feature_names=["a", "b", "c"]), 5)
    f = str(tmp_path / "m.json")
    bst.save_model(f)
    b2 = Booster(model_file=f)
    np.testing.assert_allclose(b2.inplace_predict(x), bst.inplace_predict(x), rtol=1e-6)
    assert set(b2.get_score()) <= {"a", "b", "c"}


def _dist_gbdt(rank, world, port, x, y, q):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    n = x.shape[0] // world
    bst = train({"max_depth": 5}, DMatrix(x[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]), 6)
    if rank == 0:
        q.put(bst.inplace_predict(x))
    dist.destroy_process_group()


def test_gbdt_distributed_histograms_match_single_process():
    import multiprocessing as mp
    from raydp_amd.train.trainer import _free_port
    rng = np.random.default_rng(2)
    x = rng.random((4000, 3)).astype(np.float32)
    y = (np.sin(6 * x[:, 0]) + x[:, 1] * x[:, 2]).astype(np.float32)
    single = train({"max_depth": 5}, DMatrix(x, y), 6).inplace_predict(x)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dist_gbdt, args=(r, 2, port, x, y, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(60)
    # fixed-point histograms: the all-reduced integer sums equal the single-process sums, so the
    # trees (and predictions) are identical, not merely close
    np.testing.assert_array_equal(got, single)


def test_gbdt_zero_hessian_children_do_not_make_nan():
    """lambda = 0 and min_child_weight = 0 with subsampling: children with zero hessian are
    invalid candidates (no 0/0 gains) and zero-hessian nodes get weight 0."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((3000, 4)).astype(np.float32)
    y = (x[:, 0] > 0).astype(np.float32)
    bst = train({"objective": "binary:logistic", "lambda": 0.0, "min_child_weight": 0.0, "subsample": 0.3,
                 "max_depth": 6}, DMatrix(x, y), 5)
    for (t,) in bst.trees:
        assert np.isfinite(t.value).all() and np.isfinite(t.gain).all()
    assert np.isfinite(bst.predict(DMatrix(x))).all()


def test_gbdt_max_bin_validated():
    with pytest.raises(ValueError):
        train({"max_bin": 40000}, DMatrix(np.zeros((10, 1)), np.zeros(10)), 1)


def test_split_candidates_tensor_formulation_matches_bruteforce():
    """torch_split_candidates (CPU path, and the GPU kernel's reference) against a per-threshold
    Python loop: same gains, lowest threshold on ties, -1 where nothing is valid."""
    import torch
    from raydp_amd.ops.gbdt_ops import torch_split_candidates
    g = torch.Generator().manual_seed(0)
    K, F, B = 2, 3, 12
    hist = torch.zeros(K, F, B, 2, dtype=torch.int64)
    hist[..., 0] = torch.randint(-50, 50, (K, F, B), generator=g)
    hist[..., 1] = torch.randint(0, 20, (K, F, B), generator=g)
    hist[0, 1, 3:7] = 0                                   # empty bins -> tied gains
    tot = hist[:, 0].sum(1)
    for f in range(1, F):
        hist[:, f, B - 1] += tot - hist[:, f].sum(1)
    ncuts = torch.tensor([B - 2, 5, 0])
    lam, alpha, mcw, ig, ih = 1.0, 0.0, 2.0, 0.5, 0.25
    out = torch_split_candidates(hist, tot, ncuts, None, ig, ih, lam, alpha, mcw)
    for k in range(K):
        G, H = float(tot[k, 0]) * ig, float(tot[k, 1]) * ih
        parent = G * G / (H + lam)
        for f in range(F):
            for c, dl in ((0, 1), (2, 0)):
                best, bt = -1.0, 0
                cg = ch = 0
                for t in range(B - 1):
                    cg += int(hist[k, f, t + 1, 0])
                    ch += int(hist[k, f, t + 1, 1])
                    if t >= int(ncuts[f]):
                        continue
                    lg = cg + (int(hist[k, f, 0, 0]) if dl else 0)
                    lh = ch + (int(hist[k, f, 0, 1]) if dl else 0)
                    Lg, Lh = lg * ig, lh * ih
                    Rg, Rh = (int(tot[k, 0]) - lg) * ig, (int(tot[k, 1]) - lh) * ih
                    if not (Lh >= mcw and Rh >= mcw and Lh + lam > 0 and Rh + lam > 0):
                        continue
                    gain = Lg * Lg / (Lh + lam) + Rg * Rg / (Rh + lam) - parent
                    if gain > best:
                        best, bt = gain, t
                assert float(out[k, f, c]) == best and int(out[k, f, c + 1]) == bt, (k, f, dl)


def test_tf_estimator_reports_missing_tensorflow():
    pytest.importorskip("raydp_amd.tf")
    try:
        import tensorflow  # noqa: F401
        pytest.skip("tensorflow present")
    except ImportError:
        pass
    from raydp_amd.tf import TFEstimator
    with pytest.raises(ImportError, match="TensorFlow"):
        TFEstimator(num_workers=1, model=object(), optimizer="adam", loss="mse")


_ = (os, shutil)
