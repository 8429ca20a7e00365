"""GBDT (XGBoostEstimator engine) boosting throughput on one GPU: HIP histogram kernel vs the
``index_add_`` histogram, same booster code otherwise.

Synthetic HIGGS-shaped data (n rows x 28 fp32 features, 5% missing), ``reg:squarederror`` /
``binary:logistic``, XGBoost defaults (max_depth 6, 256 bins, eta 0.3). A "step" is one boosting
round; the timed region holds ONLY boosting rounds: quantile cuts and the bin matrix are built once
(timed separately as ``setup_s``) and kept on the DMatrix, and the first ``--warmup`` rounds are
trained and discarded before the timed run. Prints one JSON line per path.

    python benchmarks/gbdt_bench.py --rows 1000000 --rounds 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from raydp_amd.ops import gbdt_ops  # noqa: E402
from raydp_amd.xgboost import gbdt  # noqa: E402


def data(n, F, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, F)).astype(np.float32)
    w = rng.normal(size=F).astype(np.float32)
    logit = x @ w * 0.3 + np.sin(x[:, 0] * 2) - np.abs(x[:, 1])
    y = (logit + rng.logistic(size=n) > 0).astype(np.float32)
    x[rng.random((n, F)) < 0.05] = np.nan
    return x, y


def run(params, dm, rounds, warmup):
    gbdt.train(params, dm, max(1, warmup), device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    bst = gbdt.train(params, dm, rounds, device="cuda")
    torch.cuda.synchronize()
    return time.perf_counter() - t, bst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--paths", default="hip,torch")
    a = ap.parse_args()
    x, y = data(a.rows, a.features)
    dm = gbdt.DMatrix(x, y)
    params = {"objective": "binary:logistic", "max_depth": a.depth, "max_bin": 256, "eta": 0.3}
    hip_hist = gbdt_ops.level_histogram
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gbdt._binned(dm, gbdt.normalize_params(params), gbdt.World(), torch.device("cuda"))
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    preds = {}
    for path in a.paths.split(","):
        if path == "torch":
            gbdt_ops.level_histogram = lambda bt, pos, g, h, K, B: gbdt_ops.torch_level_histogram(bt.t(), pos, g, h, K, B)
        else:
            gbdt_ops.level_histogram = hip_hist
        dt, bst = run(params, dm, a.rounds, a.warmup)
        gbdt_ops.level_histogram = hip_hist
        preds[path] = np.asarray(bst.predict(gbdt.DMatrix(x[:10000])))
        print(json.dumps({"metric": "GBDT boosting rounds/s", "path": path, "value": round(a.rounds / dt, 3),
                          "unit": "rounds/s", "ms_per_round": round(dt / a.rounds * 1e3, 2),
                          "rows_x_rounds_per_s": round(a.rows * a.rounds / dt), "rows": a.rows,
                          "features": a.features, "max_depth": a.depth, "max_bin": 256,
                          "objective": params["objective"], "data": "synthetic HIGGS-shaped", "n_gpus": 1,
                          "setup_s": round(setup_s, 4),
                          "timed_region": "boosting rounds only (cuts + binning done once, setup_s)"}),
              flush=True)
    if len(preds) == 2:
        v = list(preds.values())
        print(json.dumps({"max_abs_pred_diff_hip_vs_torch": float(np.abs(v[0] - v[1]).max())}), flush=True)


if __name__ == "__main__":
    main()
