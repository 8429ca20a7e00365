"""DLRM on CPU: Criteo-style preprocessing on executor processes (reference notebook
examples/pytorch_dlrm.ipynb) feeding TorchEstimator training of the Dlrm model."""
import os

import torch

from raydp_amd.models import dlrm_data as D
from raydp_amd.models.dlrm import Dlrm


def test_dlrm_preprocess_and_train(spark_on_ray_2_executors, tmp_path):
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.utils import random_split
    spark = spark_on_ray_2_executors
    path = str(tmp_path / "train.txt")
    D.synthetic_criteo(path, 2000, seed=0, vocab=[5, 9, 17, 40] + [30] * 22)
    df = spark.read.schema(D.criteo_schema()).option("sep", "\t").csv(path)
    out, sizes = D.pre_process(df.cache(), frequency_limit="3", output_ordering="total_random")
    assert len(sizes) == 26 and out.count() == 2000
    pdf = out.toPandas()
    for c, s in zip(D.CAT_COLS, sizes):
        v = pdf[f"_c{c}"]
        assert v.min() >= 0 and v.max() < s
    assert pdf[[f"_c{c}" for c in D.INT_COLS]].isna().sum().sum() == 0
    train_df, test_df = random_split(out, [0.9, 0.1], 0)
    model = Dlrm(len(D.INT_COLS), sizes, [64, 32], [64, 32, 1], 32)
    feats = [f"_c{i}" for i in range(1, 40)]
    est = TorchEstimator(num_workers=1, model=model, optimizer=torch.optim.SGD(model.parameters(), lr=0.01),
                         loss=torch.nn.BCEWithLogitsLoss(), feature_columns=feats,
                         feature_types=[torch.float32] * 13 + [torch.long] * 26, label_column="_c0",
                         label_type=torch.float, batch_size=128, num_epochs=2, use_gpu=False)
    est.fit_on_spark(train_df, test_df)
    hist = [h for h in est.results.metrics_history if "train_loss" in h]
    assert len(hist) == 2 and all(h["train_loss"] == h["train_loss"] for h in hist)
    m = est.get_model()
    assert m(torch.randn(4, 13), torch.zeros(4, 26, dtype=torch.long)).shape == (4, 1)


_ = os
