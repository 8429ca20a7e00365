"""Stroke prediction (reference: tutorials/pytorch_example.ipynb): Spark-style cleaning with
UDFs, 80/20 split, positive-class oversampling, TorchEstimator training of NET_Model (small
categorical embeddings + BatchNorm MLP). Shared by tutorials/pytorch_example.py and
benchmarks/stroke_bench.py."""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dataset", "healthcare-dataset-stroke-data.csv")


def data_preprocess(data):
    from pyspark.sql.functions import avg, col, udf
    data = data.drop("id")
    bmi_avg = data.filter(col("bmi") != "N/A").agg(avg(col("bmi").cast("double"))).head()[0]

    @udf("float")
    def fix_bmi(value):
        return float(bmi_avg) if value == "N/A" else float(value)
    data = data.withColumn("bmi", fix_bmi(col("bmi")))
    data = data.filter(data.gender != "Other")
    codes = {"gender": {"Female": 0, "Male": 1}, "ever_married": {"No": 0, "Yes": 1},
             "work_type": {"children": 0, "Govt_job": 1, "Never_worked": 2, "Private": 3, "Self-employed": 4},
             "Residence_type": {"Rural": 0, "Urban": 1},
             "smoking_status": {"formerly smoked": 0, "never smoked": 1, "smokes": 2, "Unknown": 3}}
    for name, table in codes.items():
        data = data.withColumn(name, udf(lambda v, t=table: int(t[v]), "int")(col(name)))

    @udf("int")
    def age_bucket(value):
        for k, hi in enumerate((26, 36, 46, 56)):
            if value >= (18 if k == 0 else (26, 36, 46)[k - 1]) and value < hi:
                return k
        return 4
    return data.withColumn("age_dis", age_bucket(col("age")))


class NET_Model(nn.Module):
    def __init__(self, cols):
        super().__init__()
        self.embs = nn.ModuleList([nn.Embedding(k, 1) for k in (2, 2, 2, 2, 5, 2, 4, 5)])
        self.sparse_idx = [0, 2, 3, 4, 5, 6, 9, 10]
        self.fc1, self.fc2, self.fc3 = nn.Linear(cols, 256), nn.Linear(256, 128), nn.Linear(128, 64)
        self.fc4, self.fc5 = nn.Linear(64, 16), nn.Linear(16, 1)
        self.bn1, self.bn2, self.bn3, self.bn4 = (nn.BatchNorm1d(256), nn.BatchNorm1d(128), nn.BatchNorm1d(64),
                                                  nn.BatchNorm1d(16))

    def forward(self, *x):
        x = torch.cat(x, dim=1)
        parts = [x[:, [1, 7, 8]]] + [e(x[:, i].long()) for e, i in zip(self.embs, self.sparse_idx)]
        x = torch.cat(parts, dim=1)
        x = self.bn1(F.relu(self.fc1(x)))
        x = self.bn2(F.relu(self.fc2(x)))
        x = self.bn3(F.relu(self.fc3(x)))
        x = self.bn4(F.relu(self.fc4(x)))
        return self.fc5(x)


def prepare(spark):
    from raydp.utils import random_split
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load(DATA)
    data = data_preprocess(data)
    train_df, test_df = random_split(data, [0.8, 0.2], 0)
    neg = train_df.filter(train_df.stroke == 1)
    for _ in range(3):
        train_df = train_df.unionByName(neg)
    features = [f.name for f in train_df.schema if f.name != "stroke"]
    return train_df, test_df, features


def make_estimator(features, epochs=10, workers=1, **kw):
    from raydp.torch import TorchEstimator
    model = NET_Model(len(features))
    return TorchEstimator(num_workers=workers, model=model, optimizer=torch.optim.Adam(model.parameters(), lr=0.001),
                          loss=nn.SmoothL1Loss(), feature_columns=features,
                          feature_types=[torch.float] * len(features), label_column="stroke",
                          label_type=torch.float, batch_size=64, num_epochs=epochs, metrics_name=["Accuracy"],
                          metrics_config={"Accuracy": {"task": "binary"}}, **kw)
