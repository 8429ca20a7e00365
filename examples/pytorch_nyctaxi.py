"""NYC taxi fare regression with TorchEstimator (reference: examples/pytorch_nyctaxi.py).

Runs unchanged-in-spirit on raydp-amd: Spark-style ETL on the Arrow engine, conversion to a
Dataset, and training on the MI355X (fused HIP MLP trainer) or CPU.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn
import torch.nn.functional as F

import raydp
import ray
from raydp.torch import TorchEstimator
from raydp.utils import random_split

from data_process import NYC_TRAIN_CSV, nyc_taxi_preprocess

ray.init(address="local", num_cpus=4)
spark = raydp.init_spark("NYC Taxi Fare Prediction with RayDP", 1, 1, "500M")
data = spark.read.format("csv").option("header", "true").option("inferSchema", "true") \
    .load(NYC_TRAIN_CSV)
spark.conf.set("spark.sql.session.timeZone", "UTC")
data = nyc_taxi_preprocess(data)
train_df, test_df = random_split(data, [0.9, 0.1], 0)
features = [field.name for field in list(train_df.schema) if field.name != "fare_amount"]


class NYC_Model(nn.Module):
    def __init__(self, cols):
        super().__init__()
        self.fc1 = nn.Linear(cols, 256)
        self.fc2 = nn.Linear(256, 128)
        self.fc3 = nn.Linear(128, 64)
        self.fc4 = nn.Linear(64, 16)
        self.fc5 = nn.Linear(16, 1)
        self.bn1 = nn.BatchNorm1d(256)
        self.bn2 = nn.BatchNorm1d(128)
        self.bn3 = nn.BatchNorm1d(64)
        self.bn4 = nn.BatchNorm1d(16)

    def forward(self, x):
        x = F.relu(self.fc1(x))
        x = self.bn1(x)
        x = F.relu(self.fc2(x))
        x = self.bn2(x)
        x = F.relu(self.fc3(x))
        x = self.bn3(x)
        x = F.relu(self.fc4(x))
        x = self.bn4(x)
        x = self.fc5(x)
        return x


nyc_model = NYC_Model(len(features))
criterion = nn.SmoothL1Loss()
optimizer = torch.optim.Adam(nyc_model.parameters(), lr=0.001)
estimator = TorchEstimator(num_workers=1, model=nyc_model, optimizer=optimizer, loss=criterion,
                           feature_columns=features, feature_types=torch.float,
                           label_column="fare_amount", label_type=torch.float,
                           batch_size=64, num_epochs=int(os.environ.get("NYC_EPOCHS", "30")),
                           metrics_name=["MeanAbsoluteError", "MeanSquaredError"],
                           use_ccl=False)
estimator.fit_on_spark(train_df, test_df)
for m in estimator.results.metrics_history[-2:]:
    print(m)
model = estimator.get_model()
raydp.stop_spark()
ray.shutdown()
