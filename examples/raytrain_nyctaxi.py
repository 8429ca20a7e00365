"""NYC taxi fare regression with a hand-written training loop on the worker group
(reference: examples/raytrain_nyctaxi.py -- Ray Train 1.x Trainer API). ETL runs on the
executor processes, the converted Dataset is split 90/10 and sharded over the workers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn as nn

import raydp
import ray
from ray import train
from ray.train import Trainer, TrainingCallback, get_dataset_shard

from data_process import NYC_TRAIN_CSV, nyc_taxi_preprocess
from nyc_model import NYC_Model

EPOCHS = int(os.environ.get("NYC_EPOCHS", "10"))
ray.init(address="local", num_cpus=6)
spark = raydp.init_spark("NYC Taxi Fare Prediction with RayDP", 2, 1, "500M")
data = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load(NYC_TRAIN_CSV)
spark.conf.set("spark.sql.session.timeZone", "UTC")
data = nyc_taxi_preprocess(data)
dataset = ray.data.from_spark(data)
train_dataset, test_dataset = dataset.split_at_indices([int(dataset.count() * 0.9)])
features = [f.name for f in data.schema if f.name != "fare_amount"]


class PrintingCallback(TrainingCallback):
    def handle_result(self, results, **info):
        print(results)


def run_epoch(loader, model, criterion, optimizer=None):
    model.train(optimizer is not None)
    total, sq, n, b = 0.0, 0.0, 0, 0
    with torch.set_grad_enabled(optimizer is not None):
        for b, (inputs, targets) in enumerate(loader):
            outputs = model(*[inputs[:, i].unsqueeze(1) for i in range(inputs.size(1))])
            loss = criterion(outputs, targets)
            total += loss.item()
            sq += ((outputs - targets) ** 2).sum().item()
            n += targets.size(0)
            if optimizer is not None:
                optimizer.zero_grad()
                loss.backward()
                optimizer.step()
    return sq / max(n, 1), total / (b + 1)


def train_func(config):
    kw = dict(feature_columns=features, label_column="fare_amount", label_column_dtype=torch.float,
              feature_column_dtypes=torch.float, batch_size=config["batch_size"])
    train_loader = get_dataset_shard("train").to_torch(**kw)
    test_loader = get_dataset_shard("test").to_torch(**kw)
    model = train.torch.prepare_model(NYC_Model(len(features)))
    criterion = nn.SmoothL1Loss()
    optimizer = torch.optim.Adam(model.parameters(), lr=config["lr"])
    for epoch in range(config["num_epochs"]):
        train_mse, train_loss = run_epoch(train_loader, model, criterion, optimizer)
        test_mse, test_loss = run_epoch(test_loader, model, criterion)
        train.report({"epoch": epoch, "train_loss": train_loss, "test_loss": test_loss, "test_mse": test_mse})


trainer = Trainer(backend="torch", num_workers=2)
trainer.start()
results = trainer.run(train_func, config={"num_epochs": EPOCHS, "lr": 0.001, "batch_size": 64},
                      callbacks=[PrintingCallback()], dataset={"train": train_dataset, "test": test_dataset})
trainer.shutdown()
print("final", results)
raydp.stop_spark()
ray.shutdown()
