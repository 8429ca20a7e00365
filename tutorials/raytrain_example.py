"""Stroke prediction with a raw Ray Train loop (reference: tutorials/raytrain_example.ipynb,
cells 28-42): Spark-style cleaning, 80/20 split, positive oversampling (2 extra copies),
``ray.data.from_spark``, then the Ray Train 1.x ``Trainer(backend="torch")`` running a
hand-written ``train_func`` over ``to_torch`` shards with ``prepare_model``, weighted
CrossEntropy and Adam, ``train.report`` per epoch.

Runs unchanged-in-spirit on raydp-amd: ``ray`` / ``ray.train`` are this framework's facades
(``raydp_amd.compat``), the Trainer is :class:`raydp_amd.train.legacy.Trainer`.
``RAYTRAIN_DEVICE=cuda`` moves the model and each batch to the GPU (the notebook is CPU-only).
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import torch
import torch.nn as nn

import raydp
import ray
from stroke import DATA, data_preprocess

DEVICE = os.environ.get("RAYTRAIN_DEVICE", "cpu")


class NET_Model(nn.Module):
    """The notebook's model (cell 32): one embedding per categorical column (dims 2, 2, 2, 2, 5,
    2, 4, 5), a dense branch on 3 numeric columns, concatenated into a 2-way classifier (the
    notebook's forward returns before its BN-MLP tail; the tail's layers exist but are unused)."""

    def __init__(self, cols):
        super().__init__()
        self.emb_layer_gender = nn.Embedding(2, 2)
        self.emb_layer_hypertension = nn.Embedding(2, 2)
        self.emb_layer_heart_disease = nn.Embedding(2, 2)
        self.emb_layer_ever_married = nn.Embedding(2, 2)
        self.emb_layer_work = nn.Embedding(5, 5)
        self.emb_layer_residence = nn.Embedding(2, 2)
        self.emb_layer_smoking_status = nn.Embedding(4, 4)
        self.emb_layer_age = nn.Embedding(5, 5)
        self.fc1, self.fc2, self.fc3 = nn.Linear(cols, 256), nn.Linear(256, 128), nn.Linear(128, 64)
        self.fc4, self.fc5 = nn.Linear(64, 16), nn.Linear(16, 2)
        self.fc_sparse = nn.Linear(24, 16)
        self.fc_dense = nn.Linear(3, 8)
        self.fc = nn.Linear(24, 2)
        self.bn1, self.bn2, self.bn3, self.bn4 = (nn.BatchNorm1d(256), nn.BatchNorm1d(128), nn.BatchNorm1d(64),
                                                  nn.BatchNorm1d(16))

    def forward(self, *x):
        x = torch.cat(x, dim=1)
        dense_columns = x[:, [1, 7, 8]]
        sparse = [self.emb_layer_gender(x[:, 0].long()), self.emb_layer_hypertension(x[:, 2].long()),
                  self.emb_layer_heart_disease(x[:, 3].long()), self.emb_layer_ever_married(x[:, 4].long()),
                  self.emb_layer_work(x[:, 5].long()), self.emb_layer_residence(x[:, 6].long()),
                  self.emb_layer_smoking_status(x[:, 9].long()), self.emb_layer_age(x[:, 10].long())]
        sparse_columns = torch.cat(sparse, dim=1)
        dense_feat = self.fc_dense(dense_columns)
        sparse_feat = self.fc_sparse(sparse_columns)
        return self.fc(torch.cat([dense_feat, sparse_feat], dim=1))


def train_epoch(dataset, model, criterion, optimizer):
    model.train()
    train_loss, correct, data_size, batch_idx = 0, 0, 0, 0
    for batch_idx, (inputs, targets) in enumerate(dataset):
        inputs, targets = inputs.to(DEVICE), targets.to(DEVICE)
        inputs = [inputs[:, i].unsqueeze(1) for i in range(inputs.size(1))]
        targets = targets.reshape(-1)
        outputs = model(*inputs)
        loss = criterion(outputs, targets)
        train_loss += loss.item()
        _, predicted = torch.max(outputs.data, 1)
        data_size += targets.size(0)
        correct += (predicted == targets).sum().item()
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
    return correct / max(data_size, 1), train_loss / (batch_idx + 1)


def test_epoch(dataset, model, criterion):
    model.eval()
    test_loss, correct, data_size, batch_idx = 0, 0, 0, 0
    with torch.no_grad():
        for batch_idx, (inputs, targets) in enumerate(dataset):
            inputs, targets = inputs.to(DEVICE), targets.to(DEVICE)
            inputs = [inputs[:, i].unsqueeze(1) for i in range(inputs.size(1))]
            targets = targets.reshape(-1)
            outputs = model(*inputs)
            test_loss += criterion(outputs, targets).item()
            _, predicted = torch.max(outputs.data, 1)
            data_size += targets.size(0)
            correct += (predicted == targets).sum().item()
    return correct / max(data_size, 1), test_loss / (batch_idx + 1)


def make_train_func(features):
    feature_dtype = [torch.float] * len(features)

    def train_func(config):
        from ray import train
        from ray.train import get_dataset_shard
        bs = config["batch_size"]
        # device=DEVICE: on a GPU the shard is ingested into HBM once and batches are slices of it
        train_ds = get_dataset_shard("train").to_torch(feature_columns=features, label_column="stroke",
                                                       label_column_dtype=torch.long,
                                                       feature_column_dtypes=feature_dtype, batch_size=bs,
                                                       device=DEVICE)
        test_ds = get_dataset_shard("test").to_torch(feature_columns=features, label_column="stroke",
                                                     label_column_dtype=torch.long,
                                                     feature_column_dtypes=feature_dtype, batch_size=bs,
                                                     device=DEVICE)
        model = NET_Model(len(features))
        model = train.torch.prepare_model(model).to(DEVICE)
        criterion = nn.CrossEntropyLoss(weight=torch.tensor([0.35, 0.65], device=DEVICE))
        optimizer = torch.optim.Adam(model.parameters(), lr=config["lr"])
        for epoch in range(config["num_epochs"]):
            t0 = time.perf_counter()
            train_acc, train_loss = train_epoch(train_ds, model, criterion, optimizer)
            test_acc, test_loss = test_epoch(test_ds, model, criterion)
            train.report(dict(epoch=epoch, train_acc=train_acc, train_loss=train_loss, test_acc=test_acc,
                              test_loss=test_loss, epoch_s=time.perf_counter() - t0))
    return train_func


def prepare(spark, num_executors):
    from raydp.utils import random_split
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load(DATA)
    data = data_preprocess(data)
    train_df, test_df = random_split(data, [0.8, 0.2], 0)
    neg = train_df.filter(train_df.stroke == 1)
    train_df = train_df.unionByName(neg).unionByName(neg)
    features = [f.name for f in train_df.schema if f.name != "stroke"]
    train_ds = ray.data.from_spark(train_df, parallelism=num_executors)
    test_ds = ray.data.from_spark(test_df, parallelism=num_executors)
    return train_ds, test_ds, features


def run(num_executors=1, num_epochs=10, callbacks=None):
    from ray.train import Trainer
    spark = raydp.init_spark("Stroke Prediction (Ray Train)", num_executors, 1, "500M")
    train_ds, test_ds, features = prepare(spark, num_executors)
    # (the notebook runs on CPU; on a GPU the workers are GPU workers, as Ray Train's use_gpu)
    trainer = Trainer(backend="torch", num_workers=num_executors, use_gpu=DEVICE == "cuda")
    trainer.start()
    results = trainer.run(make_train_func(features), config={"num_epochs": num_epochs, "lr": 0.001, "batch_size": 64},
                          callbacks=callbacks or [], dataset={"train": train_ds, "test": test_ds})
    trainer.shutdown()
    raydp.stop_spark()
    return results, train_ds.count(), test_ds.count()


if __name__ == "__main__":
    from ray.train import TrainingCallback

    class PrintingCallback(TrainingCallback):
        def handle_result(self, results, **info):
            print(results)

    ray.init(num_cpus=4)
    run(1, int(os.environ.get("RAYTRAIN_EPOCHS", "10")), [PrintingCallback()])
    ray.shutdown()
