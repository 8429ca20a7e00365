"""NYC taxi fare regression with the Horovod API (reference: examples/horovod_nyctaxi.py).
``horovod.torch`` resolves to raydp_amd.hvd (torch.distributed: RCCL on MI355X, gloo on CPU)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

import raydp
import ray
import horovod.torch as hvd
from ray.air import session
from ray.air.config import ScalingConfig
from ray.train.horovod import HorovodTrainer

from data_process import NYC_TRAIN_CSV, nyc_taxi_preprocess
from nyc_model import NYC_Model

parser = argparse.ArgumentParser(description="Horovod NYC taxi Example")
parser.add_argument("--batch-size", type=int, default=64)
parser.add_argument("--epochs", type=int, default=5)
parser.add_argument("--num-workers", type=int, default=2)
parser.add_argument("--lr", type=float, default=0.01)
parser.add_argument("--log-interval", type=int, default=10)
args = parser.parse_args()


def process_data(num_workers):
    spark = raydp.init_spark("NYC Taxi Fare Prediction with RayDP", 1, 1, "1g")
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load(NYC_TRAIN_CSV)
    spark.conf.set("spark.sql.session.timeZone", "UTC")
    data = nyc_taxi_preprocess(data)
    ds = ray.data.from_spark(data, parallelism=num_workers)
    return ds, [f.name for f in data.schema if f.name != "fare_amount"]


def train_fn(config):
    hvd.init()
    features = config["features"]
    loader = session.get_dataset_shard("train").to_torch(
        feature_columns=features, label_column="fare_amount", label_column_dtype=torch.float,
        feature_column_dtypes=torch.float, batch_size=config["batch_size"])
    model = NYC_Model(len(features))
    optimizer = torch.optim.Adam(model.parameters(), lr=hvd.size() * config["lr"])
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(optimizer, root_rank=0)
    optimizer = hvd.DistributedOptimizer(optimizer, named_parameters=model.named_parameters(), op=hvd.Average)
    for epoch in range(1, config["epochs"] + 1):
        model.train()
        for batch_idx, (feature, target) in enumerate(loader):
            optimizer.zero_grad()
            loss = F.smooth_l1_loss(model(feature), target)
            loss.backward()
            optimizer.step()
            if batch_idx % config["log_interval"] == 0 and hvd.rank() == 0:
                print("Train Epoch: {} \tLoss: {:.6f}".format(epoch, loss.item()))
        session.report({"epoch": epoch, "loss": loss.item()})


if __name__ == "__main__":
    ray.init(address="local", num_cpus=4)
    ds, features = process_data(args.num_workers)
    trainer = HorovodTrainer(train_loop_per_worker=train_fn,
                             train_loop_config={"features": features, "batch_size": args.batch_size,
                                                "lr": args.lr, "epochs": args.epochs,
                                                "log_interval": args.log_interval},
                             scaling_config=ScalingConfig(num_workers=args.num_workers), datasets={"train": ds})
    print(trainer.fit().metrics)
    raydp.stop_spark()
    ray.shutdown()
