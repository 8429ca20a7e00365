#!/usr/bin/env python
"""Flagship benchmark: end-to-end NYCTaxi samples/s (Spark-style ETL + conversion + training).

Metric (BASELINE.json): "end-to-end samples/sec (Spark ETL+train) NYCTaxi TorchEstimator
@1/2/4/8 GPU". One *step* = one optimizer step of the reference NYC_Model
(examples/pytorch_nyctaxi.py: 5 Linear + 4 BatchNorm1d, SmoothL1, Adam 1e-3) on a batch of 64
rows per GPU. The timed region of K steps contains EVERYTHING the reference's ``fit_on_spark``
path does for those K*64 rows per GPU: CSV read + parse, the full ``examples/data_process.py``
ETL (14 filters, 9 time features incl. 2 Python UDFs, 11 distance features incl. 8 Python-UDF
calls, 7 drops), the Spark->Dataset conversion through the shared-memory object store, the
dataset shuffle, the host->HBM ingest, K training steps (forward, backward, all-reduce across
ranks, optimizer) and the rank-0 ``model.pt`` checkpoint. Each sample passes through ETL once
(1 epoch unless ``--epochs``). Data: synthetic NYCTaxi rows with the reference generator's
distributions (examples/random_nyctaxi.py), written before timing. Weights: random init. Weak
scaling: 64 rows/step/GPU.

Launch: ``python bench.py --gpus N --steps K --warmup W``.

Topologies (``--topology``):
* ``estimator`` (default): the reference's own topology (``python/raydp/torch/estimator.py:
  331-355``): ONE driver process, ONE Spark session, ``TorchEstimator(num_workers=N,
  resources_per_worker={"GPU": 1})`` whose N worker processes (one per GPU, started by the
  worker-group trainer and kept warm between fits, as Ray's prestarted workers are) each ingest
  one equal shard of the converted dataset and train over RCCL / xGMI. Under ``torchrun
  --nproc-per-node N`` rank 0 is that driver (the launcher's rank variables are removed from its
  environment first, so the trainer starts its own group) and ranks 1..N-1 exit at once,
  before touching a GPU. The driver's wall clock spans every worker's whole fit, so it is
  already the max over ranks.
* ``spmd``: one process per GPU, each running the whole pipeline on its own rows (own Spark
  session, own executors, own CSV), training over RCCL / xGMI with its peers; the max over
  ranks of the timed region is reported. For N > 1 outside a torchrun job the script starts
  the N rank processes itself (before any GPU call).

Workloads (``--workload``, the one measured as ``value``): ``nyc`` (above); ``horovod`` (the
reference's examples/horovod_nyctaxi.py: the same ETL + conversion, then ``HorovodTrainer`` and
the user-written loop with ``hvd.DistributedOptimizer(op=Average)``, lr x size, one step = one
batch of 64 per GPU); ``dlrm`` (examples/pytorch_dlrm.ipynb: synthetic Criteo TSV -> the
notebook's preprocessing -> ``fit_on_spark`` of the DLRM, SGD 0.01, BCEWithLogits, batch 128 per
GPU, tables sharded over the workers with the all-to-all exchange when N > 1). With the ``nyc``
headline the other two run afterwards at the same N / K / W and are reported under
``config.other_workloads`` (``--extra-workloads none`` skips them), so one driver run measures
BASELINE.json configs 2-5.

Data scale (SURVEY §6 point 3): ``--rows R`` trains on R rows per GPU (instead of K*64), for
``--epochs E`` epochs, at ``--batch B``; the line then adds the object-store peak, HBM peak and
the host CPU time of the executors / workers.
"""
import argparse
import json
import math
import os
import sys
import tempfile
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "examples"))

# The reference publishes no number for this metric (BASELINE.json "published": {}), so
# vs_baseline is null. BASELINE.md B1-B4 are CPU notebook timings of a different (stroke) model.
BASELINE_SAMPLES_PER_S = None
BATCH = 64
DLRM_BATCH = 128
REFERENCE_CSV = os.path.join(HERE, "examples", "data", "fake_nyctaxi.csv")
DRIVER_TIMINGS = {}   # driver-side phases of the last run_pipeline (inside the timed region)
# torchrun / self-launch rank variables: the estimator driver must not look like an SPMD rank
_LAUNCHER_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                 "ROLE_NAME", "ROLE_WORLD_SIZE", "GROUP_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                 "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_RUN_ID",
                 "TORCHELASTIC_USE_AGENT_STORE", "TORCH_NCCL_ASYNC_ERROR_HANDLING",
                 "TORCHELASTIC_ERROR_FILE")


def make_csv(path: str, n: int, seed: int, chunk: int = 1 << 20):
    """Synthetic NYCTaxi CSV of ``n`` rows (reference examples/random_nyctaxi.py
    distributions), written in chunks so data-scale files never sit in memory whole."""
    import numpy as np
    import pyarrow as pa
    import pyarrow.csv as pacsv
    rng = np.random.default_rng(seed)
    base = np.datetime64("2010-01-01 00:00:00")
    writer = None
    try:
        for s in range(0, max(n, 1), chunk):
            m = min(chunk, n - s)
            if m <= 0:
                break
            secs = rng.integers(0, 157680000, size=m)
            dates = (base + secs.astype("timedelta64[s]")).astype(str)
            dates = np.char.add(np.char.replace(dates, "T", " "), " UTC")
            t = pa.table({
                "key": pa.array(["fake_key"] * m),
                "fare_amount": rng.uniform(3.0, 50.0, m),
                "pickup_datetime": pa.array(dates),
                "pickup_longitude": rng.uniform(-74.2, -73.8, m),
                "pickup_latitude": rng.uniform(40.7, 40.8, m),
                "dropoff_longitude": rng.uniform(-74.2, -73.8, m),
                "dropoff_latitude": rng.uniform(40.7, 40.8, m),
                "passenger_count": rng.integers(1, 5, m),
            })
            if writer is None:
                writer = pacsv.CSVWriter(path, t.schema)
            writer.write_table(t)
    finally:
        if writer is not None:
            writer.close()


def _nyc_class():
    import torch.nn as nn
    import torch.nn.functional as F

    class NYC_Model(nn.Module):
        """examples/pytorch_nyctaxi.py NYC_Model (defined once, at module level, as there)."""

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
            return self.fc5(x)
    return NYC_Model


_NYC_MODEL = None


def nyc_model(cols):
    global _NYC_MODEL
    if _NYC_MODEL is None:
        _NYC_MODEL = _nyc_class()
    return _NYC_MODEL(cols)


def _read_nyc(spark, csv_path):
    from data_process import nyc_taxi_preprocess
    t0 = time.perf_counter()
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true") \
        .load("file://" + csv_path)
    t1 = time.perf_counter()
    data = nyc_taxi_preprocess(data)
    features = [f.name for f in data.schema if f.name != "fare_amount"]
    DRIVER_TIMINGS.update(csv_schema=t1 - t0, plan_build=time.perf_counter() - t1)
    return data, features


def run_pipeline(spark, csv_path, world, storage, fused=True, topology="estimator", gpu_share=1.0,
                 batch=BATCH, epochs=1):
    """One full fit_on_spark of the NYC model over ``csv_path``."""
    import torch
    import torch.nn as nn
    from raydp_amd.torch import TorchEstimator
    data, features = _read_nyc(spark, csv_path)
    t2 = time.perf_counter()
    torch.manual_seed(0)
    model = nyc_model(len(features))
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    DRIVER_TIMINGS.update(model_init=time.perf_counter() - t2)
    extra = {"spmd_local_shards": True} if topology == "spmd" else \
        {"resources_per_worker": {"CPU": 1, "GPU": gpu_share}}
    est = TorchEstimator(num_workers=world, model=model, optimizer=opt, loss=nn.SmoothL1Loss(),
                         feature_columns=features, feature_types=torch.float,
                         label_column="fare_amount", label_type=torch.float, batch_size=batch,
                         num_epochs=epochs, metrics_name=["MeanAbsoluteError", "MeanSquaredError"],
                         drop_last=True, storage_path=storage, fused=fused, shuffle_seed=1234, **extra)
    return est.fit_on_spark(data)


def hvd_train_fn(config):
    """The reference's Horovod loop (examples/horovod_nyctaxi.py:40-60 of the reference) as a
    user writes it, on the worker's GPU: device-resident ``to_torch`` shard, Adam at lr x size,
    parameter / optimizer-state broadcast, ``DistributedOptimizer(op=Average)``, a ``loss.item()``
    every ``log_interval`` steps on rank 0."""
    import torch
    import torch.nn.functional as F
    import raydp_amd.hvd as hvd
    from raydp_amd.train import session
    hvd.init()
    dev = session.get_device() or torch.device("cpu")
    features = config["features"]
    loader = session.get_dataset_shard("train").to_torch(
        feature_columns=features, label_column="fare_amount", label_column_dtype=torch.float,
        feature_column_dtypes=torch.float, batch_size=config["batch_size"], drop_last=True, device=dev)
    torch.manual_seed(0)
    model = config["model_fn"](len(features)).to(dev)
    optimizer = torch.optim.Adam(model.parameters(), lr=hvd.size() * config["lr"])
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(optimizer, root_rank=0)
    optimizer = hvd.DistributedOptimizer(optimizer, named_parameters=model.named_parameters(), op=hvd.Average)
    logged, steps, loss = [], 0, None
    for epoch in range(1, config["epochs"] + 1):
        model.train()
        for batch_idx, (feature, target) in enumerate(loader):
            optimizer.zero_grad()
            loss = F.smooth_l1_loss(model(feature), target)
            loss.backward()
            optimizer.step()
            steps += 1
            if batch_idx % config["log_interval"] == 0 and hvd.rank() == 0:
                logged.append(loss.item())
        session.report({"epoch": epoch, "loss": loss.item() if loss is not None else None,
                        "train_rows": steps * config["batch_size"] // epoch, "steps": steps})


def run_horovod(spark, csv_path, world, storage, topology="estimator", gpu_share=1.0, batch=BATCH,
                epochs=1):
    """examples/horovod_nyctaxi.py: ETL, ``from_spark(parallelism=N)``, ``HorovodTrainer``."""
    import raydp_amd.hvd as hvd
    from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
    from raydp_amd.train.config import RunConfig, ScalingConfig
    data, features = _read_nyc(spark, csv_path)
    ds = spark_dataframe_to_ray_dataset(data, parallelism=world if topology == "estimator" else None)
    res = {"GPU": gpu_share, "CPU": 1}
    trainer = hvd.HorovodTrainer(
        train_loop_per_worker=hvd_train_fn,
        train_loop_config={"features": features, "batch_size": batch, "lr": 0.01, "epochs": epochs,
                           "log_interval": 10, "model_fn": nyc_model},
        scaling_config=ScalingConfig(num_workers=world, use_gpu=True, resources_per_worker=res),
        run_config=RunConfig(storage_path=storage), datasets={"train": ds},
        local_shards=topology == "spmd")
    return trainer.fit()


def make_dlrm_tsv(path, rows, seed):
    from raydp_amd.models import dlrm_data as D
    D.synthetic_criteo(path, rows, seed=seed)


def _dlrm_model(sizes, model_parallel, config):
    """Worker-side model creator: tables sharded over the workers (all-to-all) when N > 1."""
    import torch
    from raydp_amd.models.dlrm import Dlrm
    torch.manual_seed(0)
    return Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32, model_parallel=model_parallel)


def _dlrm_optimizer(model, config):
    import torch
    return torch.optim.SGD([q for q in model.parameters() if q.requires_grad], lr=0.01)


def run_dlrm(spark, tsv_path, world, storage, gpu_share=1.0, batch=DLRM_BATCH, epochs=1):
    """examples/pytorch_dlrm.ipynb cells 6-7, 13-14: Criteo TSV -> preprocessing -> 90/10 split
    -> ``TorchEstimator.fit_on_spark`` (train + eval epochs, ``model.pt``)."""
    import functools
    import torch
    from raydp_amd.models import dlrm_data as D
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.utils import random_split
    df = spark.read.schema(D.criteo_schema()).option("sep", "\t").csv("file://" + tsv_path)
    df, sizes = D.pre_process(df.cache(), frequency_limit="3", output_ordering="total_random",
                              no_numeric_log_col=False)
    train_df, test_df = random_split(df, [0.9, 0.1], 0)
    est = TorchEstimator(num_workers=world, model=functools.partial(_dlrm_model, list(sizes), world > 1),
                         optimizer=_dlrm_optimizer,
                         resources_per_worker={"CPU": 1, "GPU": gpu_share},
                         loss=torch.nn.BCEWithLogitsLoss(reduction="mean"),
                         feature_columns=[f"_c{i}" for i in range(1, 40)],
                         feature_types=[torch.float32] * 13 + [torch.long] * 26,
                         label_column="_c0", label_type=torch.float, batch_size=batch, drop_last=True,
                         num_epochs=epochs, storage_path=storage)
    return est.fit_on_spark(train_df, test_df)


def make_text(path, lines, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    vocab = np.array([f"w{i}" for i in range(5000)])
    with open(path, "w") as f:
        for s in range(0, lines, 10000):
            n = min(10000, lines - s)
            k = rng.integers(3, 12, n)
            z = np.minimum(rng.zipf(1.2, int(k.sum())), len(vocab)) - 1
            words = vocab[z]
            o = 0
            out = []
            for c in k:
                out.append(" ".join(words[o:o + c]))
                o += c
            f.write("\n".join(out) + "\n")


class _WordCountResult:
    """fit-result-shaped record of the word-count run (BASELINE.json config 1)."""

    def __init__(self, lines, words):
        self.metrics_history = [{"train_rows": lines, "distinct_words": words, "loss": None}]


def run_wordcount(spark, path):
    """BASELINE.json config 1: ``init_spark`` + word count + ``from_spark`` on the CPU: read the
    text, split / explode, group-by count, convert to a dataset through the object store."""
    from raydp_amd.spark import functions as F
    from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
    df = spark.read.text(path)
    counts = df.select(F.explode(F.split(F.col("value"), " ")).alias("word")).groupBy("word").count()
    ds = spark_dataframe_to_ray_dataset(counts)
    return _WordCountResult(None, ds.count())


def run_reference_config(spark, storage, epochs=30):
    """The reference example's own configuration (examples/pytorch_nyctaxi.py:50-105 of the
    reference): the 500-row fake_nyctaxi.csv, full ETL, 90/10 random_split, NYC_Model, batch 64,
    30 epochs with an evaluation pass each, one worker, through fit_on_spark. Returns
    (wall seconds, train rows)."""
    import torch
    import torch.nn as nn
    from data_process import nyc_taxi_preprocess
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.utils import random_split
    t0 = time.perf_counter()
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true") \
        .load("file://" + REFERENCE_CSV)
    data = nyc_taxi_preprocess(data)
    train_df, test_df = random_split(data, [0.9, 0.1], 0)
    features = [f.name for f in train_df.schema if f.name != "fare_amount"]
    torch.manual_seed(0)
    model = nyc_model(len(features))
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    est = TorchEstimator(num_workers=1, model=model, optimizer=opt, loss=nn.SmoothL1Loss(),
                         feature_columns=features, feature_types=torch.float,
                         label_column="fare_amount", label_type=torch.float, batch_size=BATCH,
                         num_epochs=epochs, metrics_name=["MeanAbsoluteError", "MeanSquaredError"],
                         storage_path=storage)
    res = est.fit_on_spark(train_df, test_df)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    rows = res.metrics_history[0].get("train_rows") if res.metrics_history else None
    return wall, rows, res


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n: int) -> int:
    """Start ranks 0..n-1 of this script as child processes (this process never touches the
    GPU: no exec from a HIP-initialised process), wait for all of them, return the exit code
    (the first failure's; the others are then stopped)."""
    import signal
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:          # a dead rank leaves its peers in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


class _HostSampler:
    """Object-store bytes in use (peak) and host CPU seconds of this process' children (the
    executors and training workers) over a region -- the data-scale run's resource report."""

    def __init__(self, interval_s=0.01):
        self.interval, self.peak, self._stop = interval_s, 0, threading.Event()
        self._t = None

    def _store(self):
        from raydp_amd.runtime import core
        return core.current_node_store()

    def _child_cpu(self):
        import psutil
        tot = 0.0
        for p in psutil.Process().children(recursive=True):
            try:
                c = p.cpu_times()
                tot += c.user + c.system
            except (psutil.NoSuchProcess, psutil.AccessDenied):
                pass
        return tot

    def _loop(self):
        st = self._store()
        while not self._stop.wait(self.interval):
            if st is not None:
                self.peak = max(self.peak, int(st.stats()["used"]))

    def __enter__(self):
        st = self._store()
        self.cap = int(st.stats()["capacity"]) if st is not None else None
        self.cpu0, self.t0 = self._child_cpu(), time.perf_counter()
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self._t.join()
        self.wall = time.perf_counter() - self.t0
        self.cpu = self._child_cpu() - self.cpu0

    def summary(self, n_exec):
        shm = None
        try:
            s = os.statvfs("/dev/shm")
            shm = s.f_blocks * s.f_frsize
        except OSError:
            pass
        return {"object_store_peak_mib": round(self.peak / 2 ** 20, 1),
                "object_store_capacity_mib": round(self.cap / 2 ** 20, 1) if self.cap else None,
                "dev_shm_total_mib": round(shm / 2 ** 20, 1) if shm else None,
                "child_process_cpu_s": round(self.cpu, 3),
                "executor_cpu_utilisation_upper_bound": round(self.cpu / max(self.wall * n_exec, 1e-9), 3)}


def _train_hist(res):
    return [m for m in (res.metrics_history if res is not None else []) if "train_loss" in m or "loss" in m]


def _dlrm_rows(steps, batch, n_train):
    # 90/10 split, equal shards, drop_last: enough rows that every worker gets >= steps batches
    return int(math.ceil((steps * batch * n_train + batch * n_train) / 0.9)) + 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--workload", choices=["nyc", "horovod", "dlrm"], default="nyc",
                    help="the workload measured as the line's value")
    ap.add_argument("--extra-workloads", default="horovod,dlrm,wordcount",
                    help="with the nyc headline: other workloads measured afterwards at the same "
                         "N/K/W, reported under config.other_workloads ('none' to skip)")
    ap.add_argument("--extra-timeout", type=float, default=300.0,
                    help="seconds for the extra workloads; past it the line is printed without them")
    ap.add_argument("--topology", choices=["spmd", "estimator"], default="estimator",
                    help="estimator: one driver + TorchEstimator(num_workers=N) (the reference "
                         "topology); spmd: one pipeline per GPU rank")
    ap.add_argument("--gpu-share", type=float, default=None,
                    help="estimator topology: GPUs per worker (< 1 rehearses N workers on fewer "
                         "GPUs; default 1, or the visible GPUs / N when there are fewer than N)")
    ap.add_argument("--rows", type=int, default=None,
                    help="data scale: training rows per GPU (default steps x batch)")
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (nyc/horovod 64, dlrm 128)")
    ap.add_argument("--no-fused", action="store_true")
    ap.add_argument("--no-reference-config", action="store_true",
                    help="skip the extra (untimed-by-the-driver) reference-config measurement")
    ap.add_argument("--profile-timed", default=None,
                    help="cProfile the timed region (driver process) into this text file")
    args = ap.parse_args()

    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.topology == "estimator":
        if env_world > 1:
            # launched as N ranks (torchrun): the reference topology has ONE driver -- rank 0 --
            # which starts one training worker per GPU itself. The other ranks leave now,
            # before any GPU call; torchrun waits for rank 0.
            if env_world != args.gpus:
                raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env_world}")
            if int(os.environ.get("RANK", "0")) != 0:
                return 0
            for k in _LAUNCHER_ENV:
                os.environ.pop(k, None)
        n_train, world, rank, local = args.gpus, 1, 0, 0
        import torch
        ndev = torch.cuda.device_count()        # does not initialise HIP
        share = args.gpu_share
        if share is None:
            share = 1.0 if ndev >= n_train else max(ndev, 1) / n_train
        if share < 1.0:
            # workers sharing a card cannot form an RCCL ring: gloo bootstraps them (the gradient
            # still rides the xGMI kernels between the processes)
            os.environ.setdefault("RAYDP_TRAIN_BACKEND", "gloo")
        driver_gpu = n_train == 1     # N == 1 trains in the driver process itself
    else:
        share = 1.0
        if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
            raise SystemExit(self_launch(args.gpus))
        rank = int(os.environ.get("RANK", "0"))
        world = env_world
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
        n_train = world
        driver_gpu = True
    # executors (one single-core executor per CPU): 4 for the driver-config pipelines (one CSV
    # split each); for data-scale runs one per CPU the box gives a process (16 on the one-GPU
    # box): the 1 GB+ CSVs split into whole waves of that many tasks, and the ETL is CPU-bound
    # on CSV parsing (Arrow's reader, ~1.2 M rows/s per core)
    cpus = int(os.environ.get("RAYDP_BENCH_CPUS", "16" if args.rows is not None else "4"))
    if args.topology == "estimator" and n_train > cpus:
        # one driver feeds N workers: one single-core executor per worker, within the host
        cpus = min(n_train, max(cpus, (os.cpu_count() or 8) // 4))
    if world > 1 and os.environ.get("RAYDP_BENCH_PIN", "1") != "0":
        # each SPMD rank's pipeline (driver + its executor processes, all host-bound) on its own
        # cores: ranks do not preempt each other, and the max over ranks stops paying for it
        from raydp_amd.utils import pin_to_rank_slice
        pin_to_rank_slice(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), min_per_rank=cpus + 1)
    import torch
    import torch.distributed as dist
    if driver_gpu:
        # modulo: lets a rehearsal put several ranks on a 1-GPU box (RAYDP_BENCH_BACKEND=gloo)
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if world > 1:
            backend = os.environ.get("RAYDP_BENCH_BACKEND", "nccl")
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
            else:
                dist.init_process_group(backend)

    import raydp  # noqa: F401 - API facade
    from raydp_amd import context, runtime

    workload = args.workload
    batch = args.batch or (DLRM_BATCH if workload == "dlrm" else BATCH)
    extras = [w for w in args.extra_workloads.split(",") if w and w != "none" and w != workload] \
        if workload == "nyc" else []
    if args.rows is not None:
        extras = []             # a data-scale run measures one workload
    if args.topology == "spmd" and world > 1:
        # each SPMD rank preprocesses its own Criteo file: the table sizes would differ per rank
        extras = [w for w in extras if w != "dlrm"]
        if workload == "dlrm":
            raise SystemExit("--workload dlrm needs --topology estimator when N > 1")

    tmp = tempfile.mkdtemp(prefix=f"raydp_bench_r{rank}_")
    rows_mult = 1 if args.topology == "spmd" else n_train     # rows one driver reads
    # the W warm-up steps run as two untimed pipelines of ceil(W/2) and floor(W/2) steps (one
    # when W < 2): the second one meets the caches, pinned buffers and code objects the first
    # one created, so the timed pipeline is the steady state a long-running driver sees
    warm_split = [s for s in ((args.warmup + 1) // 2, args.warmup // 2) if s > 0] or [1]
    files = {}
    for j, wl in enumerate([workload] + extras):
        b = batch if wl == workload else (DLRM_BATCH if wl == "dlrm" else BATCH)
        fl = []
        for i, ws in enumerate(warm_split + [None]):
            seed = 1000 * (j + 1) + 17 * i + rank
            if ws is None:       # the timed file
                rows = (args.rows if (args.rows is not None and wl == workload) else args.steps * b) \
                    * rows_mult
                seed += 500
            else:
                rows = ws * b * rows_mult
            if wl == "dlrm":
                p = os.path.join(tmp, f"{wl}{i}.tsv")
                make_dlrm_tsv(p, _dlrm_rows(rows // (b * rows_mult), b, rows_mult), seed)
            elif wl == "wordcount":
                p = os.path.join(tmp, f"{wl}{i}.txt")
                make_text(p, rows * 10, seed)
            else:
                p = os.path.join(tmp, f"{wl}{i}.csv")
                make_csv(p, rows, seed)
            fl.append(p)
        files[wl] = fl

    # estimator topology: one CPU per training worker on top of the executors'
    runtime.init(num_cpus=cpus + (n_train if args.topology == "estimator" else 0))
    # one single-core executor process per CPU: Arrow ETL scales without sharing a GIL
    spark = context.init_spark(f"nyc-bench-r{rank}", cpus, 1, "1G")
    spark.conf.set("spark.sql.session.timeZone", "UTC")
    storage = os.path.join(tmp, "results")

    def barrier():
        if driver_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            if driver_gpu:
                torch.cuda.synchronize()

    def run(wl, path, epochs=1, b=None):
        if wl == "nyc":
            return run_pipeline(spark, path, n_train, storage, fused=not args.no_fused,
                                topology=args.topology, gpu_share=share, batch=b or BATCH, epochs=epochs)
        if wl == "horovod":
            return run_horovod(spark, path, n_train, storage, topology=args.topology, gpu_share=share,
                               batch=b or BATCH, epochs=epochs)
        if wl == "wordcount":
            return run_wordcount(spark, path)
        return run_dlrm(spark, path, n_train, storage, gpu_share=share, batch=b or DLRM_BATCH, epochs=epochs)

    def measure(wl, b, epochs, sampler=None, profile=None):
        """Warm-up pipelines, then the timed one; -> (seconds, result, phases, driver phases)."""
        from raydp_amd.torch.estimator import LAST_TIMINGS
        from raydp_amd.utils import tracing
        from raydp_amd.utils.gcmeter import GcMeter, freeze_long_lived
        for p in files[wl][:-1]:
            run(wl, p, 1, b)
        # long-lived framework state (modules, plans, kernels) goes to the permanent GC
        # generation: a full collection over it costs ~100 ms and would land at random inside
        # the timed region. Freeze only, no gc.collect() first: collecting the warm-up's garbage
        # hands its memory back and the next pipeline pays to fault it in again (measured:
        # profiles/r3s4_warm_gap_variants.txt; scripts/dev/warm_gap.py --gc)
        freeze_long_lived()
        barrier()
        LAST_TIMINGS.clear()
        DRIVER_TIMINGS.clear()
        gcm = GcMeter()
        if profile is not None:
            profile.enable()
        t0 = time.perf_counter()
        with tracing.span("timed run", cat="bench", workload=wl), gcm:
            if sampler is not None:
                with sampler:
                    res = run(wl, files[wl][-1], epochs, b)
            else:
                res = run(wl, files[wl][-1], epochs, b)
            barrier()
        dt = time.perf_counter() - t0
        if profile is not None:
            profile.disable()
        return dt, res, dict(LAST_TIMINGS), dict(DRIVER_TIMINGS), gcm.summary()

    prof = None
    if args.profile_timed:
        import cProfile
        prof = cProfile.Profile()
    sampler = _HostSampler() if args.rows is not None else None
    dt, res, timed_phases, timed_driver, gc_summary = measure(workload, batch, args.epochs, sampler, prof)
    if prof is not None:
        import io
        import pstats
        buf = io.StringIO()
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats("cumulative").print_stats(70)
        st.sort_stats("tottime").print_stats(40)
        with open(args.profile_timed, "w") as f:
            f.write(buf.getvalue())
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    hist = _train_hist(res)
    h0 = hist[0] if hist else {}
    rows_per_gpu = h0.get("train_rows")
    if rows_per_gpu is None:
        rows_per_gpu = (args.rows if args.rows is not None else args.steps * batch)
    samples = args.epochs * rows_per_gpu * n_train
    steps_total = args.epochs * (rows_per_gpu // batch)
    value = samples / dt

    # N = 1 through a spawned worker actor (the hop every N > 1 run pays, and the one Ray Train
    # always takes: reference torch/estimator.py:348-355), measured the same way after its own
    # warm-up, so the 1 -> 2 step of a scaling curve can be read against it
    spawned_n1 = None
    if n_train == 1 and args.topology == "estimator" and workload == "nyc" and args.rows is None \
            and os.environ.get("RAYDP_BENCH_SPAWNED_N1", "1") != "0":
        os.environ["RAYDP_TRAIN_INPROCESS"] = "0"
        try:
            sdt, sres, sph, sdrv, _ = measure(workload, batch, args.epochs)
            sh = _train_hist(sres)
            srows = (sh[0].get("train_rows") if sh else None) or args.steps * batch
            spawned_n1 = {"value": round(args.epochs * srows / sdt, 1), "unit": "samples/s",
                          "ms_per_step": round(sdt * 1000.0 / max(1, args.epochs * (srows // batch)), 4),
                          "wall_s": round(sdt, 4), "engine": sh[0].get("engine") if sh else None,
                          "step_time_us": sh[0].get("step_time_us") if sh else None,
                          "breakdown_s": dict({k: round(v, 4) for k, v in sph.items()},
                                              **{k: round(v, 4) for k, v in sdrv.items()})}
        except Exception as e:  # noqa: BLE001 - never costs the headline
            spawned_n1 = {"error": repr(e)[-400:]}
        finally:
            os.environ.pop("RAYDP_TRAIN_INPROCESS", None)

    # power / HBM / activity telemetry (AMD SMI, sampled every 5 ms by a child process) over one
    # more, untimed run of the same pipeline: sampling inside the timed region slowed it (the
    # sampler competes with the executors for the host), so the timed run stays unobserved
    telemetry = None
    if os.environ.get("RAYDP_BENCH_DEVMON", "1") != "0" and args.rows is None and local == 0:
        from raydp_amd.utils.devmon import DeviceMonitor
        mon = DeviceMonitor(interval_s=0.005)
        mon.__enter__()
        err = None
        try:
            barrier()
            run(workload, files[workload][-1], 1, batch)
            barrier()
        except Exception as e:  # noqa: BLE001 - telemetry never costs the measurement
            err = repr(e)[-300:]
        mon.__exit__(None, None, None)
        telemetry = dict(mon.summary(), region="an untimed repeat of the timed pipeline")
        if err:
            telemetry["repeat_error"] = err
    elif world > 1:
        barrier()

    out = None
    if rank == 0:
        metric = {"nyc": "end-to-end samples/sec (Spark ETL+train) NYCTaxi TorchEstimator",
                  "horovod": "end-to-end samples/sec (Spark ETL+train) NYCTaxi HorovodTrainer",
                  "dlrm": "end-to-end train samples/sec (Spark ETL+train) DLRM synthetic Criteo"}[workload]
        model_name = {"nyc": "NYC_Model (examples/pytorch_nyctaxi.py, 48,513 params)",
                      "horovod": "NYC_Model under hvd.DistributedOptimizer (examples/horovod_nyctaxi.py)",
                      "dlrm": "DLRM 13 dense + 26 tables x 32, bottom 512-128-32, top 1024-1024-512-256-1 "
                              "(examples/pytorch_dlrm.ipynb)"}[workload]
        phases = dict({k: round(v, 4) for k, v in timed_phases.items()},
                      **{k: round(v, 4) for k, v in timed_driver.items()})
        phases["other"] = round(dt - sum(v for k, v in timed_phases.items() if not k.endswith("_concurrent"))
                                - sum(timed_driver.values()), 4)
        out = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": n_train,
            "steps": args.steps if args.rows is None else steps_total,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1000.0 / max(1, steps_total), 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_SAMPLES_PER_S is None else round(value / BASELINE_SAMPLES_PER_S, 2),
            "dtype": "bf16" if workload == "nyc" else "fp32 user loop" if workload == "horovod" else "bf16 towers",
            "data": ("synthetic Criteo-shaped TSV (dlrm_data.synthetic_criteo)" if workload == "dlrm" else
                     "synthetic NYCTaxi CSV (examples/random_nyctaxi.py distributions)") + ", random-init weights",
            "config": {"model": model_name, "workload": workload,
                       "global_batch": batch * n_train, "seq_len": None,
                       "parallelism": f"dp{n_train}" + ("+table-wise embedding all-to-all"
                                                         if workload == "dlrm" and n_train > 1 else ""),
                       "per_gpu_batch": batch, "epochs": args.epochs,
                       "train_rows_per_gpu": rows_per_gpu,
                       "topology": args.topology, "gpu_share": share,
                       "timing": "driver wall clock around the whole fit (spans every worker)"
                                 if args.topology == "estimator" else "max over ranks",
                       "engine": h0.get("engine"),
                       "allreduce": h0.get("allreduce"),
                       "timed_region": "csv read+ETL+from_spark+shuffle+HBM ingest+train+checkpoint",
                       "final_train_loss": hist[-1].get("train_loss", hist[-1].get("loss")) if hist else None,
                       "step_time_us": h0.get("step_time_us"),
                       "device_telemetry": telemetry,
                       "python_gc_in_timed_region": gc_summary,
                       "hbm_peak_allocated_mib": round(torch.cuda.max_memory_allocated() / 2 ** 20, 1)
                       if driver_gpu else h0.get("hbm_peak_allocated_mib"),
                       "rank0_breakdown_s": phases},
        }
        from raydp_amd.torch.estimator import STREAM_STATS
        if STREAM_STATS.get("blocks"):
            out["config"]["streamed_blocks"] = STREAM_STATS["blocks"]   # DMA'd while the conversion ran
        if spawned_n1 is not None:
            out["config"]["n1_spawned_worker"] = dict(
                spawned_n1, what="the same pipeline with the one training worker in a spawned actor "
                                 "process (the reference topology's worker hop), value = samples/s")
        if sampler is not None:
            hr = sampler.summary(cpus)
            conv = timed_phases.get("etl_and_conversion_concurrent")
            if conv:
                # the executors only work while the conversion stage runs (the upper bound above
                # divides by the whole timed region, training included)
                hr["executor_cpu_utilisation_during_conversion"] = round(
                    hr["child_process_cpu_s"] / max(conv * cpus, 1e-9), 3)
            out["config"]["host_resources"] = hr
            out["config"]["train_epoch_samples_per_s"] = [round(m.get("train_samples_per_s", 0), 1)
                                                          for m in hist if "train_samples_per_s" in m]
    if extras:
        out_extra = {}
        done = threading.Event()

        def watchdog():
            # an extra workload that hangs must not cost the headline: print without it and leave
            if not done.wait(args.extra_timeout):
                if out is not None:
                    out["config"]["other_workloads"] = dict(out_extra, timed_out_after_s=args.extra_timeout)
                    print(json.dumps(out), flush=True)
                os._exit(0)
        threading.Thread(target=watchdog, daemon=True).start()
        for wl in extras:
            b = DLRM_BATCH if wl == "dlrm" else BATCH
            try:
                edt, eres, eph, edrv, _ = measure(wl, b, 1)
                if wl == "wordcount":
                    m0 = eres.metrics_history[0]
                    lines = args.steps * BATCH * rows_mult * 10      # make_text's line count
                    out_extra[wl] = {
                        "metric": "word count + from_spark lines/s on the CPU (BASELINE.json config 1)",
                        "value": round(lines / edt, 1), "unit": "lines/s", "wall_s": round(edt, 4),
                        "lines": lines, "distinct_words": m0["distinct_words"], "executors": cpus}
                    continue
                eh = _train_hist(eres)
                rows = (eh[0].get("train_rows") if eh else None) or args.steps * b
                out_extra[wl] = {
                    "metric": {"horovod": "e2e samples/s NYCTaxi HorovodTrainer (examples/horovod_nyctaxi.py)",
                               "dlrm": "e2e train samples/s DLRM (examples/pytorch_dlrm.ipynb)"}[wl],
                    "value": round(rows * n_train / edt, 1), "unit": "samples/s", "wall_s": round(edt, 4),
                    "per_gpu_batch": b, "train_rows_per_gpu": rows,
                    "ms_per_step": round(edt * 1000.0 / max(1, rows // b), 4),
                    "engine": eh[0].get("engine") if eh else None,
                    "allreduce": eh[0].get("allreduce") if eh else None,
                    "final_loss": eh[-1].get("train_loss", eh[-1].get("loss")) if eh else None,
                    "breakdown_s": dict({k: round(v, 4) for k, v in eph.items()},
                                        **{k: round(v, 4) for k, v in edrv.items()})}
            except Exception as e:  # noqa: BLE001 - an extra never costs the headline
                out_extra[wl] = {"error": repr(e)[-400:]}
        done.set()
        if out is not None:
            out["config"]["other_workloads"] = out_extra
    if out is not None:
        if n_train == 1 and workload == "nyc" and args.rows is None and not args.no_reference_config:
            # the reference example's own config (untimed by the driver; reported alongside)
            run_reference_config(spark, storage, epochs=2)          # warm its shapes
            wall, rows, ref = run_reference_config(spark, storage)
            rh = [m for m in ref.metrics_history if "train_loss" in m]
            out["config"]["reference_config_e2e"] = {
                "what": "examples/pytorch_nyctaxi.py: 500-row fake_nyctaxi.csv, ETL, 90/10 split, "
                        "30 epochs train+eval, batch 64, fit_on_spark",
                "wall_s": round(wall, 4),
                "train_rows_per_epoch": rows,
                "train_samples_per_s_e2e": round(30 * rows / wall, 1) if rows else None,
                "final_train_loss": rh[-1]["train_loss"] if rh else None,
                "engine": rh[-1].get("engine") if rh else None}
        print(json.dumps(out), flush=True)
    context.stop_spark()
    runtime.shutdown()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
