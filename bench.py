#!/usr/bin/env python
"""Flagship benchmark: end-to-end NYCTaxi samples/s (Spark-style ETL + conversion + training).

Metric (BASELINE.json): "end-to-end samples/sec (Spark ETL+train) NYCTaxi TorchEstimator
@1/2/4/8 GPU". One *step* = one optimizer step of the reference NYC_Model
(examples/pytorch_nyctaxi.py: 5 Linear + 4 BatchNorm1d, SmoothL1, Adam 1e-3) on a batch of 64
rows per GPU. The timed region of K steps contains, per rank, EVERYTHING the reference's
``fit_on_spark`` path does for those K*64 rows: CSV read + parse, the full
``examples/data_process.py`` ETL (14 filters, 9 time features incl. 2 Python UDFs,
11 distance features incl. 8 Python-UDF calls, 7 drops), the Spark->Dataset conversion through
the shared-memory object store, the dataset shuffle, the host->HBM ingest, K training steps
(forward, backward, all-reduce across ranks, optimizer) and the rank-0 ``model.pt`` checkpoint.
Each sample passes through ETL once (1 epoch). Data: synthetic NYCTaxi rows with the
reference generator's distributions (examples/random_nyctaxi.py), written to a per-rank CSV
before timing. Weights: random init. Weak scaling: 64 rows/step/GPU.

Launch: ``python bench.py --gpus N --steps K --warmup W``. For N > 1 outside a torchrun job
the script starts the N rank processes itself (fresh child processes, before any GPU call;
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set for each) and waits
for them; under ``torchrun --nproc-per-node N ... bench.py --gpus N`` every rank runs directly.
Rank 0 prints ONE JSON line.

Topologies (``--topology``):
* ``spmd`` (default): one process per GPU, each running the whole pipeline on its own rows
  (own Spark session, own executors, own CSV) and training over RCCL/xGMI with its peers --
  the way the driver's torchrun launch scales it;
* ``estimator``: the reference's own topology (``python/raydp/torch/estimator.py:331-355``):
  ONE driver process, ONE Spark session, ``TorchEstimator(num_workers=N)`` whose N worker
  processes (one per GPU, spawned by the worker-group trainer and kept warm between fits, as
  Ray's prestarted workers are) each ingest one equal shard of the converted dataset.
"""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "examples"))

# The reference publishes no number for this metric (BASELINE.json "published": {}), so
# vs_baseline is null. BASELINE.md B1-B4 are CPU notebook timings of a different (stroke) model.
BASELINE_SAMPLES_PER_S = None
BATCH = 64
REFERENCE_CSV = os.path.join(HERE, "examples", "data", "fake_nyctaxi.csv")
DRIVER_TIMINGS = {}   # driver-side phases of the last run_pipeline (inside the timed region)


def make_csv(path: str, n: int, seed: int):
    import numpy as np
    import pyarrow as pa
    import pyarrow.csv as pacsv
    rng = np.random.default_rng(seed)
    base = np.datetime64("2010-01-01 00:00:00")
    secs = rng.integers(0, 157680000, size=n)
    dates = (base + secs.astype("timedelta64[s]")).astype(str)
    dates = np.char.add(np.char.replace(dates, "T", " "), " UTC")
    t = pa.table({
        "key": pa.array(["fake_key"] * n),
        "fare_amount": rng.uniform(3.0, 50.0, n),
        "pickup_datetime": pa.array(dates),
        "pickup_longitude": rng.uniform(-74.2, -73.8, n),
        "pickup_latitude": rng.uniform(40.7, 40.8, n),
        "dropoff_longitude": rng.uniform(-74.2, -73.8, n),
        "dropoff_latitude": rng.uniform(40.7, 40.8, n),
        "passenger_count": rng.integers(1, 5, n),
    })
    pacsv.write_csv(t, path)


def nyc_model(cols):
    import torch.nn as nn
    import torch.nn.functional as F

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
            return self.fc5(x)
    return NYC_Model(cols)


def run_pipeline(spark, csv_path, steps, world, storage, fused=True, topology="spmd", gpu_share=1.0):
    """One full fit_on_spark over a file holding exactly steps*BATCH rows (x world for the
    estimator topology, whose one driver feeds every worker)."""
    import torch
    import torch.nn as nn
    from data_process import nyc_taxi_preprocess
    from raydp_amd.torch import TorchEstimator
    t0 = time.perf_counter()
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true") \
        .load("file://" + csv_path)
    t1 = time.perf_counter()
    data = nyc_taxi_preprocess(data)
    features = [f.name for f in data.schema if f.name != "fare_amount"]
    t2 = time.perf_counter()
    torch.manual_seed(0)
    model = nyc_model(len(features))
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    DRIVER_TIMINGS.update(csv_schema=t1 - t0, plan_build=t2 - t1, model_init=time.perf_counter() - t2)
    extra = {"spmd_local_shards": True} if topology == "spmd" else \
        {"resources_per_worker": {"CPU": 1, "GPU": gpu_share}}
    est = TorchEstimator(num_workers=world, model=model, optimizer=opt, loss=nn.SmoothL1Loss(),
                         feature_columns=features, feature_types=torch.float,
                         label_column="fare_amount", label_type=torch.float, batch_size=BATCH,
                         num_epochs=1, metrics_name=["MeanAbsoluteError", "MeanSquaredError"],
                         drop_last=True, storage_path=storage, fused=fused, shuffle_seed=1234, **extra)
    res = est.fit_on_spark(data)
    return res


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--topology", choices=["spmd", "estimator"], default="spmd",
                    help="spmd: one pipeline per GPU rank; estimator: one driver + "
                         "TorchEstimator(num_workers=N) (the reference topology)")
    ap.add_argument("--gpu-share", type=float, default=1.0,
                    help="estimator topology: GPUs per worker (< 1 rehearses N workers on fewer GPUs)")
    ap.add_argument("--no-fused", action="store_true")
    ap.add_argument("--no-reference-config", action="store_true",
                    help="skip the extra (untimed-by-the-driver) reference-config measurement")
    ap.add_argument("--profile-timed", default=None,
                    help="cProfile the timed region (driver process) into this text file")
    args = ap.parse_args()

    if args.topology == "estimator" and args.gpu_share < 1.0:
        # workers sharing a card cannot form an RCCL ring: gloo bootstraps them (the gradient
        # still rides the xGMI one-shot path between the processes)
        os.environ.setdefault("RAYDP_TRAIN_BACKEND", "gloo")
    if args.topology == "spmd" and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(args.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.topology == "estimator":
        if world != 1:
            raise SystemExit("--topology estimator runs as ONE driver process (it spawns the workers)")
    elif world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cpus = int(os.environ.get("RAYDP_BENCH_CPUS", "4"))
    if world > 1 and os.environ.get("RAYDP_BENCH_PIN", "1") != "0":
        # each SPMD rank's pipeline (driver + its executor processes, all host-bound) on its own
        # cores: ranks do not preempt each other, and the max over ranks stops paying for it
        from raydp_amd.utils import pin_to_rank_slice
        pin_to_rank_slice(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), min_per_rank=cpus + 1)
    import torch
    import torch.distributed as dist
    # modulo: lets a rehearsal put several ranks on a 1-GPU box (RAYDP_BENCH_BACKEND=gloo)
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1:
        backend = os.environ.get("RAYDP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    n_train = args.gpus if args.topology == "estimator" else world   # ranks that train

    import raydp  # noqa: F401 - API facade
    from raydp_amd import context, runtime

    tmp = tempfile.mkdtemp(prefix=f"raydp_bench_r{rank}_")
    main_csv = os.path.join(tmp, "main.csv")
    rows_per = 1 if args.topology == "spmd" else n_train
    # the W warm-up steps run as two untimed pipelines of ceil(W/2) and floor(W/2) steps (one
    # when W < 2): the second one meets the caches, pinned buffers and code objects the first
    # one created, so the timed pipeline is the steady state a long-running driver sees
    warm_split = [s for s in ((args.warmup + 1) // 2, args.warmup // 2) if s > 0] or [1]
    warm_csvs = []
    for j, ws in enumerate(warm_split):
        p = os.path.join(tmp, f"warm{j}.csv")
        make_csv(p, ws * BATCH * rows_per, 1000 + 17 * j + rank)
        warm_csvs.append((p, ws))
    make_csv(main_csv, args.steps * BATCH * rows_per, 2000 + rank)

    # estimator topology: one CPU per training worker on top of the executors'
    runtime.init(num_cpus=cpus + (n_train if args.topology == "estimator" else 0))
    # one single-core executor process per CPU: Arrow ETL scales without sharing a GIL
    spark = context.init_spark(f"nyc-bench-r{rank}", int(os.environ.get("RAYDP_BENCH_CPUS", "4")), 1, "1G")
    spark.conf.set("spark.sql.session.timeZone", "UTC")
    storage = os.path.join(tmp, "results")

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    # warmup: W steps of full pipelines (compiles kernels, vectorises UDFs, warms caches)
    kw = dict(fused=not args.no_fused, topology=args.topology, gpu_share=args.gpu_share)
    for p, ws in warm_csvs:
        run_pipeline(spark, p, ws, n_train, storage, **kw)
    # long-lived framework state (modules, plans, kernels) goes to the permanent GC generation:
    # a full collection over it costs ~100 ms and would land at random inside the timed region.
    # Freeze only, no gc.collect() first: collecting the warm-up's garbage hands its memory back
    # and the next pipeline pays to fault it in again -- measured on the box, the first pipeline
    # after collect+freeze took 7.0-8.0 ms against 4.7 ms after a plain freeze, every phase of it
    # slower (profiles/r3s4_warm_gap_variants.txt; scripts/dev/warm_gap.py --gc)
    from raydp_amd.utils.gcmeter import GcMeter, freeze_long_lived
    freeze_long_lived()
    barrier()
    from raydp_amd.utils import tracing
    prof = None
    if args.profile_timed:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    gcm = GcMeter()
    t0 = time.perf_counter()
    with tracing.span("timed run", cat="bench"), gcm:
        res = run_pipeline(spark, main_csv, args.steps, n_train, storage, **kw)
        barrier()
    dt = time.perf_counter() - t0
    from raydp_amd.torch.estimator import LAST_TIMINGS
    timed_phases, timed_driver = dict(LAST_TIMINGS), dict(DRIVER_TIMINGS)   # before any other run
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats("cumulative").print_stats(70)
        st.sort_stats("tottime").print_stats(40)
        with open(args.profile_timed, "w") as f:
            f.write(buf.getvalue())
    # power / HBM / activity telemetry (AMD SMI, sampled every 5 ms by a child process on local
    # rank 0) over one more, untimed run of the same pipeline: sampling inside the timed region
    # slowed it from 5.4-7.0 to 7.2-8.5 ms on the box (the sampler competes with the executors
    # for the host), so the timed run stays unobserved
    telemetry = None
    if os.environ.get("RAYDP_BENCH_DEVMON", "1") != "0":
        from raydp_amd.utils.devmon import DeviceMonitor
        mon = DeviceMonitor(interval_s=0.005) if local == 0 else None
        if mon is not None:
            mon.__enter__()
        err = None
        try:
            barrier()
            run_pipeline(spark, main_csv, args.steps, n_train, storage, **kw)
            barrier()
        except Exception as e:  # noqa: BLE001 - telemetry never costs the measurement
            err = repr(e)[-300:]
        if mon is not None:
            mon.__exit__(None, None, None)
            telemetry = dict(mon.summary(), region="an untimed repeat of the timed pipeline")
            if err:
                telemetry["repeat_error"] = err
    t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    samples = args.steps * BATCH * n_train
    value = samples / dt
    engine = res.metrics_history[0].get("engine") if res.metrics_history else None
    if rank == 0:
        out = {
            "metric": "end-to-end samples/sec (Spark ETL+train) NYCTaxi TorchEstimator",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": n_train,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1000.0 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_SAMPLES_PER_S is None else round(value / BASELINE_SAMPLES_PER_S, 2),
            "dtype": "bf16",
            "data": "synthetic NYCTaxi CSV (examples/random_nyctaxi.py distributions), random-init weights",
            "config": {"model": "NYC_Model (examples/pytorch_nyctaxi.py, 48,513 params)",
                       "global_batch": BATCH * n_train, "seq_len": None,
                       "parallelism": f"dp{n_train}", "per_gpu_batch": BATCH, "epochs": 1,
                       "topology": args.topology,
                       "engine": engine,
                       "allreduce": res.metrics_history[0].get("allreduce") if res.metrics_history else None,
                       "timed_region": "csv read+ETL+from_spark+shuffle+HBM ingest+train+checkpoint",
                       "final_train_loss": res.metrics_history[0].get("train_loss")
                       if res.metrics_history else None,
                       "step_time_us": res.metrics_history[0].get("step_time_us") if res.metrics_history else None,
                       "device_telemetry": telemetry,
                       "python_gc_in_timed_region": gcm.summary(),
                       "hbm_peak_allocated_mib": round(torch.cuda.max_memory_allocated() / 2 ** 20, 1),
                       "rank0_breakdown_s": dict({k: round(v, 4) for k, v in timed_phases.items()},
                                                 **{k: round(v, 4) for k, v in timed_driver.items()},
                                                 other=round(dt - sum(v for k, v in timed_phases.items()
                                                                      if not k.endswith("_concurrent"))
                                                             - sum(timed_driver.values()), 4))},
        }
        if n_train == 1 and not args.no_reference_config:
            # the reference example's own config (untimed by the driver; reported alongside)
            run_reference_config(spark, storage, epochs=2)          # warm its shapes
            wall, rows, ref = run_reference_config(spark, storage)
            hist = [m for m in ref.metrics_history if "train_loss" in m]
            out["config"]["reference_config_e2e"] = {
                "what": "examples/pytorch_nyctaxi.py: 500-row fake_nyctaxi.csv, ETL, 90/10 split, "
                        "30 epochs train+eval, batch 64, fit_on_spark",
                "wall_s": round(wall, 4),
                "train_rows_per_epoch": rows,
                "train_samples_per_s_e2e": round(30 * rows / wall, 1) if rows else None,
                "final_train_loss": hist[-1]["train_loss"] if hist else None,
                "engine": hist[-1].get("engine") if hist else None}
        print(json.dumps(out), flush=True)
    context.stop_spark()
    runtime.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
