"""Tracing: Python spans and native-service events merge into one Chrome
trace covering ETL stages, executor tasks, actor life cycle and training phases."""
import json
import os
import tempfile

import raydp  # noqa: F401
import torch

from raydp_amd.utils import tracing


def test_trace_covers_etl_runtime_and_training(monkeypatch):
    d = tempfile.mkdtemp(prefix="trace_")
    path = os.path.join(d, "t")
    monkeypatch.setenv("RAYDP_TRACE", path)
    tracing.set_trace_path(path)
    try:
        from raydp_amd import runtime
        runtime.shutdown()
        runtime.init(num_cpus=4)
        import raydp_amd
        from raydp_amd.torch import TorchEstimator
        spark = raydp_amd.init_spark("trace", 1, 1, "200M")
        df = spark.range(0, 256).selectExpr("cast(id as double) as x", "cast(id * 2 as double) as y")
        est = TorchEstimator(num_workers=1, model=torch.nn.Linear(1, 1),
                             optimizer=torch.optim.SGD, loss=torch.nn.MSELoss, feature_columns=["x"],
                             label_column="y", batch_size=64, num_epochs=1)
        # optimizer given as a class: the estimator builds it (reference semantics allow creators)
        est._optimizer = lambda m, cfg: torch.optim.SGD(m.parameters(), lr=1e-4)
        res = est.fit_on_spark(df)
        first = res.metrics_history[0]
        assert first["train_samples_per_s"] > 0 and first["train_epoch_wall_s"] > 0
        raydp_amd.stop_spark()
        runtime.shutdown()
    finally:
        out = tracing.merge(path)
        tracing.set_trace_path(None)
    ev = json.load(open(out))["traceEvents"]
    names = {e["name"] for e in ev}
    cats = {e.get("cat") for e in ev}
    assert {"persist stage", "task", "etl + conversion", "ingest", "train epoch", "checkpoint"} <= names, names
    assert "actor" in cats                        # native supervisor events
    assert any(n.startswith("register executor") for n in names)  # native app master events
    pids = {e["pid"] for e in ev if e.get("ph") != "M"}
    assert len(pids) >= 3                         # driver, executor, native services


def test_actor_log_files_carry_job_id_header():
    """Logging agent (Agent.java:80-97): each worker process logs into its own file under the
    session log directory, first line ':job_id:<id>', plus one start line per (re)start."""
    import glob
    from raydp_amd import runtime
    from raydp_amd.runtime import core
    import raydp_amd
    runtime.shutdown()
    runtime.init(num_cpus=2)
    try:
        spark = raydp_amd.init_spark("logs", 1, 1, "200M")
        assert spark.range(0, 10).count() == 10
        node = core.current_node()
        files = glob.glob(os.path.join(node.session_dir, "logs", "actor-raydp-executor-0*.log"))
        assert files, os.listdir(os.path.join(node.session_dir, "logs"))
        lines = open(files[0]).read().splitlines()
        assert lines[0] == f":job_id:{node.job_id}"
        assert "start (pid" in lines[1]
        raydp_amd.stop_spark()
    finally:
        runtime.shutdown()


def test_device_monitor_and_step_histogram():
    """SURVEY §5.5 telemetry: the AMD SMI sampler never breaks the region it brackets (here no
    driver: it reports why), and the step-time histogram has the percentiles and buckets."""
    import time

    from raydp_amd.utils.devmon import DeviceMonitor, step_time_histogram
    with DeviceMonitor(interval_s=0.01) as mon:
        time.sleep(0.03)
    s = mon.summary()
    assert isinstance(s, dict) and "available" in s
    if not s["available"]:
        assert s["reason"]
    h = step_time_histogram([27.5, 28.0, 29.0, 31.0, 45.0, 1200.0])
    assert h["steps"] == 6 and h["p50"] == 30.0 and h["max"] == 1200.0
    assert sum(h["hist_us"].values()) == 6 and h["hist_us"]["1000-5000"] == 1
