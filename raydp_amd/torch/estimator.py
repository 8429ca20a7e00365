"""``TorchEstimator``: scikit-learn style distributed PyTorch training on Spark DataFrames.

API parity with ``python/raydp/torch/estimator.py`` (constructor kwargs :76-170,
``fit`` :312-356, ``fit_on_spark`` :358-390, ``get_model`` :392-396, ``train_func`` :177-270):
model instance or creator, optimizer instance (re-instantiated with ``lr=0.1`` then
``load_state_dict``, :190-196) or creator, loss class/instance/creator, per-batch LR scheduler,
per-epoch ``session.report`` dicts, rank-0 ``model.pt`` checkpoint.

Differences by design (MI355X): the worker shard is ingested into HBM once and every epoch runs
device-resident (fused HIP MLP trainer when the model allows it, otherwise a torch loop with
on-device loss/metric accumulation); ``extra_config`` is honoured (``use_gpu``, ``shuffle_seed``)
instead of being silently dropped (:163).
"""
import copy
import inspect
from concurrent.futures import wait as cf_wait
import os
import time
import tempfile
from typing import Any, Callable, Dict, List, NoReturn, Optional, Union

import torch
from torch.nn.modules.loss import _Loss as TLoss

from raydp_amd.estimator import EstimatorInterface
from raydp_amd.spark.interfaces import DF, OPTIONAL_DF, SparkEstimatorInterface
from raydp_amd.torch.config import TorchConfig
from raydp_amd.torch.metrics import TorchMetric
from raydp_amd.train import session
from raydp_amd.train.checkpoint import Checkpoint, TorchCheckpoint
from raydp_amd.train.config import FailureConfig, RunConfig, ScalingConfig
from raydp_amd.train.fast_save import save_state_dict
from raydp_amd.train.trainer import TorchTrainer

# wall-clock phase marks of the last fit in this process (bench / profiling); keys ending in
# "_concurrent" ran beside the other phases and are not part of their sequential sum
LAST_TIMINGS = {}
STREAM_STATS = {}    # {"blocks": training blocks the last fit streamed into HBM during its conversion}
_CONV_POOL = None


def _conversion_pool():
    global _CONV_POOL
    if _CONV_POOL is None:
        import concurrent.futures as cf
        _CONV_POOL = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="raydp-conversion")
    return _CONV_POOL


class _Pick:
    """Future-like view of one element of another future's tuple result."""

    def __init__(self, fut, i, need=None):
        self.fut, self.i, self.need = fut, i, need

    def result(self):
        if self.need is not None:
            self.need()     # whoever waits for the data releases a stage still held back
        return self.fut.result()[self.i]

    def done(self):
        return self.fut.done()


def _make_lr_schedule(opt_template: torch.optim.Optimizer, creator, config):
    """Per-step learning rates of ``creator(optimizer, config)`` for the fused engine."""
    dummy = torch.nn.Parameter(torch.zeros(1))
    g = dict(opt_template.param_groups[0])
    g.pop("params")
    if "initial_lr" in g:       # a resumed optimizer carries the decayed lr: restart from the base
        g["lr"] = g.pop("initial_lr")
    opt = type(opt_template)([dummy], **{k: v for k, v in g.items()
                                         if k in inspect.signature(type(opt_template)).parameters})
    sched = creator(opt, config)
    cache: List[float] = []

    def lr_at(t: int) -> float:
        while len(cache) <= t:
            cache.append(float(opt.param_groups[0]["lr"]))
            opt.step()
            sched.step()
        return cache[t]
    return lr_at


OPTIM_KEY, SCHED_KEY, META_KEY = "optim.pt", "sched.pt", "meta.json"


def _restore_optimizer(path: str, optimizer):
    op = os.path.join(path, OPTIM_KEY)
    if os.path.exists(op):
        optimizer.load_state_dict(torch.load(op, map_location="cpu", weights_only=True))


def _restore_checkpoint(path: str, model) -> int:
    """Load ``model.pt`` of a checkpoint directory into the worker's model; returns the first
    epoch still to run (``optim.pt`` is loaded by ``_restore_optimizer`` once the engine's
    scheduler exists)."""
    import json
    model.load_state_dict(torch.load(os.path.join(path, "model.pt"), map_location="cpu", weights_only=True))
    meta = os.path.join(path, META_KEY)
    if os.path.exists(meta):
        with open(meta) as f:
            return int(json.load(f).get("epoch", -1)) + 1
    return 0


def _report_epoch_checkpoint(engine, epoch: int):
    """Rank 0 writes ``model.pt`` + ``optim.pt`` (+ ``sched.pt``) + ``meta.json`` after
    ``epoch``; every rank reports so the group stays in step."""
    import json
    ckpt = None
    with tempfile.TemporaryDirectory() as d:
        if session.get_world_rank() == 0:
            save_state_dict({k: v.detach().cpu() for k, v in engine.state_dict().items()},
                            os.path.join(d, "model.pt"))
            torch.save(engine.optimizer_state_dict(), os.path.join(d, OPTIM_KEY))
            sched = getattr(engine, "scheduler", None)
            if sched is not None:
                torch.save(sched.state_dict(), os.path.join(d, SCHED_KEY))
            with open(os.path.join(d, META_KEY), "w") as f:
                json.dump({"epoch": epoch}, f)
            ckpt = Checkpoint.from_directory(d)
        session.report({"epoch": epoch, "checkpoint_epoch": epoch}, checkpoint=ckpt)


class TorchEstimator(EstimatorInterface, SparkEstimatorInterface):
    def __init__(self,
                 num_workers: int = 1,
                 resources_per_worker: Optional[Dict[str, float]] = None,
                 model: Union[torch.nn.Module, Callable] = None,
                 optimizer: Union[torch.optim.Optimizer, Callable] = None,
                 loss: Union[TLoss, Callable] = None,
                 lr_scheduler_creator: Optional[Callable] = None,
                 scheduler_step_freq="batch",
                 feature_columns: List[str] = None,
                 feature_types: Optional[List[torch.dtype]] = None,
                 label_column: str = None,
                 label_type: Optional[torch.dtype] = None,
                 batch_size: int = None,
                 drop_last: bool = False,
                 num_epochs: int = None,
                 shuffle: bool = True,
                 num_processes_for_data_loader: int = 0,
                 placement_strategy="PACK",
                 metrics_name: Optional[List[Union[str, Callable]]] = None,
                 metrics_config: Optional[Dict[str, Dict[str, Any]]] = None,
                 use_ccl: bool = False,
                 **extra_config):
        self._num_workers = num_workers
        self._resources_per_worker = resources_per_worker
        self._model = model
        self._optimizer = optimizer
        self._loss = loss
        self._lr_scheduler_creator = lr_scheduler_creator
        self._feature_columns = feature_columns
        self._feature_types = feature_types
        self._label_column = label_column
        self._label_type = label_type
        self._batch_size = batch_size
        self._drop_last = drop_last
        self._num_epochs = num_epochs
        self._shuffle = shuffle
        self._num_processes_for_data_loader = num_processes_for_data_loader
        self._placement_strategy = placement_strategy
        self._metrics = TorchMetric(metrics_name, metrics_config)
        self._use_ccl = use_ccl
        self._extra_config = extra_config
        if self._num_processes_for_data_loader > 0:
            raise TypeError("multiple processes for data loader has not supported")
        self._trainer: Optional[TorchTrainer] = None
        self._trained_results = None
        self._check()

    def _check(self):
        assert self._model is not None, "Model must be provided"
        assert self._optimizer is not None, "Optimizer must be provided"
        assert self._loss is not None, "Loss must be provided"

    # ------------------------------------------------------------------------- worker -----
    @staticmethod
    def train_func(config):
        t_setup0 = time.time_ns()
        from raydp_amd.utils import tracing
        device = session.get_device() or torch.device("cpu")
        engine = TorchEstimator._detached_fused_engine(config, device)
        if engine is not None:
            tracing.complete("worker setup", t_setup0, cat="train", engine=engine.name, detached=True)
            LAST_TIMINGS["worker_setup"] = (time.time_ns() - t_setup0) / 1e9
            return TorchEstimator._train_loop(config, engine, 0, device)
        # model
        if isinstance(config["model"], torch.nn.Module):
            model = copy.deepcopy(config["model"])
        elif callable(config["model"]):
            model = config["model"](config)
        else:
            raise Exception("Unsupported parameter, we only support torch.nn.Model instance "
                            "or a function(dict -> model)")
        # the model stays on the host until the engine is chosen: the fused engine keeps its own
        # flat device copy of the parameters (one H2D copy) and writes results back to the host
        # module in one D2H copy; the torch loop moves it to the device below
        # optimizer (instance -> re-instantiate on this worker's parameters)
        if isinstance(config["optimizer"], torch.optim.Optimizer):
            optimizer_cls = config["optimizer"].__class__
            state = config["optimizer"].state_dict()
            optimizer = optimizer_cls(model.parameters(), lr=0.1)
            optimizer.load_state_dict(state)
        elif callable(config["optimizer"]):
            optimizer = config["optimizer"](model, config)
        else:
            raise Exception("Unsupported parameter, we only support torch.optim.Optimizer subclass "
                            "instance or a function((models, dict) -> optimizer)")
        # loss
        if inspect.isclass(config["loss"]) and issubclass(config["loss"], TLoss):
            loss = config["loss"]()
        elif isinstance(config["loss"], TLoss):
            loss = config["loss"]
        elif callable(config["loss"]):
            loss = config["loss"](config)
        else:
            raise Exception("Unsupported parameter, we only support torch.nn.modules.loss._Loss "
                            "subclass, subclass instance or a function(dict -> loss)")
        metrics = config["metrics"].clone()
        # a restarted worker group resumes from the newest checkpoint an earlier attempt wrote
        start_epoch, resume_dir = 0, None
        ck = session.get_checkpoint()
        if ck is not None:
            resume_dir = ck.path
            start_epoch = _restore_checkpoint(resume_dir, model)

        from raydp_amd.torch.engine import FusedMLPEngine, TorchLoopEngine
        engine = None
        fused = None
        fused_mode = config.get("fused", None)
        if fused_mode is None:
            from raydp_amd.utils.config import get as conf_get
            fused_mode = conf_get("spark.ray.mi355x.fused")
        fused_mode = {True: "auto", False: "off"}.get(fused_mode, fused_mode)
        if fused_mode != "off":
            fused = FusedMLPEngine.applicable(model, optimizer, loss, metrics, device,
                                              config["batch_size"], config["feature_columns"],
                                              config["feature_types"])
        if fused is None and fused_mode == "on":
            raise ValueError("spark.ray.mi355x.fused=on but the model / optimizer / loss is not fusable "
                             "(FusedMLPEngine.applicable)")
        if fused is not None:
            spec, lc, oc, acc_thr = fused
            if resume_dir:
                _restore_optimizer(resume_dir, optimizer)
            lr_fn = None
            if config["lr_scheduler_creator"]:
                lr_fn = _make_lr_schedule(optimizer, config["lr_scheduler_creator"], config)
            try:
                engine = FusedMLPEngine(model, optimizer, spec, lc, oc, acc_thr, metrics, device, config, lr_fn,
                                        loss=loss)
            except ValueError:
                if fused_mode == "on":
                    raise
                fused = None   # a layout limit of the fused kernels (LDS, residency): torch loop
        if fused is None:
            model = model.to(device)       # in place: the optimizer keeps its parameter objects
            sched = config["lr_scheduler_creator"](optimizer, config) if config["lr_scheduler_creator"] else None
            if resume_dir:
                # after the scheduler: its constructor resets the group's lr, the restored
                # optimizer state puts the resumed lr back
                _restore_optimizer(resume_dir, optimizer)
                if sched is not None and os.path.exists(os.path.join(resume_dir, SCHED_KEY)):
                    sched.load_state_dict(torch.load(os.path.join(resume_dir, SCHED_KEY), weights_only=True))
            engine = TorchLoopEngine(model, optimizer, loss, metrics, device, config, sched)
        tracing.complete("worker setup", t_setup0, cat="train", engine=engine.name)
        LAST_TIMINGS["worker_setup"] = (time.time_ns() - t_setup0) / 1e9
        return TorchEstimator._train_loop(config, engine, start_epoch, device)

    @staticmethod
    def _detached_fused_engine(config, device):
        """The fused engine over the caller's own model and optimizer objects (read, never
        written: results come from the device buffers), which saves copying the model for the
        worker. Only for a fresh run of a fusable model with an optimizer instance, a loss
        instance and no LR scheduler; anything else takes the copying path."""
        model, opt, loss = config["model"], config["optimizer"], config["loss"]
        if not (isinstance(model, torch.nn.Module) and isinstance(opt, torch.optim.Optimizer)
                and isinstance(loss, TLoss)) or config["lr_scheduler_creator"] is not None \
                or session.get_checkpoint() is not None or device.type != "cuda":
            return None
        fused_mode = config.get("fused", None)
        if fused_mode is None:
            from raydp_amd.utils.config import get as conf_get
            fused_mode = conf_get("spark.ray.mi355x.fused")
        fused_mode = {True: "auto", False: "off"}.get(fused_mode, fused_mode)
        if fused_mode == "off":
            return None
        from raydp_amd.torch.engine import FusedMLPEngine
        from raydp_amd.utils import tracing
        metrics = config["metrics"].clone()
        with tracing.span("fused applicable", cat="train"):
            fused = FusedMLPEngine.applicable(model, opt, loss, metrics, device, config["batch_size"],
                                              config["feature_columns"], config["feature_types"])
        if fused is None:
            return None
        spec, lc, oc, acc_thr = fused
        try:
            return FusedMLPEngine(model, opt, spec, lc, oc, acc_thr, metrics, device, config, None,
                                  detached=True, loss=loss)
        except ValueError:
            if fused_mode == "on":
                raise
            return None     # a layout limit of the fused kernels (LDS, residency): torch loop

    @staticmethod
    def _train_loop(config, engine, start_epoch, device):
        from raydp_amd.utils import tracing
        train_ds = session.get_dataset_shard("train")
        eval_ds = session.get_dataset_shard("evaluate") if config["evaluate"] else None
        engine.epoch = start_epoch          # epoch permutations continue where the run left off
        t_wait0 = time.perf_counter()
        deferred = [ds for ds in (train_ds, eval_ds) if getattr(ds, "_pending", None) is not None]
        if deferred:   # fit_on_spark built this engine while the conversion stage ran
            with tracing.span("conversion wait", cat="train"):
                stream = getattr(train_ds, "_stream", None) if train_ds in deferred else None
                if stream is not None and hasattr(engine, "stream_ingest"):
                    # the blocks go to HBM as they land: only the last one's DMA is left after
                    with tracing.span("streamed ingest", cat="train"):
                        engine.stream_ingest(train_ds, config)
                    STREAM_STATS["blocks"] = len(getattr(engine, "_streamed", None) or ())
                for ds in deferred:
                    ds.num_blocks()
            LAST_TIMINGS["conversion_wait"] = time.perf_counter() - t_wait0
        t_load0 = time.perf_counter()
        with tracing.span("ingest", cat="train", engine=engine.name):
            engine.load(train_ds, eval_ds, config)
        LAST_TIMINGS["ingest"] = time.perf_counter() - t_load0
        t_train0 = time.perf_counter()
        config.setdefault("_engine_name", engine.name)
        timed = device.type == "cuda"
        ck_every = int(config.get("checkpoint_frequency") or 0)
        for epoch in range(start_epoch, config["num_epochs"]):
            if timed:   # device-timed epoch (HIP events; no per-step host sync)
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
            t_ep = time.perf_counter()
            with tracing.span("train epoch", cat="train", epoch=epoch):
                train_res, train_loss = engine.train_epoch()
            wall = time.perf_counter() - t_ep
            dev_s = None
            if timed:
                ev1.record()
                ev1.synchronize()
                dev_s = ev0.elapsed_time(ev1) / 1000.0
            rows = getattr(getattr(engine, "train", None), "n", None)
            perf = {}
            if rows:
                perf = {"train_rows": rows, "train_samples_per_s": rows / max(wall, 1e-9),
                        "train_epoch_wall_s": wall}
                if dev_s is not None:
                    perf["train_epoch_device_s"] = dev_s
                if getattr(engine, "last_step_times", None):
                    perf["step_time_us"] = engine.last_step_times    # device-timed, per step
            session.report(dict(epoch=epoch, train_res=train_res, train_loss=train_loss,
                                engine=engine.name, allreduce=getattr(engine, "allreduce_kind", None), **perf))
            if eval_ds is not None:
                with tracing.span("eval epoch", cat="train", epoch=epoch):
                    eval_res, test_loss = engine.evaluate_epoch()
                session.report(dict(epoch=epoch, eval_res=eval_res, test_loss=test_loss))
            if ck_every and (epoch + 1) % ck_every == 0 and epoch + 1 < config["num_epochs"]:
                with tracing.span("epoch checkpoint", cat="train", epoch=epoch):
                    _report_epoch_checkpoint(engine, epoch)
        LAST_TIMINGS["train"] = time.perf_counter() - t_train0
        t_ck0 = time.perf_counter()
        with tracing.span("checkpoint", cat="train"):
            states = engine.state_dict()
            states = {k: v.detach().cpu() for k, v in states.items()}
            if hasattr(engine, "close"):
                engine.close()
            checkpoint = None
            if session.get_world_rank() == 0:
                # model.pt is written straight into a staging dir of the run's storage and
                # renamed into place by report()
                stage = session.staging_dir()
                save_state_dict(states, os.path.join(stage, "model.pt"))
                checkpoint = Checkpoint(stage, movable=True)
            session.report({}, checkpoint=checkpoint)
        LAST_TIMINGS["checkpoint"] = time.perf_counter() - t_ck0

    # ------------------------------------------------------------------------- driver -----
    def fit(self, train_ds, evaluate_ds=None, max_retries=3) -> NoReturn:
        train_loop_config = {
            "model": self._model,
            "optimizer": self._optimizer,
            "loss": self._loss,
            "lr_scheduler_creator": self._lr_scheduler_creator,
            "feature_columns": self._feature_columns,
            "feature_types": self._feature_types,
            "label_column": self._label_column,
            "label_type": self._label_type,
            "batch_size": self._batch_size,
            "num_epochs": self._num_epochs,
            "drop_last": self._drop_last,
            "shuffle": self._shuffle,
            "evaluate": True,
            "metrics": self._metrics,
            "fused": self._extra_config.get("fused", None),
            "shuffle_seed": self._extra_config.get("shuffle_seed", None),
            # per-epoch checkpoints (model.pt + optim.pt) every N epochs; 0 = only the final
            # model.pt, as the reference
            "checkpoint_frequency": int(self._extra_config.get("checkpoint_frequency", 0) or 0),
            # the trainer splits the datasets into equal shards (every rank runs the same step
            # count without asking); SPMD ranks that bring their own rows agree once per fit
            "_equal_shards": not bool(self._extra_config.get("spmd_local_shards")),
        }
        use_gpu = self._extra_config.get("use_gpu")
        if self._resources_per_worker and "GPU" in self._resources_per_worker:
            use_gpu = self._resources_per_worker["GPU"] > 0
        scaling_config = ScalingConfig(num_workers=self._num_workers, use_gpu=use_gpu,
                                       resources_per_worker=self._resources_per_worker,
                                       placement_strategy=self._placement_strategy)
        run_config = RunConfig(failure_config=FailureConfig(max_failures=max_retries),
                               storage_path=self._extra_config.get("storage_path"))
        # The reference shuffles the dataset once before sharding (torch/estimator.py:335-338).
        # Both engines here draw a fresh device-side permutation of their whole resident shard
        # every epoch, so when every worker trains on all of its rows (one worker, or SPMD ranks
        # with local shards) the host-side pass adds nothing but a copy of the data; it stays
        # where it decides which rows land on which worker.
        local_only = self._num_workers == 1 or bool(self._extra_config.get("spmd_local_shards"))
        if self._shuffle and not local_only:
            seed = self._extra_config.get("shuffle_seed")
            train_ds = train_ds.random_shuffle(seed=seed)
            if evaluate_ds:
                evaluate_ds = evaluate_ds.random_shuffle(seed=seed)
        datasets = {"train": train_ds}
        if evaluate_ds is None:
            train_loop_config["evaluate"] = False
        else:
            datasets["evaluate"] = evaluate_ds
        # use_ccl: the reference swaps in oneCCL (torch/estimator.py:344-347); here TorchConfig
        # resolves "ccl" to RCCL on GPU workers and gloo on CPU workers
        torch_config = self._extra_config.get("torch_config")
        if torch_config is None and self._use_ccl:
            torch_config = TorchConfig(backend="ccl")
        from raydp_amd.utils import tracing
        tracing.instant("trainer start", cat="train")
        self._trainer = TorchTrainer(TorchEstimator.train_func,
                                     train_loop_config=train_loop_config,
                                     scaling_config=scaling_config,
                                     run_config=run_config,
                                     torch_config=torch_config,
                                     datasets=datasets,
                                     local_shards=bool(self._extra_config.get("spmd_local_shards")))
        self._trained_results = self._trainer.fit()
        return self._trained_results

    def fit_on_spark(self, train_df: DF, evaluate_df: OPTIONAL_DF = None, max_retries=3,
                     fs_directory: Optional[str] = None, compression: Optional[str] = None,
                     stop_spark_after_conversion=False):
        from raydp_amd.utils import tracing
        from raydp_amd.utils.config import get as conf_get
        t_conv0 = time.perf_counter()
        for k in ("conversion_wait", "etl_and_conversion_concurrent"):
            LAST_TIMINGS.pop(k, None)
        STREAM_STATS.clear()
        if fs_directory is None and not stop_spark_after_conversion \
                and conf_get("spark.ray.mi355x.overlap_conversion"):
            # The Spark stage that materialises the blocks runs on the executors while this
            # thread builds the training engine (device buffers, kernel load, parameter upload);
            # the engine awaits the blocks at ingest (Dataset.deferred). The engine build starts
            # once the driver-side stage work (plan, payload, dispatch) is done and the
            # conversion thread is blocked on the executors, and the GIL switch interval is
            # short meanwhile, so the two threads do not queue behind each other's Python.
            import sys
            import threading
            from raydp_amd.data.dataset import Dataset, DeferredDatasetError
            from raydp_amd.spark import cluster as spark_cluster
            in_flight = threading.Event()

            # one in-process worker: the training blocks stream into HBM as they land, while the
            # rest of the stage still runs (the engine's stream_ingest)
            stream = None
            if self._num_workers == 1 and conf_get("spark.ray.mi355x.stream_ingest") and \
                    conf_get("spark.ray.mi355x.train_inprocess"):
                import queue
                stream = queue.Queue()

            # N > 1 (spawned workers): the fit payload goes out FIRST and the stage after it; the
            # workers unpickle it and build their engines while the stage runs (their shards
            # follow when it is done), instead of starting only once the stage is dispatched
            early = self._num_workers > 1
            sent = threading.Event()

            def convert():
                if early:
                    sent.wait(30.0)     # (set by the trainer on every path; 30 s is a backstop)
                t0 = time.perf_counter()
                spark_cluster.set_dispatch_hook(in_flight.set)
                try:
                    with tracing.span("etl + conversion", cat="etl"):
                        out = self._convert_via_store(train_df, evaluate_df, None, stream=stream)
                finally:
                    spark_cluster.set_dispatch_hook(None)
                    in_flight.set()
                LAST_TIMINGS["etl_and_conversion_concurrent"] = time.perf_counter() - t0
                return out
            switch = sys.getswitchinterval()
            sys.setswitchinterval(min(switch, 2e-4))
            try:
                fut = _conversion_pool().submit(convert)
                # the short switch interval is only for the overlap: back to normal the moment
                # the conversion is done, not after the whole training run
                fut.add_done_callback(lambda _f: sys.setswitchinterval(switch))
                train_ds = Dataset.deferred(_Pick(fut, 0, sent.set))
                train_ds._stream = stream
                evaluate_ds = Dataset.deferred(_Pick(fut, 1, sent.set)) if evaluate_df is not None else None
                if not early:
                    in_flight.wait()
                LAST_TIMINGS["etl_and_conversion"] = time.perf_counter() - t_conv0
                from raydp_amd.train import trainer as _tr
                if early:
                    _tr.set_started_hook(sent.set)
                try:
                    return self.fit(train_ds, evaluate_ds, max_retries)
                except DeferredDatasetError as e:
                    raise e.original from None
                finally:
                    if early:
                        _tr.set_started_hook(None)
                        sent.set()     # (a fit that failed before its workers started)
                    cf_wait([fut])     # never leave a stage running behind a failed fit
            finally:
                sys.setswitchinterval(switch)
        with tracing.span("etl + conversion", cat="etl"):
            if fs_directory is None:
                from raydp_amd.spark.dataset import get_raydp_master_owner
                owner = get_raydp_master_owner(train_df.sparkSession) if stop_spark_after_conversion else None
                train_ds, evaluate_ds = self._convert_via_store(train_df, evaluate_df, owner)
            else:
                train_ds, evaluate_ds = self._convert_via_parquet(train_df, evaluate_df, fs_directory,
                                                                  compression)
        LAST_TIMINGS["etl_and_conversion"] = time.perf_counter() - t_conv0
        if stop_spark_after_conversion:
            from raydp_amd.context import stop_spark
            stop_spark(cleanup_data=False)
        return self.fit(train_ds, evaluate_ds, max_retries)

    def _convert_via_store(self, train_df, evaluate_df, owner, stream=None):
        from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
        super().fit_on_spark(train_df, evaluate_df)
        train_df = self._check_and_convert(train_df)
        if stream is not None:
            # every training partition, as its block lands: (partition, reference) into the stream
            from raydp_amd.runtime.objects import ObjectRef
            from raydp_amd.spark import cluster as spark_cluster

            def landed(i, oid, node_id, rows, ex_id):
                stream.put((i, ObjectRef(oid, owner=f"raydp-executor-{ex_id}", node_id=node_id)))
            spark_cluster.set_block_hook(landed)
        try:
            train_ds = spark_dataframe_to_ray_dataset(train_df, owner=owner)
        finally:
            if stream is not None:
                spark_cluster.set_block_hook(None)
                stream.put(None)        # end of the training blocks (the consumer blocks on get)
        evaluate_ds = None
        if evaluate_df is not None:
            evaluate_df = self._check_and_convert(evaluate_df)
            evaluate_ds = spark_dataframe_to_ray_dataset(evaluate_df, owner=owner)
        return train_ds, evaluate_ds

    def _convert_via_parquet(self, train_df, evaluate_df, fs_directory, compression):
        from raydp_amd.spark.dataset import read_spark_parquet
        super().fit_on_spark(train_df, evaluate_df)
        train_df = self._check_and_convert(train_df)
        evaluate_ds = None
        app_id = train_df.sparkSession.sparkContext.applicationId
        path = fs_directory.rstrip("/") + f"/{app_id}"
        train_df.write.parquet(path + "/train", compression=compression)
        train_ds = read_spark_parquet(path + "/train")
        if evaluate_df is not None:
            evaluate_df = self._check_and_convert(evaluate_df)
            evaluate_df.write.parquet(path + "/test", compression=compression)
            evaluate_ds = read_spark_parquet(path + "/test")
        return train_ds, evaluate_ds

    def get_model(self):
        assert self._trainer is not None, "Must call fit first"
        return TorchCheckpoint(self._trained_results.checkpoint.to_directory()).get_model(self._model)

    @property
    def results(self):
        return self._trained_results
