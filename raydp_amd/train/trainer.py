"""Worker-group trainer (Ray Train ``TorchTrainer`` equivalent), one process per GPU.

``TorchTrainer.fit()`` runs ``train_loop_per_worker(config)`` on ``num_workers`` ranks joined
by ``torch.distributed`` — backend ``"nccl"`` (= RCCL over xGMI on ROCm) when the workers own
GPUs, Gloo otherwise — with datasets split into equal row shards (equal shards keep every rank
on the same step count, so collectives never deadlock). Three launch modes:

* **in-process** — ``num_workers == 1``: the loop runs in the caller (no fork cost; config
  ``spark.ray.mi355x.train_inprocess`` off sends it through one spawned worker, as Ray Train does).
* **SPMD** — the caller already is one rank of a ``torchrun`` job (``WORLD_SIZE`` env matches):
  every process runs its own rank in-process; this is how ``bench.py`` scales to 8 GPUs.
* **spawned** — otherwise ``num_workers`` child processes are started (spawn context), each
  pinned to ``cuda:<local_rank>`` when GPUs are used.

Failures restart the whole group up to ``FailureConfig.max_failures`` times (reference:
``RunConfig(failure_config=FailureConfig(max_failures=max_retries))`` at
``python/raydp/torch/estimator.py:334``), from the newest checkpoint rank 0 reported
(``session.get_checkpoint()`` in the restarted loop), like Ray Train. The process-group backend
comes from ``TorchConfig`` (``use_ccl`` in the estimator; RCCL on GPU, gloo on CPU).
"""
import os
import pickle
import shutil
import socket
import tempfile
import time
import traceback
import uuid
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from raydp_amd.train import session as S
from raydp_amd.train.checkpoint import Checkpoint
from raydp_amd.train.config import FailureConfig, RunConfig, ScalingConfig


class TrainingFailedError(RuntimeError):
    pass


@dataclass
class Result:
    metrics: Dict[str, Any]
    checkpoint: Optional[Checkpoint]
    path: str
    error: Optional[BaseException] = None
    metrics_history: List[Dict[str, Any]] = field(default_factory=list)
    restored_from: List[str] = field(default_factory=list)   # checkpoints earlier attempts resumed from

    @property
    def metrics_dataframe(self):
        import pandas as pd
        return pd.DataFrame(self.metrics_history)

    @property
    def best_checkpoints(self):
        return [(self.checkpoint, self.metrics)] if self.checkpoint else []


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cuda_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


import threading as _threading

_launch_hooks = _threading.local()


def set_started_hook(fn) -> None:
    """``fn()`` once (this thread's next ``fit``) when a warm spawned group with deferred datasets
    has sent every rank its fit -- or right away on any other path (cold group start, eager
    shards, in-process run), which needs the data first. ``fit_on_spark`` at N > 1 starts its
    conversion stage then, so the workers' payload unpickle and engine build run beside the
    stage instead of after its dispatch."""
    _launch_hooks.on_started = fn


def _fire_started() -> None:
    fn = getattr(_launch_hooks, "on_started", None)
    _launch_hooks.on_started = None
    if fn is not None:
        fn()


def _shard_payloads(datasets: Dict[str, Any], world: int) -> List[bytes]:
    """Every rank's pickled ``{name: shard}``: each dataset split ONCE (equal shards are block
    slices, a few ids each), plain pickle first (a shard holds importable classes only; cloudpickle
    costs ~4x more per call), cloudpickle for anything else."""
    import pickle
    import cloudpickle
    splits = {k: ds.split(world, equal=True) for k, ds in (datasets or {}).items()}
    out = []
    for r in range(world):
        d = {k: sp[r] for k, sp in splits.items()}
        try:
            out.append(pickle.dumps(d, protocol=5))
        except Exception:  # noqa: BLE001 - a dataset of user objects: cloudpickle handles closures
            out.append(cloudpickle.dumps(d))
    return out


def _shard(datasets: Dict[str, Any], rank: int, world: int) -> Dict[str, Any]:
    if not datasets:
        return {}
    out = {}
    for k, ds in datasets.items():
        out[k] = ds if world == 1 else ds.split(world, equal=True)[rank]
    return out


def _init_dist(backend: str, rank: int, world: int, addr: str, port: int, timeout_s: Optional[float] = None):
    import datetime
    import torch.distributed as dist
    if dist.is_initialized():
        return False
    kw = {"timeout": datetime.timedelta(seconds=float(timeout_s))} if timeout_s else {}
    dist.init_process_group(backend, init_method=f"tcp://{addr}:{port}", rank=rank,
                            world_size=world, **kw)
    return True


def _backend(torch_config, use_gpu: bool) -> str:
    """``TorchConfig`` (reference ``python/raydp/torch/config.py:12-45``; ``use_ccl`` asks for
    oneCCL there) -> the process-group backend: RCCL (``"nccl"``) on GPU workers, gloo on CPU."""
    if torch_config is not None:
        return torch_config.resolve(use_gpu)
    forced = os.environ.get("RAYDP_TRAIN_BACKEND")
    if forced:      # rehearsals: several GPU workers sharing one card cannot form an RCCL ring
        return forced
    return "nccl" if use_gpu else "gloo"


def _checkpoint_names(storage: str) -> List[str]:
    try:
        return sorted(n for n in os.listdir(storage) if n.startswith("checkpoint_") and ".tmp" not in n)
    except OSError:
        return []


def latest_checkpoint(storage: str, exclude=(), resumable_only: bool = False) -> Optional[str]:
    """Newest ``checkpoint_*`` directory under a run's storage path (reported by rank 0).

    ``exclude``: names that existed before this fit started (a reused ``RunConfig.name``);
    ``resumable_only``: only per-epoch checkpoints, which carry ``meta.json`` (the epoch they
    follow) -- the final ``model.pt`` of a finished attempt is not a point to resume from."""
    skip = set(exclude)
    for n in reversed(_checkpoint_names(storage)):
        if n in skip:
            continue
        path = os.path.join(storage, n)
        if resumable_only and not os.path.exists(os.path.join(path, "meta.json")):
            continue
        return path
    return None


def _worker_entry(rank, world, port, payload, queue):
    """Child-process entry of a spawned worker group."""
    import cloudpickle
    try:
        fn, config, shards, use_gpu, storage, name = cloudpickle.loads(payload)
        import torch
        device = torch.device("cpu")
        if use_gpu:
            n = torch.cuda.device_count()
            torch.cuda.set_device(rank % n)
            device = torch.device("cuda", rank % n)
        backend = "nccl" if use_gpu else "gloo"
        _init_dist(backend, rank, world, "127.0.0.1", port)

        def reporter(r, metrics, ckpt):
            queue.put(("report", r, metrics, ckpt))
        ctx = S.TrainContext(rank, world, rank, world, 0, device, name, storage)
        S._set_session(S._Session(ctx, shards, reporter, storage))
        from raydp_amd.train.gpu_policy import worker_policies
        with worker_policies(use_gpu):
            fn(config) if _accepts_arg(fn) else fn()
        queue.put(("done", rank, None, None))
    except BaseException as e:  # noqa: BLE001
        queue.put(("error", rank, traceback.format_exc(), None))
        raise
    finally:
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def _accepts_arg(fn) -> bool:
    import inspect
    try:
        return len(inspect.signature(fn).parameters) >= 1
    except (TypeError, ValueError):
        return True


class DataParallelTrainer:
    backend_default = "gloo"

    def __init__(self, train_loop_per_worker: Callable, *, train_loop_config: Optional[dict] = None,
                 scaling_config: Optional[ScalingConfig] = None, run_config: Optional[RunConfig] = None,
                 datasets: Optional[Dict[str, Any]] = None, torch_config=None,
                 resume_from_checkpoint: Optional[Checkpoint] = None,
                 local_shards: bool = False, **kw):
        self.fn = train_loop_per_worker
        self.config = train_loop_config or {}
        self.scaling = scaling_config or ScalingConfig()
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.torch_config = torch_config
        self.resume = resume_from_checkpoint
        # SPMD jobs (torchrun) may pass each rank's own data: do not split it again
        self.local_shards = local_shards

    # ------------------------------------------------------------------------------------
    def _use_gpu(self) -> bool:
        if self.scaling.use_gpu is not None:
            return bool(self.scaling.use_gpu) and _cuda_available()
        r = self.scaling.resources_per_worker or {}
        if "GPU" in r:
            return float(r["GPU"]) > 0 and _cuda_available()
        return _cuda_available()

    def _storage(self) -> str:
        base = self.run_config.storage_path or os.path.join(tempfile.gettempdir(), "raydp_results")
        if base.startswith("file://"):
            base = base[len("file://"):]
        # unique per fit: two fits started in the same second must never share checkpoints
        name = self.run_config.name or \
            f"TorchTrainer_{time.strftime('%Y-%m-%d_%H-%M-%S')}_{os.getpid()}_{uuid.uuid4().hex[:8]}"
        path = os.path.join(base, name)
        os.makedirs(path, exist_ok=True)
        return path

    def fit(self) -> Result:
        """Run the worker group; on a worker failure restart it, up to
        ``FailureConfig.max_failures`` times, from the newest checkpoint any attempt reported
        (Ray Train's ``FailureConfig`` semantics, reference ``torch/estimator.py:331-334``)."""
        failures = 0
        max_f = self.run_config.failure_config.max_failures
        storage = self._storage()
        preexisting = _checkpoint_names(storage)   # a reused RunConfig.name: not this fit's
        restored = []
        while True:
            try:
                res = self._fit_once(storage)
                res.restored_from = restored
                return res
            except _WorkerFailure as e:
                failures += 1
                if max_f >= 0 and failures > max_f:
                    raise TrainingFailedError(f"training failed after {failures} attempt(s):\n{e}") from None
                # only a per-epoch checkpoint this fit wrote (meta.json): never the final
                # model.pt of an attempt whose peer died afterwards, never an earlier fit's
                ck = latest_checkpoint(storage, exclude=preexisting, resumable_only=True)
                if ck is not None:
                    self.resume = Checkpoint(ck)
                    restored.append(ck)

    def _fit_once(self, storage: Optional[str] = None) -> Result:
        world = int(self.scaling.num_workers)
        storage = storage or self._storage()
        use_gpu = self._use_gpu()
        history: List[Dict[str, Any]] = []
        ckpts: List[str] = []

        def reporter(rank, metrics, ckpt):
            if rank == 0:
                history.append(metrics)
            if ckpt:
                ckpts.append(ckpt)

        env_world = int(os.environ.get("WORLD_SIZE", "1"))
        from raydp_amd.utils.config import get as conf_get
        inproc_one = world == 1 and bool(conf_get("spark.ray.mi355x.train_inprocess"))
        if inproc_one or (env_world == world and "RANK" in os.environ and world > 1):
            _fire_started()
            self._run_inprocess(world, env_world, use_gpu, storage, reporter)
        else:
            self._run_spawned(world, use_gpu, storage, reporter)
        ck = Checkpoint(ckpts[-1]) if ckpts else None
        return Result(metrics=history[-1] if history else {}, checkpoint=ck, path=storage,
                      metrics_history=history)

    def _run_inprocess(self, world, env_world, use_gpu, storage, reporter):
        import torch
        if world > 1:
            rank = int(os.environ["RANK"])
            local = int(os.environ.get("LOCAL_RANK", rank))
        else:
            rank, local = 0, 0
        device = torch.device("cpu")
        if use_gpu:
            n = torch.cuda.device_count()
            torch.cuda.set_device(local % n)
            device = torch.device("cuda", local % n)
        created = False
        if world > 1:
            import datetime
            import torch.distributed as dist
            if not dist.is_initialized():
                kw = {}
                if self.torch_config is not None and self.torch_config.timeout_s:
                    kw["timeout"] = datetime.timedelta(seconds=float(self.torch_config.timeout_s))
                dist.init_process_group(_backend(self.torch_config, use_gpu), **kw)
                created = True
        shards = dict(self.datasets) if self.local_shards else _shard(self.datasets, rank, world)
        ctx = S.TrainContext(rank, world, local, world, 0, device, "raydp", storage)
        sess = S._Session(ctx, shards, reporter, storage, self.resume)
        S._set_session(sess)
        from raydp_amd.data.dataset import DeferredDatasetError
        from raydp_amd.train.gpu_policy import worker_policies
        try:
            with worker_policies(use_gpu):
                self.fn(self.config) if _accepts_arg(self.fn) else self.fn()
        except DeferredDatasetError:
            raise     # the input failed to materialise: restarting the workers cannot fix it
        except Exception as e:  # noqa: BLE001
            raise _WorkerFailure(traceback.format_exc()) from e
        finally:
            S._set_session(None)
            if created:
                import torch.distributed as dist
                dist.destroy_process_group()

    def _deferred_datasets(self, world) -> bool:
        """Datasets still being produced (``Dataset.deferred``) that the ranks get split."""
        return world > 1 and not self.local_shards and bool(self.datasets) and any(
            getattr(ds, "_pending", None) is not None for ds in self.datasets.values())

    def _run_spawned(self, world, use_gpu, storage, reporter):
        """Worker group of ``world`` process actors (one per rank, GPUs assigned by the
        runtime), joined into one ``torch.distributed`` group (RCCL when they own GPUs).

        Ray Train starts fresh worker actors per fit, but Ray prestarts its worker processes,
        so that costs milliseconds there. Here an actor is a new Python process that imports
        torch and initialises HIP (seconds), so a group that finished a fit cleanly is kept
        warm -- process group, RCCL / xGMI communicators, loaded kernels -- and the next fit
        with the same shape reuses it (``_GROUPS``). A failed attempt kills its group."""
        import cloudpickle
        from raydp_amd import runtime
        res = dict(self.scaling.resources_per_worker or {})
        cpus = float(res.pop("CPU", 1))
        gpus = float(res.pop("GPU", 1 if use_gpu else 0)) if use_gpu else 0.0
        strategy = self.scaling.placement_strategy if isinstance(self.scaling.placement_strategy, str) else "PACK"
        from raydp_amd.utils.config import env_for_workers
        wenv = env_for_workers()   # spark.ray.mi355x.* settings of the driver's session
        backend = _backend(self.torch_config, use_gpu)
        tmo = self.torch_config.timeout_s if self.torch_config is not None else None
        # a warm group keeps the environment it was started with: the RAYDP_* variables (the
        # env-var form of the spark.ray.mi355x.* settings) are part of its identity
        renv = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("RAYDP_")))
        key = (world, use_gpu, cpus, gpus, tuple(sorted(res.items())), strategy, backend, tmo,
               tuple(sorted(wenv.items())) if wenv else (), renv)
        group = _GROUPS.take(key)
        if group is None or not self._deferred_datasets(world):
            _fire_started()     # a cold start (seconds) or eager shards: the conversion goes first
        if group is None:
            from raydp_amd.runtime.node import ResourceError
            try:
                group = _WorkerGroup.start(world, use_gpu, cpus, gpus, res, strategy, wenv, backend, tmo, storage)
            except ResourceError:
                # warm groups of other shapes hold their CPUs / GPUs: release them and retry
                if not len(_GROUPS):
                    raise
                _GROUPS.clear()
                group = _WorkerGroup.start(world, use_gpu, cpus, gpus, res, strategy, wenv, backend, tmo, storage)
        ok = False
        try:
            workers = group.workers
            refs = []
            from raydp_amd.utils import tracing
            # the loop, its config (model, optimizer, ...) and the resume point are the same for
            # every rank: pickled once, not once per worker (~2 ms each for the NYC model)
            with tracing.span("pickle fit payload", cat="train", world=world):
                from raydp_amd.runtime import serialization as S
                try:
                    # the runtime pickler: CPU tensors as raw storage bytes (not a torch.save
                    # per storage), large Arrow tables by store reference
                    common = S.dumps((self.fn, self.config, self.resume, storage), transfer=False)
                except ValueError:
                    common = cloudpickle.dumps((self.fn, self.config, self.resume, storage))
            conv_error = None
            if self._deferred_datasets(world):
                # fit_on_spark's conversion stage is still running on the executors: start every
                # rank now (payload unpickle, engine build, kernel load, parameter upload) and send
                # each its shard the moment the stage is done -- the same overlap the in-process
                # N = 1 path gets from a deferred Dataset
                chan = uuid.uuid4().hex
                names = list(self.datasets)
                for w in workers:
                    refs.append(w.run.remote(common, None, chan, names))
                _fire_started()     # every rank has its fit: the caller may start the conversion now
                try:
                    with tracing.span("shard split", cat="train", world=world):
                        payloads = _shard_payloads(self.datasets, world)
                    for r, w in enumerate(workers):
                        w.deliver_shards.remote(chan, payloads[r])
                except Exception as e:  # noqa: BLE001 - the conversion failed: stop every rank
                    conv_error = e
                    blob = cloudpickle.dumps(RuntimeError(f"dataset conversion failed: {e!r}"))
                    for w in workers:
                        w.deliver_shards.remote(chan, None, blob)
            else:
                for r, w in enumerate(workers):
                    shards = _shard(self.datasets, r, world)
                    refs.append(w.run.remote(common, cloudpickle.dumps(shards)))
            # wait on all ranks at once: when one dies, its peers are blocked in a collective
            # that will never complete -- fail the attempt at the first error (the group is
            # killed below) instead of waiting on rank 0 forever
            outs, error = [None] * world, None
            pending = list(refs)
            while pending and error is None:
                ready, pending = runtime.wait(pending, num_returns=1)
                for ref in ready:
                    try:
                        outs[refs.index(ref)] = runtime.get(ref)
                    except Exception:  # noqa: BLE001 - a rank failed (user error or lost process)
                        error = traceback.format_exc()
                        break
            if conv_error is not None:
                # the input failed, not the workers: no group restart can fix it (the ranks have
                # all returned by now: their shards resolved to the same failure)
                for ref in pending:
                    try:
                        runtime.get(ref)
                    except Exception:  # noqa: BLE001
                        pass
                raise conv_error
            if error is not None:
                raise _WorkerFailure(error)
            for r, reports in enumerate(outs):
                for metrics, ckpt in reports:
                    reporter(r, metrics, ckpt)
            ok = True
        finally:
            if ok and _GROUPS.enabled():
                _GROUPS.put(key, group)
            else:
                group.kill()


class _WorkerGroup:
    """``world`` live ``_TrainWorker`` actors joined in one process group, plus their
    placement group."""

    def __init__(self, workers, pg):
        self.workers, self.pg = workers, pg
        from raydp_amd.runtime import core
        self.node = core.current_node()

    @classmethod
    def start(cls, world, use_gpu, cpus, gpus, res, strategy, wenv, backend, tmo, storage):
        from raydp_amd import runtime
        from raydp_amd.runtime import pgroup
        bundle = {"CPU": cpus}
        if gpus:
            bundle["GPU"] = gpus
        bundle.update(res)
        pg = pgroup.placement_group([dict(bundle) for _ in range(world)], strategy=strategy)
        port = _free_port()
        actor = runtime.remote(_TrainWorker)
        workers = []
        try:
            for r in range(world):
                opts = {"num_cpus": cpus, "num_gpus": gpus, "placement_group": pg,
                        "placement_group_bundle_index": r, "max_concurrency": 2}
                if wenv:
                    opts["runtime_env"] = {"env_vars": dict(wenv)}
                if res:
                    opts["resources"] = res
                workers.append(actor.options(**opts).remote(r, world, storage, use_gpu))
            # Like Ray Train's shared CUDA_VISIBLE_DEVICES: every worker of a node sees all of
            # that node's worker GPUs and binds its own device, so RCCL and the xGMI one-shot
            # path can map peer memory (a worker that saw only its own GPU could not)
            layout = _local_layout(workers)
            runtime.get([w.setup.remote("127.0.0.1", port, *layout[r], backend=backend, timeout_s=tmo)
                         for r, w in enumerate(workers)])
        except BaseException:
            cls(workers, pg).kill()
            raise
        return cls(workers, pg)

    def alive(self) -> bool:
        from raydp_amd.runtime import core
        return core.current_node() is self.node and all(
            not getattr(getattr(w, "_impl", None), "dead", True) for w in self.workers)

    def kill(self):
        from raydp_amd import runtime
        from raydp_amd.runtime import pgroup
        for w in self.workers:
            try:
                runtime.kill(w, no_restart=True)
            except Exception:  # noqa: BLE001
                pass
        try:
            pgroup.remove_placement_group(self.pg)
        except Exception:  # noqa: BLE001
            pass
        self.workers = []


class _GroupPool:
    """Warm worker groups keyed by their shape (at most one per key)."""

    def __init__(self):
        self._groups: Dict[Any, _WorkerGroup] = {}

    @staticmethod
    def enabled() -> bool:
        return os.environ.get("RAYDP_TRAIN_REUSE_WORKERS", "1") != "0"

    def take(self, key) -> Optional[_WorkerGroup]:
        g = self._groups.pop(key, None)
        if g is not None and not g.alive():
            g.kill()
            g = None
        return g

    def put(self, key, group: _WorkerGroup):
        old = self._groups.pop(key, None)
        if old is not None and old is not group:
            old.kill()
        self._groups[key] = group

    def clear(self):
        groups, self._groups = list(self._groups.values()), {}
        for g in groups:
            g.kill()

    def __len__(self):
        return len(self._groups)


_GROUPS = _GroupPool()


def release_worker_groups():
    """Stop the warm training worker groups (``runtime.shutdown`` does this too)."""
    _GROUPS.clear()


def _local_layout(workers):
    """Per worker: (visible GPU ids of its node, local rank, local world size, node rank,
    device index). The local rank is the worker's position among its node's workers -- unique
    even when several workers share one GPU (fractional GPUs) -- and the device index is its
    GPU's position in the node's visible list."""
    nodes, order = {}, []
    for w in workers:
        impl = getattr(w, "_impl", None)
        vn = getattr(impl, "vnode", None)
        node = vn.node_id if vn is not None else "head"
        if node not in nodes:
            nodes[node] = []
            order.append(node)
        nodes[node].append(w)
    out = []
    for w in workers:
        impl = getattr(w, "_impl", None)
        vn = getattr(impl, "vnode", None)
        node = vn.node_id if vn is not None else "head"
        peers = nodes[node]
        gpus = sorted({g for p in peers for g in (getattr(getattr(p, "_impl", None), "gpu_ids", None) or [])})
        mine = getattr(impl, "gpu_ids", None) or []
        local = peers.index(w)
        dev = gpus.index(mine[0]) if mine and mine[0] in gpus else local
        out.append((gpus or None, local, len(peers), order.index(node), dev))
    return out


class _TrainWorker:
    """One rank of a spawned worker group (a process actor). Stays alive between fits while
    its group is warm; its process group is torn down with the process."""

    def __init__(self, rank: int, world: int, storage: str, use_gpu: bool):
        import threading
        self.rank, self.world, self.storage, self.use_gpu = rank, world, storage, use_gpu
        self.local_rank, self.local_world, self.node_rank = 0, 1, rank
        self._chans: Dict[str, Any] = {}          # shard deliveries of deferred fits, by channel
        self._closed: List[str] = []              # channels whose fit already returned
        self._chan_lock = threading.Lock()

    def _chan(self, chan: str):
        import concurrent.futures as cf
        with self._chan_lock:
            return self._chans.setdefault(chan, cf.Future())

    def deliver_shards(self, chan: str, payload: Optional[bytes], error: Optional[bytes] = None) -> bool:
        """The shards of a fit started with deferred datasets (runs beside ``run`` on the
        actor's second thread): ``{name: Dataset}`` pickled, or the conversion's failure."""
        import concurrent.futures as cf
        import cloudpickle
        with self._chan_lock:
            # checked and created in ONE critical section: a fit ending in between must not leave
            # a channel behind that nothing will ever remove
            if chan in self._closed:     # the fit failed before its shards came: nothing waits
                return False
            fut = self._chans.setdefault(chan, cf.Future())
        if error is not None:
            fut.set_exception(cloudpickle.loads(error))
        else:
            fut.set_result(cloudpickle.loads(payload))
        return True

    def setup(self, addr: str, port: int, visible=None, local_rank: int = 0, local_world: int = 1,
              node_rank: int = 0, device_index: Optional[int] = None, backend: Optional[str] = None,
              timeout_s: Optional[float] = None):
        if visible and self.use_gpu:
            # before the first HIP call of this process: the node's worker GPUs, in order
            os.environ["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in visible)
            os.environ.pop("CUDA_VISIBLE_DEVICES", None)
        import torch
        self.local_rank, self.local_world, self.node_rank = local_rank, local_world, node_rank
        self.device = torch.device("cpu")
        if self.use_gpu and torch.cuda.is_available():
            dev = (local_rank if device_index is None else device_index) % max(1, torch.cuda.device_count())
            torch.cuda.set_device(dev)
            self.device = torch.device("cuda", dev)
        os.environ.update({"RANK": str(self.rank), "WORLD_SIZE": str(self.world),
                           "LOCAL_RANK": str(local_rank), "LOCAL_WORLD_SIZE": str(local_world),
                           "MASTER_ADDR": addr, "MASTER_PORT": str(port)})
        if backend is None or (backend == "nccl" and self.device.type != "cuda"):
            backend = "nccl" if self.device.type == "cuda" else "gloo"
        if backend == "nccl":
            import datetime
            import torch.distributed as dist
            kw = {"timeout": datetime.timedelta(seconds=float(timeout_s))} if timeout_s else {}
            # device_id: RCCL binds its communicator now (no lazy init inside the first step)
            dist.init_process_group(backend, init_method=f"tcp://{addr}:{port}", rank=self.rank,
                                    world_size=self.world, device_id=self.device, **kw)
        else:
            _init_dist(backend, self.rank, self.world, addr, port, timeout_s)
        return True

    def run(self, common: bytes, shard_payload: Optional[bytes], chan: Optional[str] = None,
            names: Optional[List[str]] = None):
        import cloudpickle
        from raydp_amd.utils import tracing
        with tracing.span("unpickle fit payload", cat="train", rank=self.rank):
            fn, config, resume, storage = cloudpickle.loads(common)
            if shard_payload is None and chan is not None:
                # deferred: the shards arrive through deliver_shards while the loop builds its engine
                from raydp_amd.data.dataset import Dataset
                fut = self._chan(chan)
                shards = {n: Dataset.deferred(_ShardOf(fut, n)) for n in names or []}
            else:
                shards = cloudpickle.loads(shard_payload)
        try:
            return self._run_loop(fn, config, resume, storage, shards)
        finally:
            if chan is not None:
                with self._chan_lock:
                    self._chans.pop(chan, None)
                    self._closed = (self._closed + [chan])[-32:]

    def _run_loop(self, fn, config, resume, storage, shards):
        self.storage = storage
        reports = []

        def reporter(r, metrics, ckpt):
            reports.append((metrics, ckpt))
        ctx = S.TrainContext(self.rank, self.world, self.local_rank, self.local_world, self.node_rank,
                             self.device, "raydp", self.storage)
        S._set_session(S._Session(ctx, shards, reporter, self.storage, resume))
        try:
            fn(config) if _accepts_arg(fn) else fn()
        finally:
            S._set_session(None)
        return reports


class _ShardOf:
    """Future-like view of one named shard of a delivery future's ``{name: Dataset}``."""

    def __init__(self, fut, name):
        self.fut, self.name = fut, name

    def result(self):
        return self.fut.result()[self.name]


class _WorkerFailure(Exception):
    pass


class TorchTrainer(DataParallelTrainer):
    pass


def prepare_model(model, move_to_device=True, parallel_strategy="ddp"):
    """``ray.train.torch.prepare_model``: move to the worker device, wrap in DDP if world>1."""
    import torch
    import torch.distributed as dist
    ctx = S.get_context()
    dev = ctx.device or torch.device("cpu")
    if move_to_device:
        model = model.to(dev)
    if ctx.world_size > 1 and dist.is_initialized():
        from raydp_amd.parallel.ddp import DistributedDataParallel
        model = DistributedDataParallel(model)
    elif dev.type == "cuda" and move_to_device:
        from raydp_amd.utils import config as C
        if C.get("spark.ray.mi355x.graph_user_model"):
            from raydp_amd.train.gpu_policy import graph_model
            model = graph_model(model)     # one GPU worker: training forward/backward as HIP graphs
    return model
