"""Per-worker training session (``ray.air.session`` / ``ray.train`` context equivalent).

Reference use inside ``TorchEstimator.train_func``: ``session.get_dataset_shard("train")``,
``session.report(metrics, checkpoint=...)``, ``train.get_context().get_world_rank()``
(``python/raydp/torch/estimator.py:226-270``).
"""
import os
import shutil
import tempfile
import threading
import time
from typing import Any, Callable, Dict, Optional

from raydp_amd.train.checkpoint import Checkpoint

_tls = threading.local()


class TrainContext:
    def __init__(self, world_rank=0, world_size=1, local_rank=0, local_world_size=1, node_rank=0,
                 device=None, experiment_name="raydp", trial_dir=None):
        self.world_rank, self.world_size = world_rank, world_size
        self.local_rank, self.local_world_size = local_rank, local_world_size
        self.node_rank = node_rank
        self.device = device
        self.experiment_name = experiment_name
        self.trial_dir = trial_dir

    def get_world_rank(self):
        return self.world_rank

    def get_world_size(self):
        return self.world_size

    def get_local_rank(self):
        return self.local_rank

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_dir(self):
        return self.trial_dir


class _Session:
    def __init__(self, ctx: TrainContext, datasets: Dict[str, Any], reporter: Callable,
                 storage_dir: str, start_checkpoint: Optional[Checkpoint] = None):
        self.ctx, self.datasets, self.reporter = ctx, datasets, reporter
        self.storage_dir = storage_dir
        self.iteration = 0
        self.start = time.time()
        self.last = self.start
        self.start_checkpoint = start_checkpoint

    def report(self, metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None):
        now = time.time()
        self.iteration += 1
        m = dict(metrics)
        m.setdefault("_timestamp", int(now))
        m.setdefault("_time_this_iter_s", now - self.last)
        m.setdefault("_training_iteration", self.iteration)
        self.last = now
        persisted = None
        if checkpoint is not None:
            # persist immediately (the caller's directory may be a TemporaryDirectory), under a
            # name that sorts after every checkpoint of this run, restarted attempts included:
            # the trainer resumes a failed group from the newest one
            try:
                n = sum(1 for x in os.listdir(self.storage_dir) if x.startswith("checkpoint_"))
            except OSError:
                n = 0
            dst = os.path.join(self.storage_dir, f"checkpoint_{n:06d}")
            if getattr(checkpoint, "_movable", False) and \
                    os.path.dirname(checkpoint.path) == os.path.abspath(self.storage_dir):
                os.replace(checkpoint.path, dst)   # complete staging dir: one rename
            else:
                tmp = dst + f".tmp{os.getpid()}"
                if os.path.exists(tmp):
                    shutil.rmtree(tmp)
                shutil.copytree(checkpoint.path, tmp)
                os.replace(tmp, dst)          # a crash mid-copy never leaves a partial checkpoint
            persisted = dst
        self.reporter(self.ctx.world_rank, m, persisted)


def staging_dir() -> str:
    """A fresh directory inside the run's storage (same filesystem): a checkpoint written there
    and reported as ``Checkpoint(path, movable=True)`` is renamed into place, not copied."""
    s = _get_session()
    os.makedirs(s.storage_dir, exist_ok=True)
    return tempfile.mkdtemp(prefix=".stage_", dir=s.storage_dir)


def _set_session(s: Optional[_Session]):
    _tls.session = s


def _get_session() -> _Session:
    s = getattr(_tls, "session", None)
    if s is None:
        raise RuntimeError("not inside a training worker (no active train session)")
    return s


def report(metrics: Dict[str, Any], checkpoint: Optional[Checkpoint] = None):
    _get_session().report(metrics, checkpoint)


def get_dataset_shard(name: str = "train"):
    return _get_session().datasets.get(name)


def get_context() -> TrainContext:
    return _get_session().ctx


def get_world_rank() -> int:
    return get_context().world_rank


def get_world_size() -> int:
    return get_context().world_size


def get_local_rank() -> int:
    return get_context().local_rank


def get_checkpoint() -> Optional[Checkpoint]:
    return _get_session().start_checkpoint


def get_device():
    return get_context().device
