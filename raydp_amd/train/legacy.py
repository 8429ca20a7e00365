"""Ray Train 1.x ``Trainer`` API (``Trainer(backend="torch", num_workers)``, ``start`` /
``run(train_func, config, callbacks, dataset)`` / ``shutdown``, ``TrainingCallback``), used by
the reference's ``examples/raytrain_nyctaxi.py``; runs on :class:`DataParallelTrainer`."""
from typing import Callable, Dict, List, Optional


class TrainingCallback:
    def start_training(self, logdir: str = "", **info):
        pass

    def handle_result(self, results: List[Dict], **info):
        pass

    def finish_training(self, error: bool = False, **info):
        pass


class Trainer:
    def __init__(self, backend: str = "torch", num_workers: int = 1, use_gpu: bool = False,
                 resources_per_worker: Optional[Dict[str, float]] = None, **kw):
        if backend not in ("torch", "horovod"):
            raise ValueError(f"unsupported backend {backend!r}")
        self.backend, self.num_workers, self.use_gpu = backend, num_workers, use_gpu
        self.resources = resources_per_worker
        self._started = False

    def start(self):
        self._started = True

    def run(self, train_func: Callable, config: Optional[Dict] = None,
            callbacks: Optional[List[TrainingCallback]] = None, dataset=None, checkpoint=None):
        from raydp_amd.train import ScalingConfig
        from raydp_amd.train.trainer import DataParallelTrainer
        if not self._started:
            raise RuntimeError("call Trainer.start() first")
        datasets = dataset if isinstance(dataset, dict) else ({"train": dataset} if dataset is not None else {})
        callbacks = callbacks or []
        for cb in callbacks:
            cb.start_training()
        t = DataParallelTrainer(train_func, train_loop_config=config or {},
                                scaling_config=ScalingConfig(num_workers=self.num_workers, use_gpu=self.use_gpu,
                                                             resources_per_worker=self.resources),
                                datasets=datasets)
        error = False
        try:
            res = t.fit()
            for m in res.metrics_history:
                for cb in callbacks:
                    cb.handle_result([m])
            return [res.metrics]
        except BaseException:
            error = True
            raise
        finally:
            for cb in callbacks:
                cb.finish_training(error=error)

    def shutdown(self):
        self._started = False
