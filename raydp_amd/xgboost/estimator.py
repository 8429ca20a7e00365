"""``XGBoostEstimator`` (reference: ``python/raydp/xgboost/estimator.py:29-119``).

Same constructor / ``fit`` / ``fit_on_spark`` / ``get_model`` surface. The reference hands the
datasets to xgboost-ray's ``XGBoostTrainer`` (Rabit all-reduce between workers); here each
worker of our data-parallel trainer boosts with :mod:`raydp_amd.xgboost.gbdt`, all-reducing
gradient histograms over ``torch.distributed`` (gloo on CPU, RCCL when the workers own GPUs).
Rank 0 checkpoints the booster as ``model.json`` every round (checkpoint_frequency=1,
num_to_keep=1 in the reference's ``RunConfig``).
"""
import os
import tempfile
from typing import Dict, NoReturn, Optional

from raydp_amd.estimator import EstimatorInterface
from raydp_amd.spark.interfaces import DF, OPTIONAL_DF, SparkEstimatorInterface
from raydp_amd.xgboost.gbdt import Booster, DMatrix, train

MODEL_FILE = "model.json"


def _to_dmatrix(ds, label_column: str) -> DMatrix:
    import numpy as np
    t = ds.to_arrow() if hasattr(ds, "to_arrow") else ds
    feats = [c for c in t.column_names if c != label_column]
    x = np.stack([t.column(c).to_numpy(zero_copy_only=False).astype(np.float32) for c in feats], axis=1) \
        if feats else np.zeros((t.num_rows, 0), np.float32)
    y = t.column(label_column).to_numpy(zero_copy_only=False).astype(np.float32)
    return DMatrix(x, y, feature_names=feats)


def _train_loop(config):
    from raydp_amd.train import session
    from raydp_amd.train.checkpoint import Checkpoint
    dtrain = _to_dmatrix(session.get_dataset_shard("train"), config["label_column"])
    ev = session.get_dataset_shard("evaluate")
    evals = [(dtrain, "train")]
    if ev is not None:
        evals.append((_to_dmatrix(ev, config["label_column"]), "evaluate"))
    rank = session.get_world_rank()
    params = dict(config["params"])
    rounds = int(params.pop("num_boost_round", config.get("num_boost_round", 10)))
    ckdir = tempfile.mkdtemp(prefix="raydp_xgb_")

    def on_round(rnd, bst, res):
        metrics = {f"{name}-{m}": vals[-1] for name, d in res.items() for m, vals in d.items()}
        metrics["device"] = dev                     # "cuda": histograms ran on the gfx950 kernel
        ck = None
        if rank == 0:
            bst.save_model(os.path.join(ckdir, MODEL_FILE))
            ck = Checkpoint(ckdir)
        session.report(metrics, checkpoint=ck)

    dev = "cuda" if session.get_device().type == "cuda" else "cpu"
    train(params, dtrain, rounds, evals=evals, device=dev, callback=on_round)


class XGBoostEstimator(EstimatorInterface, SparkEstimatorInterface):
    def __init__(self, xgboost_params: Dict, label_column: str, num_workers: int = 1,
                 resources_per_worker: Optional[Dict[str, float]] = None, shuffle: bool = True):
        self._xgboost_params = dict(xgboost_params or {})
        self._label_column = label_column
        self._num_workers = num_workers
        self._resources_per_worker = resources_per_worker
        self._shuffle = shuffle
        self._results = None

    def fit(self, train_ds, evaluate_ds=None, max_retries=3) -> NoReturn:
        from raydp_amd.train import CheckpointConfig, FailureConfig, RunConfig, ScalingConfig
        from raydp_amd.train.trainer import DataParallelTrainer
        if self._shuffle:
            train_ds = train_ds.random_shuffle()
            if evaluate_ds is not None:
                evaluate_ds = evaluate_ds.random_shuffle()
        datasets = {"train": train_ds}
        if evaluate_ds is not None:
            datasets["evaluate"] = evaluate_ds
        res = dict(self._resources_per_worker or {})
        scaling = ScalingConfig(num_workers=self._num_workers, resources_per_worker=res,
                                use_gpu=float(res.get("GPU", 0)) > 0)
        run = RunConfig(checkpoint_config=CheckpointConfig(num_to_keep=1, checkpoint_frequency=1),
                        failure_config=FailureConfig(max_failures=max_retries))
        trainer = DataParallelTrainer(_train_loop, train_loop_config={"params": self._xgboost_params,
                                                                      "label_column": self._label_column},
                                      scaling_config=scaling, run_config=run, datasets=datasets)
        self._results = trainer.fit()
        return self._results

    def fit_on_spark(self, train_df: DF, evaluate_df: OPTIONAL_DF = None, max_retries=3,
                     fs_directory: Optional[str] = None, compression: Optional[str] = None,
                     stop_spark_after_conversion=False):
        from raydp_amd.spark.dataset import _convert_for_estimator
        train_ds, evaluate_ds = _convert_for_estimator(self, train_df, evaluate_df, fs_directory, compression,
                                                       stop_spark_after_conversion, parallelism=self._num_workers)
        return self.fit(train_ds, evaluate_ds, max_retries)

    def get_model(self) -> Booster:
        assert self._results is not None and self._results.checkpoint is not None, "Must call fit first"
        return Booster(model_file=os.path.join(self._results.checkpoint.path, MODEL_FILE))

    @property
    def results(self):
        return self._results
