"""``TFEstimator`` (reference: ``python/raydp/tf/estimator.py:41-310``)."""
import json
import os
from typing import Any, Dict, List, Optional, Union

from raydp_amd.estimator import EstimatorInterface
from raydp_amd.spark.interfaces import DF, OPTIONAL_DF, SparkEstimatorInterface


def _require_tf():
    try:
        import tensorflow as tf  # noqa: F401
        return tf
    except ImportError as e:
        raise ImportError("TFEstimator needs TensorFlow, which is not installed in this environment; "
                          "use raydp_amd.torch.TorchEstimator (PyTorch-ROCm) instead") from e


class TFEstimator(EstimatorInterface, SparkEstimatorInterface):
    def __init__(self, num_workers: int = 1, resources_per_worker: Optional[Dict[str, float]] = None,
                 model=None, optimizer: Union[Any, str] = None, loss: Union[Any, str] = None,
                 metrics: Union[List[Any], List[str]] = None, feature_columns: Union[str, List[str]] = None,
                 label_columns: Union[str, List[str]] = None, merge_feature_columns: bool = False,
                 batch_size: int = 128, drop_last: bool = False, num_epochs: int = 1, shuffle: bool = True,
                 callbacks: Optional[List[Any]] = None, **extra_config):
        tf = _require_tf()
        keras = tf.keras
        assert model is not None, "model must be not be None"
        if not isinstance(model, keras.Model):
            raise Exception("Unsupported parameter, we only support tensorflow.keras.Model")
        assert optimizer is not None, "optimizer must not be None"
        assert loss is not None, "loss must not be None"
        self._num_workers = num_workers
        self._resources_per_worker = resources_per_worker
        self._serialized_model = model.to_json()
        self._optimizer = optimizer if isinstance(optimizer, str) else keras.optimizers.serialize(optimizer)
        self._loss = loss if isinstance(loss, str) else keras.losses.serialize(loss)
        self._metrics = [m if isinstance(m, str) else keras.metrics.serialize(m) for m in (metrics or [])]
        self._feature_columns = [feature_columns] if isinstance(feature_columns, str) else feature_columns
        self._label_columns = [label_columns] if isinstance(label_columns, str) else label_columns
        self._merge_feature_columns = merge_feature_columns
        self._batch_size = batch_size
        self._drop_last = drop_last
        self._num_epochs = num_epochs
        self._shuffle = shuffle
        self._callbacks = callbacks
        self._extra_config = extra_config
        self._results = None

    @staticmethod
    def build_and_compile_model(config):
        tf = _require_tf()
        keras = tf.keras
        model = keras.models.model_from_json(config["model"])
        opt = config["optimizer"]
        opt = opt if isinstance(opt, str) else keras.optimizers.deserialize(opt)
        loss = config["loss"]
        loss = loss if isinstance(loss, str) else keras.losses.deserialize(loss)
        metrics = [m if isinstance(m, str) else keras.metrics.deserialize(m) for m in config["metrics"]]
        model.compile(optimizer=opt, loss=loss, metrics=metrics)
        return model

    @staticmethod
    def train_func(config):
        tf = _require_tf()
        from raydp_amd.train import session
        strategy = tf.distribute.MultiWorkerMirroredStrategy()
        with strategy.scope():
            model = TFEstimator.build_and_compile_model(config)

        def to_tf(ds):
            feats, labels = config["feature_columns"], config["label_columns"]
            t = ds.to_arrow() if hasattr(ds, "to_arrow") else ds
            x = {c: t.column(c).to_numpy() for c in feats}
            if config["merge_feature_columns"]:
                import numpy as np
                x = np.stack([x[c] for c in feats], axis=1)
            y = t.column(labels[0]).to_numpy()
            d = tf.data.Dataset.from_tensor_slices((x, y))
            if config["shuffle"]:
                d = d.shuffle(10000)
            return d.batch(config["batch_size"], drop_remainder=config["drop_last"])

        train = to_tf(session.get_dataset_shard("train"))
        ev = session.get_dataset_shard("evaluate")
        hist = model.fit(train, epochs=config["num_epochs"], callbacks=config["callbacks"], verbose=0)
        out = {k: float(v[-1]) for k, v in hist.history.items()}
        if ev is not None:
            out.update({f"eval_{k}": float(v) for k, v in zip(model.metrics_names, model.evaluate(to_tf(ev),
                                                                                                    verbose=0))})
        ckpt = os.path.join(session.get_context().get_trial_dir(), "tf_model")
        model.save(ckpt)
        session.report(out, checkpoint=ckpt)

    def fit(self, train_ds, evaluate_ds=None, max_retries=3):
        from raydp_amd.train import FailureConfig, RunConfig, ScalingConfig
        from raydp_amd.train.trainer import DataParallelTrainer
        config = {"model": self._serialized_model, "optimizer": self._optimizer, "loss": self._loss,
                  "metrics": self._metrics, "feature_columns": self._feature_columns,
                  "label_columns": self._label_columns, "merge_feature_columns": self._merge_feature_columns,
                  "batch_size": self._batch_size, "drop_last": self._drop_last, "num_epochs": self._num_epochs,
                  "shuffle": self._shuffle, "callbacks": self._callbacks}
        config.update(self._extra_config)
        datasets = {"train": train_ds}
        if evaluate_ds is not None:
            datasets["evaluate"] = evaluate_ds
        trainer = DataParallelTrainer(TFEstimator.train_func, train_loop_config=config,
                                      scaling_config=ScalingConfig(num_workers=self._num_workers,
                                                                   resources_per_worker=self._resources_per_worker),
                                      run_config=RunConfig(failure_config=FailureConfig(max_failures=max_retries)),
                                      datasets=datasets)
        self._results = trainer.fit()
        return self._results

    def fit_on_spark(self, train_df: DF, evaluate_df: OPTIONAL_DF = None, fs_directory: Optional[str] = None,
                     compression: Optional[str] = None, max_retries=3, stop_spark_after_conversion=False):
        from raydp_amd.spark.dataset import _convert_for_estimator
        train_ds, evaluate_ds = _convert_for_estimator(self, train_df, evaluate_df, fs_directory, compression,
                                                       stop_spark_after_conversion)
        return self.fit(train_ds, evaluate_ds, max_retries)

    def get_model(self) -> Any:
        tf = _require_tf()
        assert self._results is not None, "Must call fit first"
        return tf.keras.models.load_model(os.path.join(self._results.checkpoint.path, "tf_model"))


_ = json  # keep the import for config serialisation helpers of user code
