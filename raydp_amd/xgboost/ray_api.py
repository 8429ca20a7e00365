"""``xgboost_ray``-compatible entry points (``RayDMatrix``, ``RayParams``, ``train``,
``predict``) over the native histogram GBDT (reference usage: ``examples/xgboost_ray_nyctaxi.py``).

``train`` shards the dataset over ``num_actors`` workers of our data-parallel trainer; each
worker builds its histograms locally and the per-level histograms are all-reduced
(torch.distributed), which is xgboost-ray's Rabit all-reduce.
"""
import os
import tempfile
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

from raydp_amd.xgboost.gbdt import Booster, DMatrix


@dataclass
class RayParams:
    num_actors: int = 1
    cpus_per_actor: int = 1
    gpus_per_actor: int = 0
    max_actor_restarts: int = 0
    elastic_training: bool = False
    resources_per_actor: Optional[Dict[str, float]] = None


class RayDMatrix:
    """A (runtime) Dataset / Arrow table / pandas frame plus the label column name."""

    def __init__(self, data, label: Optional[str] = None, feature_names: Optional[List[str]] = None, **kw):
        self.data, self.label, self.feature_names = data, label, feature_names

    def _table(self):
        import pandas as pd
        import pyarrow as pa
        d = self.data
        if hasattr(d, "to_arrow"):
            return d.to_arrow()
        if isinstance(d, pd.DataFrame):
            return pa.Table.from_pandas(d, preserve_index=False)
        return d

    def shards(self, n: int):
        d = self.data
        if hasattr(d, "split"):
            return d.split(n, equal=False)
        t = self._table()
        from raydp_amd.data.dataset import from_arrow
        return from_arrow(t).split(n, equal=False)


def _dm_from(ds, label, feature_names=None) -> DMatrix:
    import numpy as np
    t = ds.to_arrow() if hasattr(ds, "to_arrow") else ds
    feats = feature_names or [c for c in t.column_names if c != label]
    x = np.stack([t.column(c).to_numpy(zero_copy_only=False).astype(np.float32) for c in feats], axis=1)
    y = t.column(label).to_numpy(zero_copy_only=False).astype(np.float32) if label else None
    return DMatrix(x, y, feature_names=feats)


def train(params: Dict, dtrain: RayDMatrix, num_boost_round: int = 10,
          evals: Sequence[Tuple[RayDMatrix, str]] = (), evals_result: Optional[Dict] = None,
          ray_params: Optional[RayParams] = None, verbose_eval: bool = False, **kw) -> Booster:
    from raydp_amd.train import FailureConfig, RunConfig, ScalingConfig, session
    from raydp_amd.train.checkpoint import Checkpoint
    from raydp_amd.train.trainer import DataParallelTrainer
    from raydp_amd.xgboost import gbdt
    rp = ray_params or RayParams()
    n = max(1, int(rp.num_actors))
    datasets = {"train": dtrain.data}
    names = ["train"]
    for i, (dm, name) in enumerate(evals):
        datasets[f"eval{i}"] = dm.data
        names.append(name)
    label = dtrain.label
    feature_names = dtrain.feature_names

    def loop(cfg):
        dtr = _dm_from(session.get_dataset_shard("train"), label, feature_names)
        ev = [(_dm_from(session.get_dataset_shard(f"eval{i}"), label, dtr.feature_names), names[i + 1])
              for i in range(len(names) - 1)]
        res: Dict = {}
        bst = gbdt.train(params, dtr, num_boost_round, evals=ev, evals_result=res, verbose_eval=verbose_eval,
                         device="cpu")
        ck = None
        if session.get_world_rank() == 0:
            d = tempfile.mkdtemp(prefix="raydp_xgb_")
            bst.save_model(os.path.join(d, "model.json"))
            ck = Checkpoint(d)
        session.report({"evals_result": res}, checkpoint=ck)

    trainer = DataParallelTrainer(loop, scaling_config=ScalingConfig(num_workers=n, use_gpu=False),
                                  run_config=RunConfig(failure_config=FailureConfig(max_failures=rp.max_actor_restarts)),
                                  datasets=datasets)
    result = trainer.fit()
    if evals_result is not None:
        evals_result.update(result.metrics.get("evals_result", {}))
    return Booster(model_file=os.path.join(result.checkpoint.path, "model.json"))


def predict(model: Booster, data: RayDMatrix, ray_params: Optional[RayParams] = None, **kw):
    t = data._table()
    dm = _dm_from(t, data.label if data.label in t.column_names else None, model.feature_names)
    return model.predict(dm)
