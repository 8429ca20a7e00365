"""``ray`` / ``pyspark`` import facades backed by this framework.

Installed (``sys.modules`` registration) only when the real package is NOT importable, so a
real Ray or PySpark is never shadowed. They let reference-era scripts such as
``examples/pytorch_nyctaxi.py`` (``ray.init``, ``ray.data.from_spark``,
``from pyspark.sql.functions import ...``) run unchanged on the MI355X engine.
"""
import importlib.util
import sys
import types


def _missing(name: str) -> bool:
    """True when no real ``name`` package is importable (our own facade does not count)."""
    if name in sys.modules:
        return bool(getattr(sys.modules[name], "__raydp_facade__", False))
    try:
        return importlib.util.find_spec(name) is None
    except (ImportError, ValueError):
        return True


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__raydp_facade__ = True
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def install_ray():
    if not _missing("ray"):
        return
    from raydp_amd import data, runtime, train
    from raydp_amd.runtime import api
    from raydp_amd.runtime.cluster_utils import Cluster
    pg = importlib.import_module("raydp_amd.runtime.pgroup")
    from raydp_amd.utils import get_node_ip_address
    ray = _mod("ray", init=runtime.init, shutdown=runtime.shutdown,
               is_initialized=runtime.is_initialized, get=runtime.get, put=runtime.put,
               wait=api.wait, remote=api.remote, get_actor=api.get_actor, kill=api.kill,
               get_runtime_context=runtime.get_runtime_context, ObjectRef=runtime.ObjectRef,
               nodes=api.nodes, cluster_resources=api.cluster_resources,
               available_resources=api.available_resources, method=api.method,
               __version__="2.50.0-raydp-amd")
    ray.data = data
    sys.modules["ray.data"] = data
    util = _mod("ray.util", placement_group=pg.placement_group,
                remove_placement_group=pg.remove_placement_group,
                placement_group_table=pg.placement_group_table,
                get_placement_group=pg.get_placement_group,
                get_node_ip_address=get_node_ip_address)
    ray.util = util
    util.placement_group = pg.placement_group
    pgm = _mod("ray.util.placement_group", placement_group=pg.placement_group,
               PlacementGroup=pg.PlacementGroup, remove_placement_group=pg.remove_placement_group,
               placement_group_table=pg.placement_group_table,
               get_placement_group=pg.get_placement_group)
    sched = _mod("ray.util.scheduling_strategies",
                 PlacementGroupSchedulingStrategy=api.PlacementGroupSchedulingStrategy,
                 NodeAffinitySchedulingStrategy=api.NodeAffinitySchedulingStrategy)
    util.scheduling_strategies = sched
    client = _mod("ray.util.client")
    client.ray = types.SimpleNamespace(is_connected=lambda: False)
    util.client = client
    state = importlib.import_module("raydp_amd.runtime.state")
    sys.modules["ray.util.state"] = state
    util.state = state
    from raydp_amd.runtime.actors import ActorDiedError
    exc = _mod("ray.exceptions", RayActorError=ActorDiedError, ActorDiedError=ActorDiedError,
               ObjectLostError=runtime.objects.ObjectLostError, RayTaskError=Exception)
    ray.exceptions = exc
    ray.actor = _mod("ray.actor", ActorHandle=api.ActorHandle, ActorClass=api.ActorClass)
    cu = _mod("ray.cluster_utils", Cluster=Cluster)
    ray.cluster_utils = cu
    ray.train = train
    sys.modules["ray.train"] = train
    from raydp_amd.train import trainer as _tr
    sys.modules["ray.train.torch"] = train.torch
    air = _mod("ray.air", session=importlib.import_module("raydp_amd.train.session"),
               ScalingConfig=train.ScalingConfig, RunConfig=train.RunConfig,
               FailureConfig=train.FailureConfig, CheckpointConfig=train.CheckpointConfig)
    ray.air = air
    _mod("ray.air.config", ScalingConfig=train.ScalingConfig, RunConfig=train.RunConfig,
         FailureConfig=train.FailureConfig, CheckpointConfig=train.CheckpointConfig)
    sys.modules["ray.air.session"] = importlib.import_module("raydp_amd.train.session")
    _mod("ray.job_config", JobConfig=api.JobConfig)
    hvd = importlib.import_module("raydp_amd.hvd")
    train.horovod = _mod("ray.train.horovod", HorovodTrainer=hvd.HorovodTrainer)
    from raydp_amd.train import legacy
    train.Trainer = legacy.Trainer
    train.TrainingCallback = legacy.TrainingCallback
    train.get_dataset_shard = importlib.import_module("raydp_amd.train.session").get_dataset_shard
    train.report = importlib.import_module("raydp_amd.train.session").report


def install_xgboost():
    """``xgboost`` / ``xgboost_ray`` facades over the native GBDT (only when absent)."""
    from raydp_amd.xgboost import gbdt, ray_api
    if _missing("xgboost"):
        _mod("xgboost", DMatrix=gbdt.DMatrix, Booster=gbdt.Booster, train=gbdt.train,
             __version__="2.0.0-raydp-amd")
    if _missing("xgboost_ray"):
        _mod("xgboost_ray", RayDMatrix=ray_api.RayDMatrix, RayParams=ray_api.RayParams, train=ray_api.train,
             predict=ray_api.predict)


def install_horovod():
    if not _missing("horovod"):
        return
    hvd = importlib.import_module("raydp_amd.hvd")
    top = _mod("horovod", __version__="0.28.1-raydp-amd")
    top.torch = hvd
    sys.modules["horovod.torch"] = hvd


def install_pyspark():
    if not _missing("pyspark"):
        return
    from raydp_amd import spark as S
    from raydp_amd.spark import functions, pandas as ps, types as T
    from raydp_amd.spark.dataframe import StorageLevel
    py = _mod("pyspark", StorageLevel=StorageLevel, SparkConf=S.SparkConf,
              __version__="3.5.0")
    sql = _mod("pyspark.sql", SparkSession=S.SparkSession, DataFrame=S.DataFrame, Column=S.Column,
               Row=S.Row, Window=S.Window, functions=functions, types=T)
    py.sql = sql
    sys.modules["pyspark.sql.functions"] = functions
    sys.modules["pyspark.sql.types"] = T
    _mod("pyspark.sql.window", Window=S.Window)
    _mod("pyspark.sql.dataframe", DataFrame=S.DataFrame)
    py.pandas = ps
    sys.modules["pyspark.pandas"] = ps
    _mod("pyspark.storagelevel", StorageLevel=StorageLevel)
    py.version = types.SimpleNamespace(__version__="3.5.0")


def install():
    install_ray()
    install_pyspark()
    install_horovod()
    install_xgboost()


class _LazyFacades:
    """Meta-path hook: install the facades the first time user code imports one of the
    faked top-level packages (keeps worker processes from importing torch at start-up)."""
    _names = {"ray", "pyspark", "horovod", "xgboost", "xgboost_ray"}

    def find_spec(self, fullname, path=None, target=None):
        if fullname.split(".")[0] in self._names:
            sys.meta_path[:] = [f for f in sys.meta_path if f is not self]
            install()
            if fullname in sys.modules:
                import importlib.machinery
                return importlib.machinery.ModuleSpec(fullname, _Preloaded(sys.modules[fullname]))
        return None


class _Preloaded:
    def __init__(self, mod):
        self.mod = mod

    def create_module(self, spec):
        return self.mod

    def exec_module(self, module):
        pass


def install_lazy():
    if not any(isinstance(f, _LazyFacades) for f in sys.meta_path):
        sys.meta_path.insert(0, _LazyFacades())
