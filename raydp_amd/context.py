"""Global Spark-on-runtime context: ``init_spark`` / ``stop_spark``.

Parity: ``python/raydp/context.py`` — same signature (``app_name, num_executors,
executor_cores, executor_memory, enable_hive, fault_tolerant_mode, placement_group_strategy,
placement_group, placement_group_bundle_indexes, configs``), a process-global singleton under an
``RLock`` (second init raises ``"The spark environment has inited."``), placement-group
creation per strategy with one ``{CPU: cores, memory}`` bundle per executor, the
``spark.ray.placement_group`` / ``spark.ray.bundle_indexes`` confs, ``stop(cleanup_data)``
semantics (the master survives ``cleanup_data=False`` so converted data stays reachable) and an
``atexit`` hook.
"""
import atexit
from contextlib import ContextDecorator
from threading import RLock
from typing import Dict, List, Optional, Union

from raydp_amd.utils import parse_memory_size


class _SparkContext(ContextDecorator):
    _PLACEMENT_GROUP_CONF = "spark.ray.placement_group"
    _BUNDLE_INDEXES_CONF = "spark.ray.bundle_indexes"

    def __init__(self, app_name: str, num_executors: int, executor_cores: int,
                 executor_memory: Union[str, int], enable_hive: bool, fault_tolerant_mode: bool,
                 placement_group_strategy: Optional[str], placement_group,
                 placement_group_bundle_indexes: Optional[List[int]],
                 configs: Optional[Dict[str, str]] = None):
        self._app_name = app_name
        self._num_executors = num_executors
        self._executor_cores = executor_cores
        self._executor_memory = executor_memory
        self._enable_hive = enable_hive
        self._fault_tolerant_mode = fault_tolerant_mode
        self._placement_group_strategy = placement_group_strategy
        self._placement_group = placement_group
        self._placement_group_bundle_indexes = placement_group_bundle_indexes
        self._configs = {} if configs is None else dict(configs)
        self._spark_cluster = None
        self._spark_session = None

    def _get_or_create_spark_cluster(self):
        if self._spark_cluster is not None:
            return self._spark_cluster
        from raydp_amd.spark.ray_cluster import SparkCluster
        self._spark_cluster = SparkCluster(self._app_name, self._num_executors, self._executor_cores,
                                           self._executor_memory, self._enable_hive, self._configs)
        return self._spark_cluster

    def _prepare_placement_group(self):
        from raydp_amd.runtime import pgroup as pgmod
        if self._placement_group_strategy is not None:
            memory = parse_memory_size(self._executor_memory) \
                if isinstance(self._executor_memory, str) else self._executor_memory
            bundles = [{"CPU": self._executor_cores, "memory": memory}
                       for _ in range(self._num_executors)]
            pg = pgmod.placement_group(bundles, strategy=self._placement_group_strategy)
            pg.wait()
            self._placement_group = pg
            self._placement_group_bundle_indexes = None
        if self._placement_group is not None:
            self._configs[self._PLACEMENT_GROUP_CONF] = self._placement_group.id.hex()
            idx = list(range(self._placement_group.bundle_count)) \
                if self._placement_group_bundle_indexes is None else self._placement_group_bundle_indexes
            self._configs[self._BUNDLE_INDEXES_CONF] = ",".join(map(str, idx))

    def get_or_create_session(self):
        if self._spark_session is not None:
            return self._spark_session
        self._prepare_placement_group()
        cluster = self._get_or_create_spark_cluster()
        self._spark_session = cluster.get_spark_session()
        if self._fault_tolerant_mode:
            cluster.connect_spark_driver_to_ray()
        return self._spark_session

    def stop(self, cleanup_data=True):
        if self._spark_session is not None:
            self._spark_session.stop()
            self._spark_session = None
        if self._spark_cluster is not None:
            self._spark_cluster.stop(cleanup_data)
            if cleanup_data:
                self._spark_cluster = None
        if self._placement_group_strategy is not None:
            if self._placement_group is not None:
                from raydp_amd.runtime import pgroup as pgmod
                pgmod.remove_placement_group(self._placement_group)
                self._placement_group = None
            self._placement_group_strategy = None
        self._configs = None

    def __enter__(self):
        self.get_or_create_session()

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.stop()


_spark_context_lock = RLock()
_global_spark_context: Optional[_SparkContext] = None


def init_spark(app_name: str, num_executors: int, executor_cores: int,
               executor_memory: Union[str, int], enable_hive: bool = False,
               fault_tolerant_mode=True, placement_group_strategy: Optional[str] = None,
               placement_group=None, placement_group_bundle_indexes: Optional[List[int]] = None,
               configs: Optional[Dict[str, str]] = None):
    """Start executors as actor processes and return a ``SparkSession`` bound to them."""
    from raydp_amd import runtime
    if not runtime.is_initialized():
        runtime.init()
    with _spark_context_lock:
        global _global_spark_context
        if _global_spark_context is None:
            try:
                _global_spark_context = _SparkContext(
                    app_name, num_executors, executor_cores, executor_memory, enable_hive,
                    fault_tolerant_mode, placement_group_strategy, placement_group,
                    placement_group_bundle_indexes, configs)
                session = _global_spark_context.get_or_create_session()
                _freeze_driver_heap()
                return session
            except BaseException:
                if _global_spark_context is not None:
                    _global_spark_context.stop()
                _global_spark_context = None
                raise
        else:
            raise Exception("The spark environment has inited.")


def _freeze_driver_heap():
    """Everything alive once the session is up -- imported modules, the runtime, the executors'
    handles -- lives as long as the driver: out of the collector's reach it costs nothing in the
    full collections that otherwise walk it at random points of the user's job
    (``spark.ray.mi355x.driver_gc_freeze``)."""
    global _gc_frozen
    from raydp_amd.utils.config import get as conf_get
    if conf_get("spark.ray.mi355x.driver_gc_freeze"):
        from raydp_amd.utils.gcmeter import freeze_long_lived
        freeze_long_lived()
        _gc_frozen = True


_gc_frozen = False


def _unfreeze_driver_heap():
    """stop_spark: the frozen objects go back to the oldest generation, so whatever of them the
    stopped session leaves unreachable is reclaimed (repeated init/stop in one process would
    otherwise keep every session's garbage)."""
    global _gc_frozen
    if _gc_frozen:
        import gc
        gc.unfreeze()
        _gc_frozen = False


def stop_spark(cleanup_data=True):
    with _spark_context_lock:
        global _global_spark_context
        if _global_spark_context is not None:
            try:
                _global_spark_context.stop(cleanup_data)
            finally:
                if cleanup_data is True:
                    _global_spark_context = None
                    _unfreeze_driver_heap()


atexit.register(stop_spark)
