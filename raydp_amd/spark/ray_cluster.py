"""``SparkCluster``: sets up the Spark application on the actor runtime.

Parity: ``python/raydp/spark/ray_cluster.py`` (``_prepare_spark_configs`` :115-189,
``_set_up_master`` :54-78, ``get_spark_session`` :191-201, ``stop`` :203-210). The master
actor and its executor actors are provided by ``raydp_amd.spark.cluster`` (native app master +
executor processes); the returned session schedules its tasks on those executors.
"""
import logging
from typing import Any, Dict, Optional

from raydp_amd.services import Cluster
from raydp_amd.utils import get_node_ip_address, parse_memory_size

logger = logging.getLogger(__name__)

RAYDP_SPARK_MASTER_SUFFIX = "_SPARK_MASTER"
SPARK_RAY_MASTER_RESOURCE_PREFIX = "spark.ray.raydp_spark_master.actor.resource."
SPARK_RAY_MASTER_RESOURCE_PREFIX_DEPRECATED = "spark.ray.raydp_spark_master.resource."


class SparkCluster(Cluster):
    """The ``Cluster`` of a Spark application (reference ``ray_cluster.py:34``): the master is
    the native app master + driver-side backend, workers are executor actors."""

    def __init__(self, app_name: str, num_executors: int, executor_cores: int,
                 executor_memory: Any, enable_hive: bool, configs: Optional[Dict[str, str]] = None):
        super().__init__(None)
        self._app_name = app_name
        self._num_executors = num_executors
        self._executor_cores = executor_cores
        self._executor_memory = executor_memory
        self._enable_hive = enable_hive
        self._configs = dict(configs or {})
        self._prepare_spark_configs()
        self._backend = None
        self._set_up_master()
        self._spark_session = None

    def _prepare_spark_configs(self):
        c = self._configs
        c["spark.executor.instances"] = str(self._num_executors)
        c["spark.executor.cores"] = str(self._executor_cores)
        c["spark.executor.memory"] = str(self._executor_memory)
        ip = get_node_ip_address()
        c.setdefault("spark.driver.host", ip)
        c.setdefault("spark.driver.bindAddress", ip)
        c["spark.app.name"] = self._app_name
        if c.get("spark.dynamicAllocation.enabled", "false").lower() == "true" and \
                "spark.dynamicAllocation.maxExecutors" not in c:
            logger.warning("spark.dynamicAllocation.enabled is true but "
                           "spark.dynamicAllocation.maxExecutors is not set; the number of "
                           "executors will be limited by the cluster resources")
        for k in list(c):
            if k.endswith("extraJavaOptions") or k.endswith("extraClassPath") or \
                    k in ("spark.javaagent", "spark.preferClassPath", "spark.ray.preferClassPath"):
                logger.debug("JVM-only config %s is accepted and ignored", k)

    def _master_resources(self) -> Dict[str, float]:
        res = {}
        for prefix in (SPARK_RAY_MASTER_RESOURCE_PREFIX_DEPRECATED, SPARK_RAY_MASTER_RESOURCE_PREFIX):
            for k, v in self._configs.items():
                if k.startswith(prefix):
                    name = k[len(prefix):]
                    val = parse_memory_size(v) if name == "memory" else float(v)
                    res["CPU" if name.lower() == "cpu" else name] = val
        return res

    def _set_up_master(self, resources: Optional[Dict[str, float]] = None, kwargs=None):
        from raydp_amd.spark.cluster import ClusterBackend
        self._backend = ClusterBackend(self._app_name, self._configs, resources or self._master_resources())
        self._backend.start()

    def _set_up_worker(self, resources: Dict[str, float], kwargs: Dict[str, str]):
        """One more executor actor, through the app master's dynamic-allocation path (the
        reference raises "Unsupported operation" here)."""
        cur = len(self._backend.alive_executors())
        if not self._backend.request_total_executors(cur + 1):
            raise RuntimeError("the app master refused another executor (spark.dynamicAllocation.maxExecutors?)")
        self._num_nodes += 1

    def get_cluster_url(self) -> str:
        return self._backend.master_url()

    def connect_spark_driver_to_ray(self):
        self._backend.connect_driver()

    def get_spark_session(self):
        if self._spark_session is not None:
            return self._spark_session
        from raydp_amd.spark.session import SparkSession
        conf = dict(self._configs)
        conf["spark.master"] = self.get_cluster_url()
        if self._enable_hive:
            conf["spark.sql.catalogImplementation"] = "hive"
        s = SparkSession(conf, scheduler=self._backend.scheduler(), cluster=self._backend)
        SparkSession._set_active(s)
        self._spark_session = s
        return s

    def stop(self, cleanup_data=True):
        if self._spark_session is not None:
            self._spark_session.stop()
            self._spark_session = None
        if self._backend is not None:
            self._backend.stop(cleanup_data)
            if cleanup_data:
                self._backend = None
