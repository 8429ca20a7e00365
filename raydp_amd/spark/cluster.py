"""Cluster backend of a Spark-on-runtime application (driver side).

Roles of the reference's JVM control plane collapsed into one driver-side object:
``RayCoarseGrainedSchedulerBackend`` (application registration, executor target count,
dynamic allocation: ``RayCoarseGrainedSchedulerBackend.scala:123-301``), the app master
(``RayAppMaster.scala``: executor lifecycle, restart id remap) and the ``ObjectStoreWriter``
recoverable-conversion entry points (``ObjectStoreWriter.scala:164-216``).

Executors are actor processes (``raydp_amd.spark.executor``) when the actor runtime can spawn
processes; the in-process mode (``spark.raydp.executor.mode=thread``) keeps everything in the
driver for unit tests.
"""
import logging
import threading
import time
import uuid
from typing import Dict, List, Optional

import pyarrow as pa

from raydp_amd.spark import plan as P

logger = logging.getLogger(__name__)


class ClusterBackend:
    def __init__(self, app_name: str, conf: Dict[str, str], master_resources: Dict[str, float]):
        self.app_name = app_name
        self.conf = conf
        self.master_resources = master_resources
        self.app_id = f"app-{time.strftime('%Y%m%d%H%M%S')}{int(time.time() * 1000) % 1000:03d}"
        self.num_executors = int(conf.get("spark.executor.instances", "1"))
        self.cores = int(conf.get("spark.executor.cores", "1"))
        self._sched: Optional[P.TaskScheduler] = None
        self._recoverable: Dict[str, object] = {}
        self._lock = threading.RLock()
        self._started = False

    # ---------------------------------------------------------------- lifecycle ----------
    def start(self):
        par = max(1, self.num_executors * self.cores)
        self._sched = P.TaskScheduler(par)
        self._started = True

    def master_url(self) -> str:
        from raydp_amd.utils import get_node_ip_address
        return f"ray://RAY_APP_MASTER@{get_node_ip_address()}:0"

    def scheduler(self) -> P.TaskScheduler:
        return self._sched

    def connect_driver(self):
        pass

    def stop(self, cleanup_data=True):
        if cleanup_data:
            with self._lock:
                self._recoverable.clear()

    # ---------------------------------------------------------------- conversion ---------
    def prepare_recoverable(self, df, storage_level):
        from raydp_amd.runtime import objects
        df.persist(storage_level)
        rdd_id = df._id
        with self._lock:
            self._recoverable[rdd_id] = df
        refs = []
        for i, t in enumerate(df._cached.tables):
            def lineage(df=df, i=i):
                if df._cached is None:
                    df.persist()
                return df._cached.tables[i]
            refs.append(objects.put(t.replace_schema_metadata(), _lineage=lineage))
        return rdd_id, refs

    def release_recoverable(self, rdd_id):
        with self._lock:
            df = self._recoverable.pop(rdd_id, None)
        if df is not None:
            df.unpersist()

    def is_persisted(self, rdd_id) -> bool:
        with self._lock:
            return rdd_id in self._recoverable
