"""Executor actor process (reference: ``RayDPExecutor.scala`` + ``ObjectStoreWriter``).

One ``RayDPExecutor`` runs per executor as a supervised process actor named
``raydp-executor-<app>-<id>``. It executes stage tasks shipped by the driver
(``ExecutorTaskScheduler``): a task is ``(payload, partition_index)`` where ``payload`` is the
cloudpickled per-partition function of the stage (cached by digest, so a stage is
deserialised once per executor). Partition outputs travel back through the node's shared
object store (``raydp_amd.runtime.serialization``), never through the driver's heap.

``persist_partitions`` is the recoverable-conversion half of ``ObjectStoreWriter.
prepareRecoverableRDD`` + ``getRDDPartition`` (``RayDPExecutor.scala:312-355``): the partition
is computed and sealed into the executor node's store under a stable id; the driver turns
those ids into ``ObjectRef``s whose lineage recomputes a lost partition. ``block_locations``
/ ``unpersist`` back ``getBlockLocations`` and ``release_spark_recoverable``.
"""
import hashlib
import os
import threading
from typing import Dict, List, Tuple


class RayDPExecutor:
    def __init__(self, executor_id: str, app_id: str, cores: int, conf: Dict[str, str]):
        self.executor_id = executor_id
        self.app_id = app_id
        self.cores = cores
        self.conf = dict(conf)
        # the session's spark.ray.mi355x.* settings (e.g. fused_etl) reach executor-side code
        # through the environment, as they reach trainer workers
        import os
        from raydp_amd.utils.config import env_for_workers
        os.environ.update(env_for_workers(self.conf))
        self._fns: Dict[str, object] = {}
        self._fn_order: List[str] = []
        self._lock = threading.Lock()
        self._cache: Dict[Tuple[str, int], str] = {}   # (rdd_id, partition) -> store object id
        self.tasks_run = 0
        from raydp_amd.runtime import core
        self._node = core.current_node()
        self._warm_up()
        self.registration = None
        sock = self.conf.get("spark.ray.appmaster.socket")
        if sock:
            # registerToAppMaster (+ RequestAddPendingRestartedExecutor after a restart):
            # the master answers with the id this process now runs as
            from raydp_amd.spark import shuffle
            from raydp_amd.spark.appmaster import ExecutorRegistration
            restarted = int(os.environ.get("RAYDP_ACTOR_RESTART_COUNT", "0")) > 0
            self.registration = ExecutorRegistration(sock, executor_id, self._node.store.node_id, restarted)
            self.spark_executor_id = self.registration.executor_id
            shuffle.set_local_service(self.registration.shuffle_socket)
        else:
            self.spark_executor_id = executor_id

    @staticmethod
    def _warm_up():
        """Import the task-side engine and load the native kernels while the executor starts
        (executors start in parallel), so the first stage does not pay for it."""
        import numpy as np
        import pyarrow as pa
        import pyarrow.compute  # noqa: F401
        import pyarrow.csv  # noqa: F401
        from raydp_amd.spark import functions, sources, wide  # noqa: F401
        from raydp_amd.spark.plan import hash_columns
        hash_columns(pa.table({"k": np.arange(4)}), ["k"])

    # ------------------------------------------------------------------ info ------------
    def ping(self):
        return True

    def info(self):
        from raydp_amd.utils import get_node_ip_address
        return {"executor_id": self.executor_id, "pid": os.getpid(), "node_id": self._node.store.node_id,
                "ip": get_node_ip_address(), "cores": self.cores, "tasks_run": self.tasks_run,
                "restart_count": int(os.environ.get("RAYDP_ACTOR_RESTART_COUNT", "0")),
                "spark_executor_id": self.spark_executor_id,
                "shuffle_service": self.registration.shuffle_socket if self.registration else None}

    # ------------------------------------------------------------------ tasks -----------
    def _fn(self, payload):
        """Stage function from a store key ``(node_id, path, oid)`` (or raw pickled bytes)."""
        if isinstance(payload, (bytes, bytearray)):
            key = hashlib.blake2b(payload, digest_size=16).hexdigest()
        else:
            key = payload[2]
        with self._lock:
            fn = self._fns.get(key)
        if fn is None:
            from raydp_amd.runtime import serialization as S
            if isinstance(payload, (bytes, bytearray)):
                fn = S.loads(payload)
            else:
                from raydp_amd.runtime import core
                st = core.store_for(payload[0], payload[1])
                buf = st.get_buffer(payload[2]) if st is not None else None
                if buf is None:
                    raise RuntimeError("stage payload missing from the object store")
                fn = S.loads(memoryview(buf))
            with self._lock:
                self._fns[key] = fn
                self._fn_order.append(key)
                while len(self._fn_order) > 16:
                    self._fns.pop(self._fn_order.pop(0), None)
        return fn

    def run_task(self, payload: bytes, index: int):
        fn = self._fn(payload)
        from raydp_amd.spark.plan import _PartitionScope
        from raydp_amd.utils import tracing
        with tracing.span("task", cat="executor", partition=index), _PartitionScope(index):
            out = fn(index)
        self.tasks_run += 1
        return out

    def persist_partitions(self, payload: bytes, rdd_id: str, indices: List[int]):
        """Compute ``indices`` and seal them in this node's store; returns
        ``[(index, object_id, node_id, store_path, num_rows)]``."""
        import pyarrow as pa
        from raydp_amd.utils import tracing
        with tracing.span("stage unpickle", cat="executor"):
            fn = self._fn(payload)
        st = self._node.store
        out = []
        for i in indices:
            with tracing.span("task", cat="executor", partition=i, persist=rdd_id):
                t = fn(i)
            if not isinstance(t, pa.Table):
                raise TypeError(f"stage produced {type(t)} for a persisted partition")
            t = t.replace_schema_metadata()
            oid = hashlib.blake2b(f"{rdd_id}:{i}".encode(), digest_size=16).hexdigest()
            with self._lock:
                old = self._cache.pop((rdd_id, i), None)
            if old is not None or st.contains(oid):
                st.delete(oid)
            with tracing.span("store put", cat="executor", rows=t.num_rows):
                st.put(oid, t)
            with self._lock:
                self._cache[(rdd_id, i)] = oid
            out.append((i, oid, st.node_id, st.path, t.num_rows))
            self.tasks_run += 1
        return out

    def get_rdd_partition(self, rdd_id: str, index: int):
        with self._lock:
            oid = self._cache.get((rdd_id, index))
        if oid is None:
            # requestRecacheRDD (RayDPExecutor.scala:289-310): the driver agent re-materialises
            if self.registration is not None:
                self.registration.recache(rdd_id)
            return None
        found, t = self._node.store.get(oid)
        return t if found else None

    def block_locations(self, rdd_id: str) -> Dict[int, str]:
        with self._lock:
            return {i: self.executor_id for (r, i) in self._cache if r == rdd_id}

    def unpersist(self, rdd_id: str) -> int:
        st = self._node.store
        with self._lock:
            keys = [k for k in self._cache if k[0] == rdd_id]
            oids = [self._cache.pop(k) for k in keys]
        for o in oids:
            st.delete(o)
        return len(oids)

    def stop(self):
        for rdd in {k[0] for k in list(self._cache)}:
            self.unpersist(rdd)
        return True
