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

The task loop and the block cache are native (``csrc/exec/executor.cc`` through
``raydp_amd/spark/native_exec.py``): a persisted stage whose operators all lower to the
expression VM runs partition by partition on the C++ worker pool (CSV split or Arrow stream ->
VM segments -> Arrow IPC straight into the store), with the Python UDF checks called back
through the bridge; other stages, and any partition the native path hands back, run here in
Python. ``spark.ray.mi355x.native_executor=0`` keeps every stage on the Python path.
"""
import hashlib
import os
import threading
from typing import Dict, List


class RayDPExecutor:
    def __init__(self, executor_id: str, app_id: str, cores: int, conf: Dict[str, str]):
        self.executor_id = executor_id
        self.app_id = app_id
        self.cores = cores
        self.conf = dict(conf)
        self._size_thread_pools(cores)
        # the session's spark.ray.mi355x.* settings (e.g. fused_etl) reach executor-side code
        # through the environment, as they reach trainer workers
        import os
        from raydp_amd.utils.config import env_for_workers
        os.environ.update(env_for_workers(self.conf))
        self._fns: Dict[str, object] = {}
        self._fn_order: List[str] = []
        self._lock = threading.Lock()
        # native task loop (one worker per core) + the (rdd_id, partition) -> object id cache
        from raydp_amd.spark import native_exec
        self._native = native_exec.make_executor(max(1, int(cores)))
        self.tasks_run = 0
        self.native_tasks = 0
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
    def _size_thread_pools(cores) -> int:
        """An executor computes with ``spark.executor.cores`` cores, as a Spark executor does:
        Arrow's CPU pool would otherwise start one thread per CPU the host shows (256 on an
        MI355X node) in every executor, and a node of executors oversubscribes the cores it
        was given (on a CPU-quota'd host the whole job then stalls on throttling)."""
        import pyarrow as pa
        if os.environ.get("RAYDP_EXECUTOR_SIZE_POOLS", "1") == "0":     # escape hatch / A-B
            return pa.cpu_count()
        n = max(1, int(cores))
        pa.set_cpu_count(n)
        return n

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
                "shuffle_service": self.registration.shuffle_socket if self.registration else None,
                "native_tasks": self.native_tasks, "native_loop": self._native.stats()}

    # ------------------------------------------------------------------ tasks -----------
    @staticmethod
    def _key(payload) -> str:
        if isinstance(payload, (bytes, bytearray)):
            return hashlib.blake2b(payload, digest_size=16).hexdigest()
        return payload[2]

    def _fn(self, payload):
        """Stage function from a store key ``(node_id, path, oid)`` (or raw pickled bytes)."""
        key = self._key(payload)
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

    def _lower(self, fn):
        """The stage's native form (``native_exec.lower``, cached on the stage's plan) or None."""
        from raydp_amd.spark import native_exec
        if not native_exec.enabled() or not self._native.available:
            return None
        try:
            return native_exec.lower(fn)
        except Exception:  # noqa: BLE001 - lowering is an optimisation: the Python path runs
            return None

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
        from raydp_amd.utils import tracing
        with tracing.span("stage unpickle", cat="executor"):
            fn = self._fn(payload)
        st = self._node.store
        low = self._lower(fn)
        oids = {}
        for i in indices:
            oid = hashlib.blake2b(f"{rdd_id}:{i}".encode(), digest_size=16).hexdigest()
            old = self._native.cache_pop(rdd_id, i)
            if old is not None or st.contains(oid):
                st.delete(oid)
            oids[i] = oid
        rows: Dict[int, int] = {}
        if low is not None:
            # every partition of this call goes onto the native worker pool at once
            with tracing.span("native tasks", cat="executor", tasks=len(indices), persist=rdd_id):
                sub = []
                waited = set()
                try:
                    for i in indices:
                        tid, keep = self._native.submit(low, i, st, oids[i])
                        sub.append((i, tid, keep))
                    self._wait_native(sub, waited, rows)
                finally:
                    # never leave a submitted task running behind a failed submit / wait: it would
                    # keep writing the same object ids the retried partition is about to create
                    for _i, tid, _keep in sub:
                        if tid >= 0 and tid not in waited:
                            try:
                                self._native.wait(tid)
                            except Exception:  # noqa: BLE001 - draining only; the first error propagates
                                pass
        out = []
        for i in indices:
            oid = oids[i]
            if i in rows:
                self.native_tasks += 1
            else:
                rows[i] = self._persist_python(fn, i, st, oid, rdd_id)
            self._native.cache_put(rdd_id, i, oid)
            out.append((i, oid, st.node_id, st.path, rows[i]))
            self.tasks_run += 1
        return out

    def _wait_native(self, sub, waited, rows):
        from raydp_amd.spark import native_exec
        for i, tid, keep in sub:
            if tid < 0:
                continue
            status, n, _, err = self._native.wait(tid)
            waited.add(tid)
            if status == native_exec.OK:
                rows[i] = n
                native_exec.STATS["native_tasks"] += 1
                continue
            # FALLBACK / RETRY (a UDF was retired) / ERROR (e.g. the store is full):
            # the Python path computes the partition and raises its own error if any
            kind = {native_exec.RETRY: "native_retries", native_exec.ERROR: "native_errors"}
            native_exec.STATS[kind.get(status, "native_fallbacks")] += 1
            if status == native_exec.ERROR:
                native_exec.LAST_ERROR[0] = err

    def _persist_python(self, fn, i, st, oid, rdd_id) -> int:
        import pyarrow as pa
        from raydp_amd.utils import tracing
        with tracing.span("task", cat="executor", partition=i, persist=rdd_id):
            t = fn(i)
        if not isinstance(t, pa.Table):
            raise TypeError(f"stage produced {type(t)} for a persisted partition")
        t = t.replace_schema_metadata()
        if st.contains(oid):
            st.delete(oid)
        with tracing.span("store put", cat="executor", rows=t.num_rows):
            st.put(oid, t)
        return t.num_rows

    def get_rdd_partition(self, rdd_id: str, index: int):
        oid = self._native.cache_get(rdd_id, index)
        if oid is None:
            # requestRecacheRDD (RayDPExecutor.scala:289-310): the driver agent re-materialises
            if self.registration is not None:
                self.registration.recache(rdd_id)
            return None
        found, t = self._node.store.get(oid)
        return t if found else None

    def block_locations(self, rdd_id: str) -> Dict[int, str]:
        return {i: self.executor_id for i in self._native.cache_list(rdd_id)}

    def unpersist(self, rdd_id: str) -> int:
        return self._native.cache_unpersist(rdd_id, self._node.store)

    def stop(self):
        self._native.cache_unpersist(None, self._node.store)
        return True
