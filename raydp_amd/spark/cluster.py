"""Cluster backend of a Spark-on-runtime application (driver side).

Roles of the reference's JVM control plane, collapsed into one driver-side object:

* **app master** (``RayAppMaster.scala``): launches executor actors with their resources
  (``spark.ray.raydp_spark_executor.actor.resource.*``, the legacy
  ``spark.ray.actor.resource.cpu``, ``spark.executor.memory``), spreads them round-robin over
  the placement-group bundles named by ``spark.ray.placement_group`` /
  ``spark.ray.bundle_indexes`` (``RayAppMaster.scala:116-128,341-349``), restarts them without
  limit (``RayExecutorUtils.java:58``) and answers dynamic-allocation requests
  (``requestTotalExecutors`` / ``killExecutors``: ``RayCoarseGrainedSchedulerBackend.scala:
  278-301``);
* **scheduler backend**: ``ExecutorTaskScheduler`` ships stage tasks to the executor
  processes with at most ``cores`` tasks in flight per executor, and resubmits the tasks of a
  lost executor (``spark.task.maxFailures``);
* **object-store writer** (``ObjectStoreWriter.scala:164-216``): ``prepare_recoverable``
  persists a DataFrame's partitions in the executors' node stores and returns
  lineage-carrying ``ObjectRef``s; ``release_recoverable`` unpersists.

``spark.raydp.executor.mode=thread`` (or ``RAYDP_EXECUTOR_MODE=thread``) keeps all tasks on
a thread pool in the driver instead (no executor processes).
"""
import collections
import concurrent.futures as cf
import functools
import logging
import threading
import time
from typing import Dict, List, Optional

from raydp_amd.spark import plan as P
from raydp_amd.utils import parse_memory_size

logger = logging.getLogger(__name__)

EXECUTOR_RESOURCE_PREFIX = "spark.ray.raydp_spark_executor.actor.resource."
LEGACY_ACTOR_CPU = "spark.ray.actor.resource.cpu"
MASTER_SUFFIX = "_SPARK_MASTER"
_TRACE = bool(__import__("os").environ.get("RAYDP_TRACE_STAGES"))


class ExecutorInfo:
    def __init__(self, executor_id: str, handle, cores: int):
        self.executor_id = executor_id
        self.handle = handle
        self.cores = cores
        self.state = "RUNNING"
        self.launched = time.time()

    @property
    def alive(self) -> bool:
        return self.state == "RUNNING" and not self.handle._impl.dead

    def __repr__(self):
        return f"Executor({self.executor_id}, {self.state})"


class ExecutorTaskScheduler(P.TaskScheduler):
    """Runs stage tasks on the executor actor processes of one application."""

    remote = True

    def __init__(self, backend: "ClusterBackend"):
        self.backend = backend
        self.parallelism = max(1, backend.num_executors * backend.cores)
        self.max_failures = int(backend.conf.get("spark.task.maxFailures", "4"))

    def map(self, fn, indices):
        indices = list(indices)
        if not indices:
            return []
        t0 = time.perf_counter()
        payload, key = self._stage_payload(fn)
        t1 = time.perf_counter()
        try:
            return self._dispatch(lambda ex, i: ex.handle.run_task.remote(key, i), indices)
        finally:
            self._free_payload(payload, key)
            if _TRACE:
                logger.warning("stage: %d tasks, payload %d B (%d store objs), pickle %.3fs, run %.3fs",
                               len(indices), len(payload.data), len(payload.oids), t1 - t0,
                               time.perf_counter() - t1)

    @staticmethod
    def _stage_payload(fn):
        """Pickle the stage function once and seal it in the object store: each task call
        then carries only its id, and an executor maps + unpickles it once per stage."""
        import uuid
        from raydp_amd.runtime import core
        from raydp_amd.runtime import serialization as S
        payload = S.dumps_shared(fn)
        st = core.current_node_store()
        oid = uuid.uuid4().hex
        st.put(oid, payload.data)
        return payload, (st.node_id, st.path, oid)

    @staticmethod
    def _free_payload(payload, key):
        from raydp_amd.runtime import core
        payload.free()
        st = core.current_node_store()
        if st is not None:
            st.delete(key[2])

    def persist(self, fn, rdd_id: str, indices) -> List[tuple]:
        indices = list(indices)
        payload, key = self._stage_payload(fn)
        out = []
        try:
            res = self._dispatch(lambda ex, i: ex.handle.persist_partitions.remote(key, rdd_id, [i]),
                                 indices, tag=True)
        finally:
            self._free_payload(payload, key)
        for ex_id, lst in res:
            for (i, oid, node_id, path, rows) in lst:
                out.append((i, oid, node_id, path, rows, ex_id))
        return out

    def _dispatch(self, submit, indices, tag=False):
        from raydp_amd.runtime import core
        from raydp_amd.runtime.actors import ActorDiedError
        results = [None] * len(indices)
        todo = collections.deque(range(len(indices)))
        inflight: Dict[cf.Future, tuple] = {}
        load: Dict[str, int] = collections.defaultdict(int)
        failures: Dict[int, int] = collections.defaultdict(int)
        while todo or inflight:
            execs = self.backend.alive_executors()
            if not execs and not inflight:
                raise RuntimeError("no live executors to run tasks")
            while todo and execs:
                ex = min(execs, key=lambda e: load[e.executor_id])
                if load[ex.executor_id] >= ex.cores:
                    break
                pos = todo.popleft()
                try:
                    ref = submit(ex, indices[pos])
                except ActorDiedError:
                    todo.appendleft(pos)
                    self.backend.on_executor_failure(ex)
                    execs = self.backend.alive_executors()
                    continue
                load[ex.executor_id] += 1
                inflight[core.pending_result(ref)] = (pos, ex)
            if not inflight:
                time.sleep(0.01)
                continue
            done, _ = cf.wait(list(inflight), return_when=cf.FIRST_COMPLETED)
            for f in done:
                pos, ex = inflight.pop(f)
                load[ex.executor_id] -= 1
                try:
                    v = f.result()
                    results[pos] = (ex.executor_id, v) if tag else v
                except ActorDiedError:
                    failures[pos] += 1
                    self.backend.on_executor_failure(ex)
                    if failures[pos] >= self.max_failures:
                        raise RuntimeError(f"task {indices[pos]} failed {failures[pos]} times: executor lost")
                    todo.appendleft(pos)
        return results

    def shutdown(self):
        pass


class ClusterBackend:
    def __init__(self, app_name: str, conf: Dict[str, str], master_resources: Dict[str, float]):
        import os
        self.app_name = app_name
        self.conf = conf
        self.master_resources = master_resources
        self.app_id = f"app-{time.strftime('%Y%m%d%H%M%S')}-{os.getpid() % 10000:04d}"
        self.num_executors = int(conf.get("spark.executor.instances", "1"))
        self.cores = int(conf.get("spark.executor.cores", "1"))
        self.mode = conf.get("spark.raydp.executor.mode", os.environ.get("RAYDP_EXECUTOR_MODE", "process"))
        self._sched: Optional[P.TaskScheduler] = None
        self._recoverable: Dict[str, dict] = {}
        self._lock = threading.RLock()
        self._executors: Dict[str, ExecutorInfo] = {}
        self._next_id = 0
        self._bundle_rr = 0
        self.master = None
        self._master_url = None
        self._started = False

    # ---------------------------------------------------------------- lifecycle ----------
    def start(self):
        if self.mode == "thread":
            self._sched = P.TaskScheduler(max(1, self.num_executors * self.cores))
            self._started = True
            return
        from raydp_amd import runtime
        from raydp_amd.spark.master import RayDPSparkMaster
        res = dict(self.master_resources)
        opts = {"name": self.app_name + MASTER_SUFFIX, "num_cpus": res.pop("CPU", 0)}
        if "memory" in res:
            opts["memory"] = res.pop("memory")
        if res:
            opts["resources"] = res
        self.master = runtime.remote(RayDPSparkMaster).options(**opts).remote(self.app_name, self.conf)
        master_url = self.master.start_up.remote(self.master_resources)
        self.request_total_executors(self._initial_executors())
        self._master_url = runtime.get(master_url)
        # executors come up in parallel; wait until each answers
        runtime.get([e.handle.ping.remote() for e in self.alive_executors()])
        self._sched = ExecutorTaskScheduler(self)
        self._started = True

    def _initial_executors(self) -> int:
        if self.conf.get("spark.dynamicAllocation.enabled", "false").lower() == "true":
            n = self.conf.get("spark.dynamicAllocation.initialExecutors") or \
                self.conf.get("spark.dynamicAllocation.minExecutors") or "0"
            return max(int(n), 1)
        return self.num_executors

    def _executor_options(self, executor_id: str) -> dict:
        cpu = self.conf.get(EXECUTOR_RESOURCE_PREFIX + "cpu") or self.conf.get(LEGACY_ACTOR_CPU)
        opts = {"name": f"raydp-executor-{executor_id}", "num_cpus": float(cpu) if cpu else float(self.cores),
                "max_restarts": -1, "max_concurrency": max(2, self.cores)}
        mem = self.conf.get("spark.executor.memory")
        if mem:
            opts["memory"] = float(parse_memory_size(mem))
        custom = {}
        for k, v in self.conf.items():
            if k.startswith(EXECUTOR_RESOURCE_PREFIX):
                name = k[len(EXECUTOR_RESOURCE_PREFIX):]
                if name.lower() != "cpu":
                    custom[name] = float(v)
        if custom:
            opts["resources"] = custom
        pg_id = self.conf.get("spark.ray.placement_group")
        if pg_id:
            from raydp_amd.runtime import pgroup
            pg = pgroup.get_placement_group_by_id(pg_id)
            idx = [int(x) for x in self.conf.get("spark.ray.bundle_indexes", "").split(",") if x != ""] \
                or list(range(pg.bundle_count))
            opts["placement_group"] = pg
            opts["placement_group_bundle_index"] = idx[self._bundle_rr % len(idx)]
            self._bundle_rr += 1
        return opts

    def _launch_executor(self) -> ExecutorInfo:
        from raydp_amd import runtime
        from raydp_amd.spark.executor import RayDPExecutor
        from raydp_amd.spark.executor_registry import register_executor
        with self._lock:
            eid = str(self._next_id)
            self._next_id += 1
        opts = self._executor_options(eid)
        h = runtime.remote(RayDPExecutor).options(**opts).remote(eid, self.app_id, self.cores, self.conf)
        info = ExecutorInfo(eid, h, self.cores)
        with self._lock:
            self._executors[eid] = info
        register_executor(opts["name"], h)
        return info

    # ------------------------------------------------------------ dynamic allocation ----
    def request_total_executors(self, n: int) -> bool:
        """``doRequestTotalExecutors``: grow (or shrink) the executor set to ``n``."""
        max_n = self.conf.get("spark.dynamicAllocation.maxExecutors")
        if max_n is not None:
            n = min(n, int(max_n))
        alive = self.alive_executors()
        for _ in range(n - len(alive)):
            self._launch_executor()
        if n < len(alive):
            self.kill_executors([e.executor_id for e in alive[n:]])
        return True

    def kill_executors(self, ids: List[str]) -> bool:
        from raydp_amd import runtime
        from raydp_amd.spark.executor_registry import unregister_executor
        for eid in ids:
            with self._lock:
                info = self._executors.get(eid)
            if info is None or info.state != "RUNNING":
                continue
            info.state = "KILLED"
            try:
                runtime.kill(info.handle, no_restart=True)
            except Exception:  # noqa: BLE001
                pass
            unregister_executor(f"raydp-executor-{eid}")
        return True

    def alive_executors(self) -> List[ExecutorInfo]:
        with self._lock:
            return [e for e in self._executors.values() if e.alive]

    def executors(self) -> List[ExecutorInfo]:
        with self._lock:
            return list(self._executors.values())

    def on_executor_failure(self, info: ExecutorInfo):
        """A call failed with the actor dead: the supervisor restarts it (max_restarts=-1);
        only replace it when the runtime gave up on the actor."""
        if info.handle._impl.dead and info.state == "RUNNING":
            info.state = "LOST"
            logger.warning("executor %s lost; launching a replacement", info.executor_id)
            self._launch_executor()

    def master_url(self) -> str:
        if self._master_url:
            return self._master_url
        from raydp_amd.utils import get_node_ip_address
        return f"ray://{self.app_name}@{get_node_ip_address()}:0"

    def scheduler(self) -> P.TaskScheduler:
        return self._sched

    def connect_driver(self):
        """Fault-tolerant mode: nothing to connect — recoverable refs carry lineage."""

    def stop(self, cleanup_data=True):
        from raydp_amd import runtime
        with self._lock:
            recs = list(self._recoverable)
        if cleanup_data:
            for rdd in recs:
                self.release_recoverable(rdd)
        self.kill_executors([e.executor_id for e in self.executors()])
        if self.master is not None and cleanup_data:
            try:
                runtime.kill(self.master, no_restart=True)
            except Exception:  # noqa: BLE001
                pass
            self.master = None
        if self._sched is not None:
            self._sched.shutdown()

    # ---------------------------------------------------------------- conversion ---------
    def prepare_recoverable(self, df, storage_level):
        from raydp_amd.runtime.objects import ObjectRef
        plan = df._src()
        rdd_id = df._id
        sched = self._sched
        P.prepare(plan, sched)
        n = plan.num_partitions()
        if not isinstance(sched, ExecutorTaskScheduler):
            df.persist(storage_level)
            with self._lock:
                self._recoverable[rdd_id] = {"df": df}
            from raydp_amd.runtime import objects
            return rdd_id, [objects.put(t.replace_schema_metadata(),
                                        _lineage=functools.partial(self._recompute, plan, i))
                            for i, t in enumerate(df._cached.tables)]
        placed = sched.persist(plan.compute, rdd_id, range(n))
        placed.sort(key=lambda x: x[0])
        refs, loc = [], {}
        for (i, oid, node_id, path, rows, ex_id) in placed:
            refs.append(ObjectRef(oid, owner=f"raydp-executor-{ex_id}", node_id=node_id,
                                  lineage=functools.partial(self._recompute, plan, i)))
            loc[i] = ex_id
        with self._lock:
            self._recoverable[rdd_id] = {"df": df, "plan": plan, "locations": loc}
        return rdd_id, refs

    def _recompute(self, plan, i):
        """Lineage of a recoverable partition: re-run its task (``max_retries=-1`` fetch in the
        reference, with the executor re-caching the RDD block)."""
        return self._sched.map(plan.compute, [i])[0].replace_schema_metadata()

    def block_locations(self, rdd_id) -> Dict[int, str]:
        with self._lock:
            rec = self._recoverable.get(rdd_id)
        return dict(rec.get("locations", {})) if rec else {}

    def release_recoverable(self, rdd_id):
        from raydp_amd import runtime
        with self._lock:
            rec = self._recoverable.pop(rdd_id, None)
        if rec is None:
            return
        if "locations" in rec:
            refs = []
            for e in self.alive_executors():
                try:
                    refs.append(e.handle.unpersist.remote(rdd_id))
                except Exception:  # noqa: BLE001
                    pass
            for r in refs:
                try:
                    runtime.get(r)
                except Exception:  # noqa: BLE001
                    pass
        else:
            rec["df"].unpersist()

    def is_persisted(self, rdd_id) -> bool:
        with self._lock:
            return rdd_id in self._recoverable
