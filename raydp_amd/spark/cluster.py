"""Cluster backend of a Spark-on-runtime application (driver side).

The application's control state lives in the native app master (``csrc/control/app_master.cc``,
client ``raydp_amd.spark.appmaster``): application registration, executor ids, the
registration / restart-remap protocol, the executor caps, dynamic-allocation targets, the
per-node shuffle services and the RecacheRDD relay. This object is the driver half around it:

* **executor launcher** (``RayExecutorUtils.createExecutorActor``): carries out the master's
  launch orders — executor actors with their resources
  (``spark.ray.raydp_spark_executor.actor.resource.*``, the legacy
  ``spark.ray.actor.resource.cpu``, ``spark.executor.memory``), spreads them round-robin over
  the placement-group bundles named by ``spark.ray.placement_group`` /
  ``spark.ray.bundle_indexes`` (``RayAppMaster.scala:116-128,341-349``), restarts them without
  limit (``RayExecutorUtils.java:58``) and answers dynamic-allocation requests
  (``requestTotalExecutors`` / ``killExecutors``: ``RayCoarseGrainedSchedulerBackend.scala:
  278-301``);
* **scheduler backend** (``RayCoarseGrainedSchedulerBackend``): ``ExecutorTaskScheduler`` ships stage tasks to the executor
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
import os
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
# per-thread ``on_wait()`` callback: called each time a stage has its tasks in flight and the
# dispatching thread is about to block on them (fit_on_spark's overlapped conversion uses it to
# start building the training engine only once the driver-side stage work is done)
_dispatch_hooks = threading.local()


def set_dispatch_hook(fn) -> None:
    _dispatch_hooks.on_wait = fn


def set_block_hook(fn) -> None:
    """``fn(partition, object_id, node_id, rows, executor_id)`` for every partition a persist
    stage run on this thread places, as it lands (None: off). The estimator streams the blocks
    into HBM while the rest of the stage still runs (``raydp_amd/torch/engine.py`` stream_ingest)."""
    _dispatch_hooks.on_block = fn


def _seconds(v) -> float:
    v = str(v).strip().lower()
    for suf, k in (("ms", 1e-3), ("s", 1.0), ("m", 60.0)):
        if v.endswith(suf):
            return float(v[:-len(suf)]) * k
    return float(v)


class ExecutorInfo:
    def __init__(self, executor_id: str, handle, cores: int):
        self.executor_id = executor_id
        self.handle = handle
        self.cores = cores
        self.state = "RUNNING"
        self.launched = time.time()
        self.node_id: Optional[str] = None   # store node of the executor (locality)

    @property
    def alive(self) -> bool:
        return self.state == "RUNNING" and not self.handle._impl.dead

    def __repr__(self):
        return f"Executor({self.executor_id}, {self.state})"


def _driver_resident_bytes(plan, limit) -> Optional[int]:
    """Bytes of the driver-resident tables a plan reads, or None when any leaf lives elsewhere
    (files, the object store of an executor) or a wide operator is still unmaterialised."""
    from raydp_amd.spark.sources import TableSource
    total = 0
    stack = [plan]
    while stack:
        p = stack.pop()
        if isinstance(p, P.MaterializedPlan):
            total += sum(t.nbytes for t in p.tables)
        elif isinstance(p, P.SourcePlan):
            if not isinstance(p.source, TableSource):
                return None
            total += sum(t.nbytes for t in p.source.tables)
        elif isinstance(p, P.MapPlan):
            stack.append(p.child)
        elif isinstance(p, P.UnionPlan):
            stack.extend(p.plans)
        elif getattr(p, "_broadcast", None) is not None:
            total += p._broadcast.nbytes
            stack.append(p.left)
        elif isinstance(p, P.WidePlan) and getattr(p, "_out", None) is not None:
            total += sum(t.nbytes for t in p._out)
        else:
            return None
        if total > limit:
            return None
    return total


class ExecutorTaskScheduler(P.TaskScheduler):
    """Runs stage tasks on the executor actor processes of one application."""

    remote = True

    def __init__(self, backend: "ClusterBackend"):
        self.backend = backend
        self.parallelism = max(1, backend.num_executors * backend.cores)
        self.max_failures = int(backend.conf.get("spark.task.maxFailures", "4"))
        self.locality_wait = _seconds(backend.conf.get("spark.locality.wait", "3s"))

    def map(self, fn, indices, prefs=None):
        """``prefs``: optional ``{partition: node_id}`` locality hints (else taken from the plan
        when ``fn`` is a plan's ``compute``)."""
        indices = list(indices)
        if not indices:
            return []
        from raydp_amd.utils import tracing
        if self._runs_locally(fn):
            # Spark's LocalTableScan: a stage over small driver-resident tables (cached results,
            # local data) runs in the driver; shipping it costs more than computing it
            with tracing.span("local stage", cat="etl", tasks=len(indices)):
                out = []
                for i in indices:
                    with P._PartitionScope(i):
                        out.append(fn(i))
                return out
        t0 = time.perf_counter()
        payload, key = self._stage_payload(fn)
        t1 = time.perf_counter()
        try:
            with tracing.span("stage", cat="etl", tasks=len(indices), payload_bytes=len(payload.data)):
                pos_prefs = ({pos: prefs[i] for pos, i in enumerate(indices) if prefs.get(i)}
                             if prefs is not None else self._prefs(fn, indices))
                return self._dispatch(lambda ex, i: ex.handle.run_task.remote(key, i), indices,
                                      prefs=pos_prefs)
        finally:
            self._free_payload(payload, key)
            if _TRACE:
                logger.warning("stage: %d tasks, payload %d B (%d store objs), pickle %.3fs, run %.3fs",
                               len(indices), len(payload.data), len(payload.oids), t1 - t0,
                               time.perf_counter() - t1)

    def _runs_locally(self, fn) -> bool:
        plan = getattr(fn, "__self__", None)
        if not isinstance(plan, P.Plan):
            return False
        limit = self.__dict__.get("_local_bytes")
        if limit is None:
            from raydp_amd.utils import parse_memory_size
            limit = parse_memory_size(str(self.backend.conf.get(
                "spark.ray.mi355x.local_exec_bytes", os.environ.get("RAYDP_LOCAL_EXEC_BYTES", "4m"))))
            self._local_bytes = limit
        if limit <= 0:
            return False
        total = _driver_resident_bytes(plan, limit)
        return total is not None and total <= limit

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
        from raydp_amd.utils import tracing
        with tracing.span("stage payload", cat="etl"):
            payload, key = self._stage_payload(fn)
        out = []
        hook = getattr(_dispatch_hooks, "on_block", None)

        def landed(ex_id, lst):
            for (i, oid, node_id, path, rows) in lst:
                hook(i, oid, node_id, rows, ex_id)
        try:
            with tracing.span("persist stage", cat="etl", tasks=len(indices)):
                res = self._dispatch(lambda ex, i: ex.handle.persist_partitions.remote(key, rdd_id, [i]),
                                     indices, tag=True, on_done=landed if hook is not None else None)
        finally:
            self._free_payload(payload, key)
        for ex_id, lst in res:
            for (i, oid, node_id, path, rows) in lst:
                out.append((i, oid, node_id, path, rows, ex_id))
        return out

    @staticmethod
    def _prefs(fn, indices) -> Dict[int, str]:
        """Locality hints of a stage whose function is a plan's ``compute``."""
        plan = getattr(fn, "__self__", None)
        if not isinstance(plan, P.Plan):
            return {}
        out = {}
        for pos, i in enumerate(indices):
            n = P.preferred_node(plan, i)
            if n is not None:
                out[pos] = n
        return out

    def _pick(self, todo, execs, load, prefs, t_stage):
        """Next (task position, executor) under delay scheduling (``spark.locality.wait``): a
        task with a preferred node waits for a free slot there, up to the wait, unless no
        executor lives on that node; tasks without a preference take any free slot."""
        free = [e for e in execs if load[e.executor_id] < e.cores]
        if not free:
            return None
        least = min(free, key=lambda e: load[e.executor_id])
        expired = time.monotonic() - t_stage >= self.locality_wait
        for pos in todo:
            want = prefs.get(pos) if prefs else None
            if want is None:
                return pos, least
            local = [e for e in free if e.node_id == want]
            if local:
                return pos, min(local, key=lambda e: load[e.executor_id])
            if expired or not any(e.node_id == want for e in execs):
                return pos, least
        return None

    def _dispatch(self, submit, indices, tag=False, prefs=None, on_done=None):
        from raydp_amd.runtime import core
        from raydp_amd.runtime.actors import ActorDiedError
        results = [None] * len(indices)
        todo = collections.deque(range(len(indices)))
        inflight: Dict[cf.Future, tuple] = {}
        load: Dict[str, int] = collections.defaultdict(int)
        failures: Dict[int, int] = collections.defaultdict(int)
        t_stage = time.monotonic()
        while todo or inflight:
            execs = self.backend.alive_executors()
            if not execs and not inflight:
                raise RuntimeError("no live executors to run tasks")
            while todo and execs:
                pick = self._pick(todo, execs, load, prefs, t_stage)
                if pick is None:
                    break
                pos, ex = pick
                todo.remove(pos)
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
            hook = getattr(_dispatch_hooks, "on_wait", None)
            if hook is not None:
                hook()
            done, _ = cf.wait(list(inflight), return_when=cf.FIRST_COMPLETED,
                              timeout=self.locality_wait if todo and prefs else None)
            for f in done:
                pos, ex = inflight.pop(f)
                load[ex.executor_id] -= 1
                try:
                    v = f.result()
                    results[pos] = (ex.executor_id, v) if tag else v
                    if on_done is not None:
                        try:
                            on_done(ex.executor_id, v)
                        except Exception:  # noqa: BLE001 - an observer never fails the stage
                            pass
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
        self.master = None
        self.appmaster = None
        self._master_url = None
        self._started = False
        self.shuffle_service_enabled = str(conf.get("spark.shuffle.service.enabled", "false")).lower() == "true"

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
        self._start_appmaster()
        self._master_url = runtime.get(master_url)
        # executors come up in parallel; wait until each answers (and learn its node)
        execs = self.alive_executors()
        for e, inf in zip(execs, runtime.get([e.handle.info.remote() for e in execs])):
            e.node_id = inf["node_id"]
        self._sched = ExecutorTaskScheduler(self)
        self._started = True

    def _start_appmaster(self):
        """Launch the native app master, register the application and carry out the launch
        orders of its initial ``schedule()``."""
        from raydp_amd.runtime import core
        from raydp_amd.spark.appmaster import AppMasterClient
        from raydp_amd.utils import get_node_ip_address
        node = core.current_node()
        workdir = node.session_dir if node is not None and node.session_dir else __import__("tempfile").mkdtemp()
        self.appmaster = AppMasterClient.launch(workdir)
        self.conf["spark.ray.appmaster.socket"] = self.appmaster.sock_path
        cpu = self.conf.get(EXECUTOR_RESOURCE_PREFIX + "cpu") or self.conf.get(LEGACY_ACTOR_CPU)
        custom = {k[len(EXECUTOR_RESOURCE_PREFIX):]: float(v) for k, v in self.conf.items()
                  if k.startswith(EXECUTOR_RESOURCE_PREFIX) and k[len(EXECUTOR_RESOURCE_PREFIX):].lower() != "cpu"}
        mem = self.conf.get("spark.executor.memory")
        bundles = []
        if self.conf.get("spark.ray.placement_group"):
            from raydp_amd.runtime import pgroup
            pg = pgroup.get_placement_group_by_id(self.conf["spark.ray.placement_group"])
            bundles = [int(x) for x in self.conf.get("spark.ray.bundle_indexes", "").split(",") if x != ""] \
                or list(range(pg.bundle_count))
        if not bundles:
            # fail fast (with the node table in the message) when no node can ever host one
            # executor of this shape; a shortfall of capacity only warns: the app master's
            # orders queue until resources free up, as executors do under Ray
            from raydp_amd.ray_cluster_resources import plan_executors
            req = {"CPU": float(cpu) if cpu else float(self.cores), **custom}
            if mem:
                req["memory"] = float(parse_memory_size(mem))
            plan = plan_executors(self._initial_executors(), req)
            if plan.nodes and plan.capacity_total < plan.wanted:
                logger.warning("the cluster can host %d of the %d requested executors %s (%s)",
                               plan.capacity_total, plan.wanted, plan.request, plan.describe())
        dyn = self.conf.get("spark.dynamicAllocation.enabled", "false").lower() == "true"
        max_n = self.conf.get("spark.dynamicAllocation.maxExecutors")
        orders = self.appmaster.register_app(
            self.app_name, self._initial_executors(), self.cores,
            int(parse_memory_size(mem) // (1 << 20)) if mem else 1024,
            float(cpu) if cpu else float(self.cores), custom, bundles, dyn,
            int(max_n) if max_n is not None else (1 << 30), self.shuffle_service_enabled,
            self.conf.get("spark.local.dir", ""), get_node_ip_address())
        self.app_id = self.appmaster.app_id
        for o in orders:
            self._launch_executor(o)
        self.appmaster.subscribe(self._on_master_event)

    def _on_master_event(self, ev):
        """Driver agent (``RayDPDriverAgent.receive RecacheRDD``): re-materialise a persisted
        dataset whose blocks an executor lost."""
        if ev and ev[0] == "recache":
            try:
                self.recache(ev[1])
            except Exception as e:  # noqa: BLE001
                logger.warning("recache of %s failed: %s", ev[1], e)

    def recache(self, rdd_id: str) -> int:
        """Recompute the partitions of a recoverable dataset that no live executor holds."""
        with self._lock:
            rec = self._recoverable.get(rdd_id)
        if rec is None or "plan" not in rec:
            return 0
        held = {}
        for e in self.alive_executors():
            try:
                from raydp_amd import runtime
                held.update(runtime.get(e.handle.block_locations.remote(rdd_id)))
            except Exception:  # noqa: BLE001
                pass
        n = rec["plan"].num_partitions()
        missing = [i for i in range(n) if i not in held]
        if missing:
            placed = self._sched.persist(rec["plan"].compute, rdd_id, missing)
            with self._lock:
                for entry in placed:
                    rec["locations"][entry[0]] = entry[5]
                if rec.get("placed") is not None:
                    fresh = {e[0]: e for e in placed}
                    rec["placed"] = [fresh.get(e[0], e) for e in rec["placed"]]
        return len(missing)

    def _initial_executors(self) -> int:
        if self.conf.get("spark.dynamicAllocation.enabled", "false").lower() == "true":
            n = self.conf.get("spark.dynamicAllocation.initialExecutors") or \
                self.conf.get("spark.dynamicAllocation.minExecutors") or "0"
            return max(int(n), 1)
        return self.num_executors

    def _executor_options(self, order) -> dict:
        """Actor options of one launch order (``RayExecutorUtils.createExecutorActor``:
        name, CPU, memory, custom resources, bundle, ``maxRestarts=-1``)."""
        opts = {"name": f"raydp-executor-{order.executor_id}", "num_cpus": order.cpu,
                "max_restarts": -1, "max_concurrency": max(2, order.cores)}
        if self.conf.get("spark.executor.memory"):
            opts["memory"] = float(order.memory_mb) * (1 << 20)
        if order.resources:
            opts["resources"] = dict(order.resources)
        pg_id = self.conf.get("spark.ray.placement_group")
        if pg_id and order.bundle >= 0:
            from raydp_amd.runtime import pgroup
            opts["placement_group"] = pgroup.get_placement_group_by_id(pg_id)
            opts["placement_group_bundle_index"] = order.bundle
        return opts

    def _launch_executor(self, order) -> ExecutorInfo:
        from raydp_amd import runtime
        from raydp_amd.spark.executor import RayDPExecutor
        from raydp_amd.spark.executor_registry import register_executor
        eid = order.executor_id
        opts = self._executor_options(order)
        h = runtime.remote(RayDPExecutor).options(**opts).remote(eid, self.app_id, self.cores, self.conf)
        info = ExecutorInfo(eid, h, self.cores)
        with self._lock:
            self._executors[eid] = info
        register_executor(opts["name"], h)
        return info

    # ------------------------------------------------------------ dynamic allocation ----
    def request_total_executors(self, n: int) -> bool:
        """``doRequestTotalExecutors``: the master decides how many to add (its caps count
        restarted executors, ``RayAppMaster.scala:258-303``); surplus executors are killed."""
        alive = self.alive_executors()
        if n < len(alive):
            return self.kill_executors([e.executor_id for e in alive[n:]])
        for o in self.appmaster.request_executors(n):
            self._launch_executor(o)
        return True

    def _master_ids(self) -> Dict[str, str]:
        """original (actor-name) executor id -> the id the master currently knows it by."""
        cur = {}
        for new, old in sorted(self.appmaster.get_restarted().items(), key=lambda kv: int(kv[0])):
            cur[old] = new
            for k, v in list(cur.items()):  # chains of restarts
                if v == old:
                    cur[k] = new
        return cur

    def kill_executors(self, ids: List[str]) -> bool:
        from raydp_amd import runtime
        from raydp_amd.spark.executor_registry import unregister_executor
        if self.appmaster is not None:
            remap = self._master_ids()
            self.appmaster.kill_executors([remap.get(i, i) for i in ids])
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
            logger.warning("executor %s lost; asking the master for a replacement", info.executor_id)
            if self.appmaster is not None:
                self.appmaster.executor_lost(self._master_ids().get(info.executor_id, info.executor_id))
                for o in self.appmaster.request_executors(len(self.alive_executors()) + 1):
                    self._launch_executor(o)

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
        if self.appmaster is not None:
            try:
                self.appmaster.unregister_app()
            except OSError:
                pass
            self.appmaster.shutdown()
            self.appmaster = None
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
        with self._lock:
            rec = self._recoverable.get(rdd_id)
        if rec is not None and rec.get("placed") is not None and rec.get("plan") is plan:
            # the same DataFrame converted again (e.g. fit_on_spark(df, df)): its blocks are
            # already persisted under (rdd_id, i) -- hand out references to them, as Spark's
            # persist() of an already-persisted RDD is a no-op
            placed = rec["placed"]
        else:
            placed = sched.persist(plan.compute, rdd_id, range(n))
            placed.sort(key=lambda x: x[0])
        refs, loc = [], {}
        for (i, oid, node_id, path, rows, ex_id) in placed:
            refs.append(ObjectRef(oid, owner=f"raydp-executor-{ex_id}", node_id=node_id,
                                  lineage=functools.partial(self._recompute, plan, i)))
            loc[i] = ex_id
        with self._lock:
            self._recoverable[rdd_id] = {"df": df, "plan": plan, "locations": loc, "placed": placed}
        return rdd_id, refs

    def _recompute(self, plan, i):
        """Lineage of a recoverable partition: re-run its task (``max_retries=-1`` fetch in the
        reference, with the executor re-caching the RDD block)."""
        return self._sched.map(plan.compute, [i])[0].replace_schema_metadata()

    def block_locations(self, rdd_id) -> Dict[int, str]:
        """partition -> executor (actor-name id), like ``getBlockLocations`` followed by the
        restarted-executor remap of ``ObjectStoreWriter.scala:179-191``."""
        with self._lock:
            rec = self._recoverable.get(rdd_id)
        return dict(rec.get("locations", {})) if rec else {}

    def restarted_executors(self) -> Dict[str, str]:
        """new executor id -> original id (``RayAppMaster.getRestartedExecutors``)."""
        return self.appmaster.get_restarted() if self.appmaster is not None else {}

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
