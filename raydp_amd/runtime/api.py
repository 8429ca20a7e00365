"""Task / actor API (``remote``, ``get_actor``, ``kill``, ``wait``) of the actor runtime.

``@remote`` functions become tasks executed on the node's task pool; their ``ObjectRef``
carries lineage so a lost result is recomputed (``max_retries``). ``@remote`` classes become
actors. An actor lives either in a dedicated supervised *process* (``process=True``, the
default for executor-style actors created by the framework: ``raydp_amd.runtime.process``) or
in-process on its own thread pool (``max_concurrency`` threads) — the latter is what user code
gets by default here, since it shares the driver's GPU context and object-store mapping.
Named actors are registered per namespace (``get_actor(name)``), mirroring Ray's named-actor
semantics used by RayDP (``raydp-executor-<id>``, ``<app>_SPARK_MASTER``).
"""
import concurrent.futures as cf
import inspect
import os
import threading
import uuid
from typing import Any, Dict, List, Optional

from raydp_amd.runtime import core
from raydp_amd.runtime.objects import ObjectRef, get, put_with_id


class JobConfig:
    def __init__(self, code_search_path=None, runtime_env=None, **kw):
        self.code_search_path = code_search_path
        self.runtime_env = runtime_env


class PlacementGroupSchedulingStrategy:
    def __init__(self, placement_group, placement_group_bundle_index=-1,
                 placement_group_capture_child_tasks=None):
        self.placement_group = placement_group
        self.placement_group_bundle_index = placement_group_bundle_index


class NodeAffinitySchedulingStrategy:
    def __init__(self, node_id, soft=False):
        self.node_id, self.soft = node_id, soft


_pool_lock = threading.Lock()
_task_pool: Optional[cf.ThreadPoolExecutor] = None


def _pool() -> cf.ThreadPoolExecutor:
    global _task_pool
    with _pool_lock:
        if _task_pool is None:
            import os
            _task_pool = cf.ThreadPoolExecutor(max_workers=max(4, os.cpu_count() or 4),
                                               thread_name_prefix="raydp-worker")
        return _task_pool


def _resolve_args(args, kwargs):
    a = [get(x) if isinstance(x, ObjectRef) else x for x in args]
    k = {n: (get(v) if isinstance(v, ObjectRef) else v) for n, v in kwargs.items()}
    return a, k


def _submit(fn, args, kwargs, retries: int) -> ObjectRef:
    if not core.is_initialized():
        core.init()

    def run():
        a, k = _resolve_args(args, kwargs)
        return fn(*a, **k)

    ref = ObjectRef(lineage=run if retries != 0 else None)

    def task():
        attempts = 0
        while True:
            try:
                v = run()
                break
            except Exception:
                attempts += 1
                if retries >= 0 and attempts > retries:
                    raise
        put_with_id(ref.id, v)
        return v

    fut = _pool().submit(task)
    core.register_pending(ref.id, fut)
    return ref


class RemoteFunction:
    def __init__(self, fn, opts=None):
        self._fn = fn
        self._opts = dict(opts or {})
        self.__name__ = getattr(fn, "__name__", "remote_fn")

    def options(self, **opts):
        o = dict(self._opts)
        o.update(opts)
        return RemoteFunction(self._fn, o)

    def remote(self, *args, **kwargs) -> ObjectRef:
        return _submit(self._fn, args, kwargs, int(self._opts.get("max_retries", 3)))

    def __call__(self, *a, **k):
        raise TypeError("Remote functions cannot be called directly; use .remote()")


# ------------------------------------------------------------------------------ actors ----
_registry_lock = threading.RLock()
_named: Dict[tuple, "ActorHandle"] = {}


class ActorMethod:
    def __init__(self, handle, name):
        self._handle, self._name = handle, name

    def remote(self, *args, **kwargs) -> ObjectRef:
        return self._handle._call(self._name, args, kwargs)

    def options(self, **kw):
        return self


class ActorID(str):
    """Actor id (``ray.ActorID``-like: ``.hex()``)."""

    def hex(self):
        return str(self)


class ActorHandle:
    def __init__(self, impl, name=None, namespace=None):
        self._impl = impl
        self._actor_name = name
        self._namespace = namespace
        self._actor_id = ActorID(getattr(impl, "actor_id", None) or uuid.uuid4().hex)

    def __reduce__(self):
        if getattr(self._impl, "sock_path", None) is None:
            raise TypeError("in-process (thread) actor handles cannot leave their process")
        return (_attach_handle, (self._actor_id, self._actor_name, self._namespace))

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        return ActorMethod(self, item)

    def _call(self, name, args, kwargs) -> ObjectRef:
        return self._impl.call(name, args, kwargs)

    def _kill(self, no_restart=True):
        self._impl.kill(no_restart)

    def __repr__(self):
        return f"Actor({self._actor_name or self._actor_id[:8]})"


class _ThreadActor:
    """In-process actor: the instance lives in this process, calls run on its own pool."""

    def __init__(self, cls, args, kwargs, opts):
        a, k = _resolve_args(args, kwargs)
        self.instance = cls(*a, **k)
        self.pool = cf.ThreadPoolExecutor(max_workers=int(opts.get("max_concurrency", 1) or 1),
                                          thread_name_prefix=f"actor-{cls.__name__}")
        self.dead = False

    def call(self, name, args, kwargs) -> ObjectRef:
        if self.dead:
            raise RuntimeError("actor is dead")
        ref = ObjectRef()
        method = getattr(self.instance, name)

        def run():
            a, k = _resolve_args(args, kwargs)
            v = method(*a, **k)
            put_with_id(ref.id, v)
            return v
        core.register_pending(ref.id, self.pool.submit(run))
        return ref

    def kill(self, no_restart=True):
        self.dead = True
        self.pool.shutdown(wait=False, cancel_futures=True)


class ActorClass:
    def __init__(self, cls, opts=None):
        self._cls = cls
        self._opts = dict(opts or {})
        self.__name__ = cls.__name__

    def options(self, **opts):
        o = dict(self._opts)
        o.update(opts)
        return ActorClass(self._cls, o)

    def remote(self, *args, **kwargs) -> ActorHandle:
        if not core.is_initialized():
            core.init()
        name = self._opts.get("name")
        ns = self._opts.get("namespace") or core.get_runtime_context().namespace
        if name:
            with _registry_lock:
                if (ns, name) in _named and not _named[(ns, name)]._impl.dead:
                    if self._opts.get("get_if_exists"):
                        return _named[(ns, name)]
                    raise ValueError(f"actor name {name!r} already taken in namespace {ns!r}")
        if name and _named_file(ns, name) is not None and os.path.exists(_named_file(ns, name)):
            existing = _lookup_named_file(ns, name)
            if existing is not None and not existing._impl.dead:
                if self._opts.get("get_if_exists"):
                    return existing
                raise ValueError(f"actor name {name!r} already taken in namespace {ns!r}")
        if _isolation(self._opts) == "process":
            impl = core.current_node().actors.create(self._cls, args, kwargs, self._opts, name, ns)
        else:
            impl = _ThreadActor(self._cls, args, kwargs, self._opts)
        h = ActorHandle(impl, name, ns)
        if name:
            with _registry_lock:
                _named[(ns, name)] = h
            if getattr(impl, "sock_path", None) is not None:
                _write_named_file(ns, name, impl.actor_id)
        return h


def _isolation(opts) -> str:
    iso = opts.get("isolation") or os.environ.get("RAYDP_ACTOR_ISOLATION", "process")
    if iso not in ("process", "thread"):
        raise ValueError(f"isolation must be 'process' or 'thread', got {iso!r}")
    return iso


def _named_file(ns, name):
    n = core.current_node()
    if n is None or not n.session_dir:
        return None
    safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in f"{ns}__{name}")
    return os.path.join(n.session_dir, "named", safe)


def _write_named_file(ns, name, actor_id):
    p = _named_file(ns, name)
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p + ".tmp", "w") as f:
        f.write(actor_id)
    os.replace(p + ".tmp", p)


def _remove_named_file(ns, name):
    p = _named_file(ns, name)
    if p is not None and os.path.exists(p):
        try:
            os.unlink(p)
        except OSError:
            pass


def _lookup_named_file(ns, name) -> Optional["ActorHandle"]:
    p = _named_file(ns, name)
    if p is None or not os.path.exists(p):
        return None
    with open(p) as f:
        aid = f.read().strip()
    return _attach_handle(aid, name, ns)


def _attach_handle(actor_id, name=None, namespace=None) -> "ActorHandle":
    """Handle to an existing process actor (possibly created by another process)."""
    if not core.is_initialized():
        core.init()
    mgr = core.current_node().actors
    with mgr._lock:
        impl = mgr.actors.get(actor_id)
    if impl is None:
        from raydp_amd.runtime.actors import ProcessActor
        impl = ProcessActor(mgr, actor_id, name, namespace or "default", {}, owned=False)
        with mgr._lock:
            mgr.actors[actor_id] = impl
        _ = mgr.supervisor  # subscribe to death events
    return ActorHandle(impl, name, namespace)


def remote(*args, **kwargs):
    def wrap(obj, opts):
        if inspect.isclass(obj):
            return ActorClass(obj, opts)
        return RemoteFunction(obj, opts)
    if len(args) == 1 and not kwargs and callable(args[0]):
        return wrap(args[0], {})
    return lambda obj: wrap(obj, kwargs)


def method(*a, **k):
    def deco(f):
        return f
    return deco


def get_actor(name: str, namespace: Optional[str] = None) -> ActorHandle:
    ns = namespace or core.get_runtime_context().namespace
    with _registry_lock:
        h = _named.get((ns, name))
    if h is None:
        h = _lookup_named_file(ns, name)
    if h is None:
        from raydp_amd.spark.executor_registry import lookup_executor
        h = lookup_executor(name)
    if h is None or h._impl.dead:
        raise ValueError(f"Failed to look up actor with name '{name}'")
    return h


def register_named(name: str, handle, namespace: Optional[str] = None):
    ns = namespace or core.get_runtime_context().namespace
    with _registry_lock:
        _named[(ns, name)] = handle


def unregister_named(name: str, namespace: Optional[str] = None):
    ns = namespace or core.get_runtime_context().namespace
    with _registry_lock:
        _named.pop((ns, name), None)


def list_named():
    with _registry_lock:
        return [{"name": n, "namespace": ns} for (ns, n) in _named]


def kill(actor: ActorHandle, no_restart: bool = True):
    actor._kill(no_restart)
    if no_restart:
        with _registry_lock:
            for k, v in list(_named.items()):
                if v is actor or v._actor_id == actor._actor_id:
                    _named.pop(k)
                    _remove_named_file(*k)
        if actor._actor_name:
            _remove_named_file(actor._namespace or core.get_runtime_context().namespace, actor._actor_name)


def wait(refs: List[ObjectRef], num_returns: int = 1, timeout: Optional[float] = None,
         fetch_local: bool = True):
    import time
    deadline = None if timeout is None else time.time() + timeout
    ready, pending = [], list(refs)
    while len(ready) < num_returns and pending:
        for r in list(pending):
            fut = core.pending_result(r)
            if fut is None or fut.done():
                ready.append(r)
                pending.remove(r)
                if len(ready) >= num_returns:
                    break
        if len(ready) >= num_returns or (deadline is not None and time.time() > deadline):
            break
        time.sleep(0.001)
    return ready, pending


def nodes():
    n = core.current_node()
    if n is None:
        return []
    if getattr(n, "gcs", None) is not None:
        return n.gcs.call("nodes")
    return [{"NodeID": v.node_id, "Alive": v.alive, "NodeManagerAddress": v.ip,
             "Resources": dict(v.total)} for v in n.cluster.nodes.values()]


def cluster_resources():
    out: Dict[str, float] = {}
    n = core.current_node()
    if getattr(n, "gcs", None) is not None:
        return n.gcs.call("resources")[0]
    if n is not None:
        for v in n.cluster.alive_nodes():
            for k, x in v.total.items():
                out[k] = out.get(k, 0.0) + x
    return out


def available_resources():
    out: Dict[str, float] = {}
    n = core.current_node()
    if getattr(n, "gcs", None) is not None:
        return n.gcs.call("resources")[1]
    if n is not None:
        for v in n.cluster.alive_nodes():
            for k, x in v.available.items():
                out[k] = out.get(k, 0.0) + x
    return out


def _reset():
    with _registry_lock:
        for h in _named.values():
            try:
                h._impl.kill()
            except Exception:  # noqa: BLE001
                pass
        _named.clear()
