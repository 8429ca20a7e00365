"""Process actors: creation, calls, restarts and node-failure handling.

An actor created with ``isolation="process"`` runs in its own Python process spawned by the
node's native supervisor (``csrc/runtime/supervisor.cc``) and served by
``raydp_amd.runtime.actor_worker``. This module is the caller side:

* ``ActorManager`` (one per attached process) owns the supervisor client, the actor table and
  the resource reservations; it reacts to supervisor events (``died`` / ``restarted``) and to
  virtual-node removal (actors on a removed node are restarted on a surviving node while they
  have restarts left — Ray's behaviour the reference relies on for executor recovery,
  ``RayAppMaster.scala:212-244``).
* ``ProcessActor`` is one actor's connection: calls are framed over a Unix socket and resolve
  ``ObjectRef`` futures from a reader thread; a broken connection fails the in-flight calls with
  ``ActorDiedError`` and later calls reconnect to the restarted process.
"""
import concurrent.futures as cf
import itertools
import os
import socket
import sys
import threading
import time
import uuid
from typing import Dict, Optional

import cloudpickle

from raydp_amd.runtime import core
from raydp_amd.runtime.actor_worker import actor_paths, recv_frame, send_frame
from raydp_amd.runtime.objects import ObjectRef


class ActorDiedError(RuntimeError):
    """The actor process died (``ray.exceptions.RayActorError`` equivalent)."""


class ActorUnavailableError(ActorDiedError):
    pass


def _python_path() -> str:
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    paths = [root] + [p for p in sys.path if p and os.path.isdir(p)]
    seen, out = set(), []
    for p in paths + os.environ.get("PYTHONPATH", "").split(os.pathsep):
        if p and p not in seen:
            seen.add(p)
            out.append(p)
    return os.pathsep.join(out)


class ProcessActor:
    CONNECT_TIMEOUT = float(os.environ.get("RAYDP_ACTOR_CONNECT_TIMEOUT", "120"))

    def __init__(self, manager: "ActorManager", actor_id: str, name: Optional[str], namespace: str,
                 opts: dict, vnode=None, resources=None, pg=None, bundle=None, owned=True):
        self.manager = manager
        self.actor_id = actor_id
        self.name = name
        self.namespace = namespace
        self.opts = opts
        self.vnode = vnode
        self.resources = resources or {}
        self.pg, self.bundle = pg, bundle
        self.owned = owned
        self.max_restarts = int(opts.get("max_restarts", 0) or 0)
        self.restarts = 0
        self.dead = False
        self.death_cause: Optional[str] = None
        self._lock = threading.RLock()
        self._conn: Optional[socket.socket] = None
        self._send_lock = threading.Lock()
        self._pending: Dict[int, cf.Future] = {}
        self._ids = itertools.count()
        sdir = manager.node.session_dir
        self.spec_path, self.sock_path, self.err_path = actor_paths(sdir, actor_id)

    # ---------------------------------------------------------------- process control ----
    def env(self) -> Dict[str, str]:
        node = self.manager.node
        store = self.vnode.store if self.vnode is not None and self.vnode.store is not None else node.store
        e = dict(os.environ)
        e.update({"RAYDP_ACTOR_ID": self.actor_id, "RAYDP_SESSION_DIR": node.session_dir,
                  "RAYDP_STORE_PATH": store.path,
                  "RAYDP_NODE_ID": self.vnode.node_id if self.vnode is not None else node.node_id,
                  "RAYDP_HEAD_NODE_ID": node.node_id,
                  "RAYDP_SUPERVISOR_SOCK": self.manager.supervisor.sock_path,
                  "RAYDP_NAMESPACE": self.namespace, "PYTHONPATH": _python_path(),
                  "RAYDP_JOB_ID": str(getattr(node, "job_id", "") or ""),
                  "RAYDP_NODE_IP": self.vnode.ip if self.vnode is not None else ""})
        gpus = self.opts.get("_gpu_ids")
        if gpus is not None:
            e["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
        if not e["RAYDP_NODE_IP"]:
            e.pop("RAYDP_NODE_IP")
        for k, v in (self.opts.get("runtime_env") or {}).get("env_vars", {}).items():
            e[k] = str(v)
        return e

    def start(self):
        log = os.path.join(self.manager.node.session_dir, "logs", f"actor-{self.name or self.actor_id}.log")
        for p in (self.sock_path, self.err_path):
            if os.path.exists(p):
                os.unlink(p)
        self.pid = self.manager.supervisor.spawn(
            self.actor_id, [sys.executable, "-u", "-m", "raydp_amd.runtime.actor_worker"], self.env(),
            cwd=os.getcwd(), log=log, max_restarts=self.max_restarts - self.restarts if self.max_restarts >= 0 else -1)

    # ---------------------------------------------------------------------- calls ------
    def _connect(self) -> socket.socket:
        deadline = time.time() + self.CONNECT_TIMEOUT
        while True:
            if self.dead:
                raise ActorDiedError(self._died_msg())
            if os.path.exists(self.err_path):
                self._constructor_failed()
            if os.path.exists(self.sock_path):
                s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                try:
                    s.connect(self.sock_path)
                    return s
                except OSError:
                    s.close()
            if time.time() > deadline:
                raise ActorUnavailableError(f"actor {self.name or self.actor_id} did not come up within "
                                            f"{self.CONNECT_TIMEOUT}s")
            time.sleep(0.005)

    def _constructor_failed(self):
        with open(self.err_path, "rb") as f:
            exc, tb = cloudpickle.load(f)
        self.dead = True
        self.death_cause = f"actor constructor raised {exc!r}\n{tb}"
        self.manager.release(self)
        raise ActorDiedError(self.death_cause) from exc

    def _died_msg(self):
        return f"actor {self.name or self.actor_id} is dead" + (f": {self.death_cause}" if self.death_cause else "")

    def _ensure_conn(self) -> socket.socket:
        with self._lock:
            if self._conn is None:
                self._conn = self._connect()
                threading.Thread(target=self._reader, args=(self._conn,), daemon=True,
                                 name=f"actor-reader-{self.actor_id[:6]}").start()
            return self._conn

    def _reader(self, conn):
        from raydp_amd.runtime import serialization as S
        try:
            while True:
                call_id, ok, value = S.loads(recv_frame(conn))
                with self._lock:
                    fut = self._pending.pop(call_id, None)
                if fut is None:
                    continue
                if ok:
                    fut.set_result(value)
                else:
                    exc, tb = value
                    fut.set_exception(_remote_error(exc, tb))
        except (ConnectionError, OSError, EOFError):
            pass
        with self._lock:
            if self._conn is conn:
                self._conn = None
            pending, self._pending = self._pending, {}
        for f in pending.values():
            if not f.done():
                f.set_exception(ActorDiedError(f"actor {self.name or self.actor_id} died while a call was "
                                               "in flight"))

    def call(self, name, args, kwargs) -> ObjectRef:
        from raydp_amd.runtime import serialization as S
        from raydp_amd.runtime.api import _resolve_args
        if self.dead:
            raise ActorDiedError(self._died_msg())
        ref = ObjectRef()
        fut: cf.Future = cf.Future()
        core.register_pending(ref.id, fut)
        a, k = _resolve_args(args, kwargs)
        cid = next(self._ids)
        payload = S.dumps((cid, name, a, k))
        for attempt in range(2):
            try:
                conn = self._ensure_conn()
                with self._lock:
                    self._pending[cid] = fut
                send_frame(conn, self._send_lock, payload)
                break
            except (ActorDiedError,) as e:
                fut.set_exception(e)
                break
            except OSError:
                with self._lock:
                    self._pending.pop(cid, None)
                    self._conn = None
                if attempt == 1:
                    fut.set_exception(ActorDiedError(self._died_msg()))
        return ref

    def kill(self, no_restart=True):
        sup = self.manager.supervisor
        if no_restart:
            self.dead = True
            self.death_cause = self.death_cause or "killed"
        sup.kill(self.actor_id, no_restart=no_restart)
        if no_restart:
            sup.wait_dead(self.actor_id, 10)
            self.manager.release(self)
        with self._lock:
            c = self._conn
        if c is not None:
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass

    def on_event(self, ev):
        kind = ev[0]
        if kind == "died" and ev[4] == "0" and not self.manager.relocating(self):
            self.dead = True
            self.death_cause = self.death_cause or f"process exited with status {ev[3]}"
            self.manager.release(self)
        elif kind == "restarted":
            self.restarts = int(ev[3])


class _RemoteErrorBase(Exception):
    pass


def _remote_error(exc, tb):
    """Re-raise the actor's exception type when possible, with the remote traceback attached."""
    try:
        exc.__cause__ = _RemoteErrorBase(f"remote traceback:\n{tb}")
    except Exception:  # noqa: BLE001
        pass
    return exc


class ActorManager:
    def __init__(self, node):
        self.node = node
        self._sup = None
        self._lock = threading.RLock()
        self.actors: Dict[str, ProcessActor] = {}
        self._relocating = set()

    @property
    def supervisor(self):
        with self._lock:
            if self._sup is None:
                from raydp_amd.runtime.supervisor import SupervisorClient
                os.makedirs(os.path.join(self.node.session_dir, "actors"), exist_ok=True)
                if getattr(self.node, "attached", False):
                    self._sup = SupervisorClient(getattr(self.node, "supervisor_sock", None)
                                                 or os.environ["RAYDP_SUPERVISOR_SOCK"])
                else:
                    self._sup = SupervisorClient.launch(self.node.session_dir)
                self._sup.subscribe(self._on_event)
            return self._sup

    def _on_event(self, ev):
        with self._lock:
            a = self.actors.get(ev[1])
        if a is not None:
            a.on_event(ev)

    def relocating(self, a) -> bool:
        with self._lock:
            return a.actor_id in self._relocating

    def create(self, cls, args, kwargs, opts, name, namespace) -> ProcessActor:
        from raydp_amd.runtime.api import _resolve_args
        sup = self.supervisor
        gcs = getattr(self.node, "gcs", None)
        remote = None
        if gcs is not None:
            # an attached driver: the head places the actor in its cluster table
            strat = opts.get("scheduling_strategy")
            pg = opts.get("placement_group") or getattr(strat, "placement_group", None)
            bidx = opts.get("placement_group_bundle_index", getattr(strat, "placement_group_bundle_index", -1))
            req = {k: opts[k] for k in ("num_cpus", "num_gpus", "memory", "resources") if opts.get(k) is not None}
            if getattr(strat, "node_id", None):
                req["node_id"] = strat.node_id
            if opts.get("lifetime") == "detached":
                req["lifetime"] = "detached"     # the reservation outlives this driver's connection
            remote = gcs.call("place", req, pg.id.hex() if pg is not None else None, bidx)
            from raydp_amd.runtime.node import VirtualNode
            from raydp_amd.runtime.store import attach_store
            st = self.node.store if remote["store_path"] == self.node.store.path else \
                attach_store(remote["store_path"], remote["node_id"])
            vnode, res, pg, bundle = VirtualNode(remote["node_id"], {}, st, ip=remote["node_ip"] or None), {}, None, None
        else:
            vnode, res, pg, bundle = self._place(opts)
        aid = uuid.uuid4().hex[:16]
        a = ProcessActor(self, aid, name, namespace, opts, vnode, res, pg, bundle)
        a.gcs_token = remote["token"] if remote is not None else None
        ra, rk = _resolve_args(args, kwargs)
        clean = {k: v for k, v in opts.items() if k not in ("scheduling_strategy", "placement_group")}
        a.opts = dict(opts, _class_name=getattr(cls, "__name__", str(cls)))
        a.gpu_take = [] if remote is not None else self._take_gpus(vnode, res.get("GPU", 0.0))
        a.gpu_ids = list(remote["gpu_ids"]) if remote is not None else [g for g, _ in a.gpu_take]
        if a.gpu_ids:
            a.opts["_gpu_ids"] = a.gpu_ids
        with open(a.spec_path + ".tmp", "wb") as f:
            cloudpickle.dump((cls, ra, rk, clean), f)
        os.replace(a.spec_path + ".tmp", a.spec_path)
        with self._lock:
            self.actors[aid] = a
        _ = sup
        a.start()
        if remote is not None and opts.get("lifetime") == "detached" and getattr(a, "pid", None):
            try:
                gcs.call("watch", remote["token"], int(a.pid))
            except (OSError, RuntimeError):
                pass
        return a

    def _place(self, opts):
        """Pick the virtual node (and reserve resources) for a new actor."""
        node = self.node
        req = {"CPU": float(opts.get("num_cpus", 1) if opts.get("num_cpus") is not None else 1),
               "GPU": float(opts.get("num_gpus", 0) or 0)}
        if opts.get("memory"):
            req["memory"] = float(opts["memory"])
        for k, v in (opts.get("resources") or {}).items():
            req[k] = float(v)
        strat = opts.get("scheduling_strategy")
        pg = opts.get("placement_group") or getattr(strat, "placement_group", None)
        bidx = opts.get("placement_group_bundle_index", getattr(strat, "placement_group_bundle_index", -1))
        if getattr(node, "attached", False):
            return None, {}, None, None
        cl = node.cluster
        with cl.lock:
            if pg is not None and pg.state == "CREATED":
                idxs = [bidx] if bidx is not None and bidx >= 0 else list(range(pg.bundle_count))
                for i in idxs:
                    free = pg.bundle_free[i]
                    if all(free.get(k, 0.0) + 1e-9 >= v for k, v in req.items() if v):
                        for k, v in req.items():
                            if v:
                                free[k] = free.get(k, 0.0) - v
                        return cl.nodes[pg.bundle_nodes[i]], req, pg, i
                raise core_resource_error(f"placement group bundle(s) {idxs} cannot fit actor request {req}")
            prefer = getattr(strat, "node_id", None)
            vn = cl.pick_node(req, prefer=prefer)
            vn.acquire(req)
            return vn, req, None, None

    @staticmethod
    def _take_gpus(vnode, n: float):
        """GPU assignment: the actor sees exactly these devices (HIP_VISIBLE_DEVICES). A
        fractional request (``num_gpus=0.5``: several workers rehearsing on one card) packs onto
        the most-used GPU that still has that much capacity left; a whole request takes idle
        GPUs. Returns ``[(gpu id, share)]``."""
        import math
        if vnode is None or not n:
            return []
        if not hasattr(vnode, "gpu_cap"):
            vnode.gpu_cap = [1.0] * int(vnode.total.get("GPU", 0))
        cap = vnode.gpu_cap
        if n < 1.0:
            fits = [i for i, c in enumerate(cap) if c + 1e-9 >= n]
            if not fits:
                return []
            i = min(fits, key=lambda j: (cap[j], j))
            cap[i] -= n
            return [(i, float(n))]
        idle = [i for i, c in enumerate(cap) if c >= 1.0 - 1e-9][:int(math.ceil(n))]
        for i in idle:
            cap[i] = 0.0
        return [(i, 1.0) for i in idle]

    def release(self, a: ProcessActor):
        with self._lock:
            if getattr(a, "_released", False):
                return
            a._released = True
        token = getattr(a, "gcs_token", None)
        if token is not None:
            try:
                self.node.gcs.call("release", token)
            except (OSError, RuntimeError):
                pass            # head gone: its table went with it
            return
        if getattr(a, "gpu_take", None) and a.vnode is not None and hasattr(a.vnode, "gpu_cap"):
            for g, share in a.gpu_take:
                a.vnode.gpu_cap[g] = min(1.0, a.vnode.gpu_cap[g] + share)
        cl = self.node.cluster
        with cl.lock:
            if a.pg is not None:
                free = a.pg.bundle_free[a.bundle] if a.pg.state == "CREATED" else None
                if free is not None:
                    for k, v in a.resources.items():
                        if v:
                            free[k] = free.get(k, 0.0) + v
            elif a.vnode is not None and a.resources:
                a.vnode.release(a.resources)

    def on_node_removed(self, node_id):
        """Actors of a removed node die; those with restarts left come back elsewhere."""
        with self._lock:
            victims = [a for a in self.actors.values()
                       if a.vnode is not None and a.vnode.node_id == node_id and not a.dead]
        for a in victims:
            with self._lock:
                self._relocating.add(a.actor_id)
            try:
                self.supervisor.kill(a.actor_id, no_restart=True)
                self.supervisor.wait_dead(a.actor_id, 10)
            finally:
                with self._lock:
                    self._relocating.discard(a.actor_id)
            can = a.max_restarts < 0 or a.restarts < a.max_restarts
            if not can:
                a.dead = True
                a.death_cause = "node removed"
                continue
            cl = self.node.cluster
            with cl.lock:
                try:
                    vn = cl.pick_node(a.resources)
                    vn.acquire(a.resources)
                except Exception:  # noqa: BLE001
                    a.dead = True
                    a.death_cause = "node removed and no node can host the actor"
                    continue
            a.vnode, a.pg = vn, None
            a.restarts += 1
            a.start()

    def list(self):
        with self._lock:
            return list(self.actors.values())

    def kill_owned(self):
        """Kill the actors this process created (owned, not ``lifetime="detached"``)."""
        with self._lock:
            mine = [a for a in self.actors.values()
                    if a.owned and not a.dead and (a.opts or {}).get("lifetime") != "detached"]
        for a in mine:
            try:
                a.kill(no_restart=True)
            except Exception:  # noqa: BLE001 - best effort at shutdown
                pass
            if a.name:
                # (the process's current node is already unset at shutdown: use this node's dir)
                safe = "".join(c if c.isalnum() or c in "-_." else "_" for c in f"{a.namespace}__{a.name}")
                try:
                    os.unlink(os.path.join(self.node.session_dir, "named", safe))
                except OSError:
                    pass

    def shutdown(self):
        with self._lock:
            sup, self._sup = self._sup, None
            self.actors.clear()
        if sup is not None:
            if getattr(self.node, "attached", False):
                sup.close()
            else:
                sup.shutdown()


def core_resource_error(msg):
    from raydp_amd.runtime.node import ResourceError
    return ResourceError(msg)
