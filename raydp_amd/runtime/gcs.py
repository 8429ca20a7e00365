"""Head control endpoint: lets OTHER processes attach to a running node (``ray.init(address=...)``).

The reference relies on joining a running cluster in several places: every MPI rank calls
``ray.init(address=reply.ray_address)`` with the address the job driver serves
(``python/raydp/mpi/mpi_worker.py:159-160``, ``mpi/mpi_job.py:303``); ``raydp-submit`` runs an
application against an existing cluster (``doc/spark_on_ray.md:116-144``); the test fixtures
run over both a local cluster and a client address (``python/raydp/tests/conftest.py:77-84``).

Here the head process of a node (``runtime.init()`` without an address) serves a small control
protocol -- the GCS role of Ray core -- on a Unix socket inside its session directory:

* ``info``: what an attaching process needs to map the node -- session directory, object-store
  arena path, node id, supervisor socket, namespace, job id;
* ``place`` / ``release``: resource reservations (plain requests, placement-group bundles,
  GPU assignment) for actors that an attached driver creates, accounted in the head's cluster
  table like the head's own actors (released when the attached process disconnects);
* ``pg_create`` / ``pg_remove`` / ``pg_table``: placement groups in the head's table;
* ``resources`` / ``nodes``: the cluster view (``ray.cluster_resources()`` / ``ray.nodes()``);
* ``kv_put`` / ``kv_get`` / ``kv_del``: a small internal key-value store (string values).

Everything else an attached process does goes straight to the shared substrates: objects to the
shared-memory arena (zero-copy, same host), actors to their own Unix sockets, named actors through
the session directory's ``named/`` files, process lifecycle through the native supervisor.

Security: the protocol is JSON (nothing is unpickled), the Unix socket lives in the session
directory (``mkdtemp``: mode 0700, so only the node's user can connect), and the optional TCP
endpoint (``spark.ray.mi355x.runtime.port`` >= 0; off by default) binds to loopback unless
``spark.ray.mi355x.runtime.host`` says otherwise and admits a connection only after it presents
the session token (``<session>/gcs.token``, mode 0600; ``RAYDP_RUNTIME_TOKEN`` or the
``?token=`` suffix of the address on the client side).

Addresses: ``"raydp://<session dir>"`` (what ``runtime.address()`` returns), a session directory
path, ``"<host>:<port>[?token=...]"`` (the TCP endpoint), or ``"auto"`` -- the address the most
recent head on this host recorded in ``<tmp>/raydp-<uid>/raydp_current_cluster`` (Ray's
``/tmp/ray/ray_current_cluster`` convention). ``RAYDP_ADDRESS`` in the environment is used when
``init()`` gets no address.

Wire format: the actor transport's frames (8-byte little-endian length + UTF-8 JSON of
``{"op", "args"}``; reply ``{"ok", "value"}`` or ``{"ok": false, "error"}``).
"""
import hmac
import json
import os
import secrets
import socket
import tempfile
import threading
import uuid
from typing import Dict, Optional, Tuple

from raydp_amd.runtime.actor_worker import recv_frame, send_frame


def _current_file() -> str:
    return os.path.join(tempfile.gettempdir(), f"raydp-{os.getuid()}", "raydp_current_cluster")


class GcsError(RuntimeError):
    pass


def _dumps(obj) -> bytes:
    return json.dumps(obj, separators=(",", ":")).encode()


def _loads(b) -> dict:
    return json.loads(bytes(b).decode())


# actor options an attached driver may ask the head to place (JSON values only)
_PLACE_KEYS = ("num_cpus", "num_gpus", "memory", "resources")
# largest pre-authentication frame on the TCP endpoint (the hello carries a 32-hex-digit token):
# the length word is checked BEFORE anything is allocated for the frame
_MAX_HELLO = 4096
# largest control frame after authentication (control ops carry small JSON documents)
_MAX_CONTROL_FRAME = 64 << 20


def _recv_bounded(conn, limit: int) -> bytes:
    """One length-prefixed frame (``actor_worker.send_frame`` format) of at most ``limit`` bytes;
    ValueError (connection closed by the caller) past it."""
    import struct
    from raydp_amd.runtime.actor_worker import _recv_exact
    (n,) = struct.unpack("<Q", _recv_exact(conn, 8))
    if n > limit:
        raise ValueError(f"control frame of {n} bytes exceeds {limit}")
    return _recv_exact(conn, n)


class HeadService:
    """The head's control server (one per head node; threads: one acceptor per socket, one
    handler per connection)."""

    def __init__(self, node, tcp_port: int = -1, host: str = "127.0.0.1"):
        self.node = node
        self.uds_path = os.path.join(node.session_dir, "gcs.sock")
        self.token = secrets.token_hex(16)
        tok_path = os.path.join(node.session_dir, "gcs.token")
        fd = os.open(tok_path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as f:
            f.write(self.token)
        self._reservations: Dict[str, tuple] = {}
        self._kv: Dict[str, str] = {}
        self._lock = threading.RLock()
        self._closing = False
        self._socks = []
        self._conns = set()
        u = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        if os.path.exists(self.uds_path):
            os.unlink(self.uds_path)
        u.bind(self.uds_path)
        os.chmod(self.uds_path, 0o600)
        u.listen(64)
        self._socks.append((u, False))
        self.tcp_address = None
        if tcp_port is not None and int(tcp_port) >= 0:
            t = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            t.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            t.bind((host or "127.0.0.1", int(tcp_port)))
            t.listen(64)
            self._socks.append((t, True))
            self.tcp_address = f"{t.getsockname()[0]}:{t.getsockname()[1]}"
        for s, needs_token in self._socks:
            threading.Thread(target=self._accept, args=(s, needs_token), daemon=True,
                             name="raydp-gcs-accept").start()

    @property
    def address(self) -> str:
        return f"raydp://{self.node.session_dir}"

    # ------------------------------------------------------------------ serving
    def _accept(self, lsock, needs_token):
        while not self._closing:
            try:
                c, _ = lsock.accept()
            except OSError:
                return
            if c.family == socket.AF_INET:
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            with self._lock:
                self._conns.add(c)
            threading.Thread(target=self._serve, args=(c, needs_token), daemon=True,
                             name="raydp-gcs-conn").start()

    def _serve(self, conn, needs_token):
        lock = threading.Lock()
        owned = []          # reservations made over this connection: released when it closes
        try:
            if needs_token:
                # the first frame must be {"op": "hello", "args": [token]}; anything else closes
                conn.settimeout(10.0)
                msg = _loads(_recv_bounded(conn, _MAX_HELLO))
                conn.settimeout(None)
                tok = (msg.get("args") or [""])[0] if msg.get("op") == "hello" else ""
                if not hmac.compare_digest(str(tok), self.token):
                    send_frame(conn, lock, _dumps({"ok": False, "error": "bad session token"}))
                    return
                send_frame(conn, lock, _dumps({"ok": True, "value": "welcome"}))
            while True:
                msg = _loads(_recv_bounded(conn, _MAX_CONTROL_FRAME))
                try:
                    reply = {"ok": True, "value": self._handle(msg.get("op"), list(msg.get("args") or []), owned)}
                except Exception as e:  # noqa: BLE001 - reported to the caller
                    reply = {"ok": False, "error": f"{type(e).__name__}: {e}"}
                send_frame(conn, lock, _dumps(reply))
        except (ConnectionError, OSError, EOFError, ValueError, MemoryError):
            pass
        finally:
            with self._lock:
                self._conns.discard(conn)
            # (detached actors' reservations are not in `owned`: they outlive this connection and
            # are released by an explicit 'release' or when the head sees their process die)
            for token in owned:
                self._release(token)
            try:
                conn.close()
            except OSError:
                pass

    def _handle(self, op, args, owned):
        n = self.node
        if op in ("ping", "hello"):
            return "pong"
        if op == "info":
            return n.attach_info()
        if op == "place":
            token, reply = self._place(*args)
            if str(((args[0] if args else None) or {}).get("lifetime") or "") != "detached":
                owned.append(token)
            return reply
        if op == "watch":
            # a detached actor's process: its reservation is released once the process is gone
            self._watch(str(args[0]), int(args[1]))
            return True
        if op == "release":
            self._release(str(args[0]))
            if args[0] in owned:
                owned.remove(args[0])
            return True
        if op == "resources":
            from raydp_amd.runtime import api
            return [api.cluster_resources(), api.available_resources()]
        if op == "nodes":
            from raydp_amd.runtime import api
            return api.nodes()
        if op == "pg_create":
            from raydp_amd.runtime import pgroup
            bundles, strategy, name = args
            pg = pgroup.placement_group([{str(k): float(v) for k, v in b.items()} for b in bundles],
                                        str(strategy), str(name or ""))
            return [pg.id.hex(), list(pg.bundle_nodes)]
        if op == "pg_remove":
            from raydp_amd.runtime import pgroup
            try:
                pgroup.remove_placement_group(pgroup.get_placement_group_by_id(str(args[0])))
            except ValueError:
                pass
            return True
        if op == "pg_table":
            from raydp_amd.runtime import pgroup
            return pgroup.placement_group_table()
        if op == "kv_put":
            with self._lock:
                self._kv[str(args[0])] = str(args[1])
            return True
        if op == "kv_get":
            with self._lock:
                return self._kv.get(str(args[0]))
        if op == "kv_del":
            with self._lock:
                return self._kv.pop(str(args[0]), None) is not None
        raise GcsError(f"unknown control op {op!r}")

    def _place(self, opts: dict, pg_id: Optional[str] = None, bundle: Optional[int] = None) -> Tuple[str, dict]:
        """Reserve an attached driver's actor on the head's cluster table (the head's own
        ``ActorManager._place`` rules), plus its GPU assignment."""
        from raydp_amd.runtime import pgroup
        from raydp_amd.runtime.api import NodeAffinitySchedulingStrategy, PlacementGroupSchedulingStrategy
        o = {k: opts[k] for k in _PLACE_KEYS if k in (opts or {})}
        if pg_id:
            o["scheduling_strategy"] = PlacementGroupSchedulingStrategy(
                pgroup.get_placement_group_by_id(str(pg_id)), int(bundle) if bundle is not None else -1)
        elif (opts or {}).get("node_id"):
            o["scheduling_strategy"] = NodeAffinitySchedulingStrategy(str(opts["node_id"]))
        mgr = self.node.actors
        vnode, req, pg, bidx = mgr._place(o)
        take = mgr._take_gpus(vnode, req.get("GPU", 0.0)) if vnode is not None else []
        token = uuid.uuid4().hex
        with self._lock:
            self._reservations[token] = (vnode, req, pg, bidx, take)
        store = vnode.store if vnode is not None and vnode.store is not None else self.node.store
        return token, {"token": token, "node_id": vnode.node_id if vnode is not None else self.node.node_id,
                       "store_path": store.path, "node_ip": vnode.ip if vnode is not None else "",
                       "gpu_ids": [g for g, _ in take]}

    def _watch(self, token: str, pid: int):
        with self._lock:
            if token not in self._reservations:
                return
            watched = self.__dict__.setdefault("_watched", {})
            watched[token] = pid
            if getattr(self, "_watcher", None) is None:
                self._watcher = threading.Thread(target=self._watch_loop, daemon=True, name="raydp-gcs-watch")
                self._watcher.start()

    def _watch_loop(self, interval: float = 0.5):
        import time
        while not self._closing:
            with self._lock:
                items = list(self._watched.items())
            for token, pid in items:
                try:
                    os.kill(pid, 0)
                    continue
                except ProcessLookupError:
                    pass
                except PermissionError:
                    continue
                with self._lock:
                    self._watched.pop(token, None)
                self._release(token)
            time.sleep(interval)

    def _release(self, token: str):
        with self._lock:
            getattr(self, "_watched", {}).pop(token, None)
            r = self._reservations.pop(token, None)
        if r is None:
            return
        vnode, req, pg, bidx, take = r

        class _R:       # the shape ActorManager.release expects
            pass
        a = _R()
        a.vnode, a.resources, a.pg, a.bundle, a.gpu_take = vnode, req, pg, bidx, take
        self.node.actors.release(a)

    def close(self):
        self._closing = True
        for s, _ in self._socks:
            try:
                s.close()
            except OSError:
                pass
        with self._lock:
            conns, self._conns = list(self._conns), set()
        for c in conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
        for p in (self.uds_path, os.path.join(self.node.session_dir, "gcs.token")):
            try:
                os.unlink(p)
            except OSError:
                pass


# ---------------------------------------------------------------------------- client side
def resolve(address: str) -> Tuple[str, object, Optional[str]]:
    """-> ("unix", socket path, None) or ("tcp", (host, port), token) for an address string."""
    a = str(address).strip()
    if a == "auto":
        f = _current_file()
        if not os.path.exists(f):
            raise ConnectionError(f"address='auto': no running raydp_amd node recorded on this host ({f})")
        with open(f) as fh:
            a = fh.read().strip()
    for pre in ("raydp://", "ray://"):
        if a.startswith(pre):
            a = a[len(pre):]
    if os.path.isdir(a):
        return "unix", os.path.join(a, "gcs.sock"), None
    if a.endswith(".sock") and os.path.exists(a):
        return "unix", a, None
    token = os.environ.get("RAYDP_RUNTIME_TOKEN")
    if "?token=" in a:
        a, token = a.split("?token=", 1)
    host, sep, port = a.rpartition(":")
    if not sep or not port.isdigit():
        raise ValueError(f"cannot parse runtime address {address!r} (want raydp://<session dir>, a session "
                         "directory, host:port[?token=...] or 'auto')")
    return "tcp", (host or "127.0.0.1", int(port)), token


class GcsClient:
    """Thread-safe request/reply connection to a head's control endpoint."""

    def __init__(self, address: str, timeout: float = 30.0):
        kind, where, token = resolve(address)
        self.address = address
        s = socket.socket(socket.AF_UNIX if kind == "unix" else socket.AF_INET, socket.SOCK_STREAM)
        if kind == "tcp":
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.settimeout(timeout)
        try:
            s.connect(where)
        except OSError as e:
            s.close()
            raise ConnectionError(f"no raydp_amd node answers at {address!r}: {e}") from e
        s.settimeout(None)
        self._sock = s
        self._lock = threading.Lock()
        self._send_lock = threading.Lock()
        if kind == "tcp":
            if not token:
                s.close()
                raise ConnectionError(f"{address!r}: the TCP endpoint needs the session token "
                                      "(RAYDP_RUNTIME_TOKEN or '?token=' in the address)")
            self.call("hello", token)

    def call(self, op: str, *args):
        with self._lock:
            send_frame(self._sock, self._send_lock, _dumps({"op": op, "args": list(args)}))
            rep = _loads(recv_frame(self._sock))
        if not rep.get("ok"):
            raise GcsError(rep.get("error", "control request failed"))
        return rep.get("value")

    def close(self):
        try:
            self._sock.close()
        except OSError:
            pass


def record_current(address: str):
    """This host's most recent head (``address='auto'``), in a per-user 0700 directory."""
    f = _current_file()
    os.makedirs(os.path.dirname(f), mode=0o700, exist_ok=True)
    tmp = f"{f}.{os.getpid()}"
    with open(tmp, "w") as fh:
        fh.write(address)
    os.replace(tmp, f)


def clear_current(address: str):
    f = _current_file()
    try:
        with open(f) as fh:
            if fh.read().strip() != address:
                return
        os.unlink(f)
    except OSError:
        pass
