"""Python side of the native application master (``csrc/control/app_master.cc``).

``AppMasterClient.launch`` starts ``raydp_appmaster`` with a pipe on its stdin and waits for the
handshake file it writes (socket path + pid, via tmp + rename) — the reference's py4j gateway
start-up (``python/raydp/spark/ray_cluster_master.py:103-183`` with
``AppMasterEntryPoint.scala:39-94``), minus the JVM. The master dies when that pipe closes.

The driver (``ClusterBackend``) registers the application and carries out the master's launch
orders (``RayExecutorUtils.createExecutorActor``'s role); executors register themselves over a
connection they keep for life (``ExecutorRegistration``), so the master sees an executor's
death as that connection's EOF (``RayAppMaster.onDisconnected``).
"""
import os
import socket
import subprocess
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from raydp_amd.exceptions import AppMasterError
from raydp_amd.runtime.supervisor import encode, read_frame

(OP_REGISTER_APP, OP_UNREGISTER_APP, OP_REGISTER_EXECUTOR, OP_EXECUTOR_STARTED, OP_REQUEST_EXECUTORS,
 OP_KILL_EXECUTORS, OP_GET_RESTARTED, OP_APP_INFO, OP_RECACHE_RDD, OP_SUBSCRIBE, OP_PING, OP_SHUTDOWN,
 OP_MASTER_URL, OP_EXECUTOR_LOST) = range(1, 15)
OP_EVENT = 100

ENV_SOCKET = "RAYDP_APPMASTER_SOCKET"
CONN_INFO_ENV = "_RAYDP_APPMASTER_CONN_INFO_PATH"


@dataclass
class LaunchOrder:
    """One executor the master wants created (``requestNewExecutor``)."""
    executor_id: str
    cpu: float
    memory_mb: int
    cores: int
    bundle: int
    resources: Dict[str, float] = field(default_factory=dict)

    @classmethod
    def parse(cls, s: str) -> "LaunchOrder":
        kv = dict(p.split("=", 1) for p in s.split(";"))
        res = {}
        for item in filter(None, kv.get("res", "").split(",")):
            k, v = item.rsplit(":", 1)
            res[k] = float(v)
        return cls(kv["id"], float(kv["cpu"]), int(kv["memory_mb"]), int(kv["cores"]), int(kv["bundle"]), res)


class _Conn:
    def __init__(self, path: str):
        self.path = path
        self.lock = threading.Lock()
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.connect(path)

    def request(self, op: int, strs: List[str]) -> List[str]:
        with self.lock:
            self.sock.sendall(encode(op, [str(s) for s in strs]))
            _, out = read_frame(self.sock)
        return out

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


class AppMasterClient:
    def __init__(self, sock_path: str, proc: Optional[subprocess.Popen] = None):
        self.sock_path = sock_path
        self.proc = proc
        self._c = _Conn(sock_path)
        self._sub: Optional[_Conn] = None
        self.app_id: Optional[str] = None

    # ------------------------------------------------------------------ lifecycle --------
    @classmethod
    def launch(cls, workdir: str, timeout: float = 30.0) -> "AppMasterClient":
        from raydp_amd.native import loader
        exe = loader.executable("raydp_appmaster")
        try:
            shuffle = loader.executable("raydp_shuffle_service")
        except Exception:  # noqa: BLE001
            shuffle = ""
        os.makedirs(workdir, exist_ok=True)
        sock = os.path.join(workdir, f"appmaster-{os.getpid()}-{int(time.time() * 1e3) % 100000}.sock")
        info = sock + ".conn"
        log_dir = os.path.join(workdir, "logs")
        os.makedirs(log_dir, exist_ok=True)
        err = open(os.path.join(log_dir, "appmaster.err"), "ab")
        env = dict(os.environ, **{CONN_INFO_ENV: info})
        proc = subprocess.Popen([exe, sock, info] + ([shuffle] if shuffle else []), stdin=subprocess.PIPE,
                                stdout=err, stderr=err, close_fds=True, env=env)
        err.close()
        deadline = time.time() + timeout
        while not os.path.exists(info):
            if proc.poll() is not None:
                raise AppMasterError(f"app master exited with {proc.returncode} before its handshake")
            if time.time() > deadline:
                proc.kill()
                raise AppMasterError("app master handshake timed out")
            time.sleep(0.002)
        with open(info) as f:
            path, pid = f.read().split()
        if int(pid) != proc.pid:
            raise AppMasterError("handshake file from another process")
        return cls(path, proc)

    def shutdown(self):
        try:
            self._c.request(OP_SHUTDOWN, [])
        except OSError:
            pass
        self._c.close()
        if self._sub is not None:
            self._sub.close()
        if self.proc is not None:
            try:
                self.proc.stdin.close()
            except OSError:
                pass
            try:
                self.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
            self.proc = None

    def ping(self) -> bool:
        return self._c.request(OP_PING, []) == ["pong"]

    # ------------------------------------------------------------------ application ------
    def register_app(self, name: str, num_executors: int, cores: int, memory_mb: int, actor_cpu: float,
                     resources: Dict[str, float] = None, bundles: List[int] = None, dyn_alloc: bool = False,
                     max_executors: int = 0, shuffle_service: bool = False, local_dir: str = "",
                     node_ip: str = "127.0.0.1", user: str = "") -> List[LaunchOrder]:
        res = ",".join(f"{k}={v}" for k, v in (resources or {}).items())
        out = self._c.request(OP_REGISTER_APP, [
            name, num_executors, cores, memory_mb, actor_cpu, user or os.environ.get("USER", ""), res,
            ",".join(str(b) for b in (bundles or [])), int(dyn_alloc), max_executors, int(shuffle_service),
            local_dir or "", node_ip])
        if out[0] != "ok":
            raise AppMasterError(f"RegisterApplication failed: {out[1:]}")
        self.app_id, self.master_url = out[1], out[2]
        return [LaunchOrder.parse(o) for o in out[3:]]

    def unregister_app(self):
        self._c.request(OP_UNREGISTER_APP, [self.app_id or ""])

    def request_executors(self, total: int) -> List[LaunchOrder]:
        out = self._c.request(OP_REQUEST_EXECUTORS, [self.app_id, total])
        if out[0] != "ok":
            raise AppMasterError(f"RequestExecutors failed: {out[1:]}")
        return [LaunchOrder.parse(o) for o in out[1:]]

    def kill_executors(self, ids: List[str]) -> List[str]:
        out = self._c.request(OP_KILL_EXECUTORS, [self.app_id] + list(ids))
        if out[0] not in ("ok", "partial"):
            raise AppMasterError(f"KillExecutors failed: {out[1:]}")
        return out[1:]

    def executor_lost(self, executor_id: str) -> bool:
        return self._c.request(OP_EXECUTOR_LOST, [executor_id, 0])[0] == "ok"

    def get_restarted(self) -> Dict[str, str]:
        out = self._c.request(OP_GET_RESTARTED, [])
        return dict(x.split("=", 1) for x in out[1:])

    def app_info(self) -> Dict[str, object]:
        out = self._c.request(OP_APP_INFO, [])
        info: Dict[str, object] = {"executors": {}, "removed": [], "shuffle_services": {}}
        for item in out[1:]:
            k, v = item.split("=", 1)
            if k == "executor":
                eid, reg, started, node, bundle = v.split(":", 4)
                info["executors"][eid] = {"registered": reg == "registered", "started": started == "started",
                                          "node": node, "bundle": int(bundle)}
            elif k == "removed":
                info["removed"].append(v)
            elif k == "shuffle_service":
                node, path = v.split(":", 1)
                info["shuffle_services"][node] = path
            else:
                info[k] = v
        return info

    def get_master_url(self) -> str:
        return self._c.request(OP_MASTER_URL, [])[1]

    def recache_rdd(self, rdd_id: str) -> int:
        return int(self._c.request(OP_RECACHE_RDD, [rdd_id])[1])

    def subscribe(self, fn: Callable[[List[str]], None]):
        """Driver agent (``RayDPDriverAgent``): ``fn(["recache", rdd_id])`` per pushed event."""
        c = _Conn(self.sock_path)
        if c.request(OP_SUBSCRIBE, []) != ["ok"]:
            raise AppMasterError("subscribe refused")
        self._sub = c

        def loop():
            while True:
                try:
                    _, ev = read_frame(c.sock)
                except (OSError, ConnectionError):
                    return
                try:
                    fn(ev)
                except Exception:  # noqa: BLE001
                    pass
        threading.Thread(target=loop, daemon=True, name="raydp-driver-agent").start()


class ExecutorRegistration:
    """An executor's connection to the master, held open for the executor's lifetime
    (``RayDPExecutor.registerToAppMaster`` + ``ExecutorStarted``; ``RayDPExecutor.scala:58-137``)."""

    def __init__(self, sock_path: str, executor_id: str, node_id: str, restarted: bool, tries: int = 3):
        last = None
        for _ in range(tries):
            try:
                self._c = _Conn(sock_path)
                break
            except OSError as e:  # registration retried like the reference's 3 tries
                last = e
                time.sleep(0.05)
        else:
            raise AppMasterError(f"cannot reach the app master: {last}")
        out = self._c.request(OP_REGISTER_EXECUTOR, [executor_id, node_id, os.getpid(), int(restarted)])
        if out[0] != "ok":
            raise AppMasterError(f"executor {executor_id} registration refused: {out[1:]}")
        self.original_id = executor_id
        self.executor_id = out[1]
        self.shuffle_socket = out[2] or None
        self._c.request(OP_EXECUTOR_STARTED, [self.executor_id])

    def recache(self, rdd_id: str) -> int:
        return int(self._c.request(OP_RECACHE_RDD, [rdd_id])[1])

    def close(self):
        self._c.close()
