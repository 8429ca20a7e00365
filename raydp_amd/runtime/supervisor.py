"""Python client of the native actor supervisor (``csrc/runtime/supervisor.cc``).

The head process starts one ``raydp_supervisor`` per session with a pipe on its stdin: when the
head exits for any reason the pipe closes and the supervisor terminates every actor process
it spawned (the reference's launcher dies with its parent the same way,
``AppMasterEntryPoint.scala:36-55``). Other processes of the session (actors creating actors)
attach to the same Unix-domain socket.
"""
import os
import signal
import socket
import struct
import subprocess
import threading
from typing import Callable, Dict, List, Optional

OP_SPAWN, OP_KILL, OP_LIST, OP_SUBSCRIBE, OP_SHUTDOWN, OP_PING, OP_WAIT = 1, 2, 3, 4, 5, 6, 7
OP_EVENT, OP_REPLY = 100, 101


def encode(op: int, strs: List[str]) -> bytes:
    parts = [struct.pack("<II", op, len(strs))]
    for s in strs:
        b = s.encode() if isinstance(s, str) else bytes(s)
        parts.append(struct.pack("<I", len(b)))
        parts.append(b)
    payload = b"".join(parts)
    return struct.pack("<I", len(payload)) + payload


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("supervisor connection closed")
        buf += chunk
    return bytes(buf)


def read_frame(sock: socket.socket):
    (n,) = struct.unpack("<I", _recv_exact(sock, 4))
    p = _recv_exact(sock, n)
    op, cnt = struct.unpack_from("<II", p, 0)
    off, out = 8, []
    for _ in range(cnt):
        (ln,) = struct.unpack_from("<I", p, off)
        off += 4
        out.append(p[off:off + ln].decode(errors="replace"))
        off += ln
    return op, out


class SupervisorClient:
    """Request/reply connection (thread-safe) plus an optional event subscription."""

    def __init__(self, sock_path: str, proc: Optional[subprocess.Popen] = None):
        self.sock_path = sock_path
        self.proc = proc
        self._lock = threading.Lock()
        self._sock = self._connect()
        self._listeners: List[Callable[[List[str]], None]] = []
        self._event_thread = None

    def _connect(self) -> socket.socket:
        s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        s.connect(self.sock_path)
        return s

    @classmethod
    def launch(cls, session_dir: str) -> "SupervisorClient":
        from raydp_amd.native import loader
        exe = loader.executable("raydp_supervisor")
        path = os.path.join(session_dir, "sup.sock")
        proc = subprocess.Popen([exe, path], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                stderr=open(os.path.join(session_dir, "logs", "supervisor.err"), "ab"),
                                close_fds=True)
        line = proc.stdout.readline()
        if line.strip() != b"READY":
            proc.kill()
            raise RuntimeError(f"actor supervisor failed to start (got {line!r})")
        return cls(path, proc)

    def request(self, op: int, strs: List[str]) -> List[str]:
        with self._lock:
            self._sock.sendall(encode(op, strs))
            rop, out = read_frame(self._sock)
        return out

    def ping(self) -> bool:
        return self.request(OP_PING, []) == ["pong"]

    def spawn(self, actor_id: str, argv: List[str], env: Dict[str, str], cwd: str = "", log: str = "",
              max_restarts: int = 0) -> int:
        strs = [actor_id, str(int(max_restarts)), cwd, log, str(len(argv))] + list(argv)
        strs += [str(len(env))] + [f"{k}={v}" for k, v in env.items()]
        out = self.request(OP_SPAWN, strs)
        if out[0] != "ok":
            raise RuntimeError(f"spawn of actor {actor_id} failed: {out[1:]}")
        return int(out[1])

    def kill(self, actor_id: str, no_restart: bool = True, sig: int = signal.SIGKILL) -> bool:
        out = self.request(OP_KILL, [actor_id, "1" if no_restart else "0", str(int(sig))])
        return out[0] == "ok"

    def list(self) -> Dict[str, Dict]:
        res = {}
        for e in self.request(OP_LIST, []):
            aid, pid, state, restarts = e.rsplit(":", 3)
            res[aid] = {"pid": int(pid), "state": state, "restarts": int(restarts)}
        return res

    def wait_dead(self, actor_id: str, timeout: float) -> Optional[int]:
        """Exit status once the actor process is dead, None if still alive after ``timeout``."""
        s = self._connect()
        try:
            s.sendall(encode(OP_WAIT, [actor_id, str(int(timeout * 1000))]))
            _, out = read_frame(s)
        finally:
            s.close()
        return int(out[1]) if out[0] == "dead" else None

    def subscribe(self, fn: Callable[[List[str]], None]):
        self._listeners.append(fn)
        if self._event_thread is None:
            s = self._connect()
            s.sendall(encode(OP_SUBSCRIBE, []))
            read_frame(s)

            def loop():
                try:
                    while True:
                        op, ev = read_frame(s)
                        for f in list(self._listeners):
                            try:
                                f(ev)
                            except Exception:  # noqa: BLE001
                                pass
                except (ConnectionError, OSError):
                    return
            self._event_thread = threading.Thread(target=loop, name="raydp-supervisor-events", daemon=True)
            self._event_thread.start()

    def shutdown(self):
        try:
            self.request(OP_SHUTDOWN, [])
        except Exception:  # noqa: BLE001
            pass
        try:
            self._sock.close()
        except OSError:
            pass
        if self.proc is not None:
            try:
                self.proc.stdin.close()
            except OSError:
                pass
            try:
                self.proc.wait(10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait(5)
            self.proc = None

    def close(self):
        try:
            self._sock.close()
        except OSError:
            pass
