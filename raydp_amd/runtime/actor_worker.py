"""Entry point of an actor process (``python -m raydp_amd.runtime.actor_worker``).

Started by the native supervisor with ``RAYDP_ACTOR_ID`` / ``RAYDP_SESSION_DIR`` /
``RAYDP_STORE_PATH`` / ``RAYDP_NODE_ID`` / ``RAYDP_SUPERVISOR_SOCK`` in its environment. It
attaches to the node (object store + supervisor), rebuilds the actor instance from the spec
file the creator wrote (so a supervisor restart re-runs the constructor, Ray's actor-restart
semantics), then serves method calls on a Unix-domain socket:

    request  = frame(dumps((call_id, method, args, kwargs)))
    reply    = frame(dumps((call_id, ok, value_or_(exception, traceback))))

Calls run on a pool of ``max_concurrency`` threads; a sequential actor (1, Ray's default) runs
them on the connection's reader thread under one execution lock (no hand-off per call). ``__ray_terminate__`` exits cleanly (status 0: never restarted). A constructor
failure is written to ``<id>.err`` and the process exits 0 so it is not restarted.
"""
import os
import socket
import struct
import sys
import threading
import traceback
from concurrent.futures import ThreadPoolExecutor


def _recv_exact(conn, n):
    # one MSG_WAITALL receive straight into the frame buffer: the kernel fills it in a single
    # GIL-released wait (the chunked recv + concatenate loop cost a GIL round trip and a copy
    # per socket-buffer fill: 142 us for a 100 KB echo between two threads, 47 us now)
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = conn.recv_into(view[got:], n - got, socket.MSG_WAITALL)
        if not k:
            raise ConnectionError
        got += k
    return buf


def send_frame(conn, lock, data: bytes):
    hdr = struct.pack("<Q", len(data))
    with lock:
        if len(data) < 4096:
            conn.sendall(hdr + data)
            return
        # header and payload gathered by the kernel (no concatenated copy of the payload)
        sent = conn.sendmsg([hdr, data])
        if sent < len(hdr) + len(data):
            rest = memoryview(hdr + data)[sent:] if sent < len(hdr) else memoryview(data)[sent - len(hdr):]
            conn.sendall(rest)


_SPIN = []


def _spin_cfg():
    """(window ns, native poll) of the busy-poll before a blocking frame read (``RAYDP_ACTOR_SPIN_US``, default 0 = sleep
    in recv at once); see csrc/runtime/spin.cc."""
    if not _SPIN:
        try:
            us = float(os.environ.get("RAYDP_ACTOR_SPIN_US", "0") or 0)
        except ValueError:
            us = 0.0
        fn = None
        if us > 0:
            try:
                from raydp_amd.runtime.store import _lib
                lib = _lib()
                fn = lib.rt_spin_readable
                import ctypes
                fn.argtypes, fn.restype = [ctypes.c_int, ctypes.c_int64], ctypes.c_int
            except Exception:  # noqa: BLE001 - no native runtime: plain blocking reads
                fn = None
        _SPIN.append((int(us * 1000), fn))
    return _SPIN[0]


def recv_frame(conn) -> bytearray:
    ns, spin = _spin_cfg()
    if spin is not None:
        spin(conn.fileno(), ns)     # GIL released while it polls
    (n,) = struct.unpack("<Q", _recv_exact(conn, 8))
    return _recv_exact(conn, n)


class _Exit(BaseException):
    pass


def actor_paths(session_dir: str, actor_id: str):
    d = os.path.join(session_dir, "actors")
    return (os.path.join(d, f"{actor_id}.spec"), os.path.join(d, f"{actor_id}.sock"),
            os.path.join(d, f"{actor_id}.err"))


def main() -> int:
    aid = os.environ["RAYDP_ACTOR_ID"]
    sdir = os.environ["RAYDP_SESSION_DIR"]
    from raydp_amd.runtime import core
    core.attach_from_env()
    try:   # same ray / pyspark / horovod facades as the driver, installed on first import
        from raydp_amd import compat
        compat.install_lazy()
    except Exception:  # noqa: BLE001
        pass
    from raydp_amd.runtime import serialization as S
    spec_path, sock_path, err_path = actor_paths(sdir, aid)
    import cloudpickle
    with open(spec_path, "rb") as f:
        cls, args, kwargs, opts = cloudpickle.load(f)
    os.environ["RAYDP_ACTOR_NAME"] = opts.get("name") or ""
    try:
        instance = cls(*args, **kwargs)
    except BaseException as e:  # noqa: BLE001
        with open(err_path + ".tmp", "wb") as f:
            try:
                cloudpickle.dump((e, traceback.format_exc()), f)
            except Exception:  # unpicklable exception
                cloudpickle.dump((RuntimeError(repr(e)), traceback.format_exc()), f)
        os.replace(err_path + ".tmp", err_path)
        return 0
    # the actor's long-lived state (imported modules, warmed engine) moves to the permanent GC
    # generation: full collections, and heap walks such as gc.get_referrers, then skip it
    import gc
    gc.collect()
    gc.freeze()
    conc = int(opts.get("max_concurrency") or 1)
    # a sequential actor runs each call on the connection's own reader thread under one
    # execution lock (same one-call-at-a-time semantics as a one-thread pool, without the
    # queue hand-off to a second thread on every call); concurrent actors use the pool
    pool = ThreadPoolExecutor(max_workers=conc, thread_name_prefix=f"actor-{aid[:6]}") if conc > 1 else None
    exec_lock = threading.Lock()
    tmp = sock_path + ".tmp"
    for p in (tmp,):
        if os.path.exists(p):
            os.unlink(p)
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(tmp)
    srv.listen(64)
    os.replace(tmp, sock_path)     # the socket appears atomically once we can accept
    exiting = threading.Event()

    def run_call(conn, lock, call_id, method, a, k):
        if method == "__ray_terminate__":
            send_frame(conn, lock, S.dumps((call_id, True, None)))
            exiting.set()
            os._exit(0)
        try:
            if method == "__ray_ready__":
                v = True
            elif method == "__ray_call__":   # run an arbitrary fn(instance, *args)
                v = a[0](instance, *a[1:], **k)
            else:
                v = getattr(instance, method)(*a, **k)
            payload = S.dumps((call_id, True, v))
        except SystemExit as e:
            send_frame(conn, lock, S.dumps((call_id, True, None)))
            os._exit(int(e.code or 0))
        except BaseException as e:  # noqa: BLE001
            tb = traceback.format_exc()
            try:
                payload = S.dumps((call_id, False, (e, tb)))
            except Exception:  # noqa: BLE001
                payload = S.dumps((call_id, False, (RuntimeError(repr(e)), tb)))
        try:
            send_frame(conn, lock, payload)
        except OSError:
            pass

    def serve(conn):
        lock = threading.Lock()
        try:
            while True:
                call_id, method, a, k = S.loads(recv_frame(conn))
                if pool is None:
                    with exec_lock:
                        run_call(conn, lock, call_id, method, a, k)
                else:
                    pool.submit(run_call, conn, lock, call_id, method, a, k)
        except (ConnectionError, OSError, EOFError):
            pass
        finally:
            try:
                conn.close()
            except OSError:
                pass

    while not exiting.is_set():
        conn, _ = srv.accept()
        threading.Thread(target=serve, args=(conn,), daemon=True).start()
    return 0


if __name__ == "__main__":
    sys.exit(main())
