"""Shuffle exchange between stages: in-store (default) or through the per-node external
shuffle service (``spark.shuffle.service.enabled``; ``csrc/exec/shuffle_service.cc``).

A wide operator (join / aggregate / distinct / window, ``raydp_amd.spark.wide``) hash-partitions
every input partition into ``n`` buckets (map side) and then combines bucket ``j`` of every map
output (reduce side). ``exchange`` runs the map side and returns a ``Shuffle`` whose
``bucket(j)`` a reduce task calls:

* **in-store**: map tasks return their bucket tables; they travel through the node's
  shared-memory object store and the reduce stage's payload carries them.
* **service**: a map task writes its buckets as consecutive Arrow IPC streams into one file in
  its node's shuffle-service directory and registers it; it returns only ``(socket, shuffle,
  map)``. A reduce task FETCHes each map's bucket: the service answers with (offset, length)
  and passes the file descriptor itself (SCM_RIGHTS), and the task mmaps the bucket. Map
  outputs then outlive the executor that wrote them (the reference's reason for the service:
  ``RayAppMaster.scala:155-163``, ``doc/spark_on_ray.md`` dynamic allocation).
"""
import mmap
import os
import socket
import threading
import uuid
from typing import Dict, List, Optional, Tuple

import pyarrow as pa

from raydp_amd.runtime.supervisor import encode, read_frame

OP_REGISTER, OP_FETCH, OP_REMOVE, OP_LIST, OP_DATA_DIR, OP_PING, OP_SHUTDOWN = 1, 2, 3, 4, 5, 6, 7

# set in executor processes from their app-master registration (ExecutorRegistration)
_LOCAL_SERVICE: Optional[str] = None
_clients: Dict[str, "ShuffleServiceClient"] = {}
_clients_lock = threading.Lock()


def set_local_service(path: Optional[str]):
    global _LOCAL_SERVICE
    _LOCAL_SERVICE = path


def local_service() -> Optional[str]:
    return _LOCAL_SERVICE


def client(path: str) -> "ShuffleServiceClient":
    with _clients_lock:
        c = _clients.get(path)
        if c is None:
            c = _clients[path] = ShuffleServiceClient(path)
        return c


class ShuffleServiceClient:
    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()
        self._sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._sock.connect(path)
        self._dir = None

    def _req(self, op, strs):
        with self._lock:
            self._sock.sendall(encode(op, [str(s) for s in strs]))
            return read_frame(self._sock)[1]

    def ping(self) -> bool:
        return self._req(OP_PING, []) == ["pong"]

    def data_dir(self) -> str:
        if self._dir is None:
            self._dir = self._req(OP_DATA_DIR, [])[1]
        return self._dir

    def register(self, shuffle_id: str, map_id: int, path: str, offsets: List[int]):
        out = self._req(OP_REGISTER, [shuffle_id, map_id, path, ",".join(str(o) for o in offsets)])
        if out[0] != "ok":
            raise RuntimeError(f"shuffle output registration failed: {out[1:]}")

    def fetch(self, shuffle_id: str, map_id: int, reduce_id: int) -> Optional[pa.Table]:
        """Bucket ``reduce_id`` of one map output, mmapped from the descriptor the service
        passes (no copy through the service)."""
        with self._lock:
            self._sock.sendall(encode(OP_FETCH, [shuffle_id, str(map_id), str(reduce_id)]))
            first, fds, _, _ = socket.recv_fds(self._sock, 1, 1)
            if not first:
                raise ConnectionError("shuffle service closed the connection")
            # the rest of the frame: 3 more length bytes, then the payload
            rest = b""
            while len(rest) < 3:
                chunk = self._sock.recv(3 - len(rest))
                if not chunk:
                    raise ConnectionError("shuffle service closed the connection")
                rest += chunk
            import struct
            (n,) = struct.unpack("<I", first + rest)
            payload = b""
            while len(payload) < n:
                chunk = self._sock.recv(n - len(payload))
                if not chunk:
                    raise ConnectionError("shuffle service closed the connection")
                payload += chunk
        op, cnt = struct.unpack_from("<II", payload, 0)
        off, out = 8, []
        for _ in range(cnt):
            (ln,) = struct.unpack_from("<I", payload, off)
            off += 4
            out.append(payload[off:off + ln].decode())
            off += ln
        if out[0] != "ok":
            for fd in fds:
                os.close(fd)
            return None
        start, length = int(out[1]), int(out[2])
        fd = fds[0]
        try:
            if length == 0:
                return None
            page = start - start % mmap.ALLOCATIONGRANULARITY
            mm = mmap.mmap(fd, length + (start - page), prot=mmap.PROT_READ, offset=page)
        finally:
            os.close(fd)
        buf = pa.py_buffer(mm)[start - page:]
        return pa.ipc.open_stream(buf).read_all()

    def remove(self, shuffle_id: str) -> int:
        return int(self._req(OP_REMOVE, [shuffle_id])[1])

    def list(self) -> List[Tuple[str, int, int, int]]:
        out = []
        for x in self._req(OP_LIST, [])[1:]:
            sid, mid, nb, nbytes = x.rsplit(":", 3)
            out.append((sid, int(mid), int(nb), int(nbytes)))
        return out


def write_map_output(service: str, shuffle_id: str, map_id: int, buckets: List[pa.Table]) -> Tuple[str, str, int]:
    """Write ``buckets`` as consecutive IPC streams into one file and register it."""
    c = client(service)
    d = c.data_dir()
    path = os.path.join(d, f"shuffle_{shuffle_id}_{map_id}_{uuid.uuid4().hex[:8]}.data")
    offsets = [0]
    with pa.OSFile(path, "wb") as f:
        for t in buckets:
            if t.num_rows == 0:
                offsets.append(offsets[-1])
                continue
            with pa.ipc.new_stream(f, t.schema) as w:
                w.write_table(t)
            offsets.append(f.tell())
    c.register(shuffle_id, map_id, path, offsets)
    return service, shuffle_id, map_id


class Shuffle:
    """Result of the map side; ``bucket(j)`` is called by reduce tasks (any process)."""

    def __init__(self, schema: pa.Schema, pieces=None, outputs=None, shuffle_id: str = None):
        self.schema = schema
        self.pieces = pieces          # in-store: List[List[pa.Table]]
        self.outputs = outputs        # service: List[(socket, shuffle_id, map_id)]
        self.shuffle_id = shuffle_id

    def bucket(self, j: int) -> pa.Table:
        from raydp_amd.spark.plan import concat
        if self.pieces is not None:
            return concat([p[j] for p in self.pieces], self.schema)
        parts = []
        for sock, sid, mid in self.outputs:
            t = client(sock).fetch(sid, mid, j)
            if t is not None:
                parts.append(t)
        return concat(parts, self.schema)

    def release(self):
        if self.outputs:
            for sock in {o[0] for o in self.outputs}:
                try:
                    client(sock).remove(self.shuffle_id)
                except OSError:
                    pass


def _service_enabled(scheduler) -> bool:
    backend = getattr(scheduler, "backend", None)
    return bool(backend is not None and getattr(backend, "shuffle_service_enabled", False))


def exchange(scheduler, compute, n_maps: int, keys: List[str], n: int, schema: pa.Schema) -> Shuffle:
    """Run the map side of a hash shuffle of ``compute(i)`` (i < n_maps) into ``n`` buckets."""
    from raydp_amd.spark.plan import hash_partition
    if _service_enabled(scheduler):
        sid = uuid.uuid4().hex[:12]

        def map_task(i):
            svc = local_service()
            if svc is None:
                raise RuntimeError("shuffle service enabled but this executor has none")
            return write_map_output(svc, sid, i, hash_partition(compute(i), keys, n))
        outs = scheduler.map(map_task, range(n_maps))
        return Shuffle(schema, outputs=outs, shuffle_id=sid)
    pieces = scheduler.map(lambda i: hash_partition(compute(i), keys, n), range(n_maps))
    return Shuffle(schema, pieces=pieces)
