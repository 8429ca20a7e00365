"""Python front end of the native shared-memory object store (``csrc/runtime/objstore.cc``).

Arrow tables are written as Arrow IPC *directly into the arena* (size measured with a mock
stream, then serialised through a ``FixedSizeBufferWriter`` over the mapped bytes) and read
back zero-copy: the returned table's buffers point into the shared mapping and keep the object
pinned until they are garbage collected. Other values are pickled (protocol 5).

On a GPU node the arena is registered with the HIP runtime (``hipHostRegister``, in 2 MiB
chunks, lazily, by ``csrc/hip/arrow_ingest.hip:rx_pin_range``) the first time a block inside a
chunk is ingested, so a block is DMA'd to HBM straight from the store (``raydp_amd/ops/ingest.py``).
``arena_of(addr)`` finds the mapped arena holding a host address.
"""
import ctypes
import os
import pickle
import threading
import uuid
import weakref
from typing import Any, Optional, Tuple

import cloudpickle
import pyarrow as pa

from raydp_amd.native import loader

KIND_PICKLE, KIND_ARROW, KIND_BYTES = 0, 1, 2
_ID_LEN = 32


class StoreFullError(MemoryError):
    pass


_mapped_lock = threading.Lock()
_mapped = weakref.WeakSet()   # every store arena mapped in this process


def arena_of(addr: int, nbytes: int = 1) -> Optional[Tuple[int, int]]:
    """(base, capacity) of the mapped store arena holding [addr, addr + nbytes), or None."""
    with _mapped_lock:
        stores = list(_mapped)
    for st in stores:
        if st.contains_address(addr, nbytes):
            return st._base, st.capacity
    return None


def _unpin(base: int):
    """Drop this process's GPU registrations of an arena before it is unmapped."""
    import sys
    if "raydp_amd.ops._hip" not in sys.modules:
        return
    from raydp_amd.ops import _hip
    if _hip._lib is not None:
        _hip._lib.rx_unpin_arena(ctypes.c_uint64(base))


def _lib():
    lib = loader.load("raydp_runtime")
    if not getattr(lib, "_rt_typed", False):
        c = ctypes
        lib.rt_store_create.restype = c.c_void_p
        lib.rt_store_create.argtypes = [c.c_char_p, c.c_uint64, c.c_uint32]
        lib.rt_store_open.restype = c.c_void_p
        lib.rt_store_open.argtypes = [c.c_char_p]
        lib.rt_store_close.argtypes = [c.c_void_p]
        lib.rt_store_unlink.argtypes = [c.c_char_p]
        lib.rt_store_data.restype = c.c_void_p
        lib.rt_store_data.argtypes = [c.c_void_p]
        lib.rt_store_capacity.restype = c.c_uint64
        lib.rt_store_capacity.argtypes = [c.c_void_p]
        lib.rt_obj_create.restype = c.c_int64
        lib.rt_obj_create.argtypes = [c.c_void_p, c.c_char_p, c.c_uint64, c.c_int32, c.c_int64]
        for fn in ("rt_obj_seal", "rt_obj_contains", "rt_obj_release", "rt_obj_delete", "rt_obj_abort"):
            getattr(lib, fn).argtypes = [c.c_void_p, c.c_char_p]
            getattr(lib, fn).restype = c.c_int
        lib.rt_obj_get.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_uint64),
                                   c.POINTER(c.c_uint64), c.POINTER(c.c_int32)]
        lib.rt_obj_get.restype = c.c_int
        lib.rt_store_stats.argtypes = [c.c_void_p, c.POINTER(c.c_uint64), c.POINTER(c.c_uint64),
                                       c.POINTER(c.c_uint64)]
        lib.rt_store_list.argtypes = [c.c_void_p, c.c_char_p, c.c_int]
        lib.rt_store_list.restype = c.c_int
        lib._rt_typed = True
    return lib


def _key(oid: str) -> bytes:
    b = oid.encode()
    if len(b) > _ID_LEN:
        raise ValueError("object ids are at most 32 characters")
    return b


class _Pin:
    """Owner object of a zero-copy view; releases the store pin when collected."""
    __slots__ = ("store", "key", "__weakref__")

    def __init__(self, store, key):
        self.store, self.key = store, key

    def __del__(self):
        st = self.store
        if st is not None and st._h is not None:
            st._lib.rt_obj_release(st._h, self.key)


class SharedObjectStore:
    def __init__(self, path: str, node_id: str, create: bool, capacity: int = 0, nslots: int = 65536):
        self._lib = _lib()
        self.path = path
        self.node_id = node_id
        self._owner = create
        if create:
            self._h = self._lib.rt_store_create(path.encode(), int(capacity), int(nslots))
        else:
            self._h = self._lib.rt_store_open(path.encode())
        if not self._h:
            raise OSError(f"cannot {'create' if create else 'open'} object store at {path}")
        self._base = self._lib.rt_store_data(self._h)
        self.capacity = int(self._lib.rt_store_capacity(self._h))
        self._pid = os.getpid()
        self._lock = threading.Lock()
        with _mapped_lock:
            _mapped.add(self)

    # ------------------------------------------------------------------ write ------------
    def _create(self, oid: str, size: int, kind: int) -> Tuple[int, bytes]:
        key = _key(oid)
        off = self._lib.rt_obj_create(self._h, key, int(size), int(kind), self._pid)
        if off == -2:
            raise KeyError(f"object {oid} already exists")
        if off == -1:
            raise StoreFullError(f"object store full ({size} bytes requested, capacity {self.capacity})")
        if off < 0:
            raise StoreFullError("object table full")
        return off, key

    def put(self, oid: str, value: Any) -> int:
        if isinstance(value, pa.RecordBatch):
            value = pa.Table.from_batches([value])
        if isinstance(value, pa.Table):
            sink = pa.MockOutputStream()
            with pa.ipc.new_stream(sink, value.schema) as w:
                w.write_table(value)
            size = sink.size()
            off, key = self._create(oid, size, KIND_ARROW)
            try:
                buf = pa.py_buffer(memoryview((ctypes.c_char * size).from_address(self._base + off)))
                with pa.ipc.new_stream(pa.FixedSizeBufferWriter(buf), value.schema) as w:
                    w.write_table(value)
            except BaseException:
                self._lib.rt_obj_abort(self._h, key)
                raise
            self._lib.rt_obj_seal(self._h, key)
            return size
        if isinstance(value, (bytes, bytearray, memoryview)):
            raw, kind = bytes(value) if not isinstance(value, bytes) else value, KIND_BYTES
        else:
            raw, kind = cloudpickle.dumps(value, protocol=5), KIND_PICKLE
        size = len(raw)
        off, key = self._create(oid, size, kind)
        ctypes.memmove(self._base + off, raw, size)
        self._lib.rt_obj_seal(self._h, key)
        return size

    # ------------------------------------------------------------------ read -------------
    def get(self, oid: str) -> Tuple[bool, Any]:
        key = _key(oid)
        off, size, kind = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
        rc = self._lib.rt_obj_get(self._h, key, ctypes.byref(off), ctypes.byref(size), ctypes.byref(kind))
        if rc != 0:
            return False, None
        pin = _Pin(self, key)
        buf = pa.foreign_buffer(self._base + off.value, size.value, base=pin)
        k = kind.value
        if k == KIND_ARROW:
            return True, pa.ipc.open_stream(buf).read_all()
        if k == KIND_BYTES:
            return True, buf.to_pybytes()
        try:
            return True, pickle.loads(memoryview(buf))
        finally:
            del buf, pin

    def get_buffer(self, oid: str) -> Optional[pa.Buffer]:
        """Zero-copy view of the raw object bytes (pinned while referenced)."""
        key = _key(oid)
        off, size, kind = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
        if self._lib.rt_obj_get(self._h, key, ctypes.byref(off), ctypes.byref(size), ctypes.byref(kind)):
            return None
        return pa.foreign_buffer(self._base + off.value, size.value, base=_Pin(self, key))

    def contains(self, oid: str) -> bool:
        return self._lib.rt_obj_contains(self._h, _key(oid)) == 1

    def delete(self, oid: str):
        self._lib.rt_obj_delete(self._h, _key(oid))

    def stats(self):
        u, c, n = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self._lib.rt_store_stats(self._h, ctypes.byref(u), ctypes.byref(c), ctypes.byref(n))
        return {"used": u.value, "capacity": c.value, "num_objects": n.value}

    def list(self, limit: int = 1 << 16):
        buf = ctypes.create_string_buffer(limit * _ID_LEN)
        n = self._lib.rt_store_list(self._h, buf, limit)
        raw = buf.raw
        return [raw[i * _ID_LEN:(i + 1) * _ID_LEN].rstrip(b"\0").decode() for i in range(n)]

    def base_address(self) -> int:
        return self._base

    def contains_address(self, addr: int, nbytes: int = 1) -> bool:
        return self._h is not None and self._base <= addr and addr + nbytes <= self._base + self.capacity

    def close(self):
        if self._h is not None:
            with _mapped_lock:
                _mapped.discard(self)
            _unpin(self._base)
            self._lib.rt_store_close(self._h)
            self._h = None

    def destroy(self):
        self.close()
        if self._owner:
            try:
                self._lib.rt_store_unlink(self.path.encode())
            except Exception:  # noqa: BLE001
                pass


def _shm_dir() -> str:
    d = "/dev/shm"
    return d if os.path.isdir(d) and os.access(d, os.W_OK) else None


def colocated_stores() -> int:
    """How many object stores this node's processes open side by side: one per local rank of
    an SPMD job (``LOCAL_WORLD_SIZE``, set by torchrun and by bench.py's self-launch), else 1."""
    try:
        return max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    except ValueError:
        return 1


def default_capacity() -> int:
    """Arena size: 30% of the free shared memory, split between the stores co-located on this
    node (8 SPMD ranks must not each claim 30% -- 240% of /dev/shm, a SIGBUS at data scale),
    at most 64 GiB each."""
    env = os.environ.get("RAYDP_OBJECT_STORE_BYTES")
    if env:
        return int(env)
    try:
        st = os.statvfs(_shm_dir() or "/tmp")
        avail = st.f_bavail * st.f_frsize
    except OSError:
        avail = 8 << 30
    share = avail * 0.3 / colocated_stores()
    return int(min(max(share, 16 << 20), 64 << 30))


def open_store(node_id: str, capacity: Optional[int], session_dir: str) -> SharedObjectStore:
    base = _shm_dir() or session_dir
    path = os.path.join(base, f"raydp_objstore_{node_id}_{os.getpid()}")
    return SharedObjectStore(path, node_id, create=True, capacity=capacity or default_capacity())


def attach_store(path: str, node_id: str) -> SharedObjectStore:
    return SharedObjectStore(path, node_id, create=False)
