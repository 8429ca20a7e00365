"""Python side of the native executor core (``csrc/exec/executor.cc``; SURVEY §2.9 J2,
reference ``core/raydp-main/src/main/scala/org/apache/spark/executor/RayDPExecutor.scala``).

``NativeExecutor`` is one per executor process: the C++ task loop (``cores`` worker threads)
plus the partition cache (``(rdd id, partition) -> object id``, block listing, unpersist) that
``RayDPExecutor.persist_partitions`` / ``get_rdd_partition`` / ``unpersist`` use.

``lower(fn)`` turns a stage function into a native stage when the stage is a chain of narrow
operators that ``raydp_amd/spark/exprc.py`` compiled into expression-VM segments only (no host
operator in between) and every VM input has a type the C++ side checks. A lowered partition
then runs without Python:

    source  -- a byte split of a CSV file (parsed by Arrow C++ with the stage schema), or the
               chain's input table computed in Python and handed over through the Arrow C
               stream interface (in-memory / already parsed / non-CSV sources);
    VM      -- every segment's register program (``rx_expr_run``), string->timestamp inputs
               parsed natively, untouched columns gathered by the surviving rows;
    UDFs    -- a segment with inlined Python UDFs calls ``_tap`` (the UDF bridge) once with its
               exported outputs; the checks are ``exprc.Program.check_taps``, the very code the
               Python path runs, so a guard trip / failed verification decides identically;
    sink    -- Arrow IPC written straight into this node's object store under the block id.

A partition the task loop cannot finish exactly like the Python path comes back as FALLBACK
(or RETRY after a UDF was retired) and the caller computes it through ``fn(i)``.
"""
import ctypes
import itertools
import struct
import threading
import weakref
from typing import Dict, List, Optional, Tuple

import pyarrow as pa  # noqa: F401 - libarrow must be loaded (pyarrow's copy) before ours

OK, FALLBACK, RETRY, ERROR = 0, 1, 2, -1
_ERRLEN = 1024

STATS = {"native_tasks": 0, "native_fallbacks": 0, "native_retries": 0, "native_errors": 0,
         "lowered_stages": 0, "not_lowered": 0, "native_csv_reads": 0, "stage_reuse": 0}
LAST_ERROR = [None]     # message of the last native task that failed (then run in Python)

_TAPFN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                          ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                          ctypes.POINTER(ctypes.c_int64))

_lib_handle = None
_lib_lock = threading.Lock()


def _lib():
    global _lib_handle
    with _lib_lock:
        if _lib_handle is None:
            from raydp_amd.native import loader
            from raydp_amd.runtime import store as _store
            _store._lib()                      # libraydp_runtime.so first (the executor links it)
            lib = loader.load("raydp_executor")
            c = ctypes
            lib.rx_exec_create.restype = c.c_void_p
            lib.rx_exec_create.argtypes = [c.c_int]
            lib.rx_exec_destroy.argtypes = [c.c_void_p]
            lib.rx_stage_create.restype = c.c_void_p
            lib.rx_stage_create.argtypes = [c.c_char_p, c.c_int64, c.c_char_p, c.c_int]
            lib.rx_stage_destroy.argtypes = [c.c_void_p]
            lib.rx_exec_submit.restype = c.c_int64
            lib.rx_exec_submit.argtypes = [c.c_void_p, c.c_void_p, c.c_char_p, c.c_int64, c.c_int64,
                                           c.c_void_p, c.c_void_p, c.c_char_p, _TAPFN, c.c_void_p,
                                           c.c_char_p, c.c_int]
            lib.rx_exec_wait.restype = c.c_int
            lib.rx_exec_wait.argtypes = [c.c_void_p, c.c_int64, c.POINTER(c.c_int64), c.POINTER(c.c_int64),
                                         c.POINTER(c.c_int64), c.c_char_p, c.c_int]
            lib.rx_exec_stats.argtypes = [c.c_void_p, c.POINTER(c.c_int64)]
            lib.rx_cache_put.argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.c_char_p, c.c_char_p]
            for f in ("rx_cache_get", "rx_cache_pop"):
                getattr(lib, f).argtypes = [c.c_void_p, c.c_char_p, c.c_int32, c.c_char_p]
                getattr(lib, f).restype = c.c_int
            lib.rx_cache_list.argtypes = [c.c_void_p, c.c_char_p, c.POINTER(c.c_int32), c.c_int]
            lib.rx_cache_list.restype = c.c_int
            lib.rx_cache_unpersist.argtypes = [c.c_void_p, c.c_char_p, c.c_void_p]
            lib.rx_cache_unpersist.restype = c.c_int
            lib.rx_cache_rdds.argtypes = [c.c_void_p, c.c_char_p, c.c_int]
            lib.rx_cache_rdds.restype = c.c_int
            lib.rx_csv_infer.argtypes = [c.c_char_p, c.c_int64, c.c_char, c.c_void_p]
            lib.rx_csv_infer.restype = c.c_int
            _lib_handle = lib
    return _lib_handle


def enabled() -> bool:
    from raydp_amd.utils.config import get as conf_get
    return bool(conf_get("spark.ray.mi355x.native_executor"))


def read_csv_infer(data: bytes, sep: str = ",") -> Optional[pa.Table]:
    """The table pyarrow's CSV reader with type inference (header row, null token "") returns
    for ``data``, read natively in one pass (``csrc/exec/csv_infer.cc``), or None when the
    bytes hold anything that reader does not decide exactly -- then read them with pyarrow."""
    if len(sep) != 1 or not data:
        return None
    stream = ctypes.create_string_buffer(64)            # struct ArrowArrayStream
    rc = _lib().rx_csv_infer(data, len(data), sep.encode(), ctypes.addressof(stream))
    if rc != 1:
        return None
    return pa.RecordBatchReader._import_from_c(ctypes.addressof(stream)).read_all()


# ------------------------------------------------------------------------------------------
# stage lowering
# ------------------------------------------------------------------------------------------
_TYPE_NAMES = {"bool", "int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64", "float",
               "double", "string", "large_string", "binary", "large_binary", "date32[day]", "timestamp[s]",
               "timestamp[ms]", "timestamp[us]", "timestamp[ns]", "null"}


def _tname(t: pa.DataType) -> Optional[str]:
    s = str(t)
    return s if s in _TYPE_NAMES else None


class _Spec:
    """Little-endian writer of the stage layout parsed by ``csrc/exec/executor.cc``."""

    def __init__(self):
        self.parts: List[bytes] = []

    def u8(self, v):
        self.parts.append(struct.pack("<B", v))

    def u32(self, v):
        self.parts.append(struct.pack("<I", v))

    def i32(self, v):
        self.parts.append(struct.pack("<i", v))

    def s(self, v: str):
        b = v.encode()
        self.u32(len(b))
        self.parts.append(b)

    def arr(self, a, dtype):
        import numpy as np
        a = np.ascontiguousarray(np.asarray(a, dtype=dtype).reshape(-1))
        self.u32(a.size)
        self.parts.append(a.tobytes())

    def bytes(self) -> bytes:
        return b"".join(self.parts)


class Lowered:
    """A stage the native task loop can run: its C++ stage handle, the VM programs (for the UDF
    bridge) and how to produce a partition's source."""

    _ids = itertools.count(1)

    def __init__(self, top, base, progs, csv):
        self.top, self.base, self.progs, self.csv = top, base, progs, csv
        self.segs_ref = None
        self.key = next(Lowered._ids)
        self.handle = None
        self._owner = None     # _StageHandle: the C++ stage, shared by lowerings of one chain

    def _source_key(self):
        """What of the source the C++ stage spec encodes (not the file or partition: those
        come with each task)."""
        src = self.csv
        if src is None:
            return None
        return (bool(src.header), src.sep, src.null_value or "",
                tuple((f.name, str(f.type)) for f in src.schema()))

    def adopt(self, owner: "_StageHandle", segs) -> None:
        self._owner, self.handle, self.segs_ref = owner, owner.h, segs

    def build(self, segs) -> bool:
        import numpy as np
        w = _Spec()
        w.u32(0x31535852)
        if self.csv is not None:
            src = self.csv
            w.u8(1 if src.header else 0)
            sep = src.sep.encode() if isinstance(src.sep, str) else bytes([src.sep])
            if len(sep) != 1:
                return False
            w.u8(sep[0])
            w.s(src.null_value if src.null_value else "")
            fields = list(src.schema())
            names = [_tname(f.type) for f in fields]
            if any(n is None for n in names):
                self.csv = None
                return self.build(segs)
            w.u32(len(fields))
            for f, n in zip(fields, names):
                w.s(f.name)
                w.s(n)
        else:
            w.u8(0)
            w.u8(ord(","))
            w.s("")
            w.u32(0)
        w.u32(len(self.progs))
        for p in self.progs:
            w.arr(p.code, np.int32)
            w.arr(p.fconst, np.float64)
            w.arr(p.iconst, np.int64)
            w.arr(p.live, np.int32)
            w.i32(int(p.nslots))
            w.u32(len(p.inputs))
            for key in p.inputs:
                if key[0] == "col":
                    n = _tname(p.schema.field(key[1]).type)
                    if n is None:
                        return False
                    w.u8(0)
                    w.i32(int(key[1]))
                    w.s(n)
                elif key[0] == "ts":
                    w.u8(1)
                    w.i32(int(key[1]))
                    w.s("timestamp[s]")
                else:
                    return False        # host-evaluated expression input: Python path
            w.u32(len(p.out_ct))
            for ct, typ, slot in zip(p.out_ct, p.out_types, p.out_slots):
                n = _tname(typ)
                if n is None:
                    return False
                w.i32(int(ct))
                w.s(n)
                w.i32(int(slot))
            w.u8(1 if p.has_filter else 0)
            w.u8(1 if p.taps else 0)
            w.u32(len(p.columns))
            for name, ref in p.columns:
                w.s(name)
                w.u8(0 if ref[0] == "vm" else 1)
                w.i32(int(ref[1]))
        spec = w.bytes()
        lib = _lib()
        err = ctypes.create_string_buffer(_ERRLEN)
        h = lib.rx_stage_create(spec, len(spec), err, _ERRLEN)
        if not h:
            return False
        self.adopt(_StageHandle(h), segs)
        return True


class _StageHandle:
    """Owner of one C++ stage (``rx_stage_create``): destroyed when the last lowering that
    uses it and the stage cache have both let go of it."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        h, self.h = self.h, None
        if h and _lib_handle is not None:
            _lib_handle.rx_stage_destroy(h)


# (compiled chain, source spec) -> (segments, stage handle): each fit of the same pipeline
# builds a new plan tree over new data, but its chain compiles to the same cached segments
# (exprc.segments_for), so the executor reuses the C++ stage built for them instead of
# re-encoding and re-creating it on the critical path of every conversion stage.
_STAGES: "Dict[tuple, tuple]" = {}
_STAGES_MAX = 32


def lower(fn) -> Optional[Lowered]:
    """The native form of a stage function, or None (the stage runs on the Python path).
    Cached on the stage's top plan node; a recompiled chain (a UDF retired after a failed
    verification) is lowered again."""
    from raydp_amd.spark import exprc
    from raydp_amd.spark.plan import MapPlan, SourcePlan
    from raydp_amd.spark.sources import CsvSource
    top = getattr(fn, "__self__", None)
    if not isinstance(top, MapPlan) or getattr(top, "rel", None) is None or not exprc.enabled():
        return None
    if getattr(fn, "__func__", None) is not MapPlan.compute:
        return None
    nodes, base = exprc.chain_of(top)
    if not nodes:
        return None
    segs = exprc.segments_for(top, nodes, base)
    cached = top.__dict__.get("_native_lowered")
    if cached is not None and cached.segs_ref is segs:
        return cached
    if segs is None or any(s[0] != "vm" for s in segs):
        STATS["not_lowered"] += 1
        top.__dict__["_native_lowered"] = None
        return None
    csv = base.source if isinstance(base, SourcePlan) and isinstance(base.source, CsvSource) else None
    low = Lowered(top, base, [s[1] for s in segs], csv)
    try:
        skey = (id(segs), low._source_key())
    except Exception:  # noqa: BLE001 - a source whose schema cannot be read here: no reuse
        skey = None
    hit = _STAGES.get(skey) if skey is not None else None
    if hit is not None and hit[0] is segs:
        low.adopt(hit[1], segs)
        STATS["stage_reuse"] += 1
    else:
        if not low.build(segs):
            STATS["not_lowered"] += 1
            return None
        if skey is not None and low.csv is csv:     # (build drops an unencodable CSV source)
            if len(_STAGES) >= _STAGES_MAX:
                _STAGES.pop(next(iter(_STAGES)))
            _STAGES[skey] = (segs, low._owner)     # keeps segs alive: its id stays unique
    STATS["lowered_stages"] += 1
    top.__dict__["_native_lowered"] = low
    _REGISTRY[low.key] = low
    return low


# ------------------------------------------------------------------------------------------
# the UDF bridge (called from the C++ worker threads; ctypes takes the GIL)
# ------------------------------------------------------------------------------------------
# key -> Lowered, for the UDF bridge of a task in flight. Weak: a stage's Lowered lives as long
# as its plan (the executor keeps the last 16 stage functions), and a task's caller holds it
# until the task is waited for -- a strong registry kept every stage's plan tree and C++ stage
# handle for the executor's whole life.
_REGISTRY: "weakref.WeakValueDictionary[int, Lowered]" = weakref.WeakValueDictionary()


def _tap_impl(user, seg, m, vals, valids, nulls) -> int:
    try:
        from raydp_amd.spark import exprc
        low = _REGISTRY.get(int(user or 0))
        if low is None:
            return FALLBACK
        prog = low.progs[seg]
        nbits = (m + 7) // 8
        outs, out_bufs = [], []
        for j, ct in enumerate(prog.out_ct):
            size = nbits if ct == exprc.T_BOOL else m * exprc._ELEM[ct]
            vb = pa.foreign_buffer(vals[j], size)
            nj = int(nulls[j])
            mb = pa.foreign_buffer(valids[j], nbits) if nj else None
            out_bufs.append(vb)
            outs.append(pa.Array.from_buffers(prog.out_types[j], m, [mb, vb], null_count=nj))
        return prog.check_taps(outs, out_bufs, int(m))
    except Exception:  # noqa: BLE001 - any surprise: the Python path decides this partition
        return FALLBACK


_TAP = _TAPFN(_tap_impl)


# ------------------------------------------------------------------------------------------
# the per-process task loop + partition cache
# ------------------------------------------------------------------------------------------
def make_executor(threads: int):
    """The native task loop + cache, or -- when the library cannot be loaded on this host (no
    compiler, an Arrow C++ ABI that does not match the installed pyarrow) -- a Python cache
    with the same interface whose ``available`` is False (every stage takes the Python path)."""
    try:
        return NativeExecutor(threads)
    except Exception as e:  # noqa: BLE001
        import logging
        logging.getLogger(__name__).warning("native executor unavailable (%s); Python task path only", e)
        return PyCache()


class PyCache:
    """Pure-Python stand-in for the partition cache of :class:`NativeExecutor`."""
    available = False

    def __init__(self):
        self._lock = threading.Lock()
        self._c: Dict[Tuple[str, int], str] = {}

    def stats(self):
        return {"ok": 0, "fallback": 0, "error": 0, "rows": 0, "bytes": 0}

    def cache_put(self, rdd, i, oid):
        with self._lock:
            old = self._c.get((rdd, int(i)))
            self._c[(rdd, int(i))] = oid
        return old

    def cache_get(self, rdd, i):
        with self._lock:
            return self._c.get((rdd, int(i)))

    def cache_pop(self, rdd, i):
        with self._lock:
            return self._c.pop((rdd, int(i)), None)

    def cache_list(self, rdd):
        with self._lock:
            return sorted(i for (r, i) in self._c if r == rdd)

    def cache_unpersist(self, rdd, store):
        with self._lock:
            keys = [k for k in self._c if rdd is None or k[0] == rdd]
            oids = [self._c.pop(k) for k in keys]
        if store is not None:
            for o in oids:
                store.delete(o)
        return len(oids)

    def cached_rdds(self):
        with self._lock:
            return sorted({r for r, _ in self._c})

    def close(self):
        pass


class NativeExecutor:
    available = True

    def __init__(self, threads: int):
        self._lib = _lib()
        self._h = self._lib.rx_exec_create(max(1, int(threads)))

    # -- tasks ------------------------------------------------------------------------------
    def submit(self, low: Lowered, i: int, store, oid: str) -> Tuple[int, object]:
        """Queue partition ``i`` of ``low``; returns (task id, keep-alive) or (-1, error)."""
        from raydp_amd.spark.plan import _PartitionScope
        err = ctypes.create_string_buffer(_ERRLEN)
        src = low.csv
        keep = None
        if src is not None and i not in src._parsed:
            f, lo, hi = src.splits[i]
            tid = self._lib.rx_exec_submit(self._h, low.handle, f.encode(), lo, hi, None, store._h, oid.encode(),
                                           _TAP, low.key, err, _ERRLEN)
        else:
            with _PartitionScope(i):
                t = low.base.compute(i)
            reader = pa.RecordBatchReader.from_batches(t.schema, t.to_batches())
            stream = ctypes.create_string_buffer(64)         # struct ArrowArrayStream (5 pointers)
            reader._export_to_c(ctypes.addressof(stream))
            keep = (stream, reader)
            tid = self._lib.rx_exec_submit(self._h, low.handle, None, 0, 0, ctypes.addressof(stream), store._h,
                                           oid.encode(), _TAP, low.key, err, _ERRLEN)
        if tid < 0:
            return -1, err.value.decode(errors="replace")
        return tid, keep

    def wait(self, tid: int) -> Tuple[int, int, int, str]:
        """(status, rows, bytes, error) of a submitted task; the GIL is released while waiting.
        With tracing on, the task's run on its worker thread becomes a "task" span."""
        rows, nbytes = ctypes.c_int64(), ctypes.c_int64()
        times = (ctypes.c_int64 * 3)()
        err = ctypes.create_string_buffer(_ERRLEN)
        st = self._lib.rx_exec_wait(self._h, tid, ctypes.byref(rows), ctypes.byref(nbytes), times, err, _ERRLEN)
        from raydp_amd.utils import tracing
        if tracing.enabled() and times[1]:
            tracing.complete("task", times[0], cat="executor", t1_ns=times[1], tid=900000 + times[2],
                             native=True, status=st, rows=rows.value)
        return st, rows.value, nbytes.value, err.value.decode(errors="replace")

    def stats(self) -> Dict[str, int]:
        out = (ctypes.c_int64 * 5)()
        self._lib.rx_exec_stats(self._h, out)
        return dict(zip(("ok", "fallback", "error", "rows", "bytes"), list(out)))

    # -- partition cache ----------------------------------------------------------------------
    def cache_put(self, rdd: str, i: int, oid: str) -> Optional[str]:
        old = ctypes.create_string_buffer(33)
        self._lib.rx_cache_put(self._h, rdd.encode(), int(i), oid.encode(), old)
        return old.value.decode() or None

    def cache_get(self, rdd: str, i: int) -> Optional[str]:
        out = ctypes.create_string_buffer(33)
        return out.value.decode() if self._lib.rx_cache_get(self._h, rdd.encode(), int(i), out) else None

    def cache_pop(self, rdd: str, i: int) -> Optional[str]:
        out = ctypes.create_string_buffer(33)
        return out.value.decode() if self._lib.rx_cache_pop(self._h, rdd.encode(), int(i), out) else None

    def cache_list(self, rdd: str) -> List[int]:
        cap = 1024
        while True:
            buf = (ctypes.c_int32 * cap)()
            n = self._lib.rx_cache_list(self._h, rdd.encode(), buf, cap)
            if n <= cap:
                return list(buf[:n])
            cap = n

    def cache_unpersist(self, rdd: Optional[str], store) -> int:
        return self._lib.rx_cache_unpersist(self._h, None if rdd is None else rdd.encode(),
                                            None if store is None else store._h)

    def cached_rdds(self) -> List[str]:
        cap = 4096
        while True:
            buf = ctypes.create_string_buffer(cap)
            need = self._lib.rx_cache_rdds(self._h, buf, cap)
            if need <= cap:
                return [r for r in buf.value.decode().split("\n") if r]
            cap = need

    def close(self):
        h, self._h = self._h, None
        if h:
            self._lib.rx_exec_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
