"""ctypes binding of ``csrc/exec/exec_kernels.cc`` (shuffle row hashing).

The native library is built in-tree by ``__graft_entry__.build()`` / ``python -m
raydp_amd.native.build``. Hashing must agree across every process of a job, so there is one
implementation; if the library is missing it is compiled on first use.
"""
import ctypes

import numpy as np
import pyarrow as pa

from raydp_amd.native import loader

_u64p = ctypes.POINTER(ctypes.c_uint64)


def _lib():
    lib = loader.load("exec_kernels")
    if not getattr(lib, "_rx_typed", False):
        lib.rx_hash_fixed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int]
        lib.rx_hash_binary.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
        lib.rx_partition_order.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_void_p, ctypes.c_void_p]
        lib._rx_typed = True
    return lib


def _addr(buf):
    return None if buf is None else buf.address


def hash_combine(seed: np.ndarray, column) -> np.ndarray:
    """Fold one column into the per-row 64-bit hash ``seed`` (returns a new array)."""
    lib = _lib()
    out = np.array(seed, dtype=np.uint64, copy=True)
    chunks = column.chunks if isinstance(column, pa.ChunkedArray) else [column]
    pos = 0
    for arr in chunks:
        n = len(arr)
        if n == 0:
            continue
        t = arr.type
        if pa.types.is_dictionary(t):
            arr = arr.cast(t.value_type)
            t = arr.type
        if pa.types.is_timestamp(t) or pa.types.is_date(t) or pa.types.is_time(t) \
                or pa.types.is_duration(t):
            arr = arr.cast(pa.int64() if t.bit_width == 64 else pa.int32())
            t = arr.type
        if pa.types.is_boolean(t):
            arr = arr.cast(pa.int8())
            t = arr.type
        if pa.types.is_large_string(t) or pa.types.is_large_binary(t):
            arr = arr.cast(pa.string())
            t = arr.type
        bufs = arr.buffers()
        dst = out[pos:pos + n]
        if pa.types.is_string(t) or pa.types.is_binary(t):
            lib.rx_hash_binary(dst.ctypes.data, _addr(bufs[1]), _addr(bufs[2]), _addr(bufs[0]),
                               arr.offset, n)
        elif pa.types.is_integer(t) or pa.types.is_floating(t):
            lib.rx_hash_fixed(dst.ctypes.data, _addr(bufs[1]), _addr(bufs[0]), arr.offset, n,
                              t.bit_width // 8, int(pa.types.is_floating(t)))
        else:
            # nested / exotic types: hash their string rendering
            s = pa.array([None if v is None else repr(v) for v in arr.to_pylist()], pa.string())
            b = s.buffers()
            lib.rx_hash_binary(dst.ctypes.data, _addr(b[1]), _addr(b[2]), _addr(b[0]), s.offset, n)
        pos += n
    return out


def partition_order(part: np.ndarray, nparts: int):
    """Stable grouping of row indices by partition id → (order, counts)."""
    lib = _lib()
    part = np.ascontiguousarray(part, dtype=np.int64)
    counts = np.zeros(nparts, dtype=np.int64)
    order = np.empty(len(part), dtype=np.int64)
    lib.rx_partition_order(part.ctypes.data, len(part), nparts, counts.ctypes.data,
                           order.ctypes.data)
    return order, counts
