"""Arrow blocks in the object store -> device-resident training tensors.

GPU path (``csrc/hip/arrow_ingest.hip``, ``rx_ingest_dma``):

* the host never copies column bytes. For every block it computes which byte ranges of the
  block's buffers the requested columns need (values + validity, sliced to the array window)
  and hands the list to native code: ranges that are dense in the Arrow IPC body are merged
  into one DMA per block, sparse ones go buffer by buffer;
* ranges inside a store arena are pinned with ``hipHostRegister`` in 2 MiB chunks, lazily, once
  per process (``rx_pin_range``), so the copies are true DMAs out of the shared mapping;
* ``hipMemcpyAsync`` runs on a dedicated copy stream into a ring of device staging memory;
  each chunk's decode kernel waits on an event on the compute stream, so chunk k+1's DMA
  overlaps chunk k's decode (column decode, validity -> fill value, dtype cast, transpose to the
  row-major [N, stride] matrix the trainers read, 16-B loads and stores).

Counters (``ingest_stats()``): ``host_copy_bytes`` (bytes the host itself copied or converted:
casts of dictionary / timestamp / string columns, the CPU path), ``dma_pinned_bytes``,
``dma_pageable_bytes`` (sources outside any pinned arena: HIP stages those itself), ``dma_copies``,
``chunks``, plus the native pinning counters.

Reference hot site: ``python/raydp/torch/estimator.py:226-241`` (Ray Data ``to_torch`` per
batch on the CPU).
"""
import ctypes
import threading
from typing import Dict, List, Optional, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

_TYPE_CODES = {
    pa.float64(): 0, pa.float32(): 1, pa.int64(): 2, pa.int32(): 3, pa.int16(): 4, pa.int8(): 5,
    pa.uint8(): 6, pa.bool_(): 7, pa.uint16(): 8, pa.uint32(): 9,
}

_STAT_KEYS = ("host_copy_bytes", "dma_pinned_bytes", "dma_pageable_bytes", "dma_copies", "chunks")
_stats: Dict[str, int] = {k: 0 for k in _STAT_KEYS}
_lock = threading.Lock()
_copy_streams: Dict[int, "torch.cuda.Stream"] = {}
_inflight: List[tuple] = []   # (event, keep-alive refs) until the DMA + decode have completed

# staging ring: at most this many bytes of device memory per call; a chunk uses at most half
STAGE_BYTES = 256 << 20
PIN_CHUNK = 2 << 20
_REGION_ALIGN = 256


def _ru(x, m):
    return (x + m - 1) // m * m


def ingest_stats() -> Dict[str, int]:
    out = dict(_stats)
    from raydp_amd.ops import _hip
    if _hip._lib is not None:
        buf = (ctypes.c_longlong * 2)()
        _hip._lib.rx_pin_stats(buf)
        out["pin_calls"], out["pinned_arena_bytes"] = int(buf[0]), int(buf[1])
    return out


def reset_ingest_stats():
    for k in _STAT_KEYS:
        _stats[k] = 0


def _prep_array(a) -> pa.Array:
    if isinstance(a, pa.ChunkedArray):
        if a.num_chunks != 1:
            _stats["host_copy_bytes"] += a.nbytes
            a = a.combine_chunks()
        else:
            a = a.chunk(0)
    t = a.type
    if pa.types.is_dictionary(t):
        a = a.cast(t.value_type)
        _stats["host_copy_bytes"] += a.nbytes
        t = a.type
    if t not in _TYPE_CODES:
        if pa.types.is_timestamp(t) or pa.types.is_date(t) or pa.types.is_time(t) or pa.types.is_duration(t):
            a = a.view(pa.int64()) if t.bit_width == 64 else a.cast(pa.int64())
            if t.bit_width != 64:
                _stats["host_copy_bytes"] += a.nbytes
        elif pa.types.is_float16(t) or pa.types.is_uint64(t) or pa.types.is_decimal(t) \
                or pa.types.is_string(t) or pa.types.is_large_string(t):
            a = pc.cast(a, pa.float64(), safe=False)
            _stats["host_copy_bytes"] += a.nbytes
        else:
            raise TypeError(f"column type {t} cannot be ingested as a tensor")
    return a


class _Buf:
    """One host byte range a column needs: (address, length)."""
    __slots__ = ("addr", "n")

    def __init__(self, addr, n):
        self.addr, self.n = addr, n


def _column_bufs(a: pa.Array):
    """(type_code, values _Buf, bit offset of row 0, validity _Buf or None)."""
    code = _TYPE_CODES[a.type]
    bufs = a.buffers()
    n, off = len(a), a.offset
    vb = bufs[1]
    if code == 7:  # bit-packed booleans
        lo, hi = off // 8, (off + n + 7) // 8
        values, vbit = _Buf(vb.address + lo, hi - lo), off % 8
    else:
        w = a.type.bit_width // 8
        values, vbit = _Buf(vb.address + off * w, n * w), off % 8
    valid = None
    if a.null_count and bufs[0] is not None:
        lo, hi = off // 8, (off + n + 7) // 8
        valid = _Buf(bufs[0].address + lo, hi - lo)
    return code, values, vbit, valid


def _aligned(a: pa.Array) -> pa.Array:
    """The kernel splits values into 16-B vectors by element: a values buffer that is not
    aligned to its element size (never the case for Arrow IPC or pyarrow-built arrays) is
    re-materialised on the host."""
    if a.type != pa.bool_() and len(a):
        w = a.type.bit_width // 8
        if (a.buffers()[1].address + a.offset * w) % w:
            _stats["host_copy_bytes"] += a.nbytes
            return pa.concat_arrays([a.slice(0, len(a))]).take(pa.array(np.arange(len(a))))
    return a


def _numpy_matrix(tables, cols, dtype, fill=0.0, stride=None):
    n = sum(t.num_rows for t in tables)
    stride = stride or len(cols)
    out = np.zeros((n, stride), dtype=np.float32)
    r = 0
    for t in tables:
        for j, c in enumerate(cols):
            a = _prep_array(t.column(c))
            v = a.to_numpy(zero_copy_only=False).astype(np.float32, copy=False)
            if a.null_count:
                v = np.where(pc.is_valid(a).to_numpy(zero_copy_only=False), v, fill)
            out[r:r + t.num_rows, j] = v
        r += t.num_rows
    _stats["host_copy_bytes"] += int(out.nbytes)
    return torch.from_numpy(out).to(dtype)


def _numpy_int_matrix(tables, cols, fill, stride):
    n = sum(t.num_rows for t in tables)
    out = np.zeros((n, stride), dtype=np.int64)
    r = 0
    for t in tables:
        for j, c in enumerate(cols):
            a = _prep_array(t.column(c))
            v = a.fill_null(fill) if a.null_count else a
            out[r:r + t.num_rows, j] = v.to_numpy(zero_copy_only=False).astype(np.int64)
        r += t.num_rows
    _stats["host_copy_bytes"] += int(out.nbytes)
    return torch.from_numpy(out)


def _copy_stream(device) -> "torch.cuda.Stream":
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _copy_streams.get(idx)
    if s is None:
        s = torch.cuda.Stream(device=torch.device("cuda", idx))
        _copy_streams[idx] = s
    return s


def _regions(bufs: List[_Buf]):
    """Merge the byte ranges of one chunk into DMA regions: one span when the used bytes fill
    at least half of it (columns adjacent in the IPC body), else per range, merging ranges less
    than 4 KiB apart. Returns [(host_start16, nbytes, staging_off)] and a map addr -> staging off."""
    live = sorted({(b.addr, b.n) for b in bufs if b.n > 0})
    if not live:
        return [], {}, 0
    used = sum(n for _, n in live)
    lo = live[0][0] & ~15
    hi = max(a + n for a, n in live)
    if hi - lo <= 2 * used + (64 << 10):
        groups = [(lo, hi)]
    else:
        groups = []
        for a, n in live:
            s, e = a & ~15, a + n
            if groups and s - groups[-1][1] < 4096:
                groups[-1] = (groups[-1][0], max(groups[-1][1], e))
            else:
                groups.append((s, e))
    regions, off = [], 0
    for s, e in groups:
        regions.append((s, e - s, off))
        off = _ru(off + (e - s) + 16, _REGION_ALIGN)   # +16: a vector load may read past the end
    def where(addr):
        for s, n, o in regions:
            if s <= addr < s + max(n, 1) or (n == 0 and addr == s):
                return o + (addr - s)
        raise AssertionError("buffer outside every region")
    return regions, where, off


def _pin(regions) -> None:
    from raydp_amd.ops import _hip
    from raydp_amd.runtime.store import arena_of
    lib = _hip.lib()
    u64 = ctypes.c_uint64
    for s, n, _ in regions:
        ar = arena_of(s, max(n, 1))
        if ar is None:
            continue
        rc = lib.rx_pin_range(u64(ar[0]), u64(ar[1]), u64(s), u64(n), u64(PIN_CHUNK))
        if rc != 0:
            raise RuntimeError(f"hipHostRegister of the object-store arena failed (HIP error {rc})")


def _reap_inflight():
    while _inflight and _inflight[0][0].query():
        _inflight.pop(0)


def ingest_columns(tables: Sequence[pa.Table], cols: List[str], device, out_bf16: bool,
                   stride: Optional[int] = None, fill: float = 0.0,
                   stage_bytes: Optional[int] = None, out_i64: bool = False) -> torch.Tensor:
    """Build a row-major ``[N, stride]`` device matrix from ``cols``: bf16 (``out_bf16``), exact
    int64 (``out_i64``: category ids) or f32. Returns without a host synchronisation: the matrix
    is ready in stream order on the current stream."""
    device = torch.device(device)
    stride = stride or len(cols)
    n = int(sum(t.num_rows for t in tables))
    dtype = torch.int64 if out_i64 else (torch.bfloat16 if out_bf16 else torch.float32)
    if device.type != "cuda":
        if out_i64:
            return _numpy_int_matrix(tables, cols, int(fill), stride).to(device)
        return _numpy_matrix(tables, cols, dtype, fill, stride).to(device)
    from raydp_amd.ops import _hip
    lib = _hip.lib()
    if len(cols) > _hip.MAXCOLS:
        raise ValueError(f"at most {_hip.MAXCOLS} columns per ingest call")
    if len(cols) > stride:
        raise ValueError("stride must be at least the number of columns")
    out = torch.empty((max(n, 1), stride), dtype=dtype, device=device)
    if n == 0:
        return out[:0]
    if len(cols) == 0:
        return out[:n].zero_()
    cap = int(stage_bytes or STAGE_BYTES)
    max_chunk = cap // 2
    keep = []
    chunk_l, region_l, col_l = [], [], []
    row0 = 0
    total_stage = 0
    with _lock:
        _reap_inflight()
        for t in tables:
            nrows = t.num_rows
            if nrows == 0:
                continue
            arrays = [_aligned(_prep_array(t.column(c))) for c in cols]
            keep.append(arrays)
            # pin the block's whole used span with one registration (copies never straddle two)
            spans = [b for _, v, _, vd in (_column_bufs(a) for a in arrays) for b in (v, vd)
                     if b is not None and b.n > 0]
            if spans:
                lo = min(b.addr for b in spans) & ~15
                _pin([(lo, max(b.addr + b.n for b in spans) - lo, 0)])
            per_row = sum(max(1, a.type.bit_width) for a in arrays) / 8.0 + len(cols) / 8.0
            step = max(1, min(nrows, int(max_chunk / (per_row * 1.25)) - 64))
            for r in range(0, nrows, step):
                k = min(step, nrows - r)
                part = [a.slice(r, k) for a in arrays] if (r or k != nrows) else arrays
                pieces = [_column_bufs(a) for a in part]
                bufs = []
                for code, vals, vbit, valid in pieces:
                    bufs.append(vals)
                    if valid is not None:
                        bufs.append(valid)
                regions, where, nbytes = _regions(bufs)
                if nbytes > cap:
                    raise ValueError("ingest chunk larger than the staging ring")
                _pin(regions)
                chunk_l.append((k, row0 + r, nbytes, len(region_l), len(regions), len(col_l)))
                region_l.extend(regions)
                for code, vals, vbit, valid in pieces:
                    col_l.append((code, valid is not None, where(vals.addr),
                                  where(valid.addr) if valid is not None else 0, vbit, float(fill)))
                total_stage = max(total_stage, nbytes)
            row0 += nrows
        chunks = (_hip.DmaChunk * len(chunk_l))()
        for i, (k, r0, nb, fr, nr, fc) in enumerate(chunk_l):
            c = chunks[i]
            c.nrows, c.out_row0, c.bytes, c.first_region, c.nregions, c.first_col = k, r0, nb, fr, nr, fc
        regs = (_hip.DmaRegion * max(1, len(region_l)))()
        for i, (s, nb, off) in enumerate(region_l):
            regs[i].host, regs[i].bytes, regs[i].off = s, nb, off
        dcols = (_hip.DmaCol * len(col_l))()
        for i, (code, hv, vo, vo2, vbit, fl) in enumerate(col_l):
            d = dcols[i]
            d.type, d.has_valid, d.vals_off, d.valid_off, d.vbit, d.fill = code, int(hv), vo, vo2, vbit, fl
        ring = min(cap, _ru(sum(c[2] for c in chunk_l), _REGION_ALIGN))
        ring = max(ring, total_stage, _REGION_ALIGN)
        stage = torch.empty(ring, dtype=torch.uint8, device=device)
        cs = _copy_stream(device)
        compute = torch.cuda.current_stream(device)
        st = (ctypes.c_longlong * 4)()
        rc = lib.rx_ingest_dma(chunks, len(chunk_l), regs, dcols, len(cols), stride, 2 if out_i64 else int(out_bf16),
                               ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stage.data_ptr()), ring,
                               ctypes.c_void_p(compute.cuda_stream), ctypes.c_void_p(cs.cuda_stream), st)
        _hip.check(rc, "rx_ingest_dma")
        stage.record_stream(cs)
        for key, v in zip(("dma_pinned_bytes", "dma_pageable_bytes", "dma_copies", "chunks"), st):
            _stats[key] += int(v)
        ev = torch.cuda.Event()
        ev.record(compute)
        _inflight.append((ev, keep))
    return out[:n]


def random_permutation(n: int, seed: int, device) -> torch.Tensor:
    """int32 permutation of [0, n) drawn on the device (``rx_feistel_perm``: keyed Feistel
    bijection + cycle walking; one launch, no sort). CPU devices use numpy."""
    device = torch.device(device)
    if device.type != "cuda":
        rng = np.random.default_rng(seed & 0xFFFFFFFFFFFFFFFF)
        return torch.from_numpy(rng.permutation(n).astype(np.int32))
    from raydp_amd.ops import _hip
    out = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    _hip.check(_hip.lib().rx_feistel_perm(ctypes.c_void_p(out.data_ptr()), n,
                                          ctypes.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                                          _hip.stream_ptr(device)), "rx_feistel_perm")
    return out[:n]


def ingest_tables(tables, feature_columns, label_column, feature_dtype, label_dtype, device,
                  feat_stride: Optional[int] = None, feat_bf16: bool = False):
    feats = ingest_columns(tables, list(feature_columns), device, feat_bf16, feat_stride)
    labels = None
    if label_column is not None:
        labels = ingest_columns(tables, [label_column], device, False)
        if label_dtype is not None and label_dtype != torch.float32:
            labels = labels.to(label_dtype)
    if not feat_bf16 and feature_dtype is not None and feature_dtype != feats.dtype:
        feats = feats.to(feature_dtype)
    return feats, labels
