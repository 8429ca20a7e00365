"""Arrow blocks → device-resident training tensors (one DMA + HIP decode).

Host side: the raw Arrow buffers (values + validity, sliced to the array's window) of every
requested column of every block are packed into ONE pinned staging buffer; one
``non_blocking`` H2D copy moves it to HBM; ``rx_arrow_ingest`` (``csrc/hip/arrow_ingest.hip``)
then casts/null-fills/transposes into the row-major matrix the trainer consumes. On a CPU
device the same contract is implemented with numpy (tests, Gloo workers).
"""
import ctypes
from typing import List, Optional, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import torch

_TYPE_CODES = {
    pa.float64(): 0, pa.float32(): 1, pa.int64(): 2, pa.int32(): 3, pa.int16(): 4, pa.int8(): 5,
    pa.uint8(): 6, pa.bool_(): 7, pa.uint16(): 8, pa.uint32(): 9,
}


def _ru(x, m):
    return (x + m - 1) // m * m


def _prep_array(a) -> pa.Array:
    if isinstance(a, pa.ChunkedArray):
        a = a.combine_chunks() if a.num_chunks != 1 else a.chunk(0)
    t = a.type
    if pa.types.is_dictionary(t):
        a = a.cast(t.value_type)
        t = a.type
    if t not in _TYPE_CODES:
        if pa.types.is_timestamp(t) or pa.types.is_date(t):
            a = a.cast(pa.int64())
        elif pa.types.is_float16(t) or pa.types.is_uint64(t) or pa.types.is_decimal(t) \
                or pa.types.is_string(t):
            a = pc.cast(a, pa.float64(), safe=False)
        else:
            raise TypeError(f"column type {t} cannot be ingested as a tensor")
    return a


def _column_pieces(a: pa.Array):
    """(type_code, values_bytes, values_bit_offset_or_elem_offset, validity_bytes, vbit_off)."""
    code = _TYPE_CODES[a.type]
    bufs = a.buffers()
    n, off = len(a), a.offset
    if code == 7:  # bit-packed booleans
        vb = bufs[1]
        lo, hi = off // 8, (off + n + 7) // 8
        values, voff = memoryview(vb)[lo:hi], off % 8
    else:
        w = a.type.bit_width // 8
        values, voff = memoryview(bufs[1])[off * w:(off + n) * w], 0
    valid, boff = None, 0
    if a.null_count and bufs[0] is not None:
        lo, hi = off // 8, (off + n + 7) // 8
        valid, boff = memoryview(bufs[0])[lo:hi], off % 8
    return code, values, voff, valid, boff


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
    return torch.from_numpy(out).to(dtype)


def ingest_columns(tables: Sequence[pa.Table], cols: List[str], device, out_bf16: bool,
                   stride: Optional[int] = None, fill: float = 0.0) -> torch.Tensor:
    """Build a row-major ``[N, stride]`` (bf16 or f32) device matrix from ``cols``."""
    device = torch.device(device)
    stride = stride or len(cols)
    n = int(sum(t.num_rows for t in tables))
    dtype = torch.bfloat16 if out_bf16 else torch.float32
    if device.type != "cuda":
        return _numpy_matrix(tables, cols, dtype, fill, stride).to(device)
    from raydp_amd.ops import _hip
    lib = _hip.lib()
    out = torch.empty((max(n, 1), stride), dtype=dtype, device=device)
    if n == 0:
        return out[:0]
    if len(cols) > _hip.MAXCOLS:
        raise ValueError(f"at most {_hip.MAXCOLS} columns per ingest call")
    # ---- pack all buffers into one pinned staging area ----
    plan, total = [], 0
    for t in tables:
        items = []
        for c in cols:
            code, values, voff, valid, boff = _column_pieces(_prep_array(t.column(c)))
            vpos = total
            total = _ru(total + len(values), 64)
            bpos = None
            if valid is not None:
                bpos = total
                total = _ru(total + len(valid), 64)
            items.append((code, values, voff, vpos, valid, boff, bpos))
        plan.append((t.num_rows, items))
    staging = torch.empty(max(total, 64), dtype=torch.uint8, pin_memory=True)
    host = staging.numpy()
    for _, items in plan:
        for code, values, voff, vpos, valid, boff, bpos in items:
            host[vpos:vpos + len(values)] = np.frombuffer(values, dtype=np.uint8)
            if valid is not None:
                host[bpos:bpos + len(valid)] = np.frombuffer(valid, dtype=np.uint8)
    dev = staging.to(device, non_blocking=True)
    base = dev.data_ptr()
    stream = _hip.stream_ptr(device)
    row0 = 0
    for nrows, items in plan:
        args = _hip.IngestArgs()
        args.ncols, args.out_stride, args.out_bf16 = len(cols), stride, int(out_bf16)
        args.nrows, args.out_row0 = nrows, row0
        for j, (code, values, voff, vpos, valid, boff, bpos) in enumerate(items):
            col = args.col[j]
            col.type = code
            col.values = base + vpos
            col.fill = fill
            if code == 7:
                col.offset = voff
                if valid is not None and boff != voff:
                    raise ValueError("misaligned boolean validity")
            else:
                col.offset = 0
            if valid is not None:
                col.valid = base + bpos
                if code != 7 and boff != 0:
                    # the kernel indexes validity with the value offset; realign on the host
                    bits = np.unpackbits(np.frombuffer(valid, np.uint8), bitorder="little")[boff:boff + nrows]
                    packed = np.packbits(bits, bitorder="little")
                    tmp = torch.from_numpy(packed.copy()).to(device)
                    col.valid = tmp.data_ptr()
                    items[j] = items[j] + (tmp,)  # keep alive
            else:
                col.valid = None
        _hip.check(lib.rx_arrow_ingest(ctypes.byref(args), ctypes.c_void_p(out.data_ptr()), stream),
                   "rx_arrow_ingest")
        row0 += nrows
    # keep the staging buffers alive until the copies/kernels consumed them
    torch.cuda.current_stream(device).synchronize()
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
