"""GBDT gradient histograms (``csrc/hip/gbdt_hist.hip``).

``level_histogram`` builds the (node, feature, bin) -> (sum g, sum h) table of one tree level.
On a GPU it runs the gfx950 kernel (LDS-privatised fp64 atomics, one launch per level) and
raises if ``libhipkernels.so`` is missing; on the CPU it is the ``index_add_`` expression that
``torch_level_histogram`` also exposes as the numerics reference for tests.

Parity: the reference's histogram step lives inside xgboost-ray's ``hist`` tree method
(``python/raydp/xgboost/estimator.py:54-81``), not in RayDP's own code.
"""
import ctypes

import torch

from raydp_amd.ops import _hip

_bound = False


def _lib():
    global _bound
    L = _hip.lib()
    if not _bound:
        vp, i, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
        L.rx_gbdt_hist.argtypes = [vp, vp, vp, vp, vp, ll, i, i, i, vp]
        L.rx_gbdt_hist.restype = i
        L.rx_gbdt_hist_group.argtypes = [i, i]
        L.rx_gbdt_hist_group.restype = i
        d = ctypes.c_double
        L.rx_gbdt_split.argtypes = [vp, vp, vp, vp, vp, i, i, i, d, d, d, vp]
        L.rx_gbdt_split.restype = i
        L.rx_gbdt_partition.argtypes = [vp, vp, vp, vp, ll, i, vp]
        L.rx_gbdt_partition.restype = i
        _bound = True
    return L


def torch_level_histogram(bins: torch.Tensor, pos: torch.Tensor, g: torch.Tensor, h: torch.Tensor, K: int,
                          B: int) -> torch.Tensor:
    """Reference expression: ``bins`` [n, F] (row-major), ``pos`` [n] (-1 = inactive)."""
    n, F = bins.shape
    act = pos >= 0
    feat_off = (torch.arange(F, device=bins.device) * B)[None, :]
    idx = pos.clamp_min(0)[:, None] * (F * B) + feat_off + bins.long()
    gh = torch.stack([g, h], 1).double()
    hist = torch.zeros(K * F * B, 2, dtype=torch.float64, device=bins.device)
    hist.index_add_(0, idx[act].reshape(-1), gh[act].repeat_interleave(F, dim=0))
    return hist


def level_histogram(bins_t: torch.Tensor, pos: torch.Tensor, g: torch.Tensor, h: torch.Tensor, K: int,
                    B: int) -> torch.Tensor:
    """Histogram [K*F*B, 2] fp64 from column-major ``bins_t`` [F, n] int16 on a GPU."""
    F, n = bins_t.shape
    dev = bins_t.device
    if dev.type != "cuda":
        return torch_level_histogram(bins_t.t(), pos, g, h, K, B)
    if bins_t.dtype != torch.int16 or not bins_t.is_contiguous():
        raise ValueError("bins_t must be a contiguous int16 [F, n] tensor")
    L = _lib()
    if L.rx_gbdt_hist_group(int(K), int(B)) <= 0:
        raise ValueError(f"{B} bins per feature exceed the histogram kernel's LDS slice (max_bin too large)")
    pos = pos.to(torch.long).contiguous()
    g = g.to(torch.float32).contiguous()
    h = h.to(torch.float32).contiguous()
    if pos.shape[0] != n or g.shape[0] != n or h.shape[0] != n:
        raise ValueError("pos/g/h must have one entry per row of bins_t")
    for t in (pos, g, h):
        if t.device != dev:
            raise ValueError("all operands must live on the same GPU")
    hist = torch.zeros(K * F * B, 2, dtype=torch.float64, device=dev)
    _hip.check(L.rx_gbdt_hist(ctypes.c_void_p(bins_t.data_ptr()), ctypes.c_void_p(pos.data_ptr()),
                              ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(h.data_ptr()),
                              ctypes.c_void_p(hist.data_ptr()), n, F, int(B), int(K), _hip.stream_ptr(dev)),
               "rx_gbdt_hist")
    return hist


def split_candidates(hist: torch.Tensor, tot: torch.Tensor, ncuts: torch.Tensor, fmask, lam: float, alpha: float,
                     mcw: float) -> torch.Tensor:
    """Best threshold per (node, feature) for both default directions on a GPU.

    ``hist`` [K, F, B, 2] fp64, ``tot`` [K, 2] fp64 node totals, ``ncuts`` [F] int32 real cuts per
    feature, ``fmask`` [F] uint8 or None. Returns [K, F, 4] fp64: (gain, threshold) for
    default-left, then for default-right; gain -1 where no valid threshold exists.
    """
    K, F, B, two = hist.shape
    if two != 2 or hist.dtype != torch.float64 or hist.device.type != "cuda":
        raise ValueError("hist must be a [K, F, B, 2] fp64 GPU tensor")
    hist = hist.contiguous()
    tot = tot.to(torch.float64).contiguous()
    ncuts = ncuts.to(device=hist.device, dtype=torch.int32).contiguous()
    if tot.shape != (K, 2) or ncuts.shape != (F,) or (fmask is not None and fmask.shape != (F,)):
        raise ValueError("tot/ncuts/fmask shapes do not match hist")
    out = torch.empty((K, F, 4), dtype=torch.float64, device=hist.device)
    _hip.check(_lib().rx_gbdt_split(ctypes.c_void_p(hist.data_ptr()), ctypes.c_void_p(tot.data_ptr()),
                                    ctypes.c_void_p(ncuts.data_ptr()),
                                    ctypes.c_void_p(fmask.data_ptr()) if fmask is not None else None,
                                    ctypes.c_void_p(out.data_ptr()), K, F, B, float(lam), float(alpha), float(mcw),
                                    _hip.stream_ptr(hist.device)), "rx_gbdt_split")
    return out


def partition_rows_(bins_t: torch.Tensor, table: torch.Tensor, pos: torch.Tensor, leaf: torch.Tensor) -> None:
    """Move active rows one level down, in place, on a GPU.

    ``table`` [K, 5] int64 rows ``(remap, feature, split_bin, default_left, node_id)``: rows of a
    node with ``remap < 0`` get ``leaf = node_id`` and ``pos = -1``; others go to child
    ``remap + (not left)`` where left = ``default_left`` for bin 0 (missing), else
    ``bin <= split_bin``.
    """
    F, n = bins_t.shape
    if table.dtype != torch.long or table.dim() != 2 or table.shape[1] != 5:
        raise ValueError("table must be [K, 5] int64")
    if pos.dtype != torch.long or leaf.dtype != torch.long or pos.shape != (n,) or leaf.shape != (n,):
        raise ValueError("pos/leaf must be int64 [n]")
    if not (pos.is_contiguous() and leaf.is_contiguous() and bins_t.is_contiguous()):
        raise ValueError("operands must be contiguous")
    if table.shape[0] and int(table[:, 1].max()) >= F:
        raise ValueError("split feature out of range")
    table = table.to(bins_t.device).contiguous()
    _hip.check(_lib().rx_gbdt_partition(ctypes.c_void_p(bins_t.data_ptr()), ctypes.c_void_p(table.data_ptr()),
                                        ctypes.c_void_p(pos.data_ptr()), ctypes.c_void_p(leaf.data_ptr()), n,
                                        int(table.shape[0]), _hip.stream_ptr(bins_t.device)), "rx_gbdt_partition")
