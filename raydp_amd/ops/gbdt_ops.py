"""GBDT gradient histograms (``csrc/hip/gbdt_hist.hip``).

``level_histogram`` builds the (node, feature, bin) -> (sum g, sum h) table of one tree level
from fixed-point gradients (``quantise``: int32 per row, power-of-two scale per tree) into
int64 sums, so the table is exact and independent of accumulation order. On a GPU it runs the
gfx950 kernel (LDS-privatised 64-bit integer atomics, one launch per level; global atomics when
one node's bins do not fit in LDS) and raises if ``libhipkernels.so`` is missing; on the CPU it
is the ``index_add_`` expression that ``torch_level_histogram`` also exposes as the reference
for tests. Both produce the same integers bit for bit.

Parity: the reference's histogram step lives inside xgboost-ray's ``hist`` tree method
(``python/raydp/xgboost/estimator.py:54-81``), not in RayDP's own code.
"""
import ctypes
import math

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
        L.rx_gbdt_split.argtypes = [vp, vp, vp, vp, vp, i, i, i, d, d, d, d, d, vp]
        L.rx_gbdt_split.restype = i
        L.rx_gbdt_partition.argtypes = [vp, vp, vp, vp, ll, i, vp]
        L.rx_gbdt_partition.restype = i
        _bound = True
    return L


QBITS = 30   # |quantised g| <= 2**QBITS, so int64 sums hold 2**33 rows


def quant_scale(max_abs: float) -> float:
    """Power-of-two scale mapping values of magnitude <= ``max_abs`` into [-2**QBITS, 2**QBITS].
    A power of two keeps ``x * scale`` exact (no rounding before the final round-to-integer) and
    ``q / scale`` exact, on every device."""
    if not (max_abs > 0.0) or max_abs != max_abs or max_abs == float("inf"):
        return 1.0
    _, e = math.frexp(max_abs)          # max_abs < 2**e
    return math.ldexp(1.0, QBITS - e)


def quantise(x: torch.Tensor, scale: float) -> torch.Tensor:
    """round-half-even(x * scale) as int32 (identical on CPU and GPU: the product is exact)."""
    return torch.round(x.double() * scale).to(torch.int32)


def torch_level_histogram(bins: torch.Tensor, pos: torch.Tensor, gq: torch.Tensor, hq: torch.Tensor, K: int,
                          B: int) -> torch.Tensor:
    """Reference expression: ``bins`` [n, F] (row-major), ``pos`` [n] (-1 = inactive), fixed-point
    ``gq``/``hq`` [n] int32; returns [K*F*B, 2] int64 sums."""
    n, F = bins.shape
    act = pos >= 0
    feat_off = (torch.arange(F, device=bins.device) * B)[None, :]
    idx = pos.clamp_min(0)[:, None] * (F * B) + feat_off + bins.long()
    gh = torch.stack([gq, hq], 1).long()
    hist = torch.zeros(K * F * B, 2, dtype=torch.int64, device=bins.device)
    hist.index_add_(0, idx[act].reshape(-1), gh[act].repeat_interleave(F, dim=0))
    return hist


def level_histogram(bins_t: torch.Tensor, pos: torch.Tensor, gq: torch.Tensor, hq: torch.Tensor, K: int,
                    B: int) -> torch.Tensor:
    """Histogram [K*F*B, 2] int64 from column-major ``bins_t`` [F, n] int16 and fixed-point
    ``gq``/``hq`` [n] int32 on a GPU."""
    F, n = bins_t.shape
    dev = bins_t.device
    if dev.type != "cuda":
        return torch_level_histogram(bins_t.t(), pos, gq, hq, K, B)
    if bins_t.dtype != torch.int16 or not bins_t.is_contiguous():
        raise ValueError("bins_t must be a contiguous int16 [F, n] tensor")
    if not 0 < int(B) <= 32768:
        raise ValueError(f"{B} bins per feature: int16 bin ids hold at most 32768")
    if gq.dtype != torch.int32 or hq.dtype != torch.int32:
        raise ValueError("gq/hq must be fixed-point int32 (see quantise)")
    L = _lib()
    pos = pos.to(torch.long).contiguous()
    gq, hq = gq.contiguous(), hq.contiguous()
    if pos.shape[0] != n or gq.shape[0] != n or hq.shape[0] != n:
        raise ValueError("pos/gq/hq must have one entry per row of bins_t")
    for t in (pos, gq, hq):
        if t.device != dev:
            raise ValueError("all operands must live on the same GPU")
    hist = torch.zeros(K * F * B, 2, dtype=torch.int64, device=dev)
    _hip.check(L.rx_gbdt_hist(ctypes.c_void_p(bins_t.data_ptr()), ctypes.c_void_p(pos.data_ptr()),
                              ctypes.c_void_p(gq.data_ptr()), ctypes.c_void_p(hq.data_ptr()),
                              ctypes.c_void_p(hist.data_ptr()), n, F, int(B), int(K), _hip.stream_ptr(dev)),
               "rx_gbdt_hist")
    return hist


def split_gains(L: torch.Tensor, R: torch.Tensor, inv_g: float, inv_h: float, lam: float, alpha: float,
                mcw: float, parent: torch.Tensor):
    """XGBoost split gain from exact int64 (g, h) child sums ``L``/``R`` [..., 2], in the same
    operation order as the split kernel (so CPU and GPU gains agree bit for bit). Returns
    (gain, valid)."""
    Lg, Lh = L[..., 0].double() * inv_g, L[..., 1].double() * inv_h
    Rg, Rh = R[..., 0].double() * inv_g, R[..., 1].double() * inv_h
    sl, sr = soft(Lg, alpha), soft(Rg, alpha)
    gain = sl * sl / (Lh + lam) + sr * sr / (Rh + lam) - parent
    valid = (Lh >= mcw) & (Rh >= mcw) & (Lh + lam > 0) & (Rh + lam > 0)
    return gain, valid


def soft(g, alpha):
    """L1 soft threshold (identity when alpha <= 0)."""
    if alpha <= 0:
        return g
    return torch.sign(g) * torch.clamp(g.abs() - alpha, min=0.0)


def torch_split_candidates(hist: torch.Tensor, tot: torch.Tensor, ncuts: torch.Tensor, fmask, inv_g: float,
                           inv_h: float, lam: float, alpha: float, mcw: float) -> torch.Tensor:
    """Tensor formulation of :func:`split_candidates` (the CPU path and the kernel's reference)."""
    K, F, B, _ = hist.shape
    dev = hist.device
    miss = hist[:, :, 0, :]                                   # (K, F, 2)
    cum = hist[:, :, 1:, :].cumsum(2)                         # bins 1..t go left, exact int64
    G, H = tot[:, 0].double() * inv_g, tot[:, 1].double() * inv_h
    sG = soft(G, alpha)
    parent = (sG * sG / (H + lam))[:, None, None]
    tpos = torch.arange(B - 1, device=dev)[None, None, :]
    out = torch.empty((K, F, 4), dtype=torch.float64, device=dev)
    for c, dl in ((0, 1), (2, 0)):
        L = cum + (miss[:, :, None, :] if dl else 0)
        R = tot[:, None, None, :] - L
        gain, valid = split_gains(L, R, inv_g, inv_h, lam, alpha, mcw, parent)
        valid &= tpos < ncuts.to(dev)[None, :, None]
        if fmask is not None:
            valid &= fmask.to(device=dev, dtype=torch.bool)[None, :, None]
        gain = torch.where(valid, gain, torch.full_like(gain, -1.0))
        # strictly-better scan semantics: the lowest t among the maxima, -1 / t=0 when none beats -1
        best, arg = gain.max(2)
        none = ~(best > -1.0)
        out[:, :, c] = torch.where(none, torch.full_like(best, -1.0), best)
        out[:, :, c + 1] = torch.where(none, torch.zeros_like(best), arg.double())
    return out


def split_candidates(hist: torch.Tensor, tot: torch.Tensor, ncuts: torch.Tensor, fmask, inv_g: float, inv_h: float,
                     lam: float, alpha: float, mcw: float) -> torch.Tensor:
    """Best threshold per (node, feature) for both default directions on a GPU.

    ``hist`` [K, F, B, 2] int64 fixed-point sums, ``tot`` [K, 2] int64 node totals, ``inv_g`` /
    ``inv_h`` the reciprocal quantisation scales, ``ncuts`` [F] int32 real cuts per feature,
    ``fmask`` [F] uint8 or None. Returns [K, F, 4] fp64: (gain, threshold) for default-left, then
    for default-right; gain -1 where no valid threshold exists.
    """
    K, F, B, two = hist.shape
    if two != 2 or hist.dtype != torch.int64 or hist.device.type != "cuda":
        raise ValueError("hist must be a [K, F, B, 2] int64 GPU tensor")
    hist = hist.contiguous()
    tot = tot.to(torch.int64).contiguous()
    ncuts = ncuts.to(device=hist.device, dtype=torch.int32).contiguous()
    if tot.shape != (K, 2) or ncuts.shape != (F,) or (fmask is not None and fmask.shape != (F,)):
        raise ValueError("tot/ncuts/fmask shapes do not match hist")
    if fmask is not None:
        fmask = fmask.to(device=hist.device, dtype=torch.uint8).contiguous()
    out = torch.empty((K, F, 4), dtype=torch.float64, device=hist.device)
    _hip.check(_lib().rx_gbdt_split(ctypes.c_void_p(hist.data_ptr()), ctypes.c_void_p(tot.data_ptr()),
                                    ctypes.c_void_p(ncuts.data_ptr()),
                                    ctypes.c_void_p(fmask.data_ptr()) if fmask is not None else None,
                                    ctypes.c_void_p(out.data_ptr()), K, F, B, float(inv_g), float(inv_h),
                                    float(lam), float(alpha), float(mcw), _hip.stream_ptr(hist.device)),
               "rx_gbdt_split")
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
