"""Fused Linear(+bias)(+ReLU) towers on the gfx950 GEMM kernels of ``csrc/hip/linear_act.hip``.

``FusedLinearTower`` runs a chain of ``nn.Linear`` layers (each optionally followed by ReLU) as
one autograd op: per layer ONE forward kernel (GEMM + bias + ReLU epilogue, bf16 activation
out), and in backward ONE dgrad kernel (the ReLU mask of the layer below applied in its
epilogue) and ONE wgrad kernel (weight gradient + the bias gradient as a row sum of its
operand fragments). fp32 inputs (dense features, the DLRM dot-interaction output) are converted
to bf16 inside the GEMM's operand staging. The fp32 ``nn.Linear`` parameters stay the masters
(any torch optimizer updates them); their bf16 images are refreshed by one multi-tensor launch
when an optimizer step has changed them (``Tensor._version``).

This replaces the eager ``Linear``/``ReLU`` chain of the reference's DLRM ``TorchMlp``
(``examples/pytorch_dlrm.ipynb`` cell 9), whose AMP step spent ~30 % of GPU time in cast,
bias-gradient reduce, clamp and threshold kernels (``profiles/r1_dlrm_kernel_stats.csv``).
"""
import ctypes
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

from raydp_amd.ops import _hip

ROW, RED = 0, 1
FWD, DGRAD, WGRAD = 0, 1, 2


class LinOperand(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("ld", ctypes.c_longlong), ("f32", ctypes.c_int), ("lay", ctypes.c_int)]


class LinArgs(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("epi", ctypes.c_int),
        ("a", LinOperand), ("b", LinOperand),
        ("bias", ctypes.c_void_p), ("relu", ctypes.c_int), ("out_f32", ctypes.c_int),
        ("out", ctypes.c_void_p), ("ldo", ctypes.c_longlong),
        ("out2", ctypes.c_void_p), ("ldo2", ctypes.c_longlong),
        ("mask", ctypes.c_void_p), ("ldm", ctypes.c_longlong),
        ("dbias", ctypes.c_void_p), ("beta", ctypes.c_float), ("splits", ctypes.c_int),
        ("ws", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("tile", ctypes.c_int), ("pad_", ctypes.c_int),
    ]


# LinArgs.tile (csrc/hip/linear_act.hip LIN_TILE_*): 0 = the shape rx_lin_plan picks
TILE_AUTO, TILE_64x64, TILE_128x128, TILE_128x64, TILE_64x128 = 0, 1, 2, 3, 4


class LinRefresh(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("pad_", ctypes.c_int), ("src", ctypes.c_void_p * 16),
                ("dst", ctypes.c_void_p * 16), ("len", ctypes.c_longlong * 16)]


_bound = None


def _lib():
    global _bound
    L = _hip.lib()
    if _bound is not L:
        vp, ll = ctypes.c_void_p, ctypes.c_longlong
        L.rx_lin_gemm.argtypes = [vp, vp]
        L.rx_lin_mask_cast.argtypes = [vp, vp, vp, ll, vp]
        L.rx_lin_refresh.argtypes = [vp, vp]
        L.rx_lin_splits.argtypes = [ctypes.c_int] * 4
        L.rx_lin_ws_floats.argtypes = [ctypes.c_int] * 3
        L.rx_lin_splits.restype = L.rx_lin_ws_floats.restype = ctypes.c_int
        L.rx_lin_plan.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int)]
        L.rx_lin_plan.restype = ctypes.c_int
        i = ctypes.c_int
        L.rx_lin_tower_fwd.argtypes = [vp, i, i, vp, i, ll, vp, vp, vp, vp]
        L.rx_lin_tower_bwd.argtypes = [vp, i, i, vp, i, ll, vp, vp, ll, i, vp, vp, vp, vp, vp]
        L.rx_lin_tower_fwd.restype = L.rx_lin_tower_bwd.restype = i
        for name, cls in (("rx_lin_layer_size", LinLayer), ("rx_lin_scratch_size", LinScratch)):
            getattr(L, name).restype = i
            if getattr(L, name)() != ctypes.sizeof(cls):
                raise RuntimeError(f"ABI mismatch for {cls.__name__}")
        for n in ("rx_lin_gemm", "rx_lin_mask_cast", "rx_lin_refresh", "rx_lin_args_size", "rx_lin_refresh_size"):
            getattr(L, n).restype = ctypes.c_int
        for name, cls in (("rx_lin_args_size", LinArgs), ("rx_lin_refresh_size", LinRefresh)):
            if getattr(L, name)() != ctypes.sizeof(cls):
                raise RuntimeError(f"ABI mismatch for {cls.__name__}")
        _bound = L
    return L


_scratch = {}   # device index -> [workspace fp32, tile counters int32] (grown on demand)
_sizes = {}     # (device, GEMM shapes) -> (workspace floats, tiles)
_cus = {}


def plan(M: int, N: int, K: int, cus: int = 256, tile: int = TILE_AUTO):
    """(tile shape, split-K factor) the kernel library picks for one GEMM (``rx_lin_plan``)."""
    t = ctypes.c_int(0)
    sp = int(_lib().rx_lin_plan(M, N, K, cus, int(tile), ctypes.byref(t)))
    return t.value, sp


def _split_ws(device, M, N, K, force: Optional[int] = None, tile: int = TILE_AUTO):
    """(tile, split-K factor, workspace, counters) for one GEMM on ``device``."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _cus:
        _cus[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    L = _lib()
    tile, sp = plan(M, N, K, _cus[idx], tile)
    if force is not None:
        sp = int(force)
    if sp <= 1:
        return tile, 1, None, None
    need = int(L.rx_lin_ws_floats(M, N, sp))
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    ws, cnt = _scratch.get(idx, (None, None))
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=device)
    if cnt is None or cnt.numel() < tiles:
        cnt = torch.zeros(max(tiles, 1024), dtype=torch.int32, device=device)
    _scratch[idx] = (ws, cnt)
    return tile, sp, ws, cnt


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _operand(t: torch.Tensor, lay: int) -> LinOperand:
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("fused linear operands must be 2-D with a contiguous last dimension")
    if t.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"fused linear operand dtype {t.dtype}")
    return LinOperand(ctypes.c_void_p(t.data_ptr()), t.stride(0), int(t.dtype == torch.float32), lay)


def gemm(epi: int, M: int, N: int, K: int, a: torch.Tensor, a_lay: int, b: torch.Tensor, b_lay: int,
         out: torch.Tensor, bias=None, relu=False, out2=None, mask=None, dbias=None, beta=0.0,
         splits: Optional[int] = None, tile: int = TILE_AUTO):
    """One launch of the fused GEMM (host-side shape checks: the kernel itself only bounds
    rows / columns by M, N, K). ``splits`` / ``tile`` force the split-K factor / tile shape
    (default: ``plan``)."""
    def rows_cols(t, lay, rows):
        # ROW: [rows][K]; RED: [K][rows]
        want = (rows, K) if lay == ROW else (K, rows)
        if tuple(t.shape) != want:
            raise ValueError(f"operand shape {tuple(t.shape)} != {want}")
    rows_cols(a, a_lay, M)
    rows_cols(b, b_lay, N)
    if tuple(out.shape) != (M, N) or out.stride(1) != 1:
        raise ValueError(f"output shape {tuple(out.shape)} != {(M, N)}")
    if epi == WGRAD and out.dtype != torch.float32:
        raise TypeError("wgrad output is fp32")
    for t, shape in ((bias, (N,)), (dbias, (M,))):
        if t is not None and (tuple(t.shape) != shape or t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError("bias / dbias must be contiguous fp32 of the output's column / row count")
    if mask is not None and (tuple(mask.shape) != (M, N) or mask.dtype != torch.bfloat16 or mask.stride(1) != 1):
        raise ValueError("mask must be bf16 [M, N]")
    if out2 is not None and (tuple(out2.shape) != (M, N) or out2.dtype != torch.float32 or out2.stride(1) != 1):
        raise ValueError("out2 must be fp32 [M, N]")
    args = LinArgs()
    args.M, args.N, args.K, args.epi = M, N, K, epi
    args.a, args.b = _operand(a, a_lay), _operand(b, b_lay)
    args.bias, args.relu = _ptr(bias), int(relu)
    args.out_f32, args.out, args.ldo = int(out.dtype == torch.float32), _ptr(out), out.stride(0)
    args.out2, args.ldo2 = _ptr(out2), out2.stride(0) if out2 is not None else 0
    args.mask, args.ldm = _ptr(mask), mask.stride(0) if mask is not None else 0
    args.dbias, args.beta = _ptr(dbias), float(beta)
    tl, sp, ws, cnt = _split_ws(out.device, M, N, K, splits, tile)
    args.splits, args.ws, args.counters, args.tile = sp, _ptr(ws), _ptr(cnt), tl
    _hip.check(_lib().rx_lin_gemm(ctypes.byref(args), _hip.stream_ptr(out.device)), "rx_lin_gemm")
    return out


class LinLayer(ctypes.Structure):
    _fields_ = [("W", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("dW", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("N", ctypes.c_int), ("K", ctypes.c_int), ("relu", ctypes.c_int), ("pad_", ctypes.c_int)]


class LinScratch(ctypes.Structure):
    _fields_ = [("ws", ctypes.c_void_p), ("counters", ctypes.c_void_p), ("ws_floats", ctypes.c_longlong),
                ("counters_len", ctypes.c_int), ("cus", ctypes.c_int), ("pair", ctypes.c_int), ("pad_", ctypes.c_int)]


# The tower backward runs each layer's dgrad and wgrad as ONE paired launch
# (csrc/hip/linear_act.hip lin_pair_kernel); False: two launches per layer (A/B measurements).
PAIR_BACKWARD = True


def _scratch_for(device, shapes) -> LinScratch:
    """Split-K workspace covering every (M, N, K) GEMM in ``shapes`` (grown on demand); twice
    that when the backward pairs two split GEMMs in one launch (each takes one half)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _cus:
        _cus[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    key = (idx, tuple(shapes))
    hit = _sizes.get(key)
    if hit is None:
        L = _lib()
        need, tiles = 0, 1024
        for M, N, K in shapes:
            sp = int(L.rx_lin_splits(M, N, K, _cus[idx]))
            need = max(need, int(L.rx_lin_ws_floats(M, N, sp)))
            tiles = max(tiles, ((M + 63) // 64) * ((N + 63) // 64))
        hit = _sizes[key] = (2 * need, 2 * tiles)
    need, tiles = hit
    ws, cnt = _scratch.get(idx, (None, None))
    if ws is None or ws.numel() < max(need, 1):
        ws = torch.empty(max(need, 1), dtype=torch.float32, device=device)
    if cnt is None or cnt.numel() < tiles:
        cnt = torch.zeros(tiles, dtype=torch.int32, device=device)
    _scratch[idx] = (ws, cnt)
    sc = LinScratch()
    sc.ws, sc.counters, sc.ws_floats = ws.data_ptr(), cnt.data_ptr(), ws.numel()
    sc.counters_len, sc.cus, sc.pair = cnt.numel(), _cus[idx], int(PAIR_BACKWARD)
    return sc


class _TowerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tower, x, *params):
        t = tower
        t._refresh_images()
        if x.dim() != 2 or x.stride(1) != 1 or x.dtype not in (torch.float32, torch.bfloat16):
            x = x.contiguous().float()
        M = x.shape[0]
        if x.shape[1] != t.linears[0].in_features:
            raise ValueError(f"tower input has {x.shape[1]} features, expected {t.linears[0].in_features}")
        dev = x.device
        acts = [torch.empty(M, lin.out_features, dtype=torch.bfloat16, device=dev) for lin in t.linears]
        out32 = torch.empty(M, t.linears[-1].out_features, dtype=torch.float32, device=dev) if t.out_f32 else None
        layers = t._layers(None)
        ptrs = (ctypes.c_void_p * len(acts))(*[a.data_ptr() for a in acts])
        sc = _scratch_for(dev, t._shapes(M))
        _hip.check(_lib().rx_lin_tower_fwd(layers, len(acts), M, ctypes.c_void_p(x.data_ptr()),
                                           int(x.dtype == torch.float32), x.stride(0), ptrs, _ptr(out32),
                                           ctypes.byref(sc), _hip.stream_ptr(dev)), "rx_lin_tower_fwd")
        ctx.tower = t
        ctx.save_for_backward(x, *acts)
        return out32 if out32 is not None else acts[-1]

    @staticmethod
    def backward(ctx, gout):
        t = ctx.tower
        x, *acts = ctx.saved_tensors
        M = x.shape[0]
        dev = x.device
        # a producer that already applied this tower's output ReLU mask marks its gradient
        # (raydp_amd.ops.dlrm_ops: the interaction backward masks the bottom-MLP slot with X > 0)
        masked = bool(getattr(gout, "_raydp_relu_masked", False)) and t.relus[-1]
        if gout.dtype != torch.float32 or gout.dim() != 2 or gout.stride(1) != 1:
            gout = gout.contiguous().float()
        # rows of gout may be further apart than its width (a column slice of a wider gradient,
        # e.g. the DLRM interaction input's bottom-MLP slot): read in place, no copy kernel
        dWs, dbs = [], []
        for lin in t.linears:
            dWs.append(torch.empty(lin.out_features, lin.in_features, dtype=torch.float32, device=dev)
                       if lin.weight.requires_grad else None)
            dbs.append(torch.empty(lin.out_features, dtype=torch.float32, device=dev)
                       if lin.bias is not None and lin.bias.requires_grad else None)
        dx = torch.empty(x.shape, dtype=x.dtype, device=dev) if ctx.needs_input_grad[1] else None
        width = max(lin.out_features for lin in t.linears)
        g0 = torch.empty(M * width, dtype=torch.bfloat16, device=dev)
        g1 = torch.empty(M * width, dtype=torch.bfloat16, device=dev)
        layers = t._layers((dWs, dbs))
        ptrs = (ctypes.c_void_p * len(acts))(*[a.data_ptr() for a in acts])
        sc = _scratch_for(dev, t._shapes(M))
        _hip.check(_lib().rx_lin_tower_bwd(layers, len(acts), M, ctypes.c_void_p(x.data_ptr()),
                                           int(x.dtype == torch.float32), x.stride(0), ptrs, _ptr(gout),
                                           gout.stride(0) if gout.shape[0] > 1 else gout.shape[1], int(masked),
                                           _ptr(dx),
                                           _ptr(g0), _ptr(g1), ctypes.byref(sc), _hip.stream_ptr(dev)),
                   "rx_lin_tower_bwd")
        out = [dx]
        for lin, dW, db in zip(t.linears, dWs, dbs):
            out.append(dW)
            if lin.bias is not None:
                out.append(db)
        return (None,) + tuple(out)


class FusedLinearTower:
    """A chain of ``nn.Linear`` (+ReLU) layers run on the fused kernels. Holds no parameters of
    its own: the Linear modules (and so ``state_dict``) are the user's."""

    def __init__(self, linears: Sequence[nn.Linear], relus: Sequence[bool], out_f32: bool = True):
        if len(linears) != len(relus) or not linears:
            raise ValueError("one relu flag per Linear")
        if len(linears) > 16:
            raise ValueError("at most 16 layers per fused tower")
        for a, b in zip(linears[:-1], linears[1:]):
            if a.out_features != b.in_features:
                raise ValueError("Linear chain dimensions do not match")
        self.linears = list(linears)
        self.relus = [bool(r) for r in relus]
        self.out_f32 = out_f32
        self.images: List[Optional[torch.Tensor]] = [None] * len(self.linears)
        self._versions = [None] * len(self.linears)
        # images the multi-tensor optimizer writes itself (raydp_amd/ops/fused_optim.py): not
        # re-derived before a forward, not even inside a graph capture
        self._managed = [False] * len(self.linears)
        self._register()

    def _register(self):
        from raydp_amd.ops.fused_optim import register_image
        for li, lin in enumerate(self.linears):
            register_image(lin.weight, self, li)

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._managed = [False] * len(self.linears)
        self._register()

    def image_for(self, li: int) -> torch.Tensor:
        """The bf16 image buffer of layer ``li`` (allocated on first use)."""
        w = self.linears[li].weight
        img = self.images[li]
        if img is None or img.device != w.device or img.shape != w.shape:
            img = self.images[li] = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
            self._versions[li] = None
        return img

    def image_updated(self, li: int):
        """The optimizer kernel just wrote layer ``li``'s image from the updated weight."""
        w = self.linears[li].weight
        self._versions[li] = (w.data_ptr(), w._version)
        self._managed[li] = True

    def __getstate__(self):
        # device images are caches: a copied / pickled tower rebuilds them from its weights
        st = dict(self.__dict__)
        st["images"] = [None] * len(self.linears)
        st["_versions"] = [None] * len(self.linears)
        st["_managed"] = [False] * len(self.linears)
        return st

    def _refresh_images(self):
        # inside a HIP-graph capture the refresh is recorded unconditionally: a replayed step
        # must re-derive the images from the (replayed) optimizer's updates
        capturing = torch.cuda.is_current_stream_capturing()
        stale = []
        for li, lin in enumerate(self.linears):
            w = lin.weight
            img = self.images[li]
            if img is None or img.device != w.device or img.shape != w.shape:
                img = self.images[li] = torch.empty(w.shape, dtype=torch.bfloat16, device=w.device)
                self._versions[li] = None
            key = (w.data_ptr(), w._version)
            if self._versions[li] != key or (capturing and not self._managed[li]):
                stale.append(li)
                self._versions[li] = key
        if not stale:
            return
        r = LinRefresh()
        r.n = len(stale)
        for j, li in enumerate(stale):
            w = self.linears[li].weight.detach()
            if not w.is_contiguous() or w.dtype != torch.float32:
                raise ValueError("fused tower weights must be contiguous fp32")
            r.src[j], r.dst[j], r.len[j] = w.data_ptr(), self.images[li].data_ptr(), w.numel()
        _hip.check(_lib().rx_lin_refresh(ctypes.byref(r), _hip.stream_ptr(self.linears[0].weight.device)),
                   "rx_lin_refresh")

    def _layers(self, grads):
        arr = (LinLayer * len(self.linears))()
        for i, (lin, img, relu) in enumerate(zip(self.linears, self.images, self.relus)):
            L = arr[i]
            L.W, L.bias = img.data_ptr(), lin.bias.data_ptr() if lin.bias is not None else None
            L.N, L.K, L.relu = lin.out_features, lin.in_features, int(relu)
            if grads is not None:
                dW, db = grads[0][i], grads[1][i]
                L.dW = dW.data_ptr() if dW is not None else None
                L.db = db.data_ptr() if db is not None else None
        return arr

    def _shapes(self, M):
        out = []
        for lin in self.linears:
            N, K = lin.out_features, lin.in_features
            out += [(M, N, K), (N, K, M), (M, K, N)]
        return out

    def params(self):
        out = []
        for lin in self.linears:
            out.append(lin.weight)
            if lin.bias is not None:
                out.append(lin.bias)
        return out

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        return _TowerFn.apply(self, x, *self.params())


def tower_enabled() -> bool:
    from raydp_amd.utils.config import get as conf_get
    return bool(conf_get("spark.ray.mi355x.fused_linear"))
