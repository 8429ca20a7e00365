"""Multi-tensor SGD and fused BCE-with-logits for the torch-loop engine
(``csrc/hip/fused_optim.hip``).

* :func:`sgd_step` -- ``torch.optim.SGD.step()`` semantics (lr, momentum, dampening,
  nesterov, weight decay, maximize; momentum buffers kept in ``optimizer.state`` exactly as
  torch keeps them) as ONE launch per 24 dense parameter tensors, which also writes the bf16
  operand image of every weight a fused Linear tower reads (``linear_ops.FusedLinearTower``),
  so the tower does not rebuild it before the next forward. Sparse gradients (embedding rows)
  keep torch's update. :class:`FusedSGD` is the same as an optimizer class.
* :func:`adam_step` -- ``torch.optim.Adam`` / ``AdamW`` the same way (Horovod's
  ``DistributedOptimizer`` runs a wrapped Adam / AdamW / SGD through :func:`fused_step`).
* :class:`FusedBCEWithLogits` -- ``nn.BCEWithLogitsLoss()`` (mean reduction, no weights): the
  loss is one single-workgroup kernel and its gradient one elementwise kernel computed from the
  saved operands (eager torch: log-sigmoid, mean, sigmoid, sub, mul ... ~6 launches).

Reference: the DLRM notebook's ``torch.optim.SGD`` + ``nn.BCEWithLogitsLoss``
(``examples/pytorch_dlrm.ipynb`` cells 9, 14) on the estimator's loop
(``python/raydp/torch/estimator.py:272-293``).
"""
import ctypes
import weakref
from typing import Optional

import torch
import torch.nn as nn

from raydp_amd.ops import _hip

MT_MAX = 24


class MtSgd(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("first", ctypes.c_int), ("lr", ctypes.c_float), ("wd", ctypes.c_float),
                ("momentum", ctypes.c_float), ("dampening", ctypes.c_float), ("nesterov", ctypes.c_int),
                ("maximize", ctypes.c_int), ("p", ctypes.c_void_p * MT_MAX), ("g", ctypes.c_void_p * MT_MAX),
                ("buf", ctypes.c_void_p * MT_MAX), ("img", ctypes.c_void_p * MT_MAX),
                ("len", ctypes.c_longlong * MT_MAX)]


class MtAdam(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("adamw", ctypes.c_int), ("maximize", ctypes.c_int),
                ("lr", ctypes.c_float), ("b1", ctypes.c_float), ("b2", ctypes.c_float), ("eps", ctypes.c_float),
                ("wd", ctypes.c_float), ("nlr_bc1", ctypes.c_float * MT_MAX), ("rs_bc2", ctypes.c_float * MT_MAX),
                ("p", ctypes.c_void_p * MT_MAX), ("g", ctypes.c_void_p * MT_MAX), ("m", ctypes.c_void_p * MT_MAX),
                ("v", ctypes.c_void_p * MT_MAX), ("len", ctypes.c_longlong * MT_MAX)]


_bound = None


def _lib():
    global _bound
    L = _hip.lib()
    if _bound is not L:
        vp, ll = ctypes.c_void_p, ctypes.c_longlong
        L.rx_mt_sgd.argtypes = [vp, vp]
        L.rx_mt_adam.argtypes = [vp, vp]
        L.rx_bce_logits_fwd.argtypes = [vp, vp, ll, vp, vp]
        L.rx_bce_logits_bwd.argtypes = [vp, vp, vp, ll, vp, vp]
        for n in ("rx_mt_sgd", "rx_mt_adam", "rx_bce_logits_fwd", "rx_bce_logits_bwd", "rx_mt_sgd_size",
                  "rx_mt_sgd_max", "rx_mt_adam_size"):
            getattr(L, n).restype = ctypes.c_int
        if L.rx_mt_sgd_size() != ctypes.sizeof(MtSgd) or L.rx_mt_sgd_max() != MT_MAX:
            raise RuntimeError("MtSgd layout mismatch between Python and csrc/hip/fused_optim.hip")
        if L.rx_mt_adam_size() != ctypes.sizeof(MtAdam):
            raise RuntimeError("MtAdam layout mismatch between Python and csrc/hip/fused_optim.hip")
        _bound = L
    return L


def register_image(weight: torch.Tensor, tower, layer: int):
    """A fused Linear tower reads a bf16 image of ``weight``: remember (on the parameter itself,
    weakly) who owns it, so the optimizer kernel can keep the image current."""
    weight._raydp_image_owner = (weakref.ref(tower), layer)


def _image_of(p):
    ent = getattr(p, "_raydp_image_owner", None)
    if ent is None:
        return None, None, None
    tower = ent[0]()
    if tower is None:
        return None, None, None
    return tower, ent[1], tower.image_for(ent[1])


def sgd_supported(opt) -> Optional[str]:
    """None when :func:`sgd_step` reproduces ``opt.step()``; else why not."""
    if type(opt) is not torch.optim.SGD and not isinstance(opt, FusedSGD):
        return f"{type(opt).__name__} is not torch.optim.SGD"
    for g in opt.param_groups:
        if isinstance(g["lr"], torch.Tensor) or g.get("differentiable", False):
            return "tensor / differentiable learning rate"
        for p in g["params"]:
            if p.grad is not None and p.grad.is_sparse and float(g["momentum"]) != 0.0:
                # torch.optim.SGD keeps a momentum buffer for sparse gradients too (it densifies
                # the buffer): torch's own step reproduces that, this one does not
                return "sparse gradient with momentum"
            if p.grad is not None and not p.grad.is_sparse and (
                    not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous()
                    or not p.grad.is_contiguous() or p.grad.dtype != torch.float32):
                return "parameters must be contiguous fp32 CUDA tensors"
    return None


@torch.no_grad()
def sgd_step(opt) -> None:
    """One ``torch.optim.SGD`` step of ``opt`` on the multi-tensor kernel (dense gradients)."""
    L = _lib()
    for group in opt.param_groups:
        lr, mom, damp = float(group["lr"]), float(group["momentum"]), float(group["dampening"])
        wd, nest, maxim = float(group["weight_decay"]), bool(group["nesterov"]), bool(group.get("maximize", False))
        dense, fresh = [], []
        for p in group["params"]:
            if p.grad is None:
                continue
            if p.grad.is_sparse:
                # embedding rows, plain SGD (sgd_supported sends sparse + momentum to torch)
                if mom != 0.0:
                    raise RuntimeError("sgd_step: sparse gradient with momentum (use opt.step())")
                g = p.grad if not maxim else -p.grad
                if wd:
                    raise RuntimeError("weight decay with sparse gradients is not supported by SGD")
                p.add_(g, alpha=-lr)
                continue
            dense.append(p)
        # split into launches of MT_MAX tensors; tensors whose momentum buffer is new go together
        # (the kernel's `first` flag is per launch)
        if mom != 0.0:
            for p in dense:
                st = opt.state[p]
                if st.get("momentum_buffer") is None:
                    st["momentum_buffer"] = torch.empty_like(p)
                    fresh.append(p)
        fresh_ids = {id(p) for p in fresh}
        for first in (True, False):
            sel = [p for p in dense if (id(p) in fresh_ids) == first] if mom != 0.0 else (dense if not first else [])
            for k in range(0, len(sel), MT_MAX):
                chunk = sel[k:k + MT_MAX]
                a = MtSgd()
                a.n, a.first = len(chunk), int(first)
                a.lr, a.wd, a.momentum, a.dampening = lr, wd, mom, damp
                a.nesterov, a.maximize = int(nest), int(maxim)
                owners = []
                for j, p in enumerate(chunk):
                    a.p[j], a.g[j], a.len[j] = p.data_ptr(), p.grad.data_ptr(), p.numel()
                    a.buf[j] = opt.state[p]["momentum_buffer"].data_ptr() if mom != 0.0 else None
                    tower, li, img = _image_of(p)
                    a.img[j] = img.data_ptr() if img is not None else None
                    if img is not None:
                        owners.append((tower, li))
                _hip.check(L.rx_mt_sgd(ctypes.byref(a), _hip.stream_ptr(chunk[0].device)), "rx_mt_sgd")
                for tower, li in owners:
                    tower.image_updated(li)


def adam_supported(opt) -> Optional[str]:
    """None when :func:`adam_step` reproduces ``opt.step()`` of a ``torch.optim.Adam`` /
    ``AdamW`` (to fp32 rounding: the kernel's operation order is not torch's); else why not."""
    if type(opt) not in (torch.optim.Adam, torch.optim.AdamW):
        return f"{type(opt).__name__} is not torch.optim.Adam / AdamW"
    for g in opt.param_groups:
        if g.get("amsgrad") or g.get("capturable") or g.get("differentiable") or g.get("fused"):
            return "amsgrad / capturable / differentiable / fused groups keep torch's step"
        if isinstance(g["lr"], torch.Tensor) or any(isinstance(b, torch.Tensor) for b in g["betas"]):
            return "tensor hyperparameters"
        for p in g["params"]:
            if p.grad is None:
                continue
            if p.grad.is_sparse or not p.is_cuda or p.dtype != torch.float32 or not p.is_contiguous() \
                    or not p.grad.is_contiguous() or p.grad.dtype != torch.float32:
                return "parameters must be dense contiguous fp32 CUDA tensors"
            st = opt.state.get(p)
            if st and (not st["exp_avg"].is_contiguous() or not st["exp_avg_sq"].is_contiguous()
                       or st["step"].is_cuda):
                return "optimizer state not in torch's default (contiguous, host step) layout"
    return None


@torch.no_grad()
def adam_step(opt) -> None:
    """One ``torch.optim.Adam`` / ``AdamW`` step of ``opt`` on the multi-tensor kernel: one launch
    per 24 parameter tensors. The state stays torch's (``step`` a host tensor, ``exp_avg``,
    ``exp_avg_sq``), so ``state_dict()`` / checkpoints / a later ``opt.step()`` see no difference."""
    L = _lib()
    for group in opt.param_groups:
        # decoupled decay (p *= 1 - lr * wd): AdamW, or Adam(decoupled_weight_decay=True) in torch >= 2.6
        adamw = isinstance(opt, torch.optim.AdamW) or bool(group.get("decoupled_weight_decay", False))
        lr = float(group["lr"])
        b1, b2 = (float(b) for b in group["betas"])
        live = [p for p in group["params"] if p.grad is not None]
        for k in range(0, len(live), MT_MAX):
            chunk = live[k:k + MT_MAX]
            a = MtAdam()
            a.n, a.adamw, a.maximize = len(chunk), int(adamw), int(bool(group.get("maximize", False)))
            a.lr, a.b1, a.b2, a.eps, a.wd = lr, b1, b2, float(group["eps"]), float(group["weight_decay"])
            for j, p in enumerate(chunk):
                st = opt.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                t = float(st["step"])
                a.nlr_bc1[j] = -lr / (1.0 - b1 ** t)
                a.rs_bc2[j] = 1.0 / (1.0 - b2 ** t) ** 0.5
                a.p[j], a.g[j], a.len[j] = p.data_ptr(), p.grad.data_ptr(), p.numel()
                a.m[j], a.v[j] = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            _hip.check(L.rx_mt_adam(ctypes.byref(a), _hip.stream_ptr(chunk[0].device)), "rx_mt_adam")


def _has_step_hooks(opt) -> bool:
    """Optimizer step pre/post hooks (per instance or global) that ``opt.step()`` would run."""
    from torch.optim import optimizer as _o
    return bool(getattr(opt, "_optimizer_step_pre_hooks", None) or getattr(opt, "_optimizer_step_post_hooks", None)
                or getattr(_o, "_global_optimizer_pre_hooks", None) or getattr(_o, "_global_optimizer_post_hooks", None))


def fused_step(opt) -> bool:
    """``opt.step()`` on the multi-tensor kernels when they cover ``opt`` (Adam / AdamW / SGD over
    dense fp32 CUDA parameters); False (nothing done) otherwise -- also when step hooks are
    registered, which only torch's own ``step()`` runs."""
    if _has_step_hooks(opt):
        return False
    if adam_supported(opt) is None:
        adam_step(opt)
        return True
    if sgd_supported(opt) is None:
        sgd_step(opt)
        return True
    return False


class FusedSGD(torch.optim.SGD):
    """``torch.optim.SGD`` whose ``step()`` runs :func:`sgd_step` (falls back to torch's step
    for anything the kernel does not cover)."""

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if sgd_supported(self) is None:
            sgd_step(self)
        else:
            super().step()
        return loss


class _BCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        xc, yc = x.detach().contiguous(), y.detach().contiguous()
        out = torch.empty((), dtype=torch.float32, device=x.device)
        _hip.check(_lib().rx_bce_logits_fwd(ctypes.c_void_p(xc.data_ptr()), ctypes.c_void_p(yc.data_ptr()),
                                            xc.numel(), ctypes.c_void_p(out.data_ptr()),
                                            _hip.stream_ptr(x.device)), "rx_bce_logits_fwd")
        ctx.save_for_backward(xc, yc)
        ctx.shape = x.shape
        return out

    @staticmethod
    def backward(ctx, go):
        xc, yc = ctx.saved_tensors
        go = go.detach().float().contiguous()
        dx = torch.empty_like(xc)
        _hip.check(_lib().rx_bce_logits_bwd(ctypes.c_void_p(xc.data_ptr()), ctypes.c_void_p(yc.data_ptr()),
                                            ctypes.c_void_p(go.data_ptr()), xc.numel(),
                                            ctypes.c_void_p(dx.data_ptr()), _hip.stream_ptr(xc.device)),
                   "rx_bce_logits_bwd")
        return dx.view(ctx.shape), None


class FusedBCEWithLogits(nn.Module):
    """Drop-in for ``nn.BCEWithLogitsLoss()`` on fp32 CUDA tensors (other inputs: torch)."""

    def __init__(self):
        super().__init__()
        self._torch = nn.BCEWithLogitsLoss()

    def forward(self, x, y):
        if x.is_cuda and x.dtype == torch.float32 and y.dtype == torch.float32 and x.shape == y.shape \
                and x.numel() > 0:
            return _BCEFn.apply(x, y)
        return self._torch(x, y)


def fusable_bce(loss) -> bool:
    """An ``nn.BCEWithLogitsLoss`` with the defaults (mean, no weight / pos_weight)."""
    return (type(loss) is nn.BCEWithLogitsLoss and loss.reduction == "mean" and loss.weight is None
            and loss.pos_weight is None)
