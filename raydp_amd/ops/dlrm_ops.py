"""DLRM operators: fused multi-table embedding lookup and the dot interaction.

On a GPU both run the gfx950 kernels of ``csrc/hip/dlrm.hip`` (``rx_emb_gather`` /
``rx_emb_sgd`` / ``rx_dot_interaction_fwd|bwd``) and fail loudly if the library is missing; on
the CPU they use the equivalent PyTorch expressions (for tests and CPU-only hosts).
"""
import ctypes
import math
from typing import Optional, Sequence

import torch
import torch.nn as nn

from raydp_amd.ops import _hip

_bound = False


def _lib():
    global _bound
    L = _hip.lib()
    if not _bound:
        vp, i, f, ll = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_longlong
        L.rx_emb_gather.argtypes = [vp, vp, vp, vp, vp, i, i, i, i, ll, vp]
        L.rx_emb_sgd.argtypes = [vp, vp, vp, vp, i, i, i, i, f, ll, vp]
        L.rx_emb_gather_rows.argtypes = [vp, vp, vp, vp, i, i, i, ll, vp]
        L.rx_emb_sgd_rows.argtypes = [vp, vp, vp, vp, i, i, i, f, ll, vp]
        L.rx_dot_interaction_fwd.argtypes = [vp, vp, i, i, i, vp]
        L.rx_dot_interaction_bwd.argtypes = [vp, vp, vp, i, i, i, vp]
        L.rx_emb_dot_fwd.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, ll, vp]
        L.rx_dot_bwd_sgd.argtypes = [vp, vp, vp, vp, vp, vp, i, i, i, f, ll, i, vp]
        for n in ("rx_emb_gather", "rx_emb_sgd", "rx_emb_gather_rows", "rx_emb_sgd_rows", "rx_dot_interaction_fwd",
                  "rx_dot_interaction_bwd", "rx_emb_dot_fwd", "rx_dot_bwd_sgd"):
            getattr(L, n).restype = i
        _bound = True
    return L


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def tril_indices(F: int):
    rows = [i for i in range(F) for _ in range(i)]
    cols = [j for i in range(F) for j in range(i)]
    return torch.tensor(rows), torch.tensor(cols)


def dot_interaction_reference(X: torch.Tensor) -> torch.Tensor:
    """[B, F, D] -> [B, D + F(F-1)/2 + 1]: bottom row, strict lower triangle of X X^T, zero pad."""
    B, F, D = X.shape
    Z = torch.bmm(X, X.transpose(1, 2))
    r, c = tril_indices(F)
    flat = Z[:, r.to(X.device), c.to(X.device)]
    return torch.cat([X[:, 0], flat, torch.zeros(B, 1, dtype=X.dtype, device=X.device)], dim=1)


class _DotInteraction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X):
        X = X.contiguous().float()
        B, F, D = X.shape
        out = torch.empty(B, D + F * (F - 1) // 2 + 1, dtype=torch.float32, device=X.device)
        _hip.check(_lib().rx_dot_interaction_fwd(_p(X), _p(out), B, F, D, _hip.stream_ptr(X.device)),
                   "rx_dot_interaction_fwd")
        ctx.save_for_backward(X)
        return out

    @staticmethod
    def backward(ctx, g):
        (X,) = ctx.saved_tensors
        B, F, D = X.shape
        g = g.contiguous().float()
        dX = torch.empty_like(X)
        _hip.check(_lib().rx_dot_interaction_bwd(_p(X), _p(g), _p(dX), B, F, D, _hip.stream_ptr(X.device)),
                   "rx_dot_interaction_bwd")
        return dX


def dot_interaction(X: torch.Tensor) -> torch.Tensor:
    if X.is_cuda:
        if X.shape[1] > 32 or X.shape[2] not in (32, 64, 128):
            raise ValueError("HIP dot interaction supports F <= 32 and D in {32, 64, 128}")
        return _DotInteraction.apply(X)
    return dot_interaction_reference(X)


def gather_rows(weight: torch.Tensor, offsets: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """``[B, T] ids -> [B, T, D]`` rows ``weight[offsets[t] + idx[b, t]]`` (HIP on GPU)."""
    B, T = idx.shape
    D = weight.shape[1]
    if not weight.is_cuda:
        return weight[(idx.long() + offsets.view(1, -1)).reshape(-1)].view(B, T, D)
    idx = idx.contiguous().long()
    out = torch.empty(B, T, D, dtype=weight.dtype, device=weight.device)
    if B * T:
        _hip.check(_lib().rx_emb_gather_rows(_p(weight), _p(offsets), _p(idx), _p(out), B, T, D, weight.shape[0],
                                             _hip.stream_ptr(weight.device)), "rx_emb_gather_rows")
    return out


def sgd_rows_(weight: torch.Tensor, offsets: torch.Tensor, idx: torch.Tensor, grad_rows: torch.Tensor, lr: float):
    """In-place sparse SGD ``weight[offsets[t] + idx[b, t]] -= lr * grad_rows[b, t]``."""
    B, T = idx.shape
    D = weight.shape[1]
    if not weight.is_cuda:
        rows = (idx.long() + offsets.view(1, -1)).reshape(-1)
        weight.data.index_add_(0, rows, grad_rows.reshape(-1, D), alpha=-lr)
        return
    if B * T:
        _hip.check(_lib().rx_emb_sgd_rows(_p(weight), _p(offsets), _p(idx.contiguous().long()),
                                          _p(grad_rows.contiguous()), B, T, D, ctypes.c_float(lr), weight.shape[0],
                                          _hip.stream_ptr(weight.device)), "rx_emb_sgd_rows")


class _EmbedConcat(torch.autograd.Function):
    """X = [mlp_out; W[offs + idx]] ([B, 1 + T, D]); weight gradient sparse (or fused SGD)."""

    @staticmethod
    def forward(ctx, mlp_out, weight, offsets, idx, fused_lr, sync=None):
        B, T = idx.shape
        D = weight.shape[1]
        X = torch.empty(B, T + 1, D, dtype=torch.float32, device=weight.device)
        idx = idx.contiguous().long()
        head = mlp_out.contiguous()
        if head.shape != (B, D) or head.dtype != torch.float32:
            raise ValueError(f"bottom-MLP output must be fp32 [{B}, {D}]")
        # one launch writes the whole interaction input: X[:, 0] = mlp_out, X[:, 1:] = rows
        _hip.check(_lib().rx_emb_gather(_p(weight), _p(offsets), _p(idx), _p(X), _p(head), B, T, D, T + 1,
                                        weight.shape[0], _hip.stream_ptr(weight.device)), "rx_emb_gather")
        ctx.save_for_backward(weight, offsets, idx)
        ctx.fused_lr = fused_lr
        ctx.sync = sync
        return X

    @staticmethod
    def backward(ctx, dX):
        weight, offsets, idx = ctx.saved_tensors[:3]
        return _embed_backward(weight, offsets, idx, dX, ctx.fused_lr, ctx.sync)


def _embed_backward(weight, offsets, idx, dX, fused_lr, sync):
    """Gradients of X = [mlp_out; W[offs + idx]] from dX: (d_mlp, weight grad or None (fused
    SGD applied in place), None x 4)."""
    B, T = idx.shape
    D = weight.shape[1]
    dX = dX.contiguous()
    d_mlp = dX[:, 0]
    if fused_lr is not None:
        ids, rows_dx, n, lr = idx, dX, B, fused_lr
        if sync is not None:
            # replicated tables over W ranks: every rank applies every rank's rows (SGD is
            # linear: the same update as all-reducing the sparse gradient and averaging),
            # gathered over xGMI on the device -- no host round trip, capturable
            comm, W = sync
            ids = torch.empty((W,) + tuple(idx.shape), dtype=idx.dtype, device=idx.device)
            comm.allgather_(idx, ids)
            rows_dx = torch.empty((W,) + tuple(dX.shape), dtype=dX.dtype, device=dX.device)
            comm.allgather_(dX, rows_dx)
            n, lr = W * B, lr / W
        _hip.check(_lib().rx_emb_sgd(_p(weight), _p(offsets), _p(ids), _p(rows_dx), n, T, D, T + 1,
                                     ctypes.c_float(lr), weight.shape[0],
                                     _hip.stream_ptr(weight.device)), "rx_emb_sgd")
        return d_mlp, None, None, None, None, None
    rows = (idx + offsets.view(1, -1)).reshape(-1)
    grad = torch.sparse_coo_tensor(rows.unsqueeze(0), dX[:, 1:].reshape(-1, D), weight.shape)
    return d_mlp, grad, None, None, None, None


class _EmbedDot(torch.autograd.Function):
    """Z = dot_interaction([mlp_out; W[offs + idx]]) for replicated tables: forward ONE launch
    (gather + interaction, ``rx_emb_dot_fwd``); backward ONE launch when the embedding SGD is
    fused and the tables are not synchronised across ranks (``rx_dot_bwd_sgd``: interaction
    backward, bottom-MLP gradient, table rows updated in its epilogue), else the interaction
    backward followed by _EmbedConcat's backward (all-gathered rows / sparse gradient)."""

    @staticmethod
    def forward(ctx, mlp_out, weight, offsets, idx, fused_lr, sync=None, relu_head=False):
        B, T = idx.shape
        D = weight.shape[1]
        F = T + 1
        idx = idx.contiguous().long()
        head = mlp_out.contiguous()
        if head.shape != (B, D) or head.dtype != torch.float32:
            raise ValueError(f"bottom-MLP output must be fp32 [{B}, {D}]")
        X = torch.empty(B, F, D, dtype=torch.float32, device=weight.device)
        Z = torch.empty(B, D + F * (F - 1) // 2 + 1, dtype=torch.float32, device=weight.device)
        _hip.check(_lib().rx_emb_dot_fwd(_p(weight), _p(offsets), _p(idx), _p(head), _p(X), _p(Z), B, F, D,
                                         weight.shape[0], _hip.stream_ptr(weight.device)), "rx_emb_dot_fwd")
        ctx.save_for_backward(weight, offsets, idx, X)
        ctx.fused_lr = fused_lr
        ctx.sync = sync
        ctx.relu_head = bool(relu_head)
        return Z

    @staticmethod
    def backward(ctx, g):
        weight, offsets, idx, X = ctx.saved_tensors
        B, F, D = X.shape
        g = g.contiguous().float()
        stream = _hip.stream_ptr(X.device)
        if ctx.fused_lr is not None and ctx.sync is None:
            d_mlp = torch.empty(B, D, dtype=torch.float32, device=X.device)
            _hip.check(_lib().rx_dot_bwd_sgd(_p(X), _p(g), _p(d_mlp), _p(weight), _p(offsets), _p(idx), B, F, D,
                                             ctypes.c_float(ctx.fused_lr), weight.shape[0], int(ctx.relu_head),
                                             stream), "rx_dot_bwd_sgd")
            if ctx.relu_head:
                # already multiplied by the bottom MLP's output ReLU mask (raydp_amd.ops.linear_ops
                # reads this mark and skips its mask kernel; masking again would change nothing)
                d_mlp._raydp_relu_masked = True
            return d_mlp, None, None, None, None, None, None
        dX = torch.empty_like(X)
        _hip.check(_lib().rx_dot_interaction_bwd(_p(X), _p(g), _p(dX), B, F, D, stream), "rx_dot_interaction_bwd")
        return _embed_backward(weight, offsets, idx, dX, ctx.fused_lr, ctx.sync) + (None,)


class FusedEmbeddings(nn.Module):
    """All categorical tables in one [sum(rows), D] parameter (row offsets per table)."""

    def __init__(self, table_sizes: Sequence[int], dim: int, fused_sgd_lr: Optional[float] = None):
        super().__init__()
        self.table_sizes = [int(s) for s in table_sizes]
        self.dim = dim
        total = sum(self.table_sizes)
        self.weight = nn.Parameter(torch.empty(total, dim))
        self.weight._raydp_sparse_grad = fused_sgd_lr is None   # DDP: reduce as sparse rows
        offs = [0]
        for s in self.table_sizes[:-1]:
            offs.append(offs[-1] + s)
        self.register_buffer("offsets", torch.tensor(offs, dtype=torch.int64))
        self.fused_sgd_lr = fused_sgd_lr
        with torch.no_grad():
            for o, s in zip(offs, self.table_sizes):   # reference init: U(-sqrt(1/n), sqrt(1/n))
                self.weight[o:o + s].uniform_(-math.sqrt(1.0 / s), math.sqrt(1.0 / s))

    def table(self, t: int) -> torch.Tensor:
        o = int(self.offsets[t])
        return self.weight[o:o + self.table_sizes[t]]

    def forward(self, mlp_out: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        if self.weight.is_cuda:
            return _EmbedConcat.apply(mlp_out.float(), self.weight, self.offsets, idx, self.fused_sgd_lr,
                                      getattr(self, "sync", None))
        rows = idx.long() + self.offsets.view(1, -1)
        emb = nn.functional.embedding(rows, self.weight, sparse=True)
        return torch.cat([mlp_out.unsqueeze(1).float(), emb], dim=1)

    def interact(self, mlp_out: torch.Tensor, idx: torch.Tensor, relu_head: bool = False) -> torch.Tensor:
        """``dot_interaction(self(mlp_out, idx))``; on the GPU the lookup and the interaction are
        one kernel each way (``_EmbedDot``). ``relu_head``: mlp_out is a ReLU output (its
        gradient may then leave the interaction backward already masked)."""
        T = len(self.table_sizes)
        if self.weight.is_cuda and T + 1 <= 32 and self.dim in (32, 64, 128):
            return _EmbedDot.apply(mlp_out.float(), self.weight, self.offsets, idx, self.fused_sgd_lr,
                                   getattr(self, "sync", None), relu_head)
        return dot_interaction(self(mlp_out, idx))
