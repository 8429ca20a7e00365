"""Table-wise model-parallel embeddings over all-to-all (the DLRM "EP" layout).

The reference replicates every DLRM embedding table in every worker and all-reduces the dense
gradients under DDP (examples/pytorch_dlrm.ipynb cell 14 -> TorchEstimator). With 288 GB of
HBM per MI355X that still fits small Criteo-style tables, but the embedding all-reduce is the
largest collective of the step. Here each table lives on exactly one rank (greedy by size),
and one training step moves only the looked-up rows:

  forward   1. all-to-all the local batch's category ids to the owners of their tables
            2. each owner gathers rows of its tables for every rank's batch
            3. all-to-all the embeddings back -> X[b] = [bottom_mlp(b); emb_0(b); ...]
  backward  the embedding gradient rows travel back over the reverse all-to-all and become a
            sparse gradient of the owner's local table (SGD applies it without densifying).

Collectives are ``torch.distributed.all_to_all_single`` (RCCL over xGMI on MI355X, gloo on
CPU). Dense parameters (the MLPs) stay data parallel.
"""
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn


def place_tables(table_sizes: Sequence[int], world: int) -> List[int]:
    """Greedy size-balanced table -> rank assignment (largest tables first)."""
    load = [0] * world
    owner = [0] * len(table_sizes)
    for t in sorted(range(len(table_sizes)), key=lambda t: -table_sizes[t]):
        r = min(range(world), key=lambda r: (load[r], r))
        owner[t] = r
        load[r] += table_sizes[t]
    return owner


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group):
    dist.all_to_all_single(out, inp.contiguous(), output_split_sizes=out_splits, input_split_sizes=in_splits,
                           group=group)
    return out


class _ShardedLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, idx, mod):
        group, world = mod.group, mod.world
        B, T = idx.shape
        D = weight.shape[1]
        dev = weight.device
        # batch sizes of every rank (ranks may hold different local batch sizes, unless the
        # module was built with static_batch: then every rank's B equals this one's)
        if mod.static_batch:
            all_b = [B] * world
        else:
            bs = torch.tensor([B], device=dev)
            all_b = [torch.zeros_like(bs) for _ in range(world)]
            dist.all_gather(all_b, bs, group=group)
            all_b = [int(x) for x in all_b]
        # 1) ids to owners: for each destination r, my rows' ids of tables r owns ([B, n_r])
        send = torch.cat([idx[:, mod.tables_of[r]].reshape(-1) for r in range(world)]) if T else idx.reshape(-1)
        in_splits = [B * len(mod.tables_of[r]) for r in range(world)]
        out_splits = [all_b[r] * len(mod.local_tables) for r in range(world)]
        recv = torch.empty(sum(out_splits), dtype=idx.dtype, device=dev)
        _a2a(recv, send, out_splits, in_splits, group)
        # 2) owner-side gather for every source rank (HIP row gather on the GPU)
        nl = len(mod.local_tables)
        from raydp_amd.ops.dlrm_ops import gather_rows
        lidx = recv.view(-1, nl) if nl else recv.view(0, 0)
        emb = gather_rows(weight, mod.local_offsets, lidx).view(-1, D) if nl else \
            torch.empty(0, D, device=dev, dtype=weight.dtype)
        # 3) embeddings back to the requesting ranks
        back = torch.empty(sum(in_splits), D, dtype=weight.dtype, device=dev)
        _a2a(back, emb, [s for s in in_splits], [s for s in out_splits], group)
        out = torch.empty(B, T, D, dtype=weight.dtype, device=dev)
        off = 0
        for r in range(world):
            n = len(mod.tables_of[r])
            if n:
                out[:, mod.tables_of[r]] = back[off:off + B * n].view(B, n, D)
            off += B * n
        ctx.save_for_backward(lidx, weight)
        ctx.meta = (mod, B, T, D, in_splits, out_splits, weight.shape)
        return out

    @staticmethod
    def backward(ctx, g):
        lidx, weight = ctx.saved_tensors
        mod, B, T, D, in_splits, out_splits, wshape = ctx.meta
        send = torch.cat([g[:, mod.tables_of[r]].reshape(-1, D) for r in range(mod.world)]) if T else g.reshape(-1, D)
        recv = torch.empty(sum(out_splits), D, dtype=g.dtype, device=g.device)
        _a2a(recv, send, out_splits, in_splits, mod.group)
        nl = len(mod.local_tables)
        if not nl:
            return None, None, None
        if mod.fused_sgd_lr is not None:
            # apply the rows straight into the owner's tables (no sparse tensor, no optimizer pass)
            from raydp_amd.ops.dlrm_ops import sgd_rows_
            sgd_rows_(weight, mod.local_offsets, lidx, recv.view(-1, nl, D), mod.fused_sgd_lr)
            return None, None, None
        rows = (lidx + mod.local_offsets.view(1, -1)).reshape(-1)
        return torch.sparse_coo_tensor(rows.unsqueeze(0), recv, wshape), None, None


class ShardedEmbeddings(nn.Module):
    """Drop-in for :class:`raydp_amd.ops.dlrm_ops.FusedEmbeddings` across a process group."""

    def __init__(self, table_sizes: Sequence[int], dim: int, group=None, owners: Optional[List[int]] = None,
                 seed: int = 0, fused_sgd_lr: Optional[float] = None, static_batch: bool = False):
        super().__init__()
        self.fused_sgd_lr = fused_sgd_lr   # apply SGD to the local tables inside backward
        self.static_batch = static_batch   # every rank always uses the same local batch size
        import math
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.table_sizes = [int(s) for s in table_sizes]
        self.dim = dim
        self.owner = owners or place_tables(self.table_sizes, self.world)
        self.tables_of = [[t for t, o in enumerate(self.owner) if o == r] for r in range(self.world)]
        self.local_tables = self.tables_of[self.rank]
        local_sizes = [self.table_sizes[t] for t in self.local_tables]
        offs = [0]
        for s in local_sizes[:-1]:
            offs.append(offs[-1] + s)
        self.register_buffer("local_offsets", torch.tensor(offs[:len(local_sizes)], dtype=torch.int64))
        self.weight = nn.Parameter(torch.empty(max(1, sum(local_sizes)), dim))
        self.weight._raydp_model_parallel = True   # owned by this rank only: DDP leaves it alone
        # with fused_sgd_lr the weight still requires grad (so backward runs the reverse
        # all-to-all) but its .grad stays None: optimizers skip it
        self._raydp_model_parallel = True          # ... and every buffer of this module (offsets)
        with torch.no_grad():
            for t, o in zip(self.local_tables, offs):
                s = self.table_sizes[t]
                # per-table generator -> identical values to a replicated init with the same seed
                gt = torch.Generator().manual_seed(seed * 1000003 + t)
                self.weight[o:o + s] = (torch.rand(s, dim, generator=gt) * 2 - 1) * math.sqrt(1.0 / s)

    def table(self, t: int) -> torch.Tensor:
        i = self.local_tables.index(t)
        o = int(self.local_offsets[i])
        return self.weight[o:o + self.table_sizes[t]]

    def forward(self, mlp_out: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        emb = _ShardedLookup.apply(self.weight, idx.long(), self)
        return torch.cat([mlp_out.unsqueeze(1).to(emb.dtype), emb], dim=1)
