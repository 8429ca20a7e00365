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

Collectives: on GPUs whose ranks map each other's memory (one node, xGMI) the three exchanges are
the one-shot xGMI all-to-all kernel (``XgmiComm.alltoallv_``, csrc/comm/xgmi_allreduce.hip):
stream-ordered and device-sequenced, so a whole model-parallel step can be captured into a HIP
graph; otherwise ``torch.distributed.all_to_all_single`` (RCCL, gloo on CPU). The small id
exchange and the owner gather run first; the row exchange back (16x the id
bytes at D = 32 fp32) is issued ``async_op`` and overlaps the bottom MLP (``start`` / ``finish``,
``Dlrm.forward``); with the fused embedding SGD the reverse gradient exchange overlaps the
bottom MLP's backward (applied at the end of the backward pass). Batch sizes are exchanged only
when they change. Dense parameters (the MLPs) stay data parallel.
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


class _Pending:
    """A lookup in flight (``ShardedEmbeddings.start``): the ids have been exchanged and the
    owners' rows gathered; the all-to-all returning the rows (the step's largest exchange,
    B x T x D values) runs asynchronously while the bottom MLP is computed."""
    __slots__ = ("B", "T", "all_b", "in_splits", "out_splits", "recv", "work", "back", "xg")


class _ShardedLookup(torch.autograd.Function):
    """Forward: id all-to-all, owner-side row gather, and the row all-to-all issued
    ``async_op`` (its handle goes into ``pend.work``; ``finish`` waits -- a stream dependency,
    no host block -- after the bottom MLP has been enqueued). Returns the received rows in
    rank-blocked order."""

    @staticmethod
    def forward(ctx, weight, pend, mod):
        group, world = mod.group, mod.world
        B, T = pend.B, pend.T
        D = weight.shape[1]
        dev = weight.device
        in_splits, out_splits = pend.in_splits, pend.out_splits
        # 2) owner-side gather for every source rank (HIP row gather on the GPU)
        nl = len(mod.local_tables)
        from raydp_amd.ops.dlrm_ops import gather_rows
        lidx = pend.recv.view(-1, nl) if nl else pend.recv.view(0, 0)
        emb = gather_rows(weight, mod.local_offsets, lidx).view(-1, D) if nl else \
            torch.empty(0, D, device=dev, dtype=weight.dtype)
        # 3) embeddings back to the requesting ranks, in flight while the bottom MLP runs
        back = torch.empty(sum(in_splits), D, dtype=weight.dtype, device=dev)
        if pend.xg is not None:
            fo, ln, do = pend.xg["rows"]
            mod._xg.alltoallv_(emb.contiguous(), back, fo, ln, do)
            from raydp_amd.ops.comm import _Done
            pend.work = _Done()
        else:
            pend.work = dist.all_to_all_single(back, emb.contiguous(), output_split_sizes=list(in_splits),
                                               input_split_sizes=list(out_splits), group=group, async_op=True)
        ctx.save_for_backward(lidx, weight)
        ctx.meta = (mod, B, T, D, in_splits, out_splits, weight.shape, pend.xg)
        return back

    @staticmethod
    def backward(ctx, g):
        lidx, weight = ctx.saved_tensors
        mod, B, T, D, in_splits, out_splits, wshape, xg = ctx.meta
        send = g.contiguous()          # already rank-blocked: the reverse of the forward exchange
        recv = torch.empty(sum(out_splits), D, dtype=g.dtype, device=g.device)
        nl = len(mod.local_tables)
        if xg is not None:
            fo, ln, do = xg["grads"]
            mod._xg.alltoallv_(send, recv, fo, ln, do)
            if mod.fused_sgd_lr is not None:
                if nl:
                    from raydp_amd.ops.dlrm_ops import sgd_rows_
                    sgd_rows_(weight, mod.local_offsets, lidx, recv.view(-1, nl, D), mod.fused_sgd_lr)
                return None, None, None
            if not nl:
                return None, None, None
            rows = (lidx + mod.local_offsets.view(1, -1)).reshape(-1)
            return torch.sparse_coo_tensor(rows.unsqueeze(0), recv, wshape), None, None
        if mod.fused_sgd_lr is not None:
            # the reverse exchange runs while autograd continues with the bottom MLP's backward;
            # the rows are applied to the owner's tables at the end of the backward pass
            work = dist.all_to_all_single(recv, send, output_split_sizes=list(out_splits),
                                          input_split_sizes=list(in_splits), group=mod.group, async_op=True)

            def finish():
                work.wait()
                if nl:
                    from raydp_amd.ops.dlrm_ops import sgd_rows_
                    sgd_rows_(weight, mod.local_offsets, lidx, recv.view(-1, nl, D), mod.fused_sgd_lr)
            torch.autograd.Variable._execution_engine.queue_callback(finish)
            return None, None, None
        _a2a(recv, send, out_splits, in_splits, mod.group)
        if not nl:
            return None, None, None
        rows = (lidx + mod.local_offsets.view(1, -1)).reshape(-1)
        return torch.sparse_coo_tensor(rows.unsqueeze(0), recv, wshape), None, None


class ShardedEmbeddings(nn.Module):
    """Drop-in for :class:`raydp_amd.ops.dlrm_ops.FusedEmbeddings` across a process group."""

    def __init__(self, table_sizes: Sequence[int], dim: int, group=None, owners: Optional[List[int]] = None,
                 seed: int = 0, fused_sgd_lr: Optional[float] = None, static_batch="auto"):
        super().__init__()
        self.fused_sgd_lr = fused_sgd_lr   # apply SGD to the local tables inside backward
        # how ranks learn each other's batch size: True -> always equal to the local one (no
        # exchange); False -> all_gather every step (host sync); "auto" -> all_gather only when
        # the local batch size changes (ranks change sizes at the same steps: the trainer's
        # equal shards guarantee it), so a steady epoch exchanges nothing
        self.static_batch = static_batch
        self._last_b, self._all_b = None, None
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
        self._xg, self._xg_tried, self._xg_plans = None, False, {}
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

    def _batch_sizes(self, B: int, dev) -> List[int]:
        if self.static_batch is True or self.world == 1:
            return [B] * self.world
        if self.static_batch == "auto" and self._last_b == B and self._all_b is not None:
            return self._all_b
        bs = torch.tensor([B], device=dev)
        all_b = [torch.zeros_like(bs) for _ in range(self.world)]
        dist.all_gather(all_b, bs, group=self.group)
        self._all_b = [int(x) for x in torch.cat(all_b).cpu()]
        self._last_b = B
        return self._all_b

    def _xgmi(self, dev):
        """The one-shot xGMI communicator of this group (shared with the DDP buckets), created
        collectively on the first GPU lookup; None keeps torch.distributed."""
        if not self._xg_tried:
            self._xg_tried = True
            if dev.type == "cuda" and self.world > 1:
                from raydp_amd.ops.comm import XG_BUCKET_MAX_BYTES, XgmiComm
                from raydp_amd.utils.config import get as conf_get
                if conf_get("spark.ray.mi355x.allreduce") != "rccl":
                    self._xg = XgmiComm.create(XG_BUCKET_MAX_BYTES // 4, group=self.group,
                                               timeout_s=conf_get("spark.ray.mi355x.allreduce.timeout_s"))
        return self._xg

    def _xg_plan(self, all_b, D: int):
        """Word offsets of the three exchanges for batch sizes ``all_b`` (rank order):
        ids (int64, 2 words), rows back and row gradients (fp32, D words)."""
        key = (tuple(all_b), D)
        plan = self._xg_plans.get(key)
        if plan is not None:
            return plan
        W, me = self.world, self.rank
        nt = [len(self.tables_of[r]) for r in range(W)]
        cum = [sum(nt[:r]) for r in range(W)]
        nl = nt[me]
        Bme = all_b[me]

        def prefix(v):
            return [sum(v[:p]) for p in range(len(v))]
        # forward ids: rank p's send buffer is [q][B_p][nt[q]]; mine starts at B_p * cum[me]
        ids_len = [all_b[p] * nl for p in range(W)]
        ids = ([2 * all_b[p] * cum[me] for p in range(W)], [2 * n for n in ids_len], [2 * o for o in prefix(ids_len)])
        # rows back: owner p's buffer is [q][B_q][nt[p]] rows; mine at sum_{q<me} B_q * nt[p]
        rows_len = [Bme * nt[p] for p in range(W)]
        rows = ([D * sum(all_b[q] for q in range(me)) * nt[p] for p in range(W)], [D * n for n in rows_len],
                [D * o for o in prefix(rows_len)])
        # gradients: rank q's buffer is [owner p][B_q][nt[p]] rows; mine (owner) at B_q * cum[me]
        g_len = [all_b[q] * nl for q in range(W)]
        grads = ([D * all_b[q] * cum[me] for q in range(W)], [D * n for n in g_len], [D * o for o in prefix(g_len)])
        plan = {"ids": ids, "rows": rows, "grads": grads}
        self._xg_plans[key] = plan
        return plan

    def start(self, idx: torch.Tensor) -> _Pending:
        """Exchange the ids, gather the owned rows and put the row all-to-all in flight; the
        caller computes the bottom MLP next and ``finish`` completes the lookup."""
        idx = idx.long()
        B, T = idx.shape
        p = _Pending()
        p.B, p.T = B, T
        p.all_b = self._batch_sizes(B, idx.device)
        # [owner q][b][q's tables] through one cached device gather (capturable: no host index)
        send = idx.reshape(-1).index_select(0, self._send_order(B, T, idx.device)) if T else idx.reshape(-1)
        p.in_splits = [B * len(self.tables_of[r]) for r in range(self.world)]
        p.out_splits = [p.all_b[r] * len(self.local_tables) for r in range(self.world)]
        p.recv = torch.empty(sum(p.out_splits), dtype=idx.dtype, device=idx.device)
        p.xg = None
        xg = self._xgmi(idx.device)
        if xg is not None and T:
            plan = self._xg_plan(p.all_b, self.dim)
            most = max(2 * send.numel(), self.dim * max(sum(p.out_splits), sum(p.in_splits)))
            if most <= xg.max_floats:
                p.xg = plan
        if p.xg is not None:
            fo, ln, do = p.xg["ids"]
            self._xg.alltoallv_(send.contiguous(), p.recv, fo, ln, do)     # ids (8 B per lookup)
        else:
            _a2a(p.recv, send, p.out_splits, p.in_splits, self.group)
        p.back = _ShardedLookup.apply(self.weight, p, self)             # rows: async
        return p

    def finish(self, pend: _Pending, mlp_out: torch.Tensor) -> torch.Tensor:
        pend.work.wait()     # the compute stream waits for the rows (no host synchronisation)
        B, T, D = pend.B, pend.T, self.dim
        # rank-blocked rows -> [B, T, D] in table order (one gather through a cached index)
        perm = self._row_order(B, T, mlp_out.device)
        emb = pend.back.index_select(0, perm).view(B, T, D) if T else pend.back.view(B, 0, D)
        return torch.cat([mlp_out.unsqueeze(1).to(emb.dtype), emb], dim=1)

    def _send_order(self, B: int, T: int, dev) -> torch.Tensor:
        """Flat index of the local [B, T] ids in send order: for every owner q, the batch's
        ids of q's tables, row major."""
        key = (B, T, str(dev))
        cached = getattr(self, "_send_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        cols = [torch.tensor(self.tables_of[r], dtype=torch.long) for r in range(self.world)]
        order = torch.cat([(torch.arange(B).view(B, 1) * T + c.view(1, -1)).reshape(-1) for c in cols])
        order = order.to(dev)
        self._send_cache = (key, order)
        return order

    def _row_order(self, B: int, T: int, dev) -> torch.Tensor:
        """Index that maps the received rank-blocked rows ([rank][b][its tables]) to
        [b][table] order."""
        key = (B, T, str(dev))
        cached = getattr(self, "_order_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        pos = torch.empty(B, T, dtype=torch.long)
        off = 0
        for r in range(self.world):
            ts = self.tables_of[r]
            n = len(ts)
            if n:
                pos[:, ts] = off + torch.arange(B * n).view(B, n)
            off += B * n
        perm = pos.reshape(-1).to(dev)
        self._order_cache = (key, perm)
        return perm

    def forward(self, mlp_out: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
        return self.finish(self.start(idx), mlp_out)
