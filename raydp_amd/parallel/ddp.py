"""Data-parallel wrapper with bucketed, backward-overlapped gradient all-reduce.

Replaces the DDP that Ray Train's ``prepare_model`` applies in the reference
(``python/raydp/torch/estimator.py:243``; collectives K1-K3 of SURVEY §2.11). Design for
MI355X over RCCL/xGMI:

* gradients LIVE in flat buckets: every dense parameter's ``.grad`` is a view of its bucket
  (reverse parameter order = the order backward produces them), so autograd accumulates
  straight into the buffer that is all-reduced -- no per-step copy in, no copy back out. A
  bucket's all-reduce is launched the moment its last gradient is accumulated, so
  communication overlaps the rest of backward;
* fp32 buckets up to ``spark.ray.mi355x.allreduce.oneshot_max_mb`` (16 MiB) ride the xGMI
  kernels (one-shot below ``twoshot_min_mb``, all-pairs two-shot above it at world > 2) with the
  1/world average folded into the sum pass, on a dedicated comm stream (``ddp.comm_stream``,
  ``auto``: when every rank has a GPU of its own): the reduction of a finished bucket runs
  beside the rest of backward and the compute stream joins it at the end of backward; larger
  buckets go to RCCL. Ranks that share a GPU keep the buckets stream-ordered: there the early
  comm kernel spins for its peer on the CUs that peer's backward needs (5-8x slower steps,
  profiles/r4_ddp_bucket_sweep.txt);
* bucket sizes follow whether a reduction can overlap backward (:func:`bucket_caps`): with
  the comm stream (or RCCL's asynchronous collectives) on GPUs of their own, a 1 MiB first
  bucket and 4 MiB after it -- DLRM's 8.7 MB of dense gradients become 3 buckets, 2 of them
  reduced while backward still runs (torch DDP likewise starts with a small first bucket);
  stream-ordered (ranks sharing a GPU: nothing overlaps) 32 MiB, which the one-GPU sweep
  measured fastest (1 / 2 / 4 / 8 / 32 MiB, 2 and 4 ranks, profiles/r4_ddp_bucket_sweep.txt).
  The overlap itself is unmeasured until an 8-GPU run. Tiny models (NYC_Model:
  194 KB) end up in one bucket = one collective per step;
* parameters are broadcast from rank 0 at wrap time (one collective per bucket); replicated
  floating-point buffers (BatchNorm running statistics) are re-pointed into one flat tensor
  and re-broadcast before each forward with ONE collective (torch's ``broadcast_buffers``);
* with every bucket and the buffer broadcast on the one-shot kernel (device-sequenced, no
  host bookkeeping) the whole step can be captured into a HIP graph (``capturable()``;
  ``raydp_amd/torch/graphs.py``).

``zero_grad()`` zeroes the buckets in place (one fill per bucket) and keeps the views; an
optimizer's ``zero_grad(set_to_none=True)`` is tolerated (the hook copies the fresh gradient
into the bucket and re-points ``.grad``).
"""
from typing import List

import torch
import torch.distributed as dist
import torch.nn as nn


class _Bucket:
    def __init__(self, params: List[nn.Parameter]):
        self.params = params
        self.numel = sum(p.numel() for p in params)
        p0 = params[0]
        self.flat = torch.zeros(self.numel, dtype=p0.dtype, device=p0.device)
        self.pending = len(params)
        self.work = None
        self.offsets = []
        self.views = []
        off = 0
        for p in params:
            self.offsets.append(off)
            self.views.append(self.flat[off:off + p.numel()].view_as(p))
            off += p.numel()

    def reset(self):
        self.pending = len(self.params)
        self.work = None


def bucket_caps(bucket_cap_mb=None, overlaps: bool = True) -> List[int]:
    """Byte caps of the buckets in gradient-production order (the last entry repeats).

    An explicit ``bucket_cap_mb`` (or ``spark.ray.mi355x.ddp.bucket_mb`` > 0) is one uniform
    cap. Auto (0): when the reductions overlap backward, a small first bucket
    (``ddp.first_bucket_mb``) and ``ddp.overlap_bucket_mb`` after it, so the reduction of every
    bucket but the last runs beside the rest of backward; when they cannot overlap (stream-ordered
    xGMI kernels on a GPU shared by ranks) few large buckets: 32 MiB."""
    from raydp_amd.utils.config import get as conf_get
    mb = float(bucket_cap_mb or conf_get("spark.ray.mi355x.ddp.bucket_mb") or 0.0)
    if mb > 0:
        return [int(mb * (1 << 20))]
    if not overlaps:
        return [32 << 20]
    return [int(float(conf_get("spark.ray.mi355x.ddp.first_bucket_mb")) * (1 << 20)),
            int(float(conf_get("spark.ray.mi355x.ddp.overlap_bucket_mb")) * (1 << 20))]


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, bucket_cap_mb: float = None, broadcast_buffers: bool = True,
                 process_group=None):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.broadcast_buffers = broadcast_buffers
        from raydp_amd.utils.config import get as conf_get
        from raydp_amd.ops.comm import BucketAllreduce
        self._allreduce = BucketAllreduce(process_group)
        self.bucket_caps = bucket_caps(bucket_cap_mb, self._allreduce.overlaps)
        sparse_ids = set()
        for m in module.modules():
            if isinstance(m, (nn.Embedding, nn.EmbeddingBag)) and m.sparse:
                sparse_ids.add(id(m.weight))
        params, self.sparse_params = [], []
        for p in module.parameters():
            if not p.requires_grad or getattr(p, "_raydp_model_parallel", False) \
                    or getattr(p, "_raydp_grad_synced", False):
                # sharded tables (raydp_amd.parallel.embedding_mp) are not replicated; replicated
                # tables whose module synchronises its own updates (FusedEmbeddings.sync) are
                # broadcast at wrap time but never bucketed
                continue
            if id(p) in sparse_ids or getattr(p, "_raydp_sparse_grad", False):
                self.sparse_params.append(p)
            else:
                params.append(p)
        # rank-local state: tensors flagged model parallel, and everything of a module flagged so
        # (a buffer's flag would not survive .to(device), the module's does)
        local_ids = set()
        for m in module.modules():
            if getattr(m, "_raydp_model_parallel", False):
                local_ids.update(id(t) for t in list(m.parameters()) + list(m.buffers()))
        self._local_ids = local_ids
        # reverse order ~= gradient production order
        self.buckets: List[_Bucket] = []
        cur, size = [], 0
        for p in reversed(params):
            nbytes = p.numel() * p.element_size()
            cap = self.bucket_caps[min(len(self.buckets), len(self.bucket_caps) - 1)]
            if cur and (size + nbytes > cap or p.dtype != cur[0].dtype):
                self.buckets.append(_Bucket(cur))
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(_Bucket(cur))
        self._broadcast_state(params)
        self._where = {}
        for bi, b in enumerate(self.buckets):
            for pi, p in enumerate(b.params):
                self._where[p] = (bi, pi)
                p.grad = b.views[pi]          # gradient-as-bucket-view (zeros)
                p.register_post_accumulate_grad_hook(self._make_hook(p))
        for p in self.sparse_params:
            p.register_post_accumulate_grad_hook(self._sparse_hook)
        self._finalize_queued = False
        self.require_backward_grad_sync = True
        # (kind, bucket) in launch order, with ("backward_end", -1) when autograd's end-of-backward
        # callback runs: set to a list to record (tests/test_ddp_buckets.py)
        self.launch_log = None
        # sharded embedding tables (raydp_amd.parallel.embedding_mp) set up their xGMI exchange
        # here, at a point every rank reaches together, so capturable() can count on it
        self._sharded = [m for m in module.modules() if hasattr(m, "_xg_plan")]
        for m in self._sharded:
            ps = list(m.parameters())
            if ps:
                m._xgmi(ps[0].device)

    # ------------------------------------------------------------------ wrap-time state
    def _replicated(self, t) -> bool:
        return not (getattr(t, "_raydp_model_parallel", False) or id(t) in self._local_ids)

    @torch.no_grad()
    def _broadcast_state(self, params):
        """Rank 0's parameters and buffers everywhere (one collective per bucket of params, one
        per buffer dtype). Floating-point replicated buffers are re-pointed into one flat
        tensor per dtype so the per-forward broadcast is one collective."""
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        groups = {}
        for p in params + [p for p in self.module.parameters() if p not in set(params)]:
            if self._replicated(p):
                groups.setdefault((p.dtype, p.device), []).append(p.data)
        for ts in groups.values():
            flat = _flatten_dense_tensors(ts)
            dist.broadcast(flat, 0, group=self.pg)
            for t, v in zip(ts, _unflatten_dense_tensors(flat, ts)):
                t.copy_(v)
        self._buf_flats = []     # (flat, [(module, name)]) per floating dtype
        bufs = {}
        for m in self.module.modules():
            if getattr(m, "_raydp_model_parallel", False):
                continue
            for name, t in m._buffers.items():
                if t is None or not self._replicated(t):
                    continue
                bufs.setdefault((t.dtype, t.device), []).append((m, name, t))
        for (dtype, dev), ents in bufs.items():
            ts = [t for _, _, t in ents]
            flat = _flatten_dense_tensors(ts)
            dist.broadcast(flat, 0, group=self.pg)
            if dtype.is_floating_point:
                off = 0
                for m, name, t in ents:
                    m._buffers[name] = flat[off:off + t.numel()].view_as(t)
                    off += t.numel()
                self._buf_flats.append(flat)
            else:   # integer counters (num_batches_tracked) agree by construction after this
                for (m, name, t), v in zip(ents, _unflatten_dense_tensors(flat, ts)):
                    t.copy_(v)

    # ------------------------------------------------------------------ hooks
    def _sparse_hook(self, param):
        if self.require_backward_grad_sync and not self._finalize_queued:
            self._finalize_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)

    def _reduce_sparse(self, p):
        """Sum a sparse (embedding-row) gradient over ranks without densifying it."""
        g = p.grad
        if g is None:
            g = torch.sparse_coo_tensor(torch.zeros(1, 0, dtype=torch.long, device=p.device),
                                        torch.zeros(0, *p.shape[1:], dtype=p.dtype, device=p.device), p.shape)
        g = g.coalesce()
        idx, val = g.indices(), g.values()
        n = torch.tensor([idx.shape[1]], device=p.device)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n, group=self.pg)
        m = int(max(int(x) for x in ns))
        pi = torch.zeros(idx.shape[0], m, dtype=idx.dtype, device=p.device)
        pv = torch.zeros((m,) + tuple(val.shape[1:]), dtype=val.dtype, device=p.device)
        pi[:, :idx.shape[1]] = idx
        pv[:val.shape[0]] = val
        gi = [torch.empty_like(pi) for _ in range(self.world)]
        gv = [torch.empty_like(pv) for _ in range(self.world)]
        dist.all_gather(gi, pi, group=self.pg)
        dist.all_gather(gv, pv, group=self.pg)
        ai = torch.cat([x[:, :int(k)] for x, k in zip(gi, ns)], dim=1)
        av = torch.cat([x[:int(k)] for x, k in zip(gv, ns)], dim=0) / self.world
        p.grad = torch.sparse_coo_tensor(ai, av, p.shape).coalesce()

    def _make_hook(self, p):
        def hook(param):
            if not self.require_backward_grad_sync:
                return
            bi, pi = self._where[param]
            b = self.buckets[bi]
            view = b.views[pi]
            if param.grad is not view:
                # a fresh gradient tensor (the optimizer set .grad to None): move it into the
                # bucket and re-point .grad, so the next steps accumulate in place
                view.copy_(param.grad)
                param.grad = view
            b.pending -= 1
            if not self._finalize_queued:
                self._finalize_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
            if b.pending == 0:
                b.work = self._allreduce(b.flat, 1.0 / self.world)
                if self.launch_log is not None:
                    self.launch_log.append(("bucket", bi))
        return hook

    def _finalize(self):
        self._finalize_queued = False
        if self.launch_log is not None:
            self.launch_log.append(("backward_end", -1))
        for p in self.sparse_params:
            self._reduce_sparse(p)
        for b in self.buckets:
            if b.pending != 0:
                # parameters unused in this forward: reduce the zeros they contributed
                for pi, p in enumerate(b.params):
                    if p.grad is None:
                        b.views[pi].zero_()
                        p.grad = b.views[pi]
                b.work = self._allreduce(b.flat, 1.0 / self.world)
            b.work.wait()
            b.reset()

    # ------------------------------------------------------------------ API
    def zero_grad(self, set_to_none: bool = False):
        """Zero every bucket in place (one fill per bucket); ``.grad`` stays a bucket view."""
        for b in self.buckets:
            b.flat.zero_()
            for pi, p in enumerate(b.params):
                if p.grad is not b.views[pi]:
                    p.grad = b.views[pi]
        for p in self.sparse_params:
            p.grad = None

    def check_comm(self):
        """Raise ``CollectiveError`` if any xGMI exchange of this model (gradient buckets,
        sharded-table all-to-alls, replicated-table row gathers) timed out: a timed-out exchange
        leaves the communicator's error word set and every later launch skips its exchange, so
        replicas would drift apart silently. One small D2H read per communicator: call it at a
        point that syncs anyway (the trainer does at every epoch end)."""
        self._allreduce.check()
        seen = set()
        for m in self.module.modules():
            for xg in (getattr(m, "_xg", None), (getattr(m, "sync", None) or (None,))[0]):
                if xg is not None and hasattr(xg, "check") and id(xg) not in seen:
                    seen.add(id(xg))
                    xg.check()

    def capturable(self) -> bool:
        """True when one training step issues no host-synchronising collective: every
        gradient bucket and the buffer broadcast ride the one-shot xGMI kernel and no
        parameter has sparse gradients."""
        if self.sparse_params:
            return False
        if any(m._xg is None for m in self._sharded):
            return False        # a sharded table exchanges over torch.distributed
        if not all(self._allreduce.routes_to_xgmi(b.flat) for b in self.buckets):
            return False
        if self.broadcast_buffers and not all(self._allreduce.routes_to_xgmi(f) for f in self._buf_flats):
            return False
        return True

    def forward(self, *args, **kw):
        if self.broadcast_buffers and self.world > 1 and self._buf_flats:
            with torch.no_grad():
                for flat in self._buf_flats:
                    if self._allreduce.routes_to_xgmi(flat):
                        # broadcast as a one-shot sum where every rank but 0 adds zeros (exact)
                        if self.rank != 0:
                            flat.zero_()
                        self._allreduce(flat).wait()
                    else:
                        dist.broadcast(flat, 0, group=self.pg)
        return self.module(*args, **kw)

    def state_dict(self, *a, **kw):
        return self.module.state_dict(*a, **kw)

    def load_state_dict(self, *a, **kw):
        return self.module.load_state_dict(*a, **kw)
