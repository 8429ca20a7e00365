"""Horovod-compatible data-parallel API over ``torch.distributed`` (RCCL over xGMI on MI355X,
gloo on CPU).

The reference's Horovod path (``examples/horovod_nyctaxi.py:133-138``: ``hvd.init``,
``hvd.broadcast_parameters``, ``hvd.broadcast_optimizer_state``,
``hvd.DistributedOptimizer(op=hvd.Average)``, run under ``ray.train.horovod.HorovodTrainer``)
needs Horovod + MPI/Gloo controllers, neither of which exists here. This module provides the
same surface natively: collectives map to ``torch.distributed``; ``DistributedOptimizer``
registers post-accumulate-grad hooks that pack ready gradients into fusion buffers
(``HOROVOD_FUSION_THRESHOLD`` bytes, default 64 MiB -- few, large collectives suit xGMI's
point-to-point links) and all-reduce them asynchronously while backward continues; ``step``
waits, unpacks (averaging for ``op=Average``) and runs the wrapped optimizer.
"""
import contextlib
import os
import threading
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

Average, Sum, Adasum, Min, Max, Product = "Average", "Sum", "Adasum", "Min", "Max", "Product"

_state = {"init": False, "owned": False}
_lock = threading.Lock()


def _pg_ready() -> bool:
    return dist.is_available() and dist.is_initialized()


def init(comm=None, process_sets=None):
    """Join (or create) the process group. Inside a trainer worker the group already exists."""
    with _lock:
        if _state["init"]:
            return
        if not _pg_ready():
            world = int(os.environ.get("WORLD_SIZE", os.environ.get("HOROVOD_SIZE", "1")))
            rank = int(os.environ.get("RANK", os.environ.get("HOROVOD_RANK", "0")))
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if world == 1:
                # a single rank needs no rendezvous: an in-memory store (no port, nothing left
                # in the environment for the next init); the collectives below short-circuit
                dist.init_process_group(backend, store=dist.HashStore(), rank=0, world_size=1)
            else:
                dist.init_process_group(backend, rank=rank, world_size=world)
            _state["owned"] = True
        _state["init"] = True


def shutdown():
    with _lock:
        if _state["owned"] and _pg_ready():
            dist.destroy_process_group()
        _state.update(init=False, owned=False)


def is_initialized() -> bool:
    return _state["init"]


def _check():
    if not _state["init"]:
        raise ValueError("Horovod has not been initialized; use hvd.init().")


def rank() -> int:
    _check()
    return dist.get_rank()


def size() -> int:
    _check()
    return dist.get_world_size()


def local_rank() -> int:
    _check()
    return int(os.environ.get("LOCAL_RANK", dist.get_rank() % max(1, local_size())))


def local_size() -> int:
    _check()
    return int(os.environ.get("LOCAL_WORLD_SIZE", dist.get_world_size()))


def cross_rank() -> int:
    return rank() // max(1, local_size())


def cross_size() -> int:
    return max(1, size() // max(1, local_size()))


def mpi_threads_supported() -> bool:
    return False


def nccl_built() -> bool:
    return torch.cuda.is_available()


def rocm_built() -> bool:
    return getattr(torch.version, "hip", None) is not None


def _reduce_op(op):
    if op == Adasum:
        # Adasum combines gradients by projection (not a sum): returning a sum instead would
        # silently train a different algorithm
        raise NotImplementedError("hvd.Adasum is not implemented; use op=hvd.Average or hvd.Sum")
    return {Average: dist.ReduceOp.SUM, Sum: dist.ReduceOp.SUM,
            Min: dist.ReduceOp.MIN, Max: dist.ReduceOp.MAX, Product: dist.ReduceOp.PRODUCT}[op]


def _resolve_op(average, op):
    if average is not None:
        return Average if average else Sum
    return op or Average


# ---------------------------------------------------------------------------- collectives ----
class _Handle:
    def __init__(self, work, tensor, post=None):
        self.work, self.tensor, self.post = work, tensor, post
        self.done = False

    def wait(self):
        if not self.done:
            if self.work is not None:
                self.work.wait()
            self.work, self.done = None, True
            if self.post is not None:
                self.post(self.tensor)
        return self.tensor


def allreduce_async_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0):
    _check()
    op = _resolve_op(average, op)
    if prescale_factor != 1.0:
        tensor.mul_(prescale_factor)
    # one rank: every reduction is the identity (no communicator is ever built)
    work = dist.all_reduce(tensor, op=_reduce_op(op), async_op=True) if size() > 1 else None
    scale = postscale_factor / size() if op in (Average, Adasum) else postscale_factor

    def post(t):
        if scale != 1.0:
            t.mul_(scale)
    return _Handle(work, tensor, post)


def allreduce_async(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0):
    return allreduce_async_(tensor.clone(), average, name, op, prescale_factor, postscale_factor)


def synchronize(handle):
    return handle.wait()


def poll(handle) -> bool:
    return handle.done or handle.work is None or handle.work.is_completed()


def allreduce_(tensor, average=None, name=None, op=None, prescale_factor=1.0, postscale_factor=1.0):
    return synchronize(allreduce_async_(tensor, average, name, op, prescale_factor, postscale_factor))


def allreduce(tensor, average=None, name=None, compression=None, op=None, prescale_factor=1.0,
              postscale_factor=1.0):
    compression = compression or Compression.none
    t, ctx = compression.compress(tensor.detach().clone())
    out = allreduce_(t, average, name, op, prescale_factor, postscale_factor)
    return compression.decompress(out, ctx)


def grouped_allreduce(tensors, average=None, name=None, op=None):
    return [allreduce(t, average, name, op=op) for t in tensors]


def allgather(tensor, name=None):
    """Concatenate every rank's tensor along dim 0 (first dimensions may differ)."""
    _check()
    if size() == 1:
        return tensor.detach().clone()
    n = torch.tensor([tensor.shape[0]], device=tensor.device)
    sizes = [torch.zeros_like(n) for _ in range(size())]
    dist.all_gather(sizes, n)
    m = int(max(int(s) for s in sizes))
    pad = torch.zeros((m,) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    pad[:tensor.shape[0]] = tensor
    outs = [torch.empty_like(pad) for _ in range(size())]
    dist.all_gather(outs, pad)
    return torch.cat([o[:int(s)] for o, s in zip(outs, sizes)])


def broadcast_(tensor, root_rank, name=None):
    _check()
    if size() > 1:
        dist.broadcast(tensor, root_rank)
    return tensor


def broadcast(tensor, root_rank, name=None):
    return broadcast_(tensor.detach().clone(), root_rank, name)


def broadcast_object(obj, root_rank=0, name=None):
    _check()
    if size() == 1:
        return obj
    box = [obj if rank() == root_rank else None]
    dist.broadcast_object_list(box, src=root_rank)
    return box[0]


def allgather_object(obj, name=None):
    _check()
    if size() == 1:
        return [obj]
    out = [None] * size()
    dist.all_gather_object(out, obj)
    return out


def alltoall(tensor, splits=None, name=None):
    _check()
    w = size()
    if w == 1:
        return tensor.detach().clone()
    if splits is None:
        assert tensor.shape[0] % w == 0
        splits = [tensor.shape[0] // w] * w
    splits = [int(s) for s in (splits.tolist() if torch.is_tensor(splits) else splits)]
    s_t = torch.tensor(splits, device=tensor.device)
    r_t = torch.empty_like(s_t)
    dist.all_to_all_single(r_t, s_t)
    recv = [int(x) for x in r_t.tolist()]
    out = torch.empty((sum(recv),) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    dist.all_to_all_single(out, tensor.contiguous(), output_split_sizes=recv, input_split_sizes=splits)
    return out


def barrier():
    _check()
    if size() > 1:
        dist.barrier()


def join(device=-1):
    barrier()
    return size() - 1


# ------------------------------------------------------------------------ state helpers -----
def broadcast_parameters(params, root_rank: int = 0):
    """Broadcast a ``state_dict`` / ``named_parameters()`` / list of (name, tensor) in place."""
    _check()
    items = params.items() if isinstance(params, dict) else params
    for _, p in sorted(items, key=lambda kv: kv[0]) if isinstance(params, dict) else items:
        if torch.is_tensor(p) and size() > 1:
            t = p.data if isinstance(p, torch.nn.Parameter) else p
            dist.broadcast(t, root_rank)


def broadcast_optimizer_state(optimizer, root_rank: int = 0):
    """Make every rank's optimizer state (hyper-parameters and buffers) equal to ``root_rank``'s."""
    _check()
    if size() == 1:
        return
    opt = getattr(optimizer, "_inner", optimizer)
    sd = opt.state_dict()
    moved = {}
    for k, st in sd["state"].items():
        moved[k] = {n: (v.detach().cpu() if torch.is_tensor(v) else v) for n, v in st.items()}
    sd = {"state": moved, "param_groups": sd["param_groups"]}
    sd = broadcast_object(sd, root_rank)
    opt.load_state_dict(sd)


class _NoneCompressor:
    @staticmethod
    def compress(t):
        return t, None

    @staticmethod
    def decompress(t, ctx):
        return t


class _FP16Compressor:
    @staticmethod
    def compress(t):
        if t.dtype.is_floating_point:
            return t.to(torch.float16), t.dtype
        return t, None

    @staticmethod
    def decompress(t, ctx):
        return t.to(ctx) if ctx is not None else t


class _BF16Compressor(_FP16Compressor):
    @staticmethod
    def compress(t):
        if t.dtype.is_floating_point:
            return t.to(torch.bfloat16), t.dtype
        return t, None


class Compression:
    none = _NoneCompressor
    fp16 = _FP16Compressor
    bf16 = _BF16Compressor


# -------------------------------------------------------------------- DistributedOptimizer --
class _Fusion:
    """Gradient fusion buffers filled as hooks fire (reverse registration order = backward order)."""

    def __init__(self, params: List[torch.nn.Parameter], threshold: int, op, compression, gscale):
        self.op, self.compression, self.gscale = op, compression, gscale
        self._sum = None
        _reduce_op(op)      # unsupported ops fail at wrap time, not mid-step
        if op in (Average, Sum):
            from raydp_amd.ops.comm import BucketAllreduce
            self._sum = BucketAllreduce()   # one-shot xGMI for small fp32 buckets
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, cur_bytes = [], 0
        for p in reversed(params):
            nb = p.numel() * p.element_size()
            if cur and (cur_bytes + nb > threshold or p.dtype != cur[0].dtype or p.device != cur[0].device):
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): b for b, ps in enumerate(self.buckets) for p in ps}
        self.steps = 0
        self.reset()

    def reset(self):
        self.ready = [0] * len(self.buckets)
        self.pending: List[Tuple[int, torch.Tensor, object]] = []

    def mark(self, p):
        b = self.where.get(id(p))
        if b is None:
            return
        self.ready[b] += 1
        if self.ready[b] == len(self.buckets[b]):
            self._launch(b)

    def _launch(self, b):
        ps = self.buckets[b]
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
        flat = torch.cat([g.reshape(-1) for g in grads])
        flat, ctx = self.compression.compress(flat)
        scaled = False
        if self._sum is not None:
            # the average's 1/size rides in the one-shot kernel's sum pass (uncompressed fp32)
            scaled = ctx is None and self._sum.routes_to_xgmi(flat)
            work = self._sum(flat, self.gscale) if scaled else self._sum(flat)
        else:
            work = dist.all_reduce(flat, op=_reduce_op(self.op), async_op=True)
        self.pending.append((b, flat, ctx, work, scaled))

    def finish(self):
        self.steps += 1
        if self._sum is not None and self.steps % 64 == 0:
            # a timed-out xGMI exchange raises instead of drifting silently: the error word comes
            # back by a stream-ordered copy examined 64 steps later (no device sync in the loop)
            self._sum.check_async()
        for b in range(len(self.buckets)):   # buckets never completed (unused params)
            if self.ready[b] != len(self.buckets[b]) and not any(x[0] == b for x in self.pending):
                self._launch(b)
        for b, flat, ctx, work, scaled in self.pending:
            work.wait()
            flat = self.compression.decompress(flat, ctx)
            if self.gscale != 1.0 and not scaled:
                flat.mul_(self.gscale)
            off = 0
            for p in self.buckets[b]:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n
        self.reset()


def _graph_user_module(named_parameters, params):
    """The user's loop hands its module in only as ``model.named_parameters()`` (reference
    ``examples/horovod_nyctaxi.py:133-138``): when that is the module's own generator, its forward
    + backward are replayed from HIP graphs per repeated batch shape (the ``prepare_model`` policy,
    ``raydp_amd/train/gpu_policy.py`` graph_model) -- a tabular MLP step is ~40 tiny kernels each
    way whose launch cost exceeds their run time. Gradients still reach ``.grad`` through autograd
    (the accumulate hooks that start the bucket all-reduce fire as before), so the wrapped step is
    unchanged. Configs ``spark.ray.mi355x.graph_user_model`` and ``graph_hvd_model`` (off by
    default); GPU parameters only."""
    frame = getattr(named_parameters, "gi_frame", None)
    mod = frame.f_locals.get("self") if frame is not None else None
    import torch
    if not isinstance(mod, torch.nn.Module) or not params or not all(p.is_cuda for p in params):
        return None
    from raydp_amd.utils import config as C
    if not (C.get("spark.ray.mi355x.graph_user_model") and C.get("spark.ray.mi355x.graph_hvd_model")):
        return None
    from raydp_amd.train.gpu_policy import graph_model
    return graph_model(mod)


def DistributedOptimizer(optimizer, named_parameters=None, compression=None, backward_passes_per_step: int = 1,
                         op=Average, gradient_predivide_factor: float = 1.0, num_groups: int = 0,
                         groups=None, sparse_as_dense: bool = False, process_set=None):
    """Wrap ``optimizer`` so ``step()`` applies globally reduced gradients (Horovod semantics)."""
    _check()
    compression = compression or Compression.none
    params = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
    _graph_user_module(named_parameters, params)
    if named_parameters is not None:
        names = {id(p): n for n, p in named_parameters}
        missing = [p for p in params if id(p) not in names]
        if missing:
            raise ValueError("named_parameters does not cover every optimizer parameter")
    _reduce_op(op)
    threshold = int(os.environ.get("HOROVOD_FUSION_THRESHOLD", str(64 << 20)))
    world = size()
    gscale = (1.0 / world if op in (Average, Adasum) else 1.0)
    fusion = _Fusion(params, threshold, op, compression, gscale) if world > 1 else None
    counter = {"n": 0}
    base_cls = optimizer.__class__
    from raydp_amd.utils import config as C
    fused = {"on": bool(C.get("spark.ray.mi355x.fused_optimizer"))}

    class _HvdOptimizer(base_cls):
        def __init__(self):
            self.__dict__ = optimizer.__dict__   # share state with the wrapped instance
            self._inner = optimizer
            self._fusion = fusion
            self._skip_sync = False
            self._hooks = []
            if fusion is not None:
                for p in params:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._hook))

        def _hook(self, p):
            if backward_passes_per_step > 1:
                return
            self._fusion.mark(p)

        def synchronize(self):
            if self._fusion is not None:
                if backward_passes_per_step > 1:
                    for p in params:
                        self._fusion.mark(p)
                self._fusion.finish()

        @contextlib.contextmanager
        def skip_synchronize(self):
            self._skip_sync = True
            try:
                yield
            finally:
                self._skip_sync = False

        def step(self, closure=None):
            counter["n"] += 1
            if backward_passes_per_step > 1 and counter["n"] % backward_passes_per_step:
                return None
            if not self._skip_sync:
                self.synchronize()
            if closure is None and fused["on"]:
                # the wrapped Adam / AdamW / SGD on the multi-tensor HIP kernels (one launch per 24
                # tensors; torch's state layout kept): csrc/hip/fused_optim.hip
                from raydp_amd.ops.fused_optim import fused_step
                if fused_step(optimizer):
                    return None
                fused["on"] = False    # not covered (CPU / sparse / amsgrad ...): torch from now on
            return base_cls.step(self, closure)

        def zero_grad(self, set_to_none: bool = True):
            return base_cls.zero_grad(self, set_to_none)

    return _HvdOptimizer()


# -------------------------------------------------------------------------- trainer ---------
def HorovodTrainer(train_loop_per_worker, *, train_loop_config=None, scaling_config=None, run_config=None,
                   datasets=None, horovod_config=None, resume_from_checkpoint=None, **kw):
    """``ray.train.horovod.HorovodTrainer``: our data-parallel trainer (workers already share a
    ``torch.distributed`` group, so ``hvd.init()`` inside the loop simply joins it)."""
    from raydp_amd.train.trainer import DataParallelTrainer

    def loop(config):
        try:
            return train_loop_per_worker(config) if _accepts(train_loop_per_worker) else train_loop_per_worker()
        finally:
            shutdown()
    return DataParallelTrainer(loop, train_loop_config=train_loop_config, scaling_config=scaling_config,
                               run_config=run_config, datasets=datasets,
                               resume_from_checkpoint=resume_from_checkpoint, **kw)


def _accepts(fn) -> bool:
    import inspect
    try:
        return len(inspect.signature(fn).parameters) >= 1
    except (TypeError, ValueError):
        return True


__all__ = ["init", "shutdown", "is_initialized", "rank", "size", "local_rank", "local_size", "cross_rank",
           "cross_size", "allreduce", "allreduce_", "allreduce_async", "allreduce_async_", "synchronize", "poll",
           "grouped_allreduce", "allgather", "broadcast", "broadcast_", "broadcast_object", "allgather_object",
           "alltoall", "barrier", "join", "broadcast_parameters", "broadcast_optimizer_state",
           "DistributedOptimizer", "Compression", "HorovodTrainer", "Average", "Sum", "Adasum", "Min", "Max",
           "Product", "nccl_built", "rocm_built", "mpi_threads_supported"]

_ = (Dict, Iterable, Optional)
