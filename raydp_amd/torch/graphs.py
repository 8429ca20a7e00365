"""HIP-graph training loop for ``TorchLoopEngine`` (models the fused MLP kernel does not cover).

Small tabular models (the stroke tutorial's NET_Model, DLRM's MLPs) are launch bound on
MI355X: one eager step is ~60-150 tiny kernels whose launch cost dwarfs their run time. The
reference runs every step eagerly through ``DistributedDataParallel`` on CPU workers
(``python/raydp/torch/estimator.py:280-320``). Here, on a single GPU, the WHOLE step -- the
device-side batch gather from the resident shard, forward, loss, metric accumulation,
backward and optimizer update -- is captured once into a ``torch.cuda.CUDAGraph`` (a HIP graph
on ROCm) and replayed per batch. Several consecutive steps are captured into one graph
(``chunk`` steps reading a window of the epoch permutation) so a replay covers ``chunk``
batches with one launch plus one window copy.

Rules that keep it exact:
* the first two steps of the first epoch run eagerly on a side stream (lazy optimizer state,
  library workspaces), as graph capture requires;
* Adam/AdamW switch to ``capturable=True`` (device-side step counters); with an LR scheduler
  the learning rate becomes a device tensor that the scheduler ``fill_``s, and chunk = 1 so every
  step sees its own LR;
* metric state is zeroed in place between epochs (``TorchMetric.zero_``) so the captured
  accumulation keeps pointing at live storage;
* list indices in user models (``x[:, [1, 7, 8]]`` as in the reference tutorial's NET_Model) are
  an H2D copy of a pageable host list -- illegal inside capture. ``_CaptureSafeIndexing`` turns
  every integer-list index into a device tensor created during the eager warm-up and reused by
  the captured graph (identical advanced-indexing semantics);
* the last partial batch runs eagerly;
* any capture failure (an op that synchronises, sparse gradients, ...) disables graphs for the
  engine and the same batch is re-run eagerly -- results never depend on whether capture worked.
"""
import gc
import os
import traceback
from typing import Optional

import torch
from torch.overrides import TorchFunctionMode


_ADAM_LIKE = (torch.optim.Adam, torch.optim.AdamW)
_SAFE_OPT = _ADAM_LIKE + (torch.optim.SGD,)


def graphs_requested() -> bool:
    from raydp_amd.utils.config import get as conf_get
    return bool(conf_get("spark.ray.mi355x.hip_graphs"))


def supported(engine) -> Optional[str]:
    """None if the engine's step can be captured, else the reason it cannot."""
    if engine.device.type != "cuda":
        return "not on a GPU"
    if engine.world != 1:
        cap = getattr(engine.model, "capturable", None)
        if cap is None or not cap():
            return "world_size > 1 with a collective that is not capturable (RCCL bucket, sparse gradients)"
    if not engine.metrics.graph_safe():
        return "non built-in metric"
    if type(engine.optimizer) not in _SAFE_OPT:
        return f"optimizer {type(engine.optimizer).__name__} not known to be capture safe"
    if engine.scheduler is not None and type(engine.optimizer) not in _ADAM_LIKE:
        return "LR scheduler with a non-Adam optimizer"
    if any(p.is_sparse for p in engine.raw_model.parameters()):
        return "sparse parameters"
    return None


class _CaptureSafeIndexing(TorchFunctionMode):
    """Replace integer-list indices of ``Tensor.__getitem__`` by cached device index tensors."""

    def __init__(self, cache: dict):
        super().__init__()
        self.cache = cache

    def _conv(self, idx, dev):
        if type(idx) is list and idx and all(type(i) is int for i in idx):
            key = (tuple(idx), str(dev))
            v = self.cache.get(key)
            if v is None:   # first seen in the eager warm-up (outside capture)
                v = self.cache[key] = torch.tensor(idx, dtype=torch.long, device=dev)
            return v
        if type(idx) is tuple:
            parts = tuple(self._conv(i, dev) for i in idx)
            return parts if any(p is not q for p, q in zip(parts, idx)) else idx
        return idx

    def __torch_function__(self, func, types, args=(), kwargs=None):
        if func is torch.Tensor.__getitem__ and len(args) == 2 and isinstance(args[0], torch.Tensor):
            args = (args[0], self._conv(args[1], args[0].device))
        return func(*args, **(kwargs or {}))


class GraphedTrainLoop:
    def __init__(self, engine, chunk: Optional[int] = None):
        self.e = engine
        self.chunk = 1 if engine.scheduler is not None else int(chunk or os.environ.get("RAYDP_TORCH_GRAPH_CHUNK", 8))
        self.graphs = {}           # steps -> (CUDAGraph, window)
        self.pool = None
        self.warm = 0
        self.failed = None
        self.index_cache = {}
        self.total = torch.zeros((), dtype=torch.float64, device=engine.device)
        self._prepare_optimizer()

    # ------------------------------------------------------------------ setup
    def _prepare_optimizer(self):
        opt, dev = self.e.optimizer, self.e.device
        if isinstance(opt, _ADAM_LIKE):
            for g in opt.param_groups:
                g["capturable"] = True   # (the fused kernel ignores it but step() checks it)
                if self.e.scheduler is not None and not isinstance(g["lr"], torch.Tensor):
                    g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float32, device=dev)
            for st in opt.state.values():
                if "step" in st and isinstance(st["step"], torch.Tensor):
                    st["step"] = st["step"].to(device=dev, dtype=torch.float32)

    # ------------------------------------------------------------------ step bodies
    def _forward_step(self, feats, lab):
        e = self.e
        out = e.model(*feats) if e.train.multi else e.model(feats[0])
        loss = e.loss(out, lab)
        self.total += loss.detach()
        e.metrics.update(out, lab)
        e.zero_grad()
        loss.backward()
        e.opt_step()

    def _gather(self, sel):
        d = self.e.train
        return d.batch(sel)

    def _eager(self, sel):
        self._forward_step(*self._gather(sel))
        if self.e.scheduler is not None:
            self.e.scheduler.step()

    def _capture(self, steps: int):
        b = self.e.batch
        win = torch.empty(steps * b, dtype=torch.int64, device=self.e.device)
        g = torch.cuda.CUDAGraph()
        self.e.zero_grad()
        # no garbage collection while capturing: a collected object owning a graph (or any HIP
        # resource whose release is not capture-safe) would be destroyed mid-capture. No
        # gc.collect() first either: pending garbage is collected after the capture, outside it,
        # and a full collection here costs a heap walk plus re-faulting the freed memory in the
        # steps that follow (profiles/r3s4_warm_gap_variants.txt)
        gc_was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g, pool=self.pool), _CaptureSafeIndexing(self.index_cache):
                for j in range(steps):
                    self._forward_step(*self._gather(win[j * b:(j + 1) * b]))
        finally:
            if gc_was:
                gc.enable()
        if self.pool is None:
            self.pool = g.pool()
        self.graphs[steps] = (g, win)
        return g, win

    def _replay(self, steps: int, sel):
        ent = self.graphs.get(steps)
        if ent is None:
            try:
                ent = self._capture(steps)
            except Exception as exc:   # capture is best effort: fall back to eager for good
                self.failed = f"{type(exc).__name__}: {exc}\n" + "".join(traceback.format_tb(exc.__traceback__)[-4:])
                self.graphs.clear()
                torch.cuda.synchronize(self.e.device)
                self.e.zero_grad()
                b = self.e.batch
                for j in range(steps):
                    self._eager(sel[j * b:(j + 1) * b])
                return
        g, win = ent
        win.copy_(sel)
        g.replay()
        if self.e.scheduler is not None:
            self.e.scheduler.step()

    def close(self):
        """Destroy the captured graphs and their pool (no capture may be running)."""
        if self.graphs:
            torch.cuda.synchronize(self.e.device)
        self.graphs.clear()
        self.pool = None

    # ------------------------------------------------------------------ epoch
    def train_epoch(self):
        e = self.e
        e.model.train()
        d = e.train
        n, b = d.n, e.batch
        if e.shuffle:
            from raydp_amd.torch.engine import random_permutation
            idx = random_permutation(n, e.seed + e.epoch, e.device).long()
            e.epoch += 1
        else:
            idx = torch.arange(n, device=e.device)
        nfull = n // b
        self.total.zero_()
        s = 0
        # eager warm-up on a side stream (first epoch only)
        if self.warm < 2 and nfull > 0:
            side = torch.cuda.Stream(device=e.device)
            side.wait_stream(torch.cuda.current_stream(e.device))
            with torch.cuda.stream(side), _CaptureSafeIndexing(self.index_cache):
                while self.warm < 2 and s < nfull:
                    self._eager(idx[s * b:(s + 1) * b])
                    s += 1
                    self.warm += 1
            torch.cuda.current_stream(e.device).wait_stream(side)
        while s < nfull:
            if self.failed is not None:
                self._eager(idx[s * b:(s + 1) * b])
                s += 1
                continue
            k = self.chunk if nfull - s >= self.chunk else 1
            self._replay(k, idx[s * b:(s + k) * b])
            s += k
        nb = nfull
        if n % b and not e.drop_last:
            self._eager(idx[nfull * b:])
            nb += 1
        res = e.metrics.compute()
        e.metrics.zero_()
        return res, (self.total / max(nb, 1)).item()
