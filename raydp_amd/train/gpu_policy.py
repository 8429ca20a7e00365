"""Backend choices the framework makes for the user-written loops its GPU workers run, without
touching user code (Ray Train's worker setup plays the same role: device placement, process group).

* :func:`native_batchnorm` -- BatchNorm layers run on PyTorch's native kernels instead of MIOpen's
  while the worker's loop runs. At tabular batch sizes (64-1024 rows x 16-256 features) MIOpen's
  batch-norm path costs several extra launches per call and the eager step is launch-bound
  (``scripts/dev/eager_step_bench.py``: NYC_Model batch 64, 1.114 -> 0.845 ms/step). Only the
  BatchNorm call is affected -- the MIOpen switch is flipped around it and restored -- so
  convolutions keep MIOpen. The autograd node the forward picked (native_batch_norm_backward)
  carries the backward. Config ``spark.ray.mi355x.native_batchnorm``.

* :func:`fused_optimizers` -- torch's Adam / AdamW / SGD ``step()`` in the worker's loop runs on
  the multi-tensor HIP kernels (``raydp_amd/ops/fused_optim.py``), as behind
  ``hvd.DistributedOptimizer``. Config ``spark.ray.mi355x.fused_optimizer``.

* :func:`graph_model` -- ``train.torch.prepare_model`` on a one-worker GPU job replays the
  model's training forward + backward as HIP graphs (``torch.cuda.make_graphed_callables``) once
  a batch shape has repeated: a tabular MLP step is ~40 tiny kernels each way, each costing more
  host time than device time (the stroke tutorial's GPU loop was slower than its CPU loop, B4).
  Eval / no-grad calls, other shapes, kwargs and models whose forward cannot be captured (a host
  sync, data-dependent control flow) run eagerly; the capture's warm-up leaves BatchNorm running
  statistics as they were; outputs are cloned out of the graph's static buffers, so a caller may
  keep them across steps. The capture differentiates w.r.t. aliases of the parameters (fresh
  leaves on the same storage) and replays take the real parameters, so a loop that still holds
  the previous step's loss at the capture -- every plain training loop -- captures cleanly.
  Config ``spark.ray.mi355x.graph_user_model``.

Reference role: the worker set-up of Ray Train's ``TorchTrainer`` / ``HorovodTrainer``
(``tutorials/raytrain_example.ipynb`` cell 40, ``examples/horovod_nyctaxi.py:119-162``).
"""
import contextlib


@contextlib.contextmanager
def native_batchnorm(enabled: bool = True):
    """While active, ``nn.BatchNorm*`` forwards on GPU tensors bypass MIOpen (restored on exit)."""
    if not enabled:
        yield
        return
    import torch
    from torch.nn.modules.batchnorm import _BatchNorm
    orig = _BatchNorm.forward
    get, put = torch._C._get_cudnn_enabled, torch._C._set_cudnn_enabled

    def forward(self, input):
        if input.is_cuda and get():
            put(False)
            try:
                return orig(self, input)
            finally:
                put(True)
        return orig(self, input)

    forward.__wrapped__ = orig
    _BatchNorm.forward = forward
    try:
        yield
    finally:
        if _BatchNorm.forward is forward:
            _BatchNorm.forward = orig


@contextlib.contextmanager
def fused_optimizers(enabled: bool = True):
    """While active, ``torch.optim.Adam`` / ``AdamW`` / ``SGD`` steps of a user loop run on the
    multi-tensor HIP kernels (``raydp_amd.ops.fused_optim.fused_step``: one launch per 24 tensors,
    torch's state layout kept) -- what ``hvd.DistributedOptimizer`` already does -- instead of
    torch's foreach chain (~10 launches plus their host time per step). Torch's own step still
    runs for a closure, inside a graph capture, and for anything ``fused_step`` declines (step
    hooks, amsgrad / capturable / fused / differentiable groups, CPU or non-fp32 parameters):
    an optimizer it declines once keeps torch's step."""
    if not enabled:
        yield
        return
    import torch
    from torch.optim import Optimizer
    # (AdamW inherits Adam's step in recent torch: only classes that define their own are patched)
    classes = tuple(c for c in (torch.optim.Adam, torch.optim.AdamW, torch.optim.SGD) if "step" in c.__dict__)
    originals, patched = {}, {}
    for cls in classes:
        orig = cls.__dict__["step"]
        if not getattr(orig, "hooked", False):
            # what torch does to a class's step when its first optimizer is built (the wrapper
            # that runs the step hooks): done here, so the torch path below keeps the hooks
            orig = Optimizer.profile_hook_step(orig)
            orig.hooked = True
        originals[cls] = orig

    def make(orig):
        def step(self, closure=None):
            if closure is None and not self.__dict__.get("_raydp_torch_step") and \
                    not (torch.cuda.is_initialized() and torch.cuda.is_current_stream_capturing()):
                from raydp_amd.ops import fused_optim
                if fused_optim.fused_step(self):      # (declines when step hooks are registered)
                    return None
                self._raydp_torch_step = True
            return orig(self, closure)
        step.__wrapped__ = orig
        step.hooked = True       # an optimizer built under the policy must not re-wrap the class step
        return step

    for cls in classes:
        patched[cls] = cls.step = make(originals[cls])
    try:
        yield
    finally:
        for cls in classes:
            if cls.__dict__.get("step") is patched[cls]:
                cls.step = originals[cls]


def worker_policies(use_gpu: bool):
    """The context a GPU train worker runs its loop in (a no-op context on CPU workers)."""
    from raydp_amd.utils import config as C
    stack = contextlib.ExitStack()
    stack.enter_context(native_batchnorm(bool(use_gpu) and bool(C.get("spark.ray.mi355x.native_batchnorm"))))
    stack.enter_context(fused_optimizers(bool(use_gpu) and bool(C.get("spark.ray.mi355x.fused_optimizer"))))
    return stack


_MAX_SHAPES = 4        # graphed batch shapes per model (a ragged last batch stays eager)
_STEADY = 3            # calls with the same shape before it is graphed
# instance attributes graph_model adds (dropped again by copies and pickles of the module)
_PATCH_ATTRS = ("forward", "_raydp_graphed", "_raydp_graphs", "__reduce_ex__", "__deepcopy__")


def _plain_state(module):
    return {k: v for k, v in module.__dict__.items() if k not in _PATCH_ATTRS}


def _rebuild_plain(cls, state):
    """Unpickle target of a graphed module: the same class, without the graphs."""
    obj = cls.__new__(cls)
    obj.__dict__.update(state)
    return obj


def graph_model(module):
    """Patch ``module`` (in place: same object, same ``state_dict``) so its training forward runs
    from a captured HIP graph per repeated input shape; returns the module.

    A replayed graph's backward reads the activations its forward left in the graph's static
    buffers, so a second forward of the same shape before the first one's backward (twin
    networks, two losses summed, accumulation without an interleaved backward) must not replay
    the graph again: every replay marks its shape pending until the gradient of its output
    arrives, and a call on a pending shape runs eagerly. ``copy.deepcopy`` and pickling
    (``torch.save(model)``) see the plain module: the copy runs its own eager forward."""
    import copy
    import torch
    if getattr(module, "_raydp_graphed", False):
        return module
    orig = module.forward
    graphs, seen, pending = {}, {}, set()
    index_cache = {}     # integer-list indices as device tensors (see _capture)
    state = {"failed": False, "outstanding": 0}   # forwards (any shape) whose backward is still to come

    # the trainable parameters, as (owner module, attribute name, tensor)
    slots = [(sub, name, p) for sub in module.modules() for name, p in list(sub._parameters.items())
             if p is not None and p.requires_grad]

    def _fwd_aliased(*a):
        # the original forward with each parameter replaced by the alias at the same position of
        # the trailing arguments: fresh leaves sharing the parameters' storage
        xs, ps = a[:len(a) - len(slots)], a[len(a) - len(slots):]
        saved = [sub._parameters[name] for sub, name, _ in slots]
        try:
            for (sub, name, _), t in zip(slots, ps):
                sub._parameters[name] = t
            return orig(*xs)
        finally:
            for (sub, name, _), t in zip(slots, saved):
                sub._parameters[name] = t

    def _capture(args):
        bufs = [(b, b.detach().clone()) for b in module.buffers()]
        # the worker's native-BatchNorm policy (cudnn switched off around each BatchNorm call)
        # is lifted while the graph is captured: a capture of that path's backward crashed at
        # capture end on the GPU box (scripts/dev/hvd_graph_repro.py); the replay then runs the
        # default BatchNorm kernels, which is what a replay's launch cost no longer cares about
        from torch.nn.modules.batchnorm import _BatchNorm
        patched = _BatchNorm.forward
        plain = getattr(patched, "__wrapped__", None)
        if plain is not None:
            _BatchNorm.forward = plain
        try:
            # The capture differentiates w.r.t. ALIASES of the parameters (fresh leaves on the
            # same storage), not the parameters: a parameter's gradient accumulator from an
            # earlier step is still alive while the caller holds that step's loss, and the
            # capture's backward then synchronises with the default stream it was made on -- a
            # crash at capture end on this stack (scripts/dev/graph_bisect.py: gm vs gm_delloss).
            # A replay gets the real parameters (same storage: nothing copied), so autograd
            # accumulates their gradients as an eager backward would.
            samples = tuple(a.detach().clone() for a in args) + tuple(
                p.detach().requires_grad_(True) for _, _, p in slots)
            torch.cuda.synchronize()
            # a forward that indexes with a Python list (``x[:, [1, 7, 8]]``: the stroke
            # tutorial's NET_Model) copies the list to the device on every call, which a capture
            # refuses: the warm-up iterations turn each such index into a cached device tensor
            # that the captured graph then reads (the same mode the torch-loop engine's graphs use)
            from raydp_amd.torch.graphs import _CaptureSafeIndexing
            with _CaptureSafeIndexing(index_cache):
                # (parameters the forward never reads -- the tutorial's NET_Model keeps five unused
                # Linear + BatchNorm layers -- get no gradient, as in an eager backward)
                g = torch.cuda.make_graphed_callables(_fwd_aliased, samples, num_warmup_iters=3,
                                                      allow_unused_input=True)
            return g
        except Exception:  # noqa: BLE001 - not capturable: eager from now on
            state["failed"] = True
            return None
        finally:
            if plain is not None:
                _BatchNorm.forward = patched
            with torch.no_grad():       # the warm-up's BatchNorm statistics are not training steps
                for b, v in bufs:
                    b.copy_(v)

    def forward(*args, **kwargs):
        if (kwargs or state["failed"] or not module.training or not torch.is_grad_enabled()
                or not args or not all(isinstance(a, torch.Tensor) and a.is_cuda and not a.requires_grad
                                       for a in args)):
            return orig(*args, **kwargs)
        key = tuple((tuple(a.shape), a.dtype) for a in args)
        graphed = False
        if key in pending:       # this shape's last replay still waits for its backward
            out = orig(*args)
        else:
            g = graphs.get(key)
            if g is None:
                n = seen.get(key, 0) + 1
                seen[key] = n
                # capture only between iterations: with a forward of this model still waiting for
                # its backward the capture's own warm-up backward would run inside that graph
                if n >= _STEADY and len(graphs) < _MAX_SHAPES and state["outstanding"] == 0:
                    g = _capture(args)
                    if g is not None:
                        graphs[key] = g
            if g is not None:
                out, graphed = g(*args, *[p for _, _, p in slots]), True
            else:
                out = orig(*args)
        leaves = [t for t in torch.utils._pytree.tree_leaves(out)
                  if isinstance(t, torch.Tensor) and t.requires_grad]
        if leaves:
            state["outstanding"] += 1
            if graphed:
                pending.add(key)
            left = [len(leaves)]

            def arrived(grad, key=key, left=left, graphed=graphed):
                # the graphed backward runs right after the gradients of its outputs
                left[0] -= 1
                if left[0] == 0:
                    state["outstanding"] -= 1
                    if graphed:
                        pending.discard(key)
                return grad
            for t in leaves:
                t.register_hook(arrived)
        if not graphed:
            return out
        return torch.utils._pytree.tree_map(lambda t: t.clone() if isinstance(t, torch.Tensor) else t, out)

    def reduce_ex(proto):
        return _rebuild_plain, (type(module), _plain_state(module))

    def deepcopy(memo):
        new = type(module).__new__(type(module))
        memo[id(module)] = new
        new.__dict__.update(copy.deepcopy(_plain_state(module), memo))
        return new

    module.forward = forward
    module._raydp_graphed = True
    module._raydp_graphs = graphs      # captured shapes (introspection)
    module.__reduce_ex__ = reduce_ex
    module.__deepcopy__ = deepcopy
    return module
