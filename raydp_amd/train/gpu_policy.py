"""Backend choices the framework makes for the user-written loops its GPU workers run, without
touching user code (Ray Train's worker setup plays the same role: device placement, process group).

* :func:`native_batchnorm` -- BatchNorm layers run on PyTorch's native kernels instead of MIOpen's
  while the worker's loop runs. At tabular batch sizes (64-1024 rows x 16-256 features) MIOpen's
  batch-norm path costs several extra launches per call and the eager step is launch-bound
  (``scripts/dev/eager_step_bench.py``: NYC_Model batch 64, 1.114 -> 0.845 ms/step). Only the
  BatchNorm call is affected -- the MIOpen switch is flipped around it and restored -- so
  convolutions keep MIOpen. The autograd node the forward picked (native_batch_norm_backward)
  carries the backward. Config ``spark.ray.mi355x.native_batchnorm``.

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


def worker_policies(use_gpu: bool):
    """The context a GPU train worker runs its loop in (a no-op context on CPU workers)."""
    from raydp_amd.utils import config as C
    return native_batchnorm(bool(use_gpu) and bool(C.get("spark.ray.mi355x.native_batchnorm")))
