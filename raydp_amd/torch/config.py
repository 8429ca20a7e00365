"""Collective backend selection for the torch estimator.

Reference: ``python/raydp/torch/config.py`` swaps Ray Train's backend to oneCCL when
``use_ccl=True``. On MI355X the GPU backend is RCCL (``torch.distributed`` backend ``"nccl"``
binds RCCL on ROCm) and Gloo serves CPU workers; ``use_ccl`` is accepted for API parity and
maps onto the same choice.
"""
from dataclasses import dataclass


@dataclass
class TorchConfig:
    backend: str = None  # None: "nccl" (RCCL) on GPU workers, "gloo" on CPU workers
    init_method: str = "env"
    timeout_s: int = 1800

    def resolve(self, use_gpu: bool) -> str:
        if self.backend in (None, "ccl", "oneccl"):
            return "nccl" if use_gpu else "gloo"
        return self.backend
