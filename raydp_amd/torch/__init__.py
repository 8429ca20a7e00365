"""PyTorch integration (reference: ``python/raydp/torch/__init__.py``)."""
from raydp_amd.torch.estimator import TorchEstimator
from raydp_amd.torch.metrics import TorchMetric
from raydp_amd.torch.config import TorchConfig

__all__ = ["TorchEstimator", "TorchMetric", "TorchConfig"]
