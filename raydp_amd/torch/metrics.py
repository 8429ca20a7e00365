"""Training metrics (torchmetrics-compatible names), accumulated on the device.

Parity: ``python/raydp/torch/torch_metrics.py`` builds torchmetrics objects from class-name
strings (+ per-metric config) or instances and exposes ``update/compute/reset``. torchmetrics is
not installed here, so the common regression/classification metrics are implemented directly;
if torchmetrics is importable, unknown names are resolved from it. State lives in device
tensors so ``update`` never synchronises the host.
"""
from typing import Any, Dict, List, Optional, Union

import torch


class Metric:
    def __init__(self, **kwargs):
        self.kwargs = kwargs
        self.reset()

    def to(self, device):
        for k, v in list(vars(self).items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self

    def reset(self):
        raise NotImplementedError

    def update(self, preds, target):
        raise NotImplementedError

    def compute(self):
        raise NotImplementedError

    def zero_(self):
        """Reset in place (keeps tensor storage: required when ``update`` is graph-captured)."""
        for v in vars(self).values():
            if isinstance(v, torch.Tensor):
                v.zero_()


class _SumCount(Metric):
    def reset(self):
        self.total = torch.zeros((), dtype=torch.float64)
        self.count = torch.zeros((), dtype=torch.float64)

    def _dev(self, t):
        if self.total.device != t.device:
            self.total = self.total.to(t.device)
            self.count = self.count.to(t.device)

    def compute(self):
        return self.total / torch.clamp(self.count, min=1)


class MeanAbsoluteError(_SumCount):
    def update(self, preds, target):
        self._dev(preds)
        self.total += (preds.detach().double() - target.detach().double().view_as(preds)).abs().sum()
        self.count += target.numel()


class MeanSquaredError(_SumCount):
    def update(self, preds, target):
        self._dev(preds)
        self.total += (preds.detach().double() - target.detach().double().view_as(preds)).pow(2).sum()
        self.count += target.numel()

    def compute(self):
        v = super().compute()
        return v if self.kwargs.get("squared", True) else v.sqrt()


class MeanAbsolutePercentageError(_SumCount):
    def update(self, preds, target):
        self._dev(preds)
        t = target.detach().double().view_as(preds)
        self.total += ((preds.detach().double() - t).abs() / t.abs().clamp(min=1.17e-06)).sum()
        self.count += target.numel()


class Accuracy(_SumCount):
    def update(self, preds, target):
        self._dev(preds)
        p = preds.detach()
        if p.ndim > 1 and p.shape[-1] > 1:
            p = p.argmax(-1)
        else:
            thr = self.kwargs.get("threshold", 0.5)
            p = (p.reshape(-1) > thr).long() if p.is_floating_point() else p.reshape(-1)
        t = target.detach().reshape(-1).long()
        self.total += (p.reshape(-1).long() == t).sum().double()
        self.count += t.numel()


class BinaryAccuracy(Accuracy):
    pass


_BUILTIN = {c.__name__: c for c in (MeanAbsoluteError, MeanSquaredError,
                                    MeanAbsolutePercentageError, Accuracy, BinaryAccuracy)}


def _make(name: str, cfg: Dict[str, Any]):
    if name in _BUILTIN:
        return _BUILTIN[name](**cfg)
    try:
        import torchmetrics
        return getattr(torchmetrics, name)(**cfg)
    except (ImportError, AttributeError):
        raise ValueError(f"unknown metric {name!r}; built-ins: {sorted(_BUILTIN)}") from None


class TorchMetric:
    def __init__(self, metrics_name: Optional[List[Union[str, Metric]]] = None,
                 metrics_config: Optional[Dict[str, Dict[str, Any]]] = None):
        self._metrics = {}
        cfg = metrics_config or {}
        for m in metrics_name or []:
            if isinstance(m, str):
                self._metrics[m] = _make(m, cfg.get(m, {}))
            else:
                self._metrics[type(m).__name__] = m

    @property
    def names(self):
        return list(self._metrics)

    def update(self, preds, targets):
        for m in self._metrics.values():
            m.update(preds, targets)

    def compute(self):
        out = {}
        for k, m in self._metrics.items():
            v = m.compute()
            out[k] = v.item() if isinstance(v, torch.Tensor) else v
        return out

    def reset(self):
        for m in self._metrics.values():
            m.reset()

    def graph_safe(self) -> bool:
        """True if every metric is a built-in device-state metric (updates can be captured)."""
        return all(isinstance(m, Metric) and type(m).__name__ in _BUILTIN for m in self._metrics.values())

    def to(self, device):
        for m in self._metrics.values():
            if isinstance(m, Metric):
                m.to(device)
        return self

    def zero_(self):
        for m in self._metrics.values():
            m.zero_()

    def clone(self) -> "TorchMetric":
        """A fresh collection of the same metrics (state reset) for one fit: built-in metrics
        are rebuilt from their config (a deepcopy costs ~0.2 ms per fit), others deep-copied."""
        import copy
        out = TorchMetric()
        for k, m in self._metrics.items():
            out._metrics[k] = type(m)(**m.kwargs) if type(m).__name__ in _BUILTIN and type(m) is _BUILTIN[
                type(m).__name__] else copy.deepcopy(m)
        return out
