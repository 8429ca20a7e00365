"""Estimator ABC (reference: ``python/raydp/estimator.py:23-43``)."""
from abc import ABC, abstractmethod
from typing import Any, NoReturn, Optional


class EstimatorInterface(ABC):
    """A scikit-learn like API: ``fit(train_ds, evaluate_ds)`` then ``get_model()``."""

    @abstractmethod
    def fit(self, train_ds, evaluate_ds: Optional[Any] = None) -> NoReturn:
        """Train on the given datasets."""

    @abstractmethod
    def get_model(self) -> Any:
        """Return the trained model."""
