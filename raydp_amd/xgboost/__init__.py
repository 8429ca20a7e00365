"""Gradient-boosted trees estimator (reference: ``python/raydp/xgboost/``).

``XGBoostEstimator`` trains with the native histogram GBDT in :mod:`raydp_amd.xgboost.gbdt`
(``DMatrix``, ``Booster``, ``train``), distributed over ``torch.distributed``.
"""
from raydp_amd.xgboost.estimator import XGBoostEstimator
from raydp_amd.xgboost.gbdt import Booster, DMatrix, train

__all__ = ["XGBoostEstimator", "Booster", "DMatrix", "train"]
