"""Vectorised row UDFs are re-verified on every batch (value-range extremes included), so a
batch whose values take a branch the first sample never exercised falls back to exact per-row
semantics instead of returning a silently different numpy result."""
import numpy as np
import pyarrow as pa
import pytest

from raydp_amd.spark.udf import UserDefinedFunction


def _root(x):
    return x ** 0.5


def _branchy(a, b):
    if a > 0:
        return a * 2 + b
    return b - a


def test_vectorised_udf_rechecks_new_value_ranges():
    u = UserDefinedFunction(_root, "double")
    first = pa.array(np.linspace(1.0, 100.0, 500))
    out = u.evaluate([first], len(first))
    assert u.vectorized
    np.testing.assert_allclose(np.asarray(out), np.sqrt(np.linspace(1.0, 100.0, 500)))
    # a later batch reaches negative values: Python's x ** 0.5 is complex there (an error for a
    # double UDF), numpy's is NaN; the per-batch check sees the minimum row and refuses numpy
    second = pa.array(np.concatenate([np.linspace(1.0, 100.0, 499), [-4.0]]))
    with pytest.raises((TypeError, pa.ArrowInvalid)):   # per-row Python semantics, not NaN
        u.evaluate([second], len(second))
    assert not u.vectorized


def test_vectorised_udf_stays_vectorised_when_consistent():
    u = UserDefinedFunction(_branchy, "double")
    rng = np.random.default_rng(0)
    for _ in range(3):
        a, b = rng.normal(size=300), rng.normal(size=300)
        out = u.evaluate([pa.array(a), pa.array(b)], 300)
        np.testing.assert_allclose(np.asarray(out), np.where(a > 0, a * 2 + b, b - a))
    assert u.vectorized
