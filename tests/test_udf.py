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
    # double UDF), numpy's is NaN (an 'invalid' floating-point flag): that batch runs per row
    second = pa.array(np.concatenate([np.linspace(1.0, 100.0, 499), [-4.0]]))
    with pytest.raises((TypeError, pa.ArrowInvalid)):   # per-row Python semantics, not NaN
        u.evaluate([second], len(second))
    assert u.vectorized                    # only that batch left the vectorised path


def _branchy_min(a, b):
    return min(a, b) if a > -5 else max(b, a)


def test_vectorised_udf_python_min_max_and_zero_divisors():
    """Builtin min/max keep Python's NaN order semantics; a zero divisor anywhere in a batch
    runs that batch per row (ZeroDivisionError), not as numpy's inf."""
    u = UserDefinedFunction(_branchy_min, "double")
    a = np.array([1.0, np.nan, 3.0, -9.0, 2.0] * 20)
    b = np.array([np.nan, 1.0, 2.0, 4.0, 2.0] * 20)
    out = np.asarray(u.evaluate([pa.array(a), pa.array(b)], len(a)))
    want = np.array([_branchy_min(x, y) for x, y in zip(a, b)])
    np.testing.assert_array_equal(out, want)
    d = UserDefinedFunction(lambda x, y: x // y, "long")
    ok = d.evaluate([pa.array(np.arange(10)), pa.array(np.full(10, 3))], 10)
    assert ok.to_pylist() == [i // 3 for i in range(10)]
    with pytest.raises(ZeroDivisionError):
        d.evaluate([pa.array(np.arange(10)), pa.array(np.array([3, 3, 3, 0, 3, 3, 3, 3, 3, 3]))], 10)


def test_vectorised_udf_stays_vectorised_when_consistent():
    u = UserDefinedFunction(_branchy, "double")
    rng = np.random.default_rng(0)
    for _ in range(3):
        a, b = rng.normal(size=300), rng.normal(size=300)
        out = u.evaluate([pa.array(a), pa.array(b)], 300)
        np.testing.assert_allclose(np.asarray(out), np.where(a > 0, a * 2 + b, b - a))
    assert u.vectorized
