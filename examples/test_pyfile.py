"""Helper module shipped with ``raydp-submit --py-files`` (reference: examples/test_pyfile.py)."""


def compute_sum(numbers):
    return sum(numbers)
