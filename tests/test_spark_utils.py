"""Ports of python/raydp/tests/test_spark_utils.py (unit contracts of raydp.utils)."""
import math

import pytest

import raydp  # noqa: F401
import raydp.utils as utils
from raydp_amd.spark import pandas as ps


def test_df_type_check(spark_session):
    spark_df = spark_session.range(0, 10)
    koalas_df = ps.range(0, 10)
    assert utils.df_type_check(spark_df)
    assert utils.df_type_check(koalas_df)
    other_df = "df"
    with pytest.raises(Exception) as exinfo:
        utils.df_type_check(other_df)
    assert "The type: <class 'str'> is not supported" in str(exinfo.value)


def test_convert_to_spark(spark_session):
    spark_df = spark_session.range(0, 10)
    converted, is_spark_df = utils.convert_to_spark(spark_df)
    assert is_spark_df
    assert spark_df is converted
    koalas_df = ps.range(0, 10)
    converted, is_spark_df = utils.convert_to_spark(koalas_df)
    assert not is_spark_df
    assert converted.count() == 10


def test_random_split(spark_session):
    spark_df = spark_session.range(0, 10)
    splits = utils.random_split(spark_df, [0.7, 0.3])
    assert len(splits) == 2
    assert sum(s.count() for s in splits) == 10
    koalas_df = ps.range(0, 10)
    splits = utils.random_split(koalas_df, [0.7, 0.3])
    assert isinstance(splits[0], ps.DataFrame)
    assert sum(len(s) for s in splits) == 10


def test_random_split_deterministic(spark_session):
    df = spark_session.range(0, 1000, numPartitions=4)
    a = [r.id for r in utils.random_split(df, [0.5, 0.5], 7)[0].collect()]
    b = [r.id for r in utils.random_split(df, [0.5, 0.5], 7)[0].collect()]
    assert a == b and 350 < len(a) < 650


def test_memory_size_parser():
    upper_units = ["", "K", "M", "G", "T"]
    expected = [10 * math.pow(2, 10 * p) for p in range(len(upper_units))]
    for u, e in zip(upper_units, expected):
        assert utils.parse_memory_size(f"10{u}") == e
        assert utils.parse_memory_size(f"10{u.lower()}") == e
        assert utils.parse_memory_size(f"10 {u}") == e
        assert utils.parse_memory_size(f"10{u}B") == e
        assert utils.parse_memory_size(f"10 {u.lower()}b") == e
    assert utils.parse_memory_size("1.5G") == int(1.5 * 2 ** 30)
    assert utils.parse_memory_size(123) == 123


@pytest.mark.parametrize("blocks,world", [([5, 10, 15, 20, 25, 30, 35, 40], 3),
                                          ([100], 1), ([3, 3, 3, 3], 4), ([7, 1, 9, 2, 5], 2)])
@pytest.mark.parametrize("shuffle", [False, True])
def test_divide_blocks(blocks, world, shuffle):
    results = utils.divide_blocks(blocks, world, shuffle, 1)
    per_rank = int(math.ceil(sum(blocks) / world))
    assert len(results) == world
    for rank, sel in results.items():
        assert sum(n for _, n in sel) == per_rank
        for idx, n in sel:
            assert 0 < n <= blocks[idx]


def test_divide_blocks_not_enough():
    with pytest.raises(Exception):
        utils.divide_blocks([1], 2)


def test_partition_cpus_gives_disjoint_rank_slices(monkeypatch):
    import os

    from raydp_amd.utils import partition_cpus
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)))
    slices = [partition_cpus(r, 8, 5) for r in range(8)]
    assert all(len(s) == 8 for s in slices)
    flat = [c for s in slices for c in s]
    assert len(set(flat)) == 64                       # disjoint, covering every core
    assert slices[0] == list(range(8)) and slices[7] == list(range(56, 64))
    assert partition_cpus(0, 8, 9) is None            # too few cores: no pinning
    assert partition_cpus(0, 1, 2) is None
