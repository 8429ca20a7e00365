"""A window function nested inside an expression (``row_number().over(w) - 1``) is hoisted into a
temporary column (raydp_amd/spark/dataframe.py ``_hoist_windows`` / ``_has_window``); plain
expressions are left untouched."""
from raydp_amd.spark import functions as F
from raydp_amd.spark.column import ColRef
from raydp_amd.spark.dataframe import _has_window, _hoist_windows
from raydp_amd.spark.window import Window


def test_nested_window_is_found_and_hoisted():
    w = Window.partitionBy("g").orderBy("v")
    e = (F.row_number().over(w) - 1)._expr
    assert _has_window(e)
    ne, hoisted = _hoist_windows(e)
    assert len(hoisted) == 1 and ne is not e
    plain = (F.col("v") * 2 + F.lit(1))._expr
    assert not _has_window(plain)
    assert _hoist_windows(plain) == (plain, [])
    assert not _has_window(ColRef("x"))


def test_nested_window_column_values(spark_session=None):
    from raydp_amd import context
    spark = context.init_spark("win", 1, 1, "500M")
    try:
        df = spark.createDataFrame([(1, "a", 3.0), (2, "a", 1.0), (3, "b", 2.0)], ["id", "g", "v"])
        w = Window.partitionBy("g").orderBy("v")
        rows = df.withColumn("rn", F.row_number().over(w) - 1).orderBy("id").collect()
        assert [(r.id, r.rn) for r in rows] == [(1, 1), (2, 0), (3, 0)]
        assert df.withColumn("rn", F.row_number().over(w) - 1).columns == ["id", "g", "v", "rn"]
    finally:
        context.stop_spark()
