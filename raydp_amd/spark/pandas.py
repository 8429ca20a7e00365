"""Pandas-on-Spark (``pyspark.pandas``) subset used by the reference tests.

Only what ``python/raydp/tests/test_torch.py`` and ``raydp.utils.random_split`` exercise:
``ps.range``, column assignment with arithmetic (``df["z"] = df["x"] * 3 + 5``),
``astype``, ``to_spark``/``to_pandas`` and wrapping a Spark-style DataFrame.
"""
import pyarrow as pa

from raydp_amd.spark.column import Column
from raydp_amd.spark.types import parse_type_string

_PANDAS_TO_SPARK = {"float": "double", "float64": "double", "float32": "float", "int": "bigint",
                    "int64": "bigint", "int32": "int", "str": "string", "bool": "boolean"}


class Series:
    def __init__(self, df: "DataFrame", col: Column):
        self._df, self._col = df, col

    def _op(self, other, f):
        o = other._col if isinstance(other, Series) else other
        return Series(self._df, f(self._col, o))

    def __add__(self, o): return self._op(o, lambda a, b: a + b)
    def __radd__(self, o): return self._op(o, lambda a, b: b + a)
    def __sub__(self, o): return self._op(o, lambda a, b: a - b)
    def __rsub__(self, o): return self._op(o, lambda a, b: b - a)
    def __mul__(self, o): return self._op(o, lambda a, b: a * b)
    def __rmul__(self, o): return self._op(o, lambda a, b: b * a)
    def __truediv__(self, o): return self._op(o, lambda a, b: a / b)

    def astype(self, dtype):
        return Series(self._df, self._col.cast(_PANDAS_TO_SPARK.get(str(dtype), str(dtype))))

    def to_pandas(self):
        return self._df._sdf.select(self._col).toPandas().iloc[:, 0]


class DataFrame:
    def __init__(self, data=None):
        from raydp_amd.spark.dataframe import DataFrame as SDF
        if isinstance(data, SDF):
            self._sdf = data
        elif isinstance(data, DataFrame):
            self._sdf = data._sdf
        else:
            import pandas as pd
            from raydp_amd.spark.session import SparkSession
            spark = SparkSession.getActiveSession() or SparkSession.builder.getOrCreate()
            self._sdf = spark.createDataFrame(pd.DataFrame(data))

    def __getitem__(self, key):
        if isinstance(key, str):
            return Series(self, self._sdf[key])
        return DataFrame(self._sdf.select(*key))

    def __setitem__(self, key, value):
        col = value._col if isinstance(value, Series) else value
        if not isinstance(col, Column):
            from raydp_amd.spark.functions import lit
            col = lit(col)
        self._sdf = self._sdf.withColumn(key, col)

    def astype(self, dtype):
        t = _PANDAS_TO_SPARK.get(str(dtype), str(dtype))
        return DataFrame(self._sdf.select(*[self._sdf[c].cast(t).alias(c) for c in self._sdf.columns]))

    @property
    def columns(self):
        return self._sdf.columns

    def to_spark(self, index_col=None):
        return self._sdf

    def to_pandas(self):
        return self._sdf.toPandas()

    def __len__(self):
        return self._sdf.count()

    def head(self, n=5):
        return DataFrame(self._sdf.limit(n))


def range(start, end=None, step=1, num_partitions=None):  # noqa: A001
    from raydp_amd.spark.session import SparkSession
    spark = SparkSession.getActiveSession() or SparkSession.builder.getOrCreate()
    return DataFrame(spark.range(start, end, step, num_partitions))


def from_pandas(pdf):
    return DataFrame(pdf)
