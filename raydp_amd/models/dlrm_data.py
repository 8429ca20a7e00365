"""Criteo-style DLRM preprocessing on the Spark-compatible engine, plus a synthetic generator.

Behaviour follows the reference notebook ``examples/pytorch_dlrm.ipynb`` (cells 4-7): for
every categorical column, count each value's frequency (``posexplode(array(...))`` +
``groupBy(column_id, data).count()``), drop values rarer than ``frequency_limit``, assign
dense ids by descending frequency (``row_number`` over a window per column), replace each
categorical value by its id with a left join (unseen/rare values -> 0), ``log(x + 3)`` the
integer features, null -> 0, and optionally shuffle rows through a random ordinal
(``repartition(ordinal).sortWithinPartitions(ordinal)``). Label is column ``_c0``, integer
features ``_c1.._c13``, categorical ``_c14.._c39``.

All of it runs as stages on the executor processes (joins / window / shuffles included).
"""
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

LABEL_COL = 0
INT_COLS = list(range(1, 14))
CAT_COLS = list(range(14, 40))


def _limits(frequency_limit) -> Tuple[Optional[int], Dict[int, int]]:
    """'3' -> default 3; '3,15:10' -> default 3 and column 15 at 10."""
    if frequency_limit in (None, "", 0):
        return None, {}
    default, per_col = None, {}
    for part in str(frequency_limit).split(","):
        bits = part.split(":")
        if len(bits) == 1:
            default = int(bits[0])
        else:
            per_col[int(bits[0])] = int(bits[1])
    return default, per_col


def value_counts(df, frequency_limit=None):
    """(column_id, data, count) for every categorical value that survives the limit."""
    from raydp_amd.spark.functions import array, col, posexplode
    names = [f"_c{i}" for i in CAT_COLS]
    counts = (df.select(posexplode(array(*names)))
                .withColumnRenamed("pos", "column_id")
                .withColumnRenamed("col", "data")
                .filter("data is not null")
                .groupBy("column_id", "data").count())
    default, per_col = _limits(frequency_limit)
    for c, lim in per_col.items():
        counts = counts.filter((col("column_id") != c - CAT_COLS[0]) | (col("count") >= lim))
    if default:
        rest = [c - CAT_COLS[0] for c in CAT_COLS if c not in per_col]
        counts = counts.filter((~col("column_id").isin(rest)) | (col("count") >= default))
    return counts


def assign_ids(counts):
    """Dense id per (column, value): rank by descending frequency, 0-based."""
    from raydp_amd.spark import Window
    from raydp_amd.spark.functions import desc, row_number
    w = Window.partitionBy("column_id").orderBy(desc("count"))
    return counts.withColumn("id", row_number().over(w) - 1).withColumnRenamed("count", "model_count")


def column_models(with_ids):
    for c in CAT_COLS:
        yield c, with_ids.filter(f"column_id == {c - CAT_COLS[0]}").drop("column_id")


def apply_models(df, models: Sequence[Tuple[int, object]]):
    for c, model in models:
        name = f"_c{c}"
        m = model.drop("model_count").withColumnRenamed("data", name)
        df = df.join(m, name, how="left").drop(name).withColumnRenamed("id", name)
    return df.fillna(0, [f"_c{c}" for c in CAT_COLS])


def transform_log(df, do_log: bool = True):
    from raydp_amd.spark.functions import log
    names = [f"_c{c}" for c in INT_COLS]
    if do_log:
        # one projection for the 13 columns (13 withColumn calls type the 26-join plan 13 times)
        logged = set(names)
        df = df.select(*[(log(df[n] + 3).alias(n) if n in logged else df[n]) for n in df.columns])
    return df.fillna(0, names)


def pre_process(df, frequency_limit="3", output_ordering: str = "total_random", no_numeric_log_col: bool = False):
    """-> (processed DataFrame, categorical table sizes)."""
    from raydp_amd.spark.functions import count, lit, monotonically_increasing_id, rand
    from raydp_amd.spark.types import LongType
    ids = assign_ids(value_counts(df, frequency_limit)).cache()
    # every table's size from ONE aggregation over the id table (the notebook counts each
    # column's model separately: 26 jobs of a few ms each for a few KB of ids)
    per_col = {int(r["column_id"]): int(r["size"])
               for r in ids.groupBy("column_id").agg(count(lit(1)).alias("size")).collect()}
    models = [(c, m.cache()) for c, m in column_models(ids)]
    sizes = [per_col.get(c - CAT_COLS[0], 0) + 1 for c, _ in models]
    if output_ordering == "total_random":
        df = df.withColumn("ordinal", (rand() * (1 << 52)).cast(LongType()))
    elif output_ordering == "input":
        df = df.withColumn("ordinal", monotonically_increasing_id())
    df = apply_models(df, models)
    df = transform_log(df, not no_numeric_log_col)
    if output_ordering == "total_random":
        df = df.repartition("ordinal").sortWithinPartitions("ordinal").drop("ordinal")
    elif output_ordering == "input":
        df = df.sortWithinPartitions("ordinal").drop("ordinal")
    return df, sizes


def criteo_schema():
    from raydp_amd.spark.types import IntegerType, StringType, StructField, StructType
    return StructType([StructField(f"_c{LABEL_COL}", IntegerType())]
                      + [StructField(f"_c{i}", IntegerType()) for i in INT_COLS]
                      + [StructField(f"_c{i}", StringType()) for i in CAT_COLS])


def synthetic_criteo(path: str, rows: int, seed: int = 0, vocab: Sequence[int] = None, null_frac: float = 0.05):
    """Write a Criteo-shaped TSV (label, 13 ints, 26 hex categoricals) with Zipf-like
    categorical frequencies, so frequency limits and id assignment behave as on real data."""
    rng = np.random.default_rng(seed)
    vocab = list(vocab or [max(4, int(v)) for v in np.geomspace(8, 5000, len(CAT_COLS))])
    cols = [rng.integers(0, 2, rows).astype(str)]
    for _ in INT_COLS:
        v = rng.poisson(5.0, rows).astype(object)
        v[rng.random(rows) < null_frac] = ""
        cols.append(v.astype(str))
    for k in vocab:
        z = np.minimum(rng.zipf(1.3, rows), k) - 1
        v = np.array([f"{(h * 2654435761) & 0xffffffff:08x}" for h in range(k)], dtype=object)[z]
        v[rng.random(rows) < null_frac] = ""
        cols.append(v.astype(str))
    with open(path, "w") as f:
        for r in range(rows):
            f.write("\t".join(c[r] for c in cols) + "\n")
    return vocab


_ = List
