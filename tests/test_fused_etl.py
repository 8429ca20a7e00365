"""Fused narrow-operator execution (raydp_amd/spark/exprc.py + csrc/exec/expr/expr_vm.cc).

Every case runs the same DataFrame twice - once through the native expression VM and once
through the per-operator Arrow path (RAYDP_FUSED_ETL=0) - and requires identical tables:
same schema, same rows, same nulls, bit-identical values."""
import math

import numpy as np
import pyarrow as pa
import pytest

from raydp_amd.spark import exprc
from raydp_amd.spark import functions as F
from raydp_amd.spark.functions import col, lit, udf


def _collect(df, fused, monkeypatch):
    monkeypatch.setenv("RAYDP_FUSED_ETL", "1" if fused else "0")
    plan = df._plan
    parts = [plan.compute(i) for i in range(plan.num_partitions())]
    return pa.concat_tables(parts) if parts else None


def _check_static_schemas(df):
    """Statically inferred operator schemas equal the ones the Arrow path produces."""
    nodes, _ = exprc.chain_of(df._plan)
    for n in nodes:
        st = exprc.static_schema(n)
        if st is not None:
            assert st == n.empty().schema, (n.desc, st, n.empty().schema)


def _same(df, monkeypatch):
    _check_static_schemas(df)
    before = dict(exprc.STATS)
    ref = _collect(df, False, monkeypatch)
    got = _collect(df, True, monkeypatch)
    assert ref.schema == got.schema, (ref.schema, got.schema)
    assert ref.num_rows == got.num_rows
    for name in ref.column_names:
        a, b = ref.column(name).combine_chunks(), got.column(name).combine_chunks()
        assert _equal(a, b), (name, a[:8], b[:8])
    return {k: exprc.STATS[k] - before[k] for k in before}


def _equal(a, b):
    """Arrow equality that also treats NaN == NaN (bit-identical values, identical nulls)."""
    if not pa.types.is_floating(a.type):
        return a.equals(b)
    if a.type != b.type or not a.is_null().equals(b.is_null()):
        return False
    x = a.fill_null(0).to_numpy(zero_copy_only=False)
    y = b.fill_null(0).to_numpy(zero_copy_only=False)
    return np.array_equal(x, y, equal_nan=True)


def _table(n=2000, seed=0, nulls=True):
    rng = np.random.default_rng(seed)

    def mask():
        return rng.random(n) < 0.1 if nulls else None

    ts = (np.datetime64("1969-06-01T00:00:00") +
          rng.integers(0, 80 * 365 * 86400, n).astype("timedelta64[s]"))
    strs = np.char.add(np.char.replace(np.datetime_as_string(ts, unit="s"), "T", " "), " UTC")
    return pa.table({
        "i32": pa.array(rng.integers(-50, 50, n).astype(np.int32), mask=mask()),
        "i64": pa.array(rng.integers(-10 ** 6, 10 ** 6, n), mask=mask()),
        "f32": pa.array(rng.normal(size=n).astype(np.float32), mask=mask()),
        "f64": pa.array(np.where(rng.random(n) < 0.02, np.nan, rng.normal(scale=30, size=n)),
                        mask=mask()),
        "b": pa.array(rng.random(n) < 0.5, mask=mask()),
        "ts": pa.array(ts.astype("datetime64[ms]"), mask=mask()),
        "s": pa.array(strs, mask=mask()),
        "name": pa.array([f"k{i % 7}" for i in range(n)]),
    })


@pytest.fixture
def spark(spark_session):
    spark_session.conf.set("spark.sql.session.timeZone", "UTC")
    return spark_session


def test_arithmetic_compare_logic_with_nulls(spark, monkeypatch):
    df = spark.createDataFrame(_table())
    df = df.withColumn("a", col("i32") + col("i64")) \
        .withColumn("b2", col("i32") * 3 - col("f32")) \
        .withColumn("c", col("f64") / col("i32")) \
        .withColumn("d", col("f64") % 7.5) \
        .withColumn("e", -col("f32") + 1.5) \
        .withColumn("g", F.abs(col("i64") - 17)) \
        .withColumn("h", F.sqrt(F.abs(col("f64")))) \
        .withColumn("k", (col("i32") > 3) & (col("f64") <= 10.0) | col("b")) \
        .withColumn("m", ~col("b") | col("f32").isNull()) \
        .withColumn("p", col("i32").eqNullSafe(col("i64"))) \
        .withColumn("q", F.isnan(col("f64"))) \
        .withColumn("r", col("f32") ** 2) \
        .withColumn("one", lit(1)) \
        .withColumn("i32", col("i32") + 1)
    d = _same(df, monkeypatch)
    assert d["fused_partitions"] > 0 and d["fallback_partitions"] == 0


def test_filters_then_projections(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=1))
    df = df.filter(col("f64") > -20).filter(col("i32") != 0).filter(col("b") | col("i64").isNull()) \
        .withColumn("x", col("f64") * col("i32")) \
        .filter(col("x") < 100) \
        .select("name", "x", (col("i64") + 1).alias("y"), col("ts"), col("s")) \
        .drop("s")
    d = _same(df, monkeypatch)
    assert d["fused_partitions"] > 0


def test_datetime_fields_from_strings_and_timestamps(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=2))
    for name, f in [("year", F.year), ("month", F.month), ("day", F.dayofmonth),
                    ("hour", F.hour), ("minute", F.minute), ("second", F.second),
                    ("dow", F.dayofweek), ("woy", F.weekofyear), ("q", F.quarter),
                    ("doy", F.dayofyear)]:
        df = df.withColumn("s_" + name, f(col("s"))).withColumn("t_" + name, f(col("ts")))
    df = df.filter(col("s_hour") > 3).withColumn("late", F.hour(col("s")) - 2)
    d = _same(df, monkeypatch)
    assert d["fused_partitions"] > 0


def test_casts_and_case_when(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=3))
    df = df.withColumn("fi", col("f64").cast("int")) \
        .withColumn("fl", col("f32").cast("bigint")) \
        .withColumn("if", col("i32").cast("double")) \
        .withColumn("bi", col("b").cast("int")) \
        .withColumn("ff", col("f64").cast("float")) \
        .withColumn("ib", col("i64").cast("boolean")) \
        .withColumn("cw", F.when(col("i32") > 10, col("i64")).when(col("b"), 5).otherwise(col("i32"))) \
        .withColumn("cn", F.when(col("f64") > 0, col("f64")))
    _same(df, monkeypatch)


def test_nyc_etl_chain_matches(spark, monkeypatch, tmp_path):
    import bench
    from data_process import nyc_taxi_preprocess
    p = str(tmp_path / "nyc.csv")
    bench.make_csv(p, 3000, 7)
    df = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load("file://" + p)
    df = nyc_taxi_preprocess(df)
    d = _same(df, monkeypatch)
    assert d["fused_partitions"] > 0 and d["fallback_partitions"] == 0
    # the whole 35-operator chain is one VM segment (no host operators)
    nodes, base = exprc.chain_of(df._plan)
    segs = exprc.segments_for(df._plan, nodes, base)
    assert [s[0] for s in segs] == ["vm"]


@udf("int")
def _night(hour, weekday):
    if ((16 <= hour <= 20) and (weekday < 5)):
        return int(1)
    else:
        return int(0)


@udf("float")
def _dist(a, b, c, d):
    return float(np.abs(c - a) + math.fabs(d - b))


@udf("double")
def _mixed(x, y):
    z = x * 2 + 1
    return min(z, y) if x > 0 else max(z // 3, y % 4)


@udf("string")
def _label(x):
    return "big" if x > 0 else "small"


def test_udfs_inline_and_host(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=4, nulls=False))
    df = df.withColumn("n", _night(F.hour(col("s")), F.dayofweek(col("s")) - 2)) \
        .withColumn("dd", _dist("f64", "f32", lit(-74.0), lit(40.7))) \
        .filter(col("dd") < 80) \
        .withColumn("mx", _mixed("i64", "f64")) \
        .withColumn("lab", _label("f64"))          # string UDF after a filter: host operator
    d = _same(df, monkeypatch)
    assert d["fused_partitions"] > 0
    nodes, base = exprc.chain_of(df._plan)
    kinds = [s[0] for s in exprc.segments_for(df._plan, nodes, base)]
    assert kinds == ["vm", "host"]


@udf("int")
def _is3(x):
    return 1 if x == 3 else 0      # compilable, and defined for None (Python: None == 3 is False)


def test_udf_null_arguments_take_row_path(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=5, nulls=True))
    df = df.withColumn("e3", _is3("i32"))
    ref = _collect(df, False, monkeypatch)
    before = exprc.STATS["fallback_partitions"]
    got = _collect(df, True, monkeypatch)
    assert exprc.STATS["fallback_partitions"] > before
    assert all(_equal(ref.column(n).combine_chunks(), got.column(n).combine_chunks())
               for n in ref.column_names)


def _complexish(x):
    return x ** 0.5


def test_python_raising_rows_take_the_row_path(spark, monkeypatch):
    # numpy gives NaN for a negative base, Python a complex number (an error for a double UDF):
    # the compile-time guard (base >= 0 of a fractional power) sends the partition holding the
    # negative row to the per-row path, which raises like Spark would
    u = udf(_complexish, "double")
    t = pa.table({"x": pa.array(np.concatenate([np.linspace(1, 9, 50), [-4.0]]))})
    df = spark.createDataFrame(t).withColumn("r", u("x"))
    monkeypatch.setenv("RAYDP_FUSED_ETL", "1")
    before = exprc.STATS["udf_guard_fallbacks"]
    with pytest.raises((TypeError, pa.ArrowInvalid)):
        [df._plan.compute(i) for i in range(df._plan.num_partitions())]
    assert exprc.STATS["udf_guard_fallbacks"] > before


def _ratio(a, b):
    return a / b + a // b + a % b


def test_zero_divisor_mid_range_takes_the_row_path(spark, monkeypatch):
    """A zero divisor in the middle of the value range (never a sampled extreme) must not come
    back as inf/nan: Python raises ZeroDivisionError there."""
    u = udf(_ratio, "double")
    x = np.arange(-3, 4, dtype=np.int64).repeat(30)          # divisor -3..3, zeros mid-range
    t = pa.table({"a": pa.array(np.arange(len(x), dtype=np.int64) + 7), "b": pa.array(x)})
    df = spark.createDataFrame(t).withColumn("r", u("a", "b"))
    monkeypatch.setenv("RAYDP_FUSED_ETL", "1")
    before = exprc.STATS["udf_guard_fallbacks"]
    with pytest.raises(Exception) as ei:
        [df._plan.compute(i) for i in range(df._plan.num_partitions())]
    assert "ZeroDivision" in repr(ei.value) or "division" in str(ei.value)
    assert exprc.STATS["udf_guard_fallbacks"] > before
    # without zeros the same UDF stays inlined and matches the row path exactly
    t2 = pa.table({"a": pa.array(np.arange(200, dtype=np.int64) - 50),
                   "b": pa.array(np.where(np.arange(200) % 2, 3, -2).astype(np.int64))})
    d = _same(spark.createDataFrame(t2).withColumn("r", u("a", "b")), monkeypatch)
    assert d["fused_partitions"] > 0


LIMIT = 100.0


def _clip(x):
    return x if x < LIMIT else -x


def test_udf_verification_follows_new_value_ranges(spark, monkeypatch):
    """Partitions inside the value range already checked at a call site only get spread rows
    checked; a later partition that leaves that range has its extreme rows checked. Here the
    Python function's behaviour changes above x = 5 after compilation (a module global the
    compiled program captured), which only rows beyond the checked range expose: the
    mismatch is caught there and the UDF retired to the row path."""
    global LIMIT
    u = udf(_clip, "double")
    good = np.linspace(1, 4.9, 200)
    monkeypatch.setenv("RAYDP_FUSED_ETL", "1")
    before = exprc.STATS["udf_retired"]

    def run(t):   # same chain structure: the same compiled program (and checked ranges) serves all
        df = spark.createDataFrame(t).withColumn("r", u("x"))
        return pa.concat_tables([df._plan.compute(i) for i in range(df._plan.num_partitions())])
    try:
        for t in (pa.table({"x": pa.array(good)}), pa.table({"x": pa.array(good[::-1].copy())})):
            np.testing.assert_allclose(np.asarray(run(t).column("r")), np.asarray(t.column("x")))
        assert exprc.STATS["udf_retired"] == before
        LIMIT = 5.0
        t3 = pa.table({"x": pa.array(np.concatenate([good[:150], [9.0], good[150:]]))})
        r = np.asarray(run(t3).column("r"))
        assert r[150] == -9.0            # the row path's answer, not the stale program's
        assert exprc.STATS["udf_retired"] > before
    finally:
        LIMIT = 100.0


def test_all_rows_filtered_and_empty_input(spark, monkeypatch):
    df = spark.createDataFrame(_table(seed=6)).filter(col("i32") > 1000).withColumn("z", col("f64") + 1)
    _same(df, monkeypatch)
    empty = spark.createDataFrame(_table(seed=6).slice(0, 0)).withColumn("z", col("f64") * 2) \
        .filter(col("z") > 0)
    _same(empty, monkeypatch)


def test_program_register_reuse_is_safe():
    """Widening casts and selects never write a register that one of their operands occupies."""
    t = pa.table({"a": pa.array(np.arange(3000, dtype=np.int32)),
                  "c": pa.array(np.arange(3000) % 3 == 0)})
    cc = exprc._ChainCompiler(t.schema)
    from raydp_amd.spark.column import BinOp, Cast, ColRef, CaseWhen, Lit
    from raydp_amd.spark.types import parse_type_string
    cc.op(("with", "w", Cast(ColRef("a"), parse_type_string("double"))))
    cc.op(("with", "s", CaseWhen([(ColRef("c"), BinOp("+", ColRef("a"), Lit(1)))], ColRef("a"))))
    prog = cc.finish()
    out = prog.run(t)
    np.testing.assert_array_equal(out.column("w").to_numpy(), np.arange(3000, dtype=np.float64))
    want = np.where(np.arange(3000) % 3 == 0, np.arange(3000) + 1, np.arange(3000))
    np.testing.assert_array_equal(out.column("s").to_numpy(), want)


def test_small_csv_inference_parse_is_the_partition(tmp_path):
    """A single-split file parsed whole by schema inference ships that parse as its partition;
    it must equal what the task-side parse with the inferred schema produces."""
    import os
    import bench
    from raydp_amd.spark.sources import CsvSource
    for p in (str(tmp_path / "nyc.csv"), os.path.join(os.path.dirname(bench.__file__), "examples",
                                                       "data", "fake_nyctaxi.csv")):
        if not os.path.exists(p):
            bench.make_csv(p, 2000, 11)
        src = CsvSource(p, header=True, infer_schema=True)
        assert 0 in src._parsed
        fast = src.load(0)
        src._parsed.clear()
        slow = src.load(0)
        assert fast.schema == slow.schema and fast.equals(slow)


@pytest.mark.parametrize("how", ["left", "inner"])
def test_broadcast_lookup_join_matches_hash_join(spark, monkeypatch, how):
    """Dimension-table joins run as a narrow hash lookup (left order kept); rows, values and
    nulls must equal Arrow's hash join (compared order-insensitively)."""
    rng = np.random.default_rng(3)
    n = 3000
    keys = np.array([f"v{i}" for i in range(60)], dtype=object)
    left = pa.table({"k": pa.array(keys[rng.integers(0, 60, n)], mask=rng.random(n) < 0.05),
                     "x": pa.array(rng.normal(size=n))})
    dim = pa.table({"k": pa.array(keys[:40]), "id": pa.array(np.arange(40, dtype=np.int64))})
    out = spark.createDataFrame(left).join(spark.createDataFrame(dim), "k", how=how)
    plan = out._plan
    from raydp_amd.spark.plan import get_scheduler, prepare
    prepare(plan, get_scheduler())
    assert plan._broadcast is not None
    got = pa.concat_tables([plan.compute(i) for i in range(plan.num_partitions())])
    ref = pa.concat_tables([plan._join(plan.left.compute(i), plan._broadcast)
                            for i in range(plan.num_partitions())])
    assert got.schema == ref.schema
    key = [("x", "ascending")]
    assert got.sort_by(key).equals(ref.sort_by(key))


@pytest.mark.parametrize("how", ["inner", "left", "right", "outer", "left_semi", "left_anti"])
@pytest.mark.parametrize("same_keys", [True, False])
def test_static_join_schema_matches_arrow_join(spark, how, same_keys):
    left = pa.table({"k": pa.array([1, 2, 3], pa.int64()), "x": pa.array([1.0, 2.0, 3.0]),
                     "s": pa.array(["a", "b", "c"])})
    right = pa.table({("k" if same_keys else "rk"): pa.array([2, 3, 4], pa.int64()),
                      "y": pa.array([5, 6, 7], pa.int32()), "s2": pa.array(["u", "v", "w"])})
    a, b = spark.createDataFrame(left), spark.createDataFrame(right)
    on = "k" if same_keys else (a["k"] == b["rk"])
    plan = a.join(b, on, how=how)._plan
    ran = plan._join(plan.left.schema.empty_table(), plan.right.schema.empty_table()).schema
    st = plan.static_schema()
    assert st is None or st == ran
    assert plan.schema == ran


def test_adaptive_repartition_coalesces_buckets_and_keeps_keys_together(spark):
    rng = np.random.default_rng(9)
    t = pa.table({"k": pa.array(rng.integers(0, 500, 20000)), "v": pa.array(rng.normal(size=20000))})
    df = spark.createDataFrame(t).repartition("k")             # 200 requested, tiny data
    parts = df._session._run(df._src())
    assert 1 <= len(parts) < 200 and len(parts) == df._src().num_partitions()
    assert sum(p.num_rows for p in parts) == 20000
    seen = {}
    for j, p in enumerate(parts):
        for k in set(p.column("k").to_pylist()):
            assert seen.setdefault(k, j) == j                  # every key in exactly one partition
    # an explicit count is honoured, and so is a count someone sized itself on beforehand
    assert spark.createDataFrame(t).repartition(7, "k")._src().num_partitions() == 7
    df2 = spark.createDataFrame(t).repartition("k")
    n_seen = df2._src().num_partitions()          # sized on before the shuffle ran
    assert len(df2._session._run(df2._src())) == n_seen == 200
    df3 = spark.createDataFrame(t).repartition("k")
    assert df3.rdd.getNumPartitions() == len(df3._session._run(df3._src())) < 200


def test_map_output_travels_as_one_table():
    import pickle
    from raydp_amd.spark.plan import MapOutput, hash_partition
    t = pa.table({"k": pa.array(np.arange(1000) % 37), "v": pa.array(np.arange(1000.0))})
    mo = hash_partition(t, ["k"], 16)
    assert isinstance(mo, MapOutput) and len(mo) == 16
    assert sum(b.num_rows for b in mo) == 1000
    back = pickle.loads(pickle.dumps(mo))
    assert all(a.equals(b) for a, b in zip(mo, back))
