"""Spark SQL statements (raydp_amd/spark/sql.py) against the same computation written with the
DataFrame API. Reference flow: doc/spark_on_ray.md:187-201 (Hive tables through
``spark.sql("select * from db.xxx")`` on a Spark-on-Ray session)."""
import numpy as np
import pyarrow as pa
import pytest

from raydp_amd.spark import functions as F


@pytest.fixture
def spark(spark_session, tmp_path):
    spark_session.conf.set("spark.sql.warehouse.dir", str(tmp_path / "warehouse"))
    spark_session.conf.set("spark.sql.session.timeZone", "UTC")
    yield spark_session
    for v in list(spark_session._catalog):
        spark_session._catalog.pop(v, None)
    if hasattr(spark_session, "_sql_catalog"):
        del spark_session._sql_catalog


def _sales(spark):
    rng = np.random.default_rng(0)
    n = 400
    t = pa.table({"store": pa.array(rng.integers(0, 7, n)), "item": pa.array([f"i{k}" for k in rng.integers(0, 5, n)]),
                  "qty": pa.array(rng.integers(1, 10, n)), "price": pa.array(np.round(rng.uniform(1, 20, n), 2))})
    df = spark.createDataFrame(t)
    df.createOrReplaceTempView("sales")
    stores = spark.createDataFrame(pa.table({"store": pa.array(np.arange(6)),
                                             "city": pa.array(["a", "b", "c", "a", "b", "d"])}))
    stores.createOrReplaceTempView("stores")
    return df, stores


def _rows(df, key=None):
    rows = [tuple(r) for r in df.collect()]
    return sorted(rows, key=key or (lambda r: tuple(str(x) for x in r)))


def test_select_where_order_limit(spark):
    df, _ = _sales(spark)
    got = spark.sql("SELECT store, item, qty * price AS amount FROM sales "
                    "WHERE qty > 3 AND item <> 'i2' ORDER BY amount DESC, store LIMIT 15")
    want = df.filter((F.col("qty") > 3) & (F.col("item") != "i2")) \
        .select("store", "item", (F.col("qty") * F.col("price")).alias("amount")) \
        .orderBy(F.col("amount").desc(), "store").limit(15)
    assert got.columns == ["store", "item", "amount"]
    assert [tuple(r) for r in got.collect()] == [tuple(r) for r in want.collect()]


def test_group_by_having_aggregates(spark):
    df, _ = _sales(spark)
    got = spark.sql("""
        SELECT store, count(*) AS n, sum(qty) AS total, round(avg(price), 3) AS avg_price
        FROM sales GROUP BY store HAVING sum(qty) > 100 AND count(*) >= 10 ORDER BY total DESC""")
    want = df.groupBy("store").agg(F.count(F.lit(1)).alias("n"), F.sum("qty").alias("total"),
                                   F.round(F.avg("price"), 3).alias("avg_price")) \
        .filter((F.col("total") > 100) & (F.col("n") >= 10)).orderBy(F.col("total").desc())
    assert [tuple(r) for r in got.collect()] == [tuple(r) for r in want.collect()]
    # HAVING on a select alias, ORDER BY an aggregate that is not selected, a grouping expression
    got2 = spark.sql("SELECT item, max(price) AS top FROM sales GROUP BY item HAVING top > 5 "
                     "ORDER BY sum(qty) DESC")
    w2 = df.groupBy("item").agg(F.max("price").alias("top"), F.sum("qty").alias("q")) \
        .filter(F.col("top") > 5).orderBy(F.col("q").desc()).select("item", "top")
    assert [tuple(r) for r in got2.collect()] == [tuple(r) for r in w2.collect()]
    got3 = spark.sql("SELECT store % 2 AS parity, count(*) AS c FROM sales GROUP BY store % 2 ORDER BY parity")
    w3 = df.groupBy((F.col("store") % 2).alias("parity")).agg(F.count(F.lit(1)).alias("c")).orderBy("parity")
    assert [tuple(r) for r in got3.collect()] == [tuple(r) for r in w3.collect()]


@pytest.mark.parametrize("how,sql", [("inner", "JOIN"), ("left", "LEFT OUTER JOIN"), ("left_semi", "LEFT SEMI JOIN"),
                                     ("left_anti", "LEFT ANTI JOIN")])
def test_joins(spark, how, sql):
    df, stores = _sales(spark)
    cols = "s.*, t.city" if how in ("inner", "left") else "s.*"
    got = spark.sql(f"SELECT {cols} FROM sales s {sql} stores t ON s.store = t.store")
    want = df.join(stores, "store", how)
    assert sorted(got.columns) == sorted(want.columns)
    assert _rows(got.select(*sorted(got.columns))) == _rows(want.select(*sorted(want.columns)))


def test_join_using_and_aggregate_over_join_with_cte(spark):
    df, stores = _sales(spark)
    got = spark.sql("""
        WITH big AS (SELECT * FROM sales WHERE qty >= 5)
        SELECT city, sum(qty * price) AS revenue FROM big JOIN stores USING (store)
        GROUP BY city ORDER BY city""")
    want = df.filter(F.col("qty") >= 5).join(stores, "store") \
        .groupBy("city").agg(F.sum(F.col("qty") * F.col("price")).alias("revenue")).orderBy("city")
    g, w = [tuple(r) for r in got.collect()], [tuple(r) for r in want.collect()]
    assert [r[0] for r in g] == [r[0] for r in w]
    np.testing.assert_allclose([r[1] for r in g], [r[1] for r in w], rtol=1e-12)


def test_union_distinct_subquery_and_case(spark):
    df, _ = _sales(spark)
    got = spark.sql("""
        SELECT DISTINCT item FROM (SELECT item FROM sales WHERE store < 2
                                   UNION ALL SELECT item FROM sales WHERE store > 4) x ORDER BY item""")
    want = df.filter(F.col("store") < 2).select("item").union(df.filter(F.col("store") > 4).select("item")) \
        .distinct().orderBy("item")
    assert [tuple(r) for r in got.collect()] == [tuple(r) for r in want.collect()]
    got2 = spark.sql("SELECT store, CASE WHEN qty > 5 THEN 'hi' ELSE 'lo' END AS band, CAST(price AS INT) AS p "
                     "FROM sales WHERE store IN (1, 3) AND price BETWEEN 2 AND 9")
    want2 = df.filter(F.col("store").isin([1, 3]) & (F.col("price") >= 2) & (F.col("price") <= 9)) \
        .select("store", F.when(F.col("qty") > 5, "hi").otherwise("lo").alias("band"),
                F.col("price").cast("int").alias("p"))
    assert _rows(got2) == _rows(want2)


def test_hive_style_tables_persist_in_the_warehouse(spark, tmp_path):
    """doc/spark_on_ray.md:187-201: create a database and a table, then
    spark.sql("select * from db.xxx") -- the table lives in the warehouse directory, so a new
    session (same warehouse) reads it too."""
    df, _ = _sales(spark)
    spark.sql("CREATE DATABASE IF NOT EXISTS db")
    spark.sql("CREATE TABLE db.xxx AS SELECT store, sum(qty) AS q FROM sales GROUP BY store")
    assert (tmp_path / "warehouse" / "db.db" / "xxx").is_dir()
    got = spark.sql("select * from db.xxx order by store")
    want = df.groupBy("store").agg(F.sum("qty").alias("q")).orderBy("store")
    assert [tuple(r) for r in got.collect()] == [tuple(r) for r in want.collect()]
    assert ("db", "xxx", False) in [tuple(r) for r in spark.sql("SHOW TABLES IN db").collect()]
    assert "db" in [r[0] for r in spark.sql("SHOW DATABASES").collect()]
    # saveAsTable + insertInto + INSERT INTO, then a fresh catalog (a new session) reads it
    df.filter(F.col("store") == 0).write.saveAsTable("s0")
    with pytest.raises(ValueError):
        df.write.saveAsTable("s0")                       # errorifexists
    spark.sql("INSERT INTO s0 SELECT * FROM sales WHERE store = 1")
    n01 = df.filter(F.col("store") <= 1).count()
    del spark._sql_catalog
    spark._catalog.clear()
    assert spark.table("s0").count() == n01
    assert spark.sql("SELECT count(*) AS c FROM s0").collect()[0][0] == n01
    spark.sql("USE db")
    assert spark.sql("SELECT count(*) FROM xxx").collect()[0][0] == 7
    spark.sql("USE default")
    spark.sql("CREATE OR REPLACE TEMP VIEW v AS SELECT store FROM s0 WHERE store = 1")
    assert spark.sql("select * from v").count() == df.filter(F.col("store") == 1).count()
    spark.sql("DROP VIEW v")
    spark.sql("DROP TABLE IF EXISTS s0")
    assert not spark.tableExists("s0")
    desc = spark.sql("DESCRIBE db.xxx").collect()
    assert [r[0] for r in desc] == ["store", "q"]
    spark.sql("DROP DATABASE db CASCADE")
    assert not (tmp_path / "warehouse" / "db.db").exists()


def _pairs(spark):
    rng = np.random.default_rng(3)
    ta = pa.table({"k": pa.array(rng.integers(0, 6, 50)), "j": pa.array(rng.integers(0, 6, 50)),
                   "va": pa.array(np.arange(50))})
    tb = pa.table({"k": pa.array(rng.integers(0, 6, 40)), "j": pa.array(rng.integers(0, 6, 40)),
                   "vb": pa.array(np.arange(100, 140))})
    spark.createDataFrame(ta).createOrReplaceTempView("ta")
    spark.createDataFrame(tb).createOrReplaceTempView("tb")
    return ta.to_pandas(), tb.to_pandas()


@pytest.mark.parametrize("on", ["b.k = a.j", "a.j = b.k"])
def test_join_on_resolves_sides_by_qualifier(spark, on):
    # both tables have k and j: a bare-name guess would join a.k = b.j instead of a.j = b.k
    pa_, pb = _pairs(spark)
    got = spark.sql(f"SELECT a.va, b.vb FROM ta a JOIN tb b ON {on}")
    want = pa_.merge(pb, left_on="j", right_on="k")
    assert sorted((int(r[0]), int(r[1])) for r in got.collect()) == \
        sorted(zip(want["va"].tolist(), want["vb"].tolist()))


def test_self_join_on_qualified_columns(spark):
    pa_, _ = _pairs(spark)
    got = spark.sql("SELECT count(*) AS n FROM ta x JOIN ta y ON x.j = y.k")
    assert int(got.collect()[0][0]) == len(pa_.merge(pa_, left_on="j", right_on="k"))


def test_join_on_ambiguous_bare_name_raises(spark):
    from raydp_amd.spark.sql import SqlError
    _pairs(spark)
    with pytest.raises(SqlError, match="ambiguous"):
        spark.sql("SELECT a.va FROM ta a JOIN tb b ON k = j").collect()
    with pytest.raises(SqlError, match="unknown qualifier"):
        spark.sql("SELECT a.va FROM ta a JOIN tb b ON c.k = a.j").collect()


def test_dataframe_join_with_residual_condition(spark_session):
    """``a.join(b, (a.k == b.k) & (a.x < b.y))``: the equality is the hash key, the rest decides
    which key-matched pairs match -- for inner, outer, semi and anti joins (Spark semantics), and
    the same rows as the SQL front end's ``JOIN ... ON a.k = b.k AND a.x < b.x``."""
    s = spark_session
    a = s.createDataFrame([(1, 1.0, "a"), (1, 5.0, "b"), (2, 3.0, "c"), (3, 9.0, "d")], ["k", "x", "la"])
    b = s.createDataFrame([(1, 2.0, "p"), (2, 1.0, "q"), (2, 4.0, "r"), (4, 0.0, "z")], ["k", "x", "lb"])

    def rows(df):
        return sorted(map(tuple, df.collect()), key=str)
    cond = (a.k == b.k) & (a.x < b["x"])
    assert rows(a.join(b, cond)) == [(1, 1.0, "a", 2.0, "p"), (2, 3.0, "c", 4.0, "r")]
    assert rows(a.join(b, cond, "left")) == [(1, 1.0, "a", 2.0, "p"), (1, 5.0, "b", None, None),
                                             (2, 3.0, "c", 4.0, "r"), (3, 9.0, "d", None, None)]
    assert rows(a.join(b, cond, "right")) == [(1, 1.0, "a", 2.0, "p"), (2, 3.0, "c", 4.0, "r"),
                                              (2, None, None, 1.0, "q"), (4, None, None, 0.0, "z")]
    assert len(rows(a.join(b, cond, "full"))) == 6
    assert rows(a.join(b, cond, "left_semi")) == [(1, 1.0, "a"), (2, 3.0, "c")]
    assert rows(a.join(b, cond, "left_anti")) == [(1, 5.0, "b"), (3, 9.0, "d")]
    # distinct-named residual columns need no side
    c = b.withColumnRenamed("x", "y")
    assert rows(a.join(c, [a.k == c.k, a.x < c.y]).select("la", "lb")) == [("a", "p"), ("c", "r")]
    a.createOrReplaceTempView("ja")
    b.createOrReplaceTempView("jb")
    sql = s.sql("SELECT ja.la, jb.lb FROM ja JOIN jb ON ja.k = jb.k AND ja.x < jb.x")
    assert rows(sql) == [("a", "p"), ("c", "r")]
