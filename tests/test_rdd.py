"""RDD API on executor processes (sc.parallelize, narrow/wide transformations, df.rdd, toDF)."""


def test_rdd_ops(spark_on_ray_2_executors):
    sc = spark_on_ray_2_executors.sparkContext
    r = sc.parallelize(range(100), 4)
    assert r.getNumPartitions() == 4
    assert r.map(lambda x: x * 2).filter(lambda x: x % 3 == 0).sum() == sum(x * 2 for x in range(100) if (x * 2) % 3 == 0)
    assert r.flatMap(lambda x: [x, x]).count() == 200
    assert sorted(r.map(lambda x: (x % 5, 1)).reduceByKey(lambda a, b: a + b).collect()) == [(k, 20) for k in range(5)]
    g = dict(r.map(lambda x: ("k%d" % (x % 3), x)).groupByKey().mapValues(len).collect())
    assert g == {"k0": 34, "k1": 33, "k2": 33}
    assert sorted(sc.parallelize([1, 1, 2, 3, 3, 3]).distinct().collect()) == [1, 2, 3]
    assert r.reduce(lambda a, b: a + b) == 4950
    assert r.take(3) == [0, 1, 2] and r.first() == 0
    assert r.repartition(7).getNumPartitions() == 7 and r.repartition(7).count() == 100
    assert r.coalesce(2).glom().map(len).collect() == [50, 50]
    assert r.zipWithIndex().filter(lambda xi: xi[0] != xi[1]).count() == 0
    assert r.sortBy(lambda x: -x).take(2) == [99, 98]
    assert r.mapPartitionsWithIndex(lambda i, it: [(i, sum(1 for _ in it))]).collect() == [(0, 25), (1, 25), (2, 25), (3, 25)]
    c = r.map(lambda x: x + 1).cache()
    assert c.is_cached and c.count() == 100


def test_rdd_dataframe_roundtrip(spark_on_ray_2_executors):
    spark = spark_on_ray_2_executors
    sc = spark.sparkContext
    rows = sc.parallelize([("a", 1, 2.5), ("b", 2, None), ("c", 3, 1.0)], 2)
    df = spark.createDataFrame(rows, ["name", "n", "v"])
    assert df.count() == 3
    assert [r.name for r in df.orderBy("n").collect()] == ["a", "b", "c"]
    df2 = rows.toDF(["x", "y", "z"])
    assert df2.columns == ["x", "y", "z"]
    back = df.rdd.map(lambda row: row.n * 10).collect()
    assert sorted(back) == [10, 20, 30]
    assert df.rdd.getNumPartitions() == 2
