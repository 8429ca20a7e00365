"""Native executor core (``csrc/exec/executor.cc`` via ``raydp_amd/spark/native_exec.py``;
reference ``RayDPExecutor.scala``): a lowered stage's partitions run on the C++ task loop and
must produce exactly what the Python path (``plan.compute``) produces -- CSV byte splits,
in-memory sources, filters, datetime fields, inlined UDFs through the bridge -- and anything
the loop cannot reproduce exactly must come back as a fallback, never as a different result."""
import os
import uuid

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import pytest

import raydp  # noqa: F401
from raydp_amd.spark import exprc, native_exec


@pytest.fixture
def store():
    from raydp_amd.runtime.store import SharedObjectStore
    st = SharedObjectStore(f"/dev/shm/rxnt_{uuid.uuid4().hex[:10]}", "n0", True, 64 << 20)
    yield st
    st.destroy()


@pytest.fixture
def spark():
    from raydp_amd.spark.session import SparkSession
    s = SparkSession.builder.master("local[2]").appName("native-exec").getOrCreate()
    yield s
    s.stop()


def _csv(tmp_path, n=6000, seed=0, bad_ts=False):
    rng = np.random.default_rng(seed)
    ts = pa.array(rng.integers(1_200_000_000, 1_400_000_000, n), pa.timestamp("s")).cast(pa.string())
    tss = [s + " UTC" for s in ts.to_pylist()]
    if bad_ts:
        tss[n // 2] = "2012-02-30 10:00:00"      # not a date: strptime decides (null)
    a = rng.integers(-50, 50, n).astype(object)
    a[::97] = None                                 # nulls through the VM and the gather
    t = pa.table({"a": pa.array(list(a), pa.int64()), "b": rng.standard_normal(n),
                  "s": pa.array([f"x{i % 7}" * (i % 3 + 1) for i in range(n)]), "t": pa.array(tss)})
    p = os.path.join(str(tmp_path), "d.csv")
    pacsv.write_csv(t, p)
    return p


def _run_all(low, fn, store, nparts):
    ex = native_exec.NativeExecutor(3)
    try:
        statuses = []
        subs = []
        for i in range(nparts):
            oid = uuid.uuid4().hex
            tid, keep = ex.submit(low, i, store, oid)
            assert tid > 0, keep
            subs.append((i, tid, oid, keep))
        for i, tid, oid, _ in subs:
            st, rows, nbytes, err = ex.wait(tid)
            statuses.append(st)
            want = fn(i)
            if st == native_exec.OK:
                ok, got = store.get(oid)
                assert ok and got.num_rows == rows
                assert got.schema == want.schema, (got.schema, want.schema)
                assert got.equals(want), i
            else:
                assert st in (native_exec.FALLBACK, native_exec.RETRY), err
        return statuses, ex.stats()
    finally:
        ex.close()


def _etl(df):
    import raydp_amd.spark.functions as F
    return (df.filter(F.col("a") > -20)
              .withColumn("c", F.col("a") * 2 + F.col("b"))
              .withColumn("h", F.hour(F.col("t")))
              .withColumn("dow", F.dayofweek(F.col("t")))
              .withColumn("y", F.year(F.col("t")))
              .filter(F.col("b") < 1.5)
              .drop("b"))


def test_csv_splits_run_natively_and_match(spark, tmp_path, store):
    spark.conf.set("spark.sql.files.maxPartitionBytes", str(40 << 10))
    df = _etl(spark.read.csv(_csv(tmp_path), header=True, inferSchema=True))
    plan = df._src()
    n = plan.num_partitions()
    assert n >= 4
    low = native_exec.lower(plan.compute)
    assert low is not None and low.csv is not None          # CSV byte splits parsed in C++
    statuses, stats = _run_all(low, plan.compute, store, n)
    assert statuses == [native_exec.OK] * n
    assert stats["ok"] == n and stats["rows"] == sum(plan.compute(i).num_rows for i in range(n))


def test_in_memory_source_goes_through_the_c_stream(spark, store):
    import pandas as pd
    import raydp_amd.spark.functions as F
    rng = np.random.default_rng(1)
    pdf = pd.DataFrame({"x": rng.standard_normal(3000), "k": rng.integers(0, 9, 3000),
                        "name": [f"n{i}" for i in range(3000)]})
    df = spark.createDataFrame(pdf)
    df = df.withColumn("z", F.col("x") * F.col("k")).filter(F.col("k") != 3).withColumn("w", F.abs(F.col("z")))
    plan = df._src()
    low = native_exec.lower(plan.compute)
    assert low is not None and low.csv is None
    statuses, _ = _run_all(low, plan.compute, store, plan.num_partitions())
    assert statuses and all(s == native_exec.OK for s in statuses)


def test_inlined_udf_is_checked_through_the_bridge(spark, tmp_path, store):
    import raydp_amd.spark.functions as F
    from raydp_amd.spark.types import DoubleType

    def scale(a, b):
        return a * 0.5 + (b if b > 0 else -b)
    u = F.udf(scale, DoubleType())
    spark.conf.set("spark.sql.files.maxPartitionBytes", str(60 << 10))
    df = spark.read.csv(_csv(tmp_path, seed=2), header=True, inferSchema=True)
    df = df.filter(F.col("a").isNotNull()).withColumn("u", u(F.col("a"), F.col("b")))
    plan = df._src()
    low = native_exec.lower(plan.compute)
    assert low is not None and any(p.taps for p in low.progs), "the UDF should be inlined into the VM"
    statuses, _ = _run_all(low, plan.compute, store, plan.num_partitions())
    assert all(s == native_exec.OK for s in statuses)
    assert all(all(p.verified) for p in low.progs if p.taps)   # the Python checks ran via the bridge


def test_udf_guard_trip_falls_back_to_python(spark, store):
    import pandas as pd
    import raydp_amd.spark.functions as F
    from raydp_amd.spark.types import DoubleType

    def ratio(a, b):
        return a / b
    u = F.udf(ratio, DoubleType())
    pdf = pd.DataFrame({"a": np.arange(100, dtype=np.float64), "b": np.r_[np.ones(99), 0.0]})
    df = spark.createDataFrame(pdf).withColumn("r", u(F.col("a"), F.col("b")))
    plan = df._src()
    low = native_exec.lower(plan.compute)
    if low is None or not any(p.taps for p in low.progs):
        pytest.skip("division UDF not inlined")
    last = plan.num_partitions() - 1                  # the partition holding the zero divisor
    ex = native_exec.NativeExecutor(1)
    tid, _ = ex.submit(low, last, store, uuid.uuid4().hex)
    st, _, _, _ = ex.wait(tid)
    ex.close()
    assert st == native_exec.FALLBACK                 # the zero divisor trips the guard ...
    with pytest.raises(ZeroDivisionError):            # ... and Python fails the task, as Spark does
        plan.compute(last)


def test_unparseable_timestamp_falls_back(spark, tmp_path, store):
    spark.conf.set("spark.sql.files.maxPartitionBytes", str(1 << 30))
    df = _etl(spark.read.csv(_csv(tmp_path, n=800, bad_ts=True), header=True, inferSchema=True))
    plan = df._src()
    low = native_exec.lower(plan.compute)
    assert low is not None
    statuses, _ = _run_all(low, plan.compute, store, plan.num_partitions())
    assert statuses == [native_exec.FALLBACK]


def test_host_operator_is_not_lowered(spark):
    import raydp_amd.spark.functions as F
    df = spark.range(100).withColumn("s", F.concat(F.lit("a"), F.col("id").cast("string")))
    assert native_exec.lower(df._src().compute) is None


def test_partition_cache(store):
    ex = native_exec.NativeExecutor(1)
    for i in range(3):
        oid = uuid.uuid4().hex
        store.put(oid, pa.table({"x": [i]}))
        assert ex.cache_put("rddA", i, oid) is None
    oid_b = uuid.uuid4().hex
    store.put(oid_b, pa.table({"x": [9]}))
    ex.cache_put("rddB", 0, oid_b)
    assert ex.cache_list("rddA") == [0, 1, 2]
    assert sorted(ex.cached_rdds()) == ["rddA", "rddB"]
    a1 = ex.cache_get("rddA", 1)
    assert store.get(a1)[1].column("x").to_pylist() == [1]
    assert ex.cache_pop("rddA", 1) == a1 and ex.cache_get("rddA", 1) is None
    assert ex.cache_unpersist("rddA", store) == 2
    assert ex.cache_list("rddA") == [] and store.contains(oid_b)
    assert ex.cache_unpersist(None, store) == 1 and not store.contains(oid_b)
    ex.close()


def test_cluster_conversion_runs_on_the_native_loop(tmp_path):
    """End to end: executors persist a converted ETL DataFrame on their native task loops."""
    import ray
    import raydp_amd
    from raydp_amd.spark.session import SparkSession
    ray.shutdown()
    ray.init(num_cpus=4)
    try:
        spark = raydp_amd.init_spark("native", 2, 1, "300M",
                                     configs={"spark.sql.files.maxPartitionBytes": str(40 << 10)})
        df = _etl(spark.read.csv(_csv(tmp_path, seed=3), header=True, inferSchema=True))
        ds = raydp.spark.from_spark_recoverable(df)
        want = pa.concat_tables([df._src().compute(i) for i in range(df._src().num_partitions())])
        got = pa.concat_tables([ray.get(r) for b in ds.iter_internal_ref_bundles() for r, _ in b.blocks])
        assert got.equals(want)
        backend = SparkSession.getActiveSession()._cluster
        infos = ray.get([e.handle.info.remote() for e in backend.alive_executors()])
        assert sum(i["native_tasks"] for i in infos) == df._src().num_partitions()
        raydp_amd.stop_spark()
    finally:
        ray.shutdown()


def test_disabled_keeps_python_path(monkeypatch):
    monkeypatch.setenv("RAYDP_NATIVE_EXECUTOR", "0")
    assert not native_exec.enabled()
    assert exprc.TAPS_OK == native_exec.OK and exprc.TAPS_FALLBACK == native_exec.FALLBACK


def test_python_cache_fallback_has_the_same_interface(store):
    c = native_exec.PyCache()
    oid = uuid.uuid4().hex
    store.put(oid, pa.table({"x": [1]}))
    assert c.cache_put("r", 0, oid) is None and c.cache_get("r", 0) == oid
    assert c.cache_list("r") == [0] and c.cached_rdds() == ["r"]
    assert c.cache_unpersist("r", store) == 1 and not store.contains(oid)
    assert not c.available and native_exec.NativeExecutor.available


def test_lowered_stages_do_not_outlive_their_plans(spark, store):
    """The UDF bridge's key -> stage registry is weak: an executor that runs stage after stage
    keeps only the stages whose plans are still alive (it caches the last 16 stage functions),
    not every plan tree and C++ stage handle it ever lowered."""
    import gc

    import pandas as pd
    import raydp_amd.spark.functions as F
    before = len(native_exec._REGISTRY)
    keys = []
    for k in range(6):
        df = spark.createDataFrame(pd.DataFrame({"x": np.arange(100.0) + k}))
        plan = df.withColumn("y", F.col("x") * 2.0)._src()
        low = native_exec.lower(plan.compute)
        assert low is not None
        keys.append(low.key)
        statuses, _ = _run_all(low, plan.compute, store, plan.num_partitions())
        assert all(s == native_exec.OK for s in statuses)
        del df, plan, low
    gc.collect()
    assert not any(k in native_exec._REGISTRY for k in keys)
    assert len(native_exec._REGISTRY) <= before


def test_refit_of_the_same_chain_reuses_the_native_stage(spark, tmp_path, store):
    """A second pipeline of the same shape over new data compiles to the same cached segments:
    its lowering adopts the C++ stage built for the first one (no re-encode / re-create on the
    executor's critical path) and still produces exactly the Python path's result."""
    lows = []
    for seed in (3, 4):
        spark.conf.set("spark.sql.files.maxPartitionBytes", str(80 << 10))
        df = _etl(spark.read.csv(_csv(tmp_path, seed=seed), header=True, inferSchema=True))
        plan = df._src()
        before = native_exec.STATS["stage_reuse"]
        low = native_exec.lower(plan.compute)
        assert low is not None
        statuses, _ = _run_all(low, plan.compute, store, plan.num_partitions())
        assert all(s == native_exec.OK for s in statuses)
        lows.append((low, native_exec.STATS["stage_reuse"] - before))
    (a, _), (b, reused) = lows
    assert reused == 1 and a is not b and a.handle == b.handle and a.key != b.key
