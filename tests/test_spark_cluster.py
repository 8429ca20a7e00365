"""Spark-on-runtime cluster behaviour (port of the reference's
python/raydp/tests/test_spark_cluster.py and test_spark_master_memory.py).

Executors are real actor processes under the native supervisor; multi-node cases use the
virtual-node cluster (ray.cluster_utils.Cluster equivalent) with one store arena per node."""
import os
import time

import pyarrow
import pytest

import raydp  # noqa: F401  (installs the ray / pyspark facades when those are absent)
import ray
import raydp.utils as utils
from ray.cluster_utils import Cluster
from ray.util.placement_group import placement_group_table


@pytest.fixture
def local_rt():
    ray.shutdown()
    ray.init(num_cpus=6)
    yield
    raydp.stop_spark()
    ray.shutdown()


def test_spark(spark_on_ray_small):
    assert spark_on_ray_small.range(0, 10).count() == 10


def test_executors_are_processes(spark_on_ray_2_executors):
    from raydp_amd.spark.session import SparkSession
    backend = SparkSession.getActiveSession()._cluster
    infos = ray.get([e.handle.info.remote() for e in backend.alive_executors()])
    assert len({i["pid"] for i in infos}) == 2 and os.getpid() not in {i["pid"] for i in infos}
    assert ray.get_actor("raydp-executor-0") is not None
    assert ray.get_actor("test2_SPARK_MASTER") is not None


def test_legacy_spark_on_fractional_cpu():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 2})
    spark = raydp.init_spark(app_name="test_cpu_fraction", num_executors=1, executor_cores=3,
                             executor_memory="500M", configs={"spark.ray.actor.resource.cpu": "0.1"})
    assert spark.range(0, 10).count() == 10
    raydp.stop_spark()
    cluster.shutdown()


def test_spark_executor_on_fractional_cpu():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 2})
    spark = raydp.init_spark(app_name="test_cpu_fraction", num_executors=1, executor_cores=3,
                             executor_memory="500M",
                             configs={"spark.ray.raydp_spark_executor.actor.resource.cpu": "0.1"})
    assert spark.range(0, 10).count() == 10
    raydp.stop_spark()
    cluster.shutdown()


def test_spark_executor_node_affinity():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    node = cluster.add_node(num_cpus=2, resources={"spark_executor": 10})
    spark = raydp.init_spark(app_name="test_executor_node_affinity", num_executors=1, executor_cores=2,
                             executor_memory="500M",
                             configs={"spark.ray.raydp_spark_executor.actor.resource.spark_executor": "1"})
    assert spark.range(0, 10).count() == 10
    from ray.util.state import list_actors
    ex = [a for a in list_actors() if a.name == "raydp-executor-0"][0]
    assert ex.node_id == node.node_id and ex.required_resources["spark_executor"] == 1
    raydp.stop_spark()
    cluster.shutdown()


def test_spark_remote(local_rt):
    @ray.remote
    class SparkRemote:
        def __init__(self):
            import raydp as rdp
            self.spark = rdp.init_spark(app_name="test_spark_remote", num_executors=1, executor_cores=1,
                                        executor_memory="500MB")

        def run(self):
            return self.spark.range(0, 100).count()

        def stop(self):
            import raydp as rdp
            self.spark.stop()
            rdp.stop_spark()

    driver = SparkRemote.remote()
    assert ray.get(driver.run.remote()) == 100
    ray.get(driver.stop.remote())


def test_spark_driver_and_executor_hostname(spark_on_ray_small):
    conf = spark_on_ray_small.conf
    ip = ray.util.get_node_ip_address()
    assert conf.get("spark.driver.host") == ip
    assert conf.get("spark.driver.bindAddress") == ip


def test_ray_dataset_roundtrip():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 6})
    spark = raydp.init_spark(app_name="test_ray_dataset_roundtrip", num_executors=2, executor_cores=1,
                             executor_memory="500M")
    spark_df = spark.createDataFrame([(1, "a"), (2, "b"), (3, "c")], ["one", "two"])
    rows = [(r.one, r.two) for r in spark_df.take(3)]
    ds = ray.data.from_spark(spark_df)
    values = [(r["one"], r["two"]) for r in ds.take(6)]
    assert values == rows
    block_refs = [b for bundle in ds.iter_internal_ref_bundles() for b, _ in bundle.blocks]
    df = raydp.spark.dataset.ray_dataset_to_spark_dataframe(spark, ds.schema(), block_refs)
    assert [(r.one, r.two) for r in df.take(3)] == values
    raydp.stop_spark()
    cluster.shutdown()


def test_ray_dataset_to_spark(spark_on_ray_2_executors):
    spark = spark_on_ray_2_executors
    n = 5
    ds = ray.data.from_arrow(pyarrow.Table.from_pydict({"value": list(range(n))}))
    values = [r["value"] for r in ds.take(n)]
    refs = [b for bundle in ds.iter_internal_ref_bundles() for b, _ in bundle.blocks]
    df = raydp.spark.dataset.ray_dataset_to_spark_dataframe(spark, ds.schema(), refs)
    assert [r.value for r in df.take(n)] == values
    ds2 = ray.data.from_items([{"id": i} for i in range(n)])
    ids = [r["id"] for r in ds2.take(n)]
    refs2 = [b for bundle in ds2.iter_internal_ref_bundles() for b, _ in bundle.blocks]
    df2 = raydp.spark.dataset.ray_dataset_to_spark_dataframe(spark, ds2.schema(), refs2)
    assert [r.id for r in df2.take(n)] == ids


def test_placement_group(local_rt):
    for strategy in ["PACK", "STRICT_PACK", "SPREAD", "STRICT_SPREAD"]:
        spark = raydp.init_spark(f"test_strategy_{strategy}_1", 1, 1, "500M", placement_group_strategy=strategy)
        assert spark.range(0, 10, numPartitions=10).count() == 10
        raydp.stop_spark()
        pg = ray.util.placement_group([{"CPU": 1, "memory": utils.parse_memory_size("500M")}], strategy=strategy)
        ray.get(pg.ready())
        spark = raydp.init_spark(f"test_bundle_{strategy}_2", 1, 1, "500M", placement_group=pg,
                                 placement_group_bundle_indexes=[0])
        assert spark.range(0, 10, numPartitions=10).count() == 10
        from ray.util.state import list_actors
        ex = [a for a in list_actors() if a.name == "raydp-executor-0" and a.state == "ALIVE"][0]
        assert ex.placement_group_id == pg.id.hex()
        raydp.stop_spark()
        spark = raydp.init_spark(f"test_bundle_{strategy}_3", 1, 1, "500M", placement_group=pg)
        assert spark.range(0, 10, numPartitions=10).count() == 10
        raydp.stop_spark()
        ray.util.remove_placement_group(pg)
    assert len([p for p in placement_group_table().values() if p["state"] != "REMOVED"]) == 0


def test_reconstruction():
    """Remove the node holding converted partitions; every block is still gettable."""
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    node_to_kill = cluster.add_node(num_cpus=1, object_store_memory=10 ** 8)
    spark = raydp.init_spark("a", 2, 1, "500m", fault_tolerant_mode=True)
    df = spark.range(100000)
    ds = raydp.spark.from_spark_recoverable(df)
    locations = {r.node_id for bundle in ds.iter_internal_ref_bundles() for r, _ in bundle.blocks}
    assert node_to_kill.node_id in locations   # one executor (and its partitions) lives there
    cluster.add_node(num_cpus=1, object_store_memory=10 ** 8)
    cluster.remove_node(node_to_kill)           # arena destroyed, executor relocated
    cluster.add_node(num_cpus=1, object_store_memory=10 ** 8)
    total = 0
    for bundle in ds.iter_internal_ref_bundles():
        for block_ref, _ in bundle.blocks:
            total += ray.get(block_ref).num_rows
    assert total == 100000
    assert ds.count() == 100000
    raydp.stop_spark()
    cluster.shutdown()


def test_executor_killed_tasks_retried(spark_on_ray_2_executors):
    """An executor process dying mid-job: its tasks rerun and the supervisor restarts it."""
    spark = spark_on_ray_2_executors
    from raydp_amd.spark.session import SparkSession
    backend = SparkSession.getActiveSession()._cluster
    ex = backend.alive_executors()[0]
    pid = ray.get(ex.handle.info.remote())["pid"]
    os.kill(pid, 9)
    assert spark.range(0, 1000, numPartitions=8).count() == 1000
    info = ray.get(ex.handle.info.remote())
    assert info["pid"] != pid and info["restart_count"] >= 1


def test_recoverable_survives_gc():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 6})
    spark = raydp.init_spark("test_gc", 1, 1, "500M")
    df = spark.range(1000)
    ds = raydp.spark.from_spark_recoverable(df)
    import gc
    gc.collect()
    time.sleep(0.2)
    assert ds.count() == 1000
    raydp.stop_spark()
    cluster.shutdown()


def test_release_spark_recoverable():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 6})
    spark = raydp.init_spark("test_release", 1, 1, "500M")
    df = spark.range(100)
    ds = raydp.spark.from_spark_recoverable(df)
    from raydp.spark.dataset import _recoverable_rdd_ids
    backend = spark._cluster
    rdd_id = _recoverable_rdd_ids[df]
    assert backend.is_persisted(rdd_id)
    assert ds.count() == 100
    raydp.spark.release_spark_recoverable(df)
    assert not backend.is_persisted(rdd_id)
    assert df not in _recoverable_rdd_ids
    raydp.stop_spark()
    cluster.shutdown()


def test_dynamic_allocation(local_rt):
    spark = raydp.init_spark("dyn", 1, 1, "200M", configs={
        "spark.dynamicAllocation.enabled": "true", "spark.dynamicAllocation.initialExecutors": "1",
        "spark.dynamicAllocation.maxExecutors": "3"})
    backend = spark._cluster
    assert len(backend.alive_executors()) == 1
    backend.request_total_executors(5)          # capped at maxExecutors
    assert len(backend.alive_executors()) == 3
    assert spark.range(0, 300, numPartitions=6).count() == 300
    backend.request_total_executors(1)
    assert len(backend.alive_executors()) == 1
    assert spark.range(0, 30).count() == 30


def test_spark_master_memory_custom():
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 2, "resources": {"master": 10}})
    custom_memory = 100 * 1024 * 1024
    app = "test_spark_master_memory_custom"
    spark = raydp.init_spark(app_name=app, num_executors=1, executor_cores=1, executor_memory="500M",
                             configs={"spark.ray.raydp_spark_master.actor.resource.memory": str(custom_memory),
                                      "spark.ray.raydp_spark_master.actor.resource.master": "1"})
    assert spark.createDataFrame([(1, 2)], ["a", "b"]).count() == 1
    actor = ray.get_actor(f"{app}_SPARK_MASTER")
    from ray.util.state import list_actors
    st = list_actors(filters=[("actor_id", "=", actor._actor_id.hex())], detail=True)[0]
    assert st.required_resources["memory"] == custom_memory
    assert st.required_resources["master"] == 1
    raydp.stop_spark()
    cluster.shutdown()


def test_restarted_executor_registers_under_a_new_id(spark_on_ray_2_executors):
    """RayDPExecutor.scala:82-94 + RayAppMaster.scala:192-209: a restarted executor actor keeps
    its name but asks the master for a new executor id; the master records new -> old."""
    spark = spark_on_ray_2_executors
    backend = spark._cluster
    ex = [e for e in backend.alive_executors() if e.executor_id == "1"][0]
    before = ray.get(ex.handle.info.remote())
    assert before["spark_executor_id"] == "1"
    os.kill(before["pid"], 9)
    assert spark.range(0, 100, numPartitions=4).count() == 100
    after = ray.get(ex.handle.info.remote())
    assert after["pid"] != before["pid"]
    assert after["spark_executor_id"] not in ("0", "1")
    assert backend.restarted_executors() == {after["spark_executor_id"]: "1"}
    info = backend.appmaster.app_info()
    assert info["executors"][after["spark_executor_id"]]["registered"]


def test_external_shuffle_service(local_rt):
    """spark.shuffle.service.enabled: map outputs go through the per-node native service
    (RayAppMaster.scala:155-163) and the results equal the in-store shuffle's."""
    import pandas as pd
    from raydp_amd.spark import functions as F
    from raydp_amd.spark import shuffle as S
    spark = raydp.init_spark("shuf", 2, 1, "200M", configs={"spark.shuffle.service.enabled": "true"})
    backend = spark._cluster
    assert backend.shuffle_service_enabled
    pdf = pd.DataFrame({"k": [i % 7 for i in range(5000)], "v": [float(i) for i in range(5000)]})
    df = spark.createDataFrame(pdf).repartition(4)
    got = df.groupBy("k").agg(F.sum("v").alias("s")).toPandas().sort_values("k").reset_index(drop=True)
    want = pdf.groupby("k", as_index=False)["v"].sum().rename(columns={"v": "s"})
    assert got["k"].tolist() == want["k"].tolist()
    assert got["s"].tolist() == pytest.approx(want["s"].tolist())
    assert df.select("k").distinct().count() == 7
    services = backend.appmaster.app_info()["shuffle_services"]
    assert len(services) == 1
    sock = next(iter(services.values()))
    assert S.client(sock).list() == []      # map outputs released after the reduce stage
    infos = ray.get([e.handle.info.remote() for e in backend.alive_executors()])
    assert {i["shuffle_service"] for i in infos} == {sock}


def test_to_spark_tasks_run_where_blocks_live():
    """RayDatasetRDD.getPreferredLocations (RayDatasetRDD.scala:35-57): a DataFrame built over
    dataset blocks schedules each partition's task on an executor of the block's node."""
    cluster = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    cluster.add_node(num_cpus=1, object_store_memory=10 ** 8)
    cluster.add_node(num_cpus=1, object_store_memory=10 ** 8)
    spark = raydp.init_spark("loc", 2, 1, "200M")
    df = spark.range(0, 4000, numPartitions=8)
    ds = raydp.spark.from_spark_recoverable(df)
    refs = [r for bundle in ds.iter_internal_ref_bundles() for r, _ in bundle.blocks]
    homes = [r.node_id for r in refs]
    assert len(set(homes)) == 2            # blocks spread over both executors' nodes
    back = ds.to_spark(spark)

    def where(it):
        import os as _os
        rows = list(it)
        yield (_os.environ.get("RAYDP_NODE_ID"), len(rows))
    ran = back.rdd.mapPartitions(where).collect()
    assert [n for n, _ in ran] == homes
    assert sum(c for _, c in ran) == 4000
    raydp.stop_spark()
    cluster.shutdown()


def test_fault_inject_helpers(spark_on_ray_2_executors):
    """raydp_amd.runtime.fault_inject: kill an executor by name, wait for its restart, and the
    application keeps working (tasks retried, restart registered with a new id)."""
    from raydp_amd.runtime import fault_inject as FI
    spark = spark_on_ray_2_executors
    old = FI.kill_executor("0")
    new = FI.wait_restarted("raydp-executor-0", old)
    assert new != old
    assert spark.range(0, 500, numPartitions=5).count() == 500
    assert "0" in spark._cluster.restarted_executors().values()


def test_colocated_stores_share_the_node_shm_budget(monkeypatch):
    """Eight SPMD ranks of one node (LOCAL_WORLD_SIZE=8) each open an object store: together
    they never reserve more than the free /dev/shm (30% of it, split eight ways)."""
    import os
    import tempfile

    from raydp_amd.runtime import store as S
    monkeypatch.delenv("RAYDP_OBJECT_STORE_BYTES", raising=False)
    st = os.statvfs(S._shm_dir() or "/tmp")
    avail = st.f_bavail * st.f_frsize
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    stores = []
    try:
        with tempfile.TemporaryDirectory() as d:
            for r in range(8):
                stores.append(S.open_store(f"budget-test-{r}", None, d))
            total = sum(s.capacity for s in stores)
            assert total <= avail, (total, avail)
            assert total <= 0.3 * avail + (8 << 24), (total, avail)
    finally:
        for s in stores:
            s.destroy()
    # a lone process keeps the whole 30% (unless the 64 GiB cap binds)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    one = S.default_capacity()
    assert one >= min(64 << 30, 4 * max(s.capacity for s in stores)), one


def test_executor_sizes_arrow_pool_to_its_cores():
    """An executor's Arrow CPU pool is its spark.executor.cores, not the host's CPU count."""
    import pyarrow as pa

    from raydp_amd.spark.executor import RayDPExecutor
    before = pa.cpu_count()
    try:
        assert RayDPExecutor._size_thread_pools(2) == 2 and pa.cpu_count() == 2
        assert RayDPExecutor._size_thread_pools(0) == 1 and pa.cpu_count() == 1
    finally:
        pa.set_cpu_count(before)
