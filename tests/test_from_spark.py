"""from_spark API compatibility (port of tests/test_from_spark.py): converting must not leak
resources, and converted data stays readable after GC."""
import time

import raydp  # noqa: F401
import ray


def gen_test_data(spark):
    data = []
    tmp = [("ming", 20, 15552211521), ("hong", 19, 13287994007), ("dave", 21, 15552211523),
           ("john", 40, 15322211523), ("wong", 50, 15122211523)]
    for _ in range(10):
        data += tmp
    rdd = spark.sparkContext.parallelize(data)
    return spark.createDataFrame(rdd, ["Name", "Age", "Phone"])


def test_api_compatibility(runtime_local):
    spark = raydp.init_spark(app_name="test_api_compatibility", num_executors=1, executor_cores=1,
                             executor_memory="500M")
    df_train = gen_test_data(spark)
    cpu_cnt = ray.available_resources()["CPU"]
    ds = ray.data.from_spark(df_train)
    ds.show(1)
    import gc
    gc.collect()
    time.sleep(0.2)
    assert ray.available_resources()["CPU"] == cpu_cnt
    assert ds.count() == 50
    raydp.stop_spark()


def test_from_spark_owner_keeps_data_after_stop(runtime_local):
    """stop_spark(cleanup_data=False) with the master as owner: blocks stay readable."""
    spark = raydp.init_spark(app_name="owner_test", num_executors=1, executor_cores=1, executor_memory="500M")
    df = spark.range(0, 1000)
    ds = raydp.spark.spark_dataframe_to_ray_dataset(df, owner=raydp.spark.get_raydp_master_owner(spark))
    raydp.stop_spark(cleanup_data=False)
    assert ds.count() == 1000
    raydp.stop_spark()
