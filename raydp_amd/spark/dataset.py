"""Spark DataFrame ⇄ Dataset conversion (``raydp.spark`` conversion API).

Parity: ``python/raydp/spark/dataset.py``.

* ``from_spark_recoverable(df)`` (:172-222): the DataFrame's Arrow partitions are materialised
  and *pinned* in the executors' partition cache (``ObjectStoreWriter.prepareRecoverableRDD``,
  ``ObjectStoreWriter.scala:164-204``); each Dataset block is an ``ObjectRef`` whose lineage
  re-fetches the partition from its executor — recomputing it from the DataFrame plan if the
  cached copy was lost (``RayDPExecutor.getRDDPartition`` + ``requestRecacheRDD``,
  ``RayDPExecutor.scala:289-355``).
* ``release_spark_recoverable(df)`` (:224-237) unpins the cached partitions.
* ``ray_dataset_to_spark_dataframe(spark, schema, blocks)`` (:293-313) builds a DataFrame whose
  partitions are the Dataset's Arrow blocks (read zero-copy from the object store).
"""
import logging
import uuid
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Union

import pyarrow as pa

from raydp_amd.data.dataset import Dataset
from raydp_amd.runtime.objects import ObjectRef
from raydp_amd.spark.dataframe import DataFrame, StorageLevel

logger = logging.getLogger(__name__)

RAYDP_SPARK_MASTER_SUFFIX = "_SPARK_MASTER"
_recoverable_rdd_ids: Dict[DataFrame, str] = {}


@dataclass
class PartitionObjectsOwner:
    actor_name: str
    set_reference_as_state: Callable


def get_raydp_master_owner(spark=None) -> PartitionObjectsOwner:
    from raydp_amd.spark.session import SparkSession
    if spark is None:
        spark = SparkSession.getActiveSession()
    name = spark.sparkContext.appName + RAYDP_SPARK_MASTER_SUFFIX

    def set_state(master, objects):
        return master.add_objects(uuid.uuid4().hex, objects)
    return PartitionObjectsOwner(name, set_state)


def spark_dataframe_to_ray_dataset(df: DataFrame, parallelism: Optional[int] = None,
                                   owner: Union[PartitionObjectsOwner, None] = None) -> Dataset:
    if owner is not None:
        logger.debug("spark_dataframe_to_ray_dataset uses recoverable conversion; owner ignored")
    return from_spark_recoverable(df, parallelism=parallelism)


def from_spark_recoverable(df: DataFrame, storage_level=StorageLevel.MEMORY_AND_DISK,
                           parallelism: Optional[int] = None) -> Dataset:
    original = df
    if parallelism is not None and parallelism != df._src().num_partitions():
        df = df.repartition(parallelism)
    backend = df.sparkSession._cluster
    if backend is not None:
        rdd_id, refs = backend.prepare_recoverable(df, storage_level)
    else:
        rdd_id, refs = _prepare_local(df)
    _recoverable_rdd_ids[original] = rdd_id
    return Dataset(refs, df.arrow_schema)


def _prepare_local(df: DataFrame):
    """Driver-local path (a plain ``SparkSession`` without an executor cluster)."""
    from raydp_amd.runtime import objects
    df.persist()
    tables = df._cached.tables
    rdd_id = df._id
    refs = []
    for i, t in enumerate(tables):
        def lineage(df=df, i=i):
            if df._cached is None:
                df.persist()
            return df._cached.tables[i]
        refs.append(objects.put(t.replace_schema_metadata(), _lineage=lineage))
    return rdd_id, refs


def release_spark_recoverable(df: DataFrame) -> None:
    rdd_id = _recoverable_rdd_ids.pop(df, None)
    if rdd_id is None:
        return
    backend = df.sparkSession._cluster
    if backend is not None:
        backend.release_recoverable(rdd_id)
    else:
        df.unpersist()


def ray_dataset_to_spark_dataframe(spark, arrow_schema, blocks: List[ObjectRef],
                                   locations=None) -> DataFrame:
    from raydp_amd.runtime.objects import get
    from raydp_amd.spark import plan as P
    from raydp_amd.spark.sources import Source
    if hasattr(arrow_schema, "base_schema"):
        arrow_schema = arrow_schema.base_schema
    if not isinstance(arrow_schema, pa.Schema):
        raise RuntimeError(f"Schema is {type(arrow_schema)}, required pyarrow.lib.Schema. \n"
                           f"to_spark does not support converting non-arrow ray datasets.")

    class _BlockSource(Source):
        def num_partitions(self):
            return len(blocks)

        def load(self, i):
            b = get(blocks[i])
            if isinstance(b, (bytes, bytearray, memoryview)):
                b = pa.ipc.open_stream(pa.py_buffer(b)).read_all()
            if isinstance(b, pa.Table):
                return b.cast(arrow_schema) if b.schema != arrow_schema else b
            raise RuntimeError("ray.to_spark only supports arrow type blocks")

        def schema(self):
            return arrow_schema

        def preferred_node(self, i):
            # RayDatasetRDD / RayObjectRefRDD: run the task where the block lives
            return getattr(blocks[i], "node_id", None)

    return DataFrame(P.SourcePlan(_BlockSource()), spark)


def read_spark_parquet(path: str) -> Dataset:
    from raydp_amd.data import dataset as D
    return D.read_parquet(path, file_extensions=["parquet"])


def _convert_for_estimator(est, train_df, evaluate_df=None, fs_directory: Optional[str] = None,
                           compression: Optional[str] = None, stop_spark_after_conversion: bool = False,
                           parallelism: Optional[int] = None):
    """Shared ``fit_on_spark`` conversion of the estimators (reference: the identical blocks in
    ``python/raydp/tf/estimator.py:272-304`` and ``xgboost/estimator.py:83-116``): via a
    parquet directory when ``fs_directory`` is given, else through the object store."""
    train_df = est._check_and_convert(train_df)
    evaluate_ds = None
    if fs_directory is not None:
        app_id = train_df.sparkSession.sparkContext.applicationId
        path = fs_directory.rstrip("/") + f"/{app_id}"
        train_df.write.parquet(path + "/train", compression=compression)
        train_ds = read_spark_parquet(path + "/train")
        if evaluate_df is not None:
            evaluate_df = est._check_and_convert(evaluate_df)
            evaluate_df.write.parquet(path + "/test", compression=compression)
            evaluate_ds = read_spark_parquet(path + "/test")
    else:
        owner = get_raydp_master_owner(train_df.sparkSession) if stop_spark_after_conversion else None
        train_ds = spark_dataframe_to_ray_dataset(train_df, parallelism=parallelism, owner=owner)
        if evaluate_df is not None:
            evaluate_df = est._check_and_convert(evaluate_df)
            evaluate_ds = spark_dataframe_to_ray_dataset(evaluate_df, parallelism=parallelism, owner=owner)
    if stop_spark_after_conversion:
        from raydp_amd.context import stop_spark
        stop_spark(cleanup_data=False)
    return train_ds, evaluate_ds
