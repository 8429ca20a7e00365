"""Spark-compatible, Arrow-native DataFrame engine + the ``raydp.spark`` conversion API.

Engine surface (``pyspark.sql`` equivalents): ``SparkSession``, ``DataFrame``, ``Column``,
``Row``, ``functions``, ``types``, ``Window``. Conversion surface (reference
``python/raydp/spark/__init__.py:18-36``): ``spark_dataframe_to_ray_dataset``,
``from_spark_recoverable``, ``release_spark_recoverable``, ``ray_dataset_to_spark_dataframe``,
``get_raydp_master_owner``, ``PartitionObjectsOwner``, ``SparkCluster``,
``SparkEstimatorInterface``.
"""
from raydp_amd.spark.column import Column
from raydp_amd.spark.dataframe import DataFrame, GroupedData, StorageLevel
from raydp_amd.spark.row import Row
from raydp_amd.spark.session import SparkSession, SparkConf
from raydp_amd.spark.window import Window
from raydp_amd.spark import functions, types

_LAZY = {
    "PartitionObjectsOwner": "raydp_amd.spark.dataset",
    "get_raydp_master_owner": "raydp_amd.spark.dataset",
    "spark_dataframe_to_ray_dataset": "raydp_amd.spark.dataset",
    "ray_dataset_to_spark_dataframe": "raydp_amd.spark.dataset",
    "from_spark_recoverable": "raydp_amd.spark.dataset",
    "release_spark_recoverable": "raydp_amd.spark.dataset",
    "SparkEstimatorInterface": "raydp_amd.spark.interfaces",
    "SparkCluster": "raydp_amd.spark.ray_cluster",
}


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError(name)
    import importlib
    return getattr(importlib.import_module(mod), name)


__all__ = [
    "SparkCluster", "SparkEstimatorInterface", "PartitionObjectsOwner", "get_raydp_master_owner",
    "spark_dataframe_to_ray_dataset", "ray_dataset_to_spark_dataframe", "from_spark_recoverable",
    "release_spark_recoverable", "SparkSession", "DataFrame", "Column", "Row", "functions",
    "types", "Window", "StorageLevel", "GroupedData", "SparkConf",
]
