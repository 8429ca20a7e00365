"""Spark-facing estimator interface (reference: ``python/raydp/spark/interfaces.py:27-39``)."""
from typing import NoReturn, Optional, Union

from raydp_amd.utils import convert_to_spark

DF = Union["raydp_amd.spark.DataFrame", "raydp_amd.spark.pandas.DataFrame"]
OPTIONAL_DF = Union[Optional["raydp_amd.spark.DataFrame"], Optional["raydp_amd.spark.pandas.DataFrame"]]


class SparkEstimatorInterface:
    def _check_and_convert(self, df):
        train_df, _ = convert_to_spark(df)
        return train_df

    def fit_on_spark(self, train_df: DF, evaluate_df: OPTIONAL_DF = None) -> NoReturn:
        """Fit on a Spark-style DataFrame (or pandas-on-Spark); subclasses convert and train."""
