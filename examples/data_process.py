"""NYC taxi ETL (reference: examples/data_process.py) on the raydp-amd DataFrame engine."""
import os

import sys
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import raydp  # noqa: F401  (installs the pyspark facade when PySpark is absent)
from pyspark.sql.functions import (abs as functions_abs, col, dayofmonth, dayofweek, hour, lit,
                                   month, quarter, udf, weekofyear, year)

NYC_TRAIN_CSV = "file://" + os.path.join(os.path.dirname(os.path.realpath(__file__)), "data",
                                         "fake_nyctaxi.csv")


def clean_up(data):
    return data.filter(col("pickup_longitude") <= -72) \
        .filter(col("pickup_longitude") >= -76) \
        .filter(col("dropoff_longitude") <= -72) \
        .filter(col("dropoff_longitude") >= -76) \
        .filter(col("pickup_latitude") <= 42) \
        .filter(col("pickup_latitude") >= 38) \
        .filter(col("dropoff_latitude") <= 42) \
        .filter(col("dropoff_latitude") >= 38) \
        .filter(col("passenger_count") <= 6) \
        .filter(col("passenger_count") >= 1) \
        .filter(col("fare_amount") > 0) \
        .filter(col("fare_amount") < 250) \
        .filter(col("dropoff_longitude") != col("pickup_longitude")) \
        .filter(col("dropoff_latitude") != col("pickup_latitude"))


def add_time_features(data):
    data = data.withColumn("day", dayofmonth(col("pickup_datetime")))
    data = data.withColumn("hour_of_day", hour(col("pickup_datetime")))
    data = data.withColumn("day_of_week", dayofweek(col("pickup_datetime")) - 2)
    data = data.withColumn("week_of_year", weekofyear(col("pickup_datetime")))
    data = data.withColumn("month_of_year", month(col("pickup_datetime")))
    data = data.withColumn("quarter_of_year", quarter(col("pickup_datetime")))
    data = data.withColumn("year", year(col("pickup_datetime")))

    @udf("int")
    def night(hour, weekday):
        if ((16 <= hour <= 20) and (weekday < 5)):
            return int(1)
        else:
            return int(0)

    @udf("int")
    def late_night(hour):
        if ((hour <= 6) or (hour >= 20)):
            return int(1)
        else:
            return int(0)
    data = data.withColumn("night", night("hour_of_day", "day_of_week"))
    data = data.withColumn("late_night", late_night("hour_of_day"))
    return data


def add_distance_features(data):
    @udf("float")
    def manhattan(lat1, lon1, lat2, lon2):
        return float(np.abs(lat2 - lat1) + np.abs(lon2 - lon1))
    ny = (-74.0063889, 40.7141667)
    jfk = (-73.7822222222, 40.6441666667)
    ewr = (-74.175, 40.69)
    lgr = (-73.87, 40.77)
    data = data.withColumn("abs_diff_longitude", functions_abs(col("dropoff_longitude") - col("pickup_longitude"))) \
        .withColumn("abs_diff_latitude", functions_abs(col("dropoff_latitude") - col("pickup_latitude")))
    data = data.withColumn("manhattan", col("abs_diff_latitude") + col("abs_diff_longitude"))
    for name, (lon, lat) in (("jfk", jfk), ("ewr", ewr), ("lgr", lgr), ("downtown", ny)):
        data = data.withColumn(f"pickup_distance_{name}",
                               manhattan("pickup_longitude", "pickup_latitude", lit(lon), lit(lat)))
        data = data.withColumn(f"dropoff_distance_{name}",
                               manhattan("dropoff_longitude", "dropoff_latitude", lit(lon), lit(lat)))
    return data


def drop_col(data):
    return data.drop("pickup_datetime").drop("pickup_longitude").drop("pickup_latitude") \
        .drop("dropoff_longitude").drop("dropoff_latitude").drop("passenger_count").drop("key")


def nyc_taxi_preprocess(data):
    data = clean_up(data)
    data = add_time_features(data)
    data = add_distance_features(data)
    return drop_col(data)
