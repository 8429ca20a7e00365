"""Monte-Carlo pi (the PySpark examples/src/main/python/pi.py program the reference's
examples/raydp-submit.py submits). Run: bin/raydp-submit --conf spark.executor.instances=2 examples/pi.py 4"""
import sys
from operator import add
from random import random

from pyspark.sql import SparkSession

if __name__ == "__main__":
    spark = SparkSession.builder.appName("PythonPi").getOrCreate()
    partitions = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = 100000 * partitions

    def f(_):
        x = random() * 2 - 1
        y = random() * 2 - 1
        return 1 if x ** 2 + y ** 2 <= 1 else 0

    count = spark.sparkContext.parallelize(range(1, n + 1), partitions).map(f).reduce(add)
    print("Pi is roughly %f" % (4.0 * count / n))
    spark.stop()
