import os, sys, time, tempfile
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "examples"))
import raydp
from raydp_amd import context, runtime
from bench import make_csv, BATCH
from data_process import nyc_taxi_preprocess
tmp = tempfile.mkdtemp()
p = os.path.join(tmp, "m.csv"); make_csv(p, 3000 * BATCH, 1)
runtime.init(num_cpus=4)
spark = context.init_spark("e", int(os.environ.get("NE","1")), int(os.environ.get("NC","4")), "2G")
spark.conf.set("spark.sql.session.timeZone", "UTC")
from raydp_amd.spark.dataset import from_spark_recoverable
for it in range(4):
    t = time.perf_counter()
    d = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load("file://" + p)
    d = nyc_taxi_preprocess(d)
    ds = from_spark_recoverable(d)
    n = ds.count()
    print(os.environ.get("RAYDP_EXECUTOR_MODE", "process"), n, round(time.perf_counter() - t, 4))
context.stop_spark(); runtime.shutdown()
