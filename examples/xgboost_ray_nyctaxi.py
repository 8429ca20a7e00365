"""NYC taxi fare regression with gradient-boosted trees (reference:
examples/xgboost_ray_nyctaxi.py). ``xgboost_ray`` resolves to raydp_amd.xgboost.ray_api: the
native histogram GBDT with histograms all-reduced across ``num_actors`` workers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raydp
import ray
from raydp.utils import random_split
from xgboost_ray import RayDMatrix, RayParams, train

from data_process import NYC_TRAIN_CSV, nyc_taxi_preprocess

ray.init(address="local", num_cpus=4)
spark = raydp.init_spark("NYC Taxi Fare Prediction with RayDP", 1, 1, "500M")
data = spark.read.format("csv").option("header", "true").option("inferSchema", "true").load(NYC_TRAIN_CSV)
spark.conf.set("spark.sql.session.timeZone", "UTC")
data = nyc_taxi_preprocess(data)
train_df, test_df = random_split(data, [0.9, 0.1], 0)
dtrain = RayDMatrix(ray.data.from_spark(train_df), label="fare_amount")
dtest = RayDMatrix(ray.data.from_spark(test_df), label="fare_amount")
evals_result = {}
bst = train({"tree_method": "hist", "eval_metric": ["rmse", "mae"]}, dtrain, evals=[(dtest, "eval")],
            evals_result=evals_result, ray_params=RayParams(max_actor_restarts=1, num_actors=2, cpus_per_actor=1),
            num_boost_round=10)
print("Final validation rmse: {:.4f}".format(evals_result["eval"]["rmse"][-1]))
raydp.stop_spark()
ray.shutdown()
