"""Stroke prediction with RayDP on MI355X (reference: tutorials/pytorch_example.ipynb)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import raydp
import ray

from stroke import make_estimator, prepare

ray.init(num_cpus=6)
spark = raydp.init_spark("Stoke Prediction with RayDP", 1, 1, "500M")
train_df, test_df, features = prepare(spark)
estimator = make_estimator(features, epochs=int(os.environ.get("STROKE_EPOCHS", "10")))
estimator.fit_on_spark(train_df, test_df)
for h in estimator.results.metrics_history:
    if "train_loss" in h or "test_loss" in h:
        print(h)
raydp.stop_spark()
ray.shutdown()
