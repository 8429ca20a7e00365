"""NYC taxi with TFEstimator (reference: examples/tensorflow_nyctaxi.py — Keras regression,
2 workers, batch 256). TensorFlow is not part of the MI355X image: the estimator raises a clear
ImportError and this script reports that and exits 0; where TF is installed it trains."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raydp  # noqa: E402
from raydp.tf import TFEstimator
from raydp.utils import random_split

from data_process import nyc_taxi_preprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    spark = raydp.init_spark(app_name="NYC Taxi Fare Prediction with TF", num_executors=1, executor_cores=1,
                             executor_memory="500M")
    data = spark.read.format("csv").option("header", "true").option("inferSchema", "true") \
        .load("file://" + os.path.join(HERE, "data", "fake_nyctaxi.csv"))
    data = nyc_taxi_preprocess(data)
    train_df, test_df = random_split(data, [0.9, 0.1], 0)
    features = [f.name for f in list(train_df.schema) if f.name != "fare_amount"]
    try:
        import tensorflow as tf
    except ImportError:
        print("TensorFlow is not installed: TFEstimator is unavailable here "
              "(use raydp.torch.TorchEstimator on PyTorch-ROCm)")
        raydp.stop_spark()
        return 0
    keras = tf.keras
    inp = keras.Input(shape=(len(features),))
    x = keras.layers.Dense(256, activation="relu")(inp)
    x = keras.layers.BatchNormalization()(x)
    x = keras.layers.Dense(128, activation="relu")(x)
    x = keras.layers.Dense(64, activation="relu")(x)
    out = keras.layers.Dense(1)(x)
    model = keras.Model(inp, out)
    est = TFEstimator(num_workers=2, model=model, optimizer=keras.optimizers.Adam(0.001), loss="mse",
                      metrics=["mae"], feature_columns=features, label_columns="fare_amount",
                      merge_feature_columns=True, batch_size=256, num_epochs=10)
    est.fit_on_spark(train_df, test_df)
    print(est.get_model().evaluate)
    raydp.stop_spark()
    return 0


if __name__ == "__main__":
    sys.exit(main())
