"""Like-for-like reproduction of the reference's only published measurements (BASELINE.md
B1-B3: tutorials/pytorch_example.ipynb cell 38 -- stroke dataset, NET_Model, batch 64, Adam
1e-3, 1 worker, 30 train + 30 eval epochs, whole ``fit_on_spark``).

Prints one JSON line: fit_on_spark wall time, median steady-state train / eval epoch time and
the derived samples/s, next to the reference's numbers (Colab CPU VM)."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tutorials"))
import raydp
import ray

from stroke import make_estimator, prepare

REF = {"train_epoch_s": 1.008, "eval_epoch_s": 0.101, "fit_wall_s": 36.0, "train_samples_per_s": 4600,
       "fit_samples_per_s": 3900}


def main():
    epochs = int(os.environ.get("STROKE_EPOCHS", "30"))
    ray.init(num_cpus=6)
    spark = raydp.init_spark("Stoke Prediction with RayDP", 1, 1, "500M")
    # warm-up run (process start-up, UDF vectorisation, kernel compilation)
    tr, te, feats = prepare(spark)
    make_estimator(feats, epochs=1).fit_on_spark(tr, te)
    t0 = time.perf_counter()
    tr, te, feats = prepare(spark)
    est = make_estimator(feats, epochs=epochs)
    est.fit_on_spark(tr, te)
    wall = time.perf_counter() - t0
    hist = est.results.metrics_history
    train_t = [h["_time_this_iter_s"] for h in hist if "train_loss" in h][1:]
    eval_t = [h["_time_this_iter_s"] for h in hist if "test_loss" in h][1:]
    n_train = tr.count()
    n_test = te.count()
    out = {"metric": "stroke tutorial fit_on_spark (30 train + 30 eval epochs)", "fit_wall_s": round(wall, 3),
           "train_epoch_s_median": round(statistics.median(train_t), 6),
           "eval_epoch_s_median": round(statistics.median(eval_t), 6),
           "train_rows": n_train, "test_rows": n_test,
           "train_samples_per_s": round(n_train / statistics.median(train_t), 1),
           "fit_samples_per_s": round(n_train * epochs / wall, 1),
           "engine": hist[0].get("engine"), "reference": REF,
           "speedup_fit": round(REF["fit_wall_s"] / wall, 2),
           "final_train": {k: v for k, v in [h for h in hist if "train_loss" in h][-1].items()
                           if not k.startswith("_")},
           "final_eval": {k: v for k, v in ([h for h in hist if "test_loss" in h] or [{}])[-1].items()
                          if not k.startswith("_")}}
    print(json.dumps(out))
    raydp.stop_spark()
    ray.shutdown()


if __name__ == "__main__":
    main()
