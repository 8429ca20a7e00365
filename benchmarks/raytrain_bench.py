"""Like-for-like reproduction of BASELINE.md B4: the reference's raw Ray Train tutorial
(tutorials/raytrain_example.ipynb cell 40: stroke data, NET_Model, CrossEntropy with class
weights, Adam 1e-3, batch 64, 1 worker, 10 epochs of train + test). The reference's
steady-state train+test epoch was 0.596 s median (Colab CPU VM).

One JSON line with the median steady-state epoch time (epochs 2..N), per device.
  python benchmarks/raytrain_bench.py            # CPU, as the notebook
  RAYTRAIN_DEVICE=cuda python benchmarks/raytrain_bench.py
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tutorials"))

REF = {"epoch_s_median": 0.596, "first_epoch_s": 0.880, "train_rows": 4486, "test_rows": 1022}


def main():
    import raydp  # noqa: F401 - installs the ray facade
    import ray
    import raytrain_example as R
    from ray.train import TrainingCallback

    epochs = int(os.environ.get("RAYTRAIN_EPOCHS", "10"))
    hist = []

    class Keep(TrainingCallback):
        def handle_result(self, results, **info):
            hist.extend(results)

    ray.init(num_cpus=4)
    t0 = time.perf_counter()
    _, n_train, n_test = R.run(1, epochs, [Keep()])
    wall = time.perf_counter() - t0
    ep = [h["epoch_s"] for h in hist if "epoch_s" in h]
    steady = statistics.median(ep[1:]) if len(ep) > 1 else ep[0]
    print(json.dumps({
        "metric": "Ray Train stroke tutorial: train+test epoch time (B4)", "device": R.DEVICE,
        "epoch_s_median": round(steady, 4), "first_epoch_s": round(ep[0], 4), "epochs": len(ep),
        "train_rows": n_train, "test_rows": n_test,
        "train_samples_per_s": round(n_train / steady, 1),
        "whole_run_s": round(wall, 3), "final_test_acc": hist[-1].get("test_acc") if hist else None,
        "reference": REF, "speedup_epoch": round(REF["epoch_s_median"] / steady, 2)}), flush=True)
    ray.shutdown()


if __name__ == "__main__":
    main()
