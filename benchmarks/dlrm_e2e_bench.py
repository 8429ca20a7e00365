"""DLRM end to end through the Spark path (BASELINE.json config 5): the reference notebook's
flow (examples/pytorch_dlrm.ipynb cells 6-7, 13-14) on a synthetic Criteo-shaped TSV.

  read TSV with the Criteo schema -> pre_process (posexplode value counts, frequency limit 3,
  dense ids by window row_number, left joins, log(x+3), random row order) -> random_split
  0.9/0.1 -> TorchEstimator.fit_on_spark(Dlrm(13, sizes, [512,128,32], [1024,1024,512,256,1]),
  SGD lr 0.01, BCEWithLogits, batch --batch, --epochs) on the GPU.

One JSON line: end-to-end train samples/s over the WHOLE pipeline (ETL + conversion + HBM
ingest + training + evaluation + checkpoint), and the per-phase breakdown. Weights random,
data synthetic (no network for the Kaggle file).

  python benchmarks/dlrm_e2e_bench.py --rows 200000 --epochs 2 --batch 2048
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--epochs", type=int, default=2)
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--executors", type=int, default=4)
    ap.add_argument("--fused-sgd", action="store_true", help="embedding SGD applied inside backward")
    args = ap.parse_args()
    import torch

    import raydp_amd as raydp
    from raydp_amd import runtime
    from raydp_amd.models import dlrm_data as D
    from raydp_amd.models.dlrm import Dlrm
    from raydp_amd.torch import TorchEstimator
    from raydp_amd.torch.estimator import LAST_TIMINGS
    from raydp_amd.utils import random_split

    tmp = tempfile.mkdtemp(prefix="dlrm_e2e_")
    path = os.path.join(tmp, "train.txt")
    t_gen = time.perf_counter()
    D.synthetic_criteo(path, args.rows, seed=0)
    gen_s = time.perf_counter() - t_gen
    runtime.init(num_cpus=max(4, args.executors))
    spark = raydp.init_spark("dlrm-e2e", args.executors, 1, "2GB")
    torch.cuda.set_device(0)
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    df = spark.read.schema(D.criteo_schema()).option("sep", "\t").csv("file://" + path)
    df, sizes = D.pre_process(df.cache(), frequency_limit="3", output_ordering="total_random",
                              no_numeric_log_col=False)
    train_df, test_df = random_split(df, [0.9, 0.1], 0)
    t_plan = time.perf_counter()
    torch.manual_seed(0)
    model = Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32,
                 fused_embedding_sgd_lr=0.01 if args.fused_sgd else None)
    est = TorchEstimator(num_workers=1, model=model,
                         optimizer=torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=0.01),
                         loss=torch.nn.BCEWithLogitsLoss(reduction="mean"),
                         feature_columns=[f"_c{i}" for i in range(1, 40)],
                         feature_types=[torch.float32] * 13 + [torch.long] * 26,
                         label_column="_c0", label_type=torch.float, batch_size=args.batch,
                         num_epochs=args.epochs, storage_path=os.path.join(tmp, "results"))
    res = est.fit_on_spark(train_df, test_df)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    hist = [m for m in res.metrics_history if "train_loss" in m]
    rows = hist[-1].get("train_rows") if hist else None
    out = {
        "metric": "DLRM end-to-end train samples/s (Spark ETL + conversion + train), synthetic Criteo",
        "value": round(args.epochs * rows / wall, 1) if rows else None, "unit": "samples/s", "n_gpus": 1,
        "wall_s": round(wall, 3), "rows": args.rows, "train_rows": rows, "epochs": args.epochs,
        "batch": args.batch, "tables": len(sizes), "table_rows_total": int(sum(sizes)),
        "engine": hist[-1].get("engine") if hist else None,
        "train_epoch_samples_per_s": [round(m.get("train_samples_per_s", 0), 1) for m in hist],
        "final_train_loss": hist[-1]["train_loss"] if hist else None,
        "phases_s": {"plan_build": round(t_plan - t0, 4),
                     **{k: round(v, 4) for k, v in LAST_TIMINGS.items()}},
        "synthetic_generation_s (untimed)": round(gen_s, 2),
        "data": "synthetic Criteo-shaped TSV (dlrm_data.synthetic_criteo), random-init weights",
    }
    print(json.dumps(out), flush=True)
    raydp.stop_spark()
    runtime.shutdown()


if __name__ == "__main__":
    main()
