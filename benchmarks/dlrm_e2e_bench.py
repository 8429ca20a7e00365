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
    ap.add_argument("--workers", type=int, default=1,
                    help="TorchEstimator num_workers (the notebook uses 2); > GPUs rehearses on a share "
                         "of one GPU (gloo bootstrap)")
    ap.add_argument("--fused-sgd", action="store_true", help="embedding SGD applied inside backward")
    ap.add_argument("--gc-freeze", type=int, default=1,
                    help="move the warmed-up process state to the permanent GC generation before timing")
    ap.add_argument("--profile-timed", default=None, help="cProfile the timed region into this file")
    ap.add_argument("--warmup-rows", type=int, default=20_000,
                    help="rows of an untimed warm-up run of the same pipeline (0: none)")
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
    warm = os.path.join(tmp, "warm.txt")
    if args.warmup_rows:
        D.synthetic_criteo(warm, args.warmup_rows, seed=1)
    if args.workers > torch.cuda.device_count():
        os.environ.setdefault("RAYDP_TRAIN_BACKEND", "gloo")   # several workers share a card
    runtime.init(num_cpus=max(4, args.executors) + args.workers)
    spark = raydp.init_spark("dlrm-e2e", args.executors, 1, "2GB")
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
    from raydp_amd.utils import tracing

    def pipeline(p, epochs):
        """The notebook's flow on file ``p``: returns (result, sizes, t_plan_done, t_est_start)."""
        df = spark.read.schema(D.criteo_schema()).option("sep", "\t").csv("file://" + p)
        df, sizes = D.pre_process(df.cache(), frequency_limit="3", output_ordering="total_random",
                                  no_numeric_log_col=False)
        train_df, test_df = random_split(df, [0.9, 0.1], 0)
        t_plan = time.perf_counter()
        torch.manual_seed(0)
        model = Dlrm(13, sizes, [512, 128, 32], [1024, 1024, 512, 256, 1], 32,
                     fused_embedding_sgd_lr=0.01 if args.fused_sgd else None)
        share = min(1.0, torch.cuda.device_count() / args.workers)
        est = TorchEstimator(num_workers=args.workers, model=model,
                             resources_per_worker={"CPU": 1, "GPU": share},
                             optimizer=torch.optim.SGD([q for q in model.parameters() if q.requires_grad], lr=0.01),
                             loss=torch.nn.BCEWithLogitsLoss(reduction="mean"),
                             feature_columns=[f"_c{i}" for i in range(1, 40)],
                             feature_types=[torch.float32] * 13 + [torch.long] * 26,
                             label_column="_c0", label_type=torch.float, batch_size=args.batch,
                             num_epochs=epochs, storage_path=os.path.join(tmp, "results"))
        t_est = time.perf_counter()
        return est.fit_on_spark(train_df, test_df), sizes, t_plan, t_est

    if args.warmup_rows:
        # untimed warm-up of the same pipeline on a small file (library imports such as
        # torch._dynamo on the first optimizer, pandas on the first empty Arrow table, kernel
        # code-object loads, executor-side compiled ETL programs), as bench.py does for NYC
        pipeline(warm, 1)
    from raydp_amd.utils.gcmeter import GcMeter, freeze_long_lived
    if args.gc_freeze:
        freeze_long_lived()
    prof = None
    if args.profile_timed:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t_ns = time.time_ns()
    gcm = GcMeter()
    t0 = time.perf_counter()
    with gcm:
        res, sizes, t_plan, t_est = pipeline(path, args.epochs)
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tracing.complete("timed run", t_ns, cat="bench")
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats("cumulative").print_stats(60)
        st.sort_stats("tottime").print_stats(30)
        with open(args.profile_timed, "w") as f:
            f.write(buf.getvalue())
    hist = [m for m in res.metrics_history if "train_loss" in m]
    rows = hist[-1].get("train_rows") if hist else None
    out = {
        "metric": "DLRM end-to-end train samples/s (Spark ETL + conversion + train), synthetic Criteo",
        "value": round(args.epochs * rows * args.workers / wall, 1) if rows else None, "unit": "samples/s",
        "n_gpus": torch.cuda.device_count(), "workers": args.workers,
        "allreduce": hist[-1].get("allreduce") if hist else None,
        "wall_s": round(wall, 3), "rows": args.rows, "train_rows": rows, "epochs": args.epochs,
        "batch": args.batch, "tables": len(sizes), "table_rows_total": int(sum(sizes)),
        "engine": hist[-1].get("engine") if hist else None,
        "train_epoch_samples_per_s": [round(m.get("train_samples_per_s", 0), 1) for m in hist],
        "final_train_loss": hist[-1]["train_loss"] if hist else None,
        "phases_s": {"plan_build": round(t_plan - t0, 4), "model_and_estimator_init": round(t_est - t_plan, 4),
                     **{k: round(v, 4) for k, v in LAST_TIMINGS.items()}},
        "python_gc_in_timed_region": gcm.summary(), "gc_freeze": bool(args.gc_freeze),
        "synthetic_generation_s (untimed)": round(gen_s, 2),
        "warmup_rows (untimed)": args.warmup_rows,
        "data": "synthetic Criteo-shaped TSV (dlrm_data.synthetic_criteo), random-init weights",
    }
    print(json.dumps(out), flush=True)
    raydp.stop_spark()
    runtime.shutdown()


if __name__ == "__main__":
    main()
