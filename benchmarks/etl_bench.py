"""NYC ETL throughput of the DataFrame engine: fused expression VM vs per-operator Arrow path.

Runs ``examples/data_process.py``'s ``nyc_taxi_preprocess`` (14 filters, 9 time features,
2 + 8 Python UDF calls, 7 drops; the reference's ``examples/data_process.py:97-101``) over a
synthetic NYCTaxi CSV and reports rows/s for

* the whole chain on parsed partitions (``ops``: CSV parse excluded, one partition per task),
* CSV read + chain (``e2e``), on ``--executors`` executor processes through ``init_spark``,

with ``RAYDP_FUSED_ETL=1`` (one native program per partition, ``csrc/exec/expr/expr_vm.cc``)
and ``=0`` (one or more pyarrow kernels per expression node, a table per operator). Outputs
are compared for equality before timing.

  python benchmarks/etl_bench.py --rows 2000000 --partitions 16
"""
import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "examples"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--partitions", type=int, default=16)
    ap.add_argument("--executors", type=int, default=4)
    ap.add_argument("--repeat", type=int, default=3)
    args = ap.parse_args()
    import pyarrow as pa

    import bench
    from data_process import nyc_taxi_preprocess
    from raydp_amd import context, runtime
    from raydp_amd.spark import exprc

    tmp = tempfile.mkdtemp(prefix="raydp_etl_bench_")
    csv = os.path.join(tmp, "nyc.csv")
    bench.make_csv(csv, args.rows, 3)
    size = os.path.getsize(csv)
    out = {"bench": "nyc_etl", "rows": args.rows, "csv_mb": round(size / 2 ** 20, 1),
           "partitions": args.partitions}

    # -- ops: the chain over in-memory partitions, in this process ---------------------------
    from raydp_amd.spark import SparkSession
    s = SparkSession.builder.master("local[1]").appName("etl-bench").getOrCreate()
    s.conf.set("spark.sql.session.timeZone", "UTC")
    raw = s.read.format("csv").option("header", "true").option("inferSchema", "true") \
        .load("file://" + csv)
    table = pa.concat_tables([raw._plan.compute(i) for i in range(raw._plan.num_partitions())])
    parts = [table.slice(k * (table.num_rows // args.partitions),
                         table.num_rows // args.partitions) for k in range(args.partitions)]
    src_df = s.createDataFrame(pa.concat_tables(parts))
    results = {}
    ref = None
    for mode in ("0", "1"):
        os.environ["RAYDP_FUSED_ETL"] = mode
        d = nyc_taxi_preprocess(src_df)
        plan = d._plan
        n = plan.num_partitions()
        got = pa.concat_tables([plan.compute(i) for i in range(n)])   # warm (compile, verify)
        if ref is None:
            ref = got
        else:
            assert got.num_rows == ref.num_rows and got.schema == ref.schema
        best = float("inf")
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            for i in range(n):
                plan.compute(i)
            best = min(best, time.perf_counter() - t0)
        results[mode] = best
    out["ops_rows_per_s"] = {"per_operator": round(table.num_rows / results["0"]),
                             "fused_vm": round(table.num_rows / results["1"])}
    out["ops_speedup"] = round(results["0"] / results["1"], 2)
    out["ops_partitions_in_process"] = src_df._plan.num_partitions()
    s.stop()

    # -- e2e: CSV read + chain on executor processes ----------------------------------------
    runtime.init(num_cpus=args.executors)
    e2e = {}
    for mode in ("0", "1"):
        # executor processes inherit the switch when the session starts
        os.environ["RAYDP_FUSED_ETL"] = mode
        spark = context.init_spark("etl-bench", args.executors, 1, "2G")
        spark.conf.set("spark.sql.session.timeZone", "UTC")
        best = float("inf")
        for r in range(args.repeat + 1):
            t0 = time.perf_counter()
            d = nyc_taxi_preprocess(spark.read.format("csv").option("header", "true")
                                    .option("inferSchema", "true").load("file://" + csv))
            cnt = d.count()
            dt = time.perf_counter() - t0
            if r:
                best = min(best, dt)
        e2e[mode] = best
        context.stop_spark()
    out["e2e_rows_per_s"] = {"per_operator": round(args.rows / e2e["0"]),
                             "fused_vm": round(args.rows / e2e["1"])}
    out["e2e_output_rows"] = cnt
    out["executors"] = args.executors
    out["stats"] = dict(exprc.STATS)
    runtime.shutdown()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
