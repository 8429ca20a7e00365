"""Synthetic NYC-taxi CSV generator (reference: examples/random_nyctaxi.py — same columns and
value ranges: fares U(3, 50), longitudes U(-74.2, -73.8), latitudes U(40.7, 40.8), 1-4
passengers, pickup times uniform over five years from 2010-01-01, "YYYY-MM-DD HH:MM:SS UTC").

Written column-wise with Arrow (no per-row Python), so tens of millions of rows take seconds:
    python examples/random_nyctaxi.py --num-records 2000 [--output path.csv] [--seed 0]
"""
import argparse
import os

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv


def generate(n: int, seed=None) -> pa.Table:
    rng = np.random.default_rng(seed)
    secs = rng.integers(0, 157_680_000, size=n)
    stamps = (np.datetime64("2010-01-01 00:00:00") + secs.astype("timedelta64[s]")).astype(str)
    stamps = np.char.add(np.char.replace(stamps, "T", " "), " UTC")
    return pa.table({
        "key": pa.array(np.full(n, "fake_key")),
        "fare_amount": rng.uniform(3.0, 50.0, n),
        "pickup_datetime": pa.array(stamps),
        "pickup_longitude": rng.uniform(-74.2, -73.8, n),
        "pickup_latitude": rng.uniform(40.7, 40.8, n),
        "dropoff_longitude": rng.uniform(-74.2, -73.8, n),
        "dropoff_latitude": rng.uniform(40.7, 40.8, n),
        "passenger_count": rng.integers(1, 5, n),
    })


def main(argv=None):
    ap = argparse.ArgumentParser(description="Random NYC taxi generator")
    ap.add_argument("--num-records", type=int, default=2000, metavar="N")
    ap.add_argument("--output", default=os.path.join(os.path.dirname(os.path.realpath(__file__)), "fake_nyctaxi.csv"))
    ap.add_argument("--seed", type=int, default=None)
    a = ap.parse_args(argv)
    pacsv.write_csv(generate(a.num_records, a.seed), a.output)
    print(f"wrote {a.num_records} rows to {a.output}")


if __name__ == "__main__":
    main()
