"""Object store -> HBM ingest throughput (raydp_amd/ops/ingest.py, csrc/hip/arrow_ingest.hip).

A table of ``--rows`` x ``--cols`` float64 columns (default 10M x 20 = 1.6 GB) is written into
the shared-memory object store in ``--blocks`` blocks, read back zero-copy (as an executor's
persisted partitions are) and ingested into a bf16 [rows, 32] training matrix: pinned DMA out of
the arena on the copy stream, decode kernel on the compute stream. Reports GB/s of Arrow bytes
moved against the PCIe Gen5 x16 host link (~63 GB/s), for the first call (arena pages pinned on
the way) and for steady-state calls, plus the pageable baseline (same table outside the store).

  python benchmarks/ingest_bench.py --rows 10000000 --cols 20
"""
import argparse
import json
import os
import sys
import time
import uuid

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--cols", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--repeat", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import pyarrow as pa
    import torch

    from raydp_amd.ops import ingest
    from raydp_amd.runtime.store import SharedObjectStore

    torch.cuda.set_device(0)
    rng = np.random.default_rng(0)
    per = args.rows // args.blocks
    nbytes = per * args.blocks * args.cols * 8
    store = SharedObjectStore(f"/dev/shm/raydp_ingest_bench_{uuid.uuid4().hex[:8]}", "bench", create=True,
                              capacity=int(nbytes * 1.1) + (256 << 20))
    try:
        host_tables, views = [], []
        for b in range(args.blocks):
            t = pa.table({f"c{j}": rng.standard_normal(per) for j in range(args.cols)})
            oid = uuid.uuid4().hex
            store.put(oid, t)
            _, v = store.get(oid)
            views.append(v)
            host_tables.append(t)
        cols = [f"c{j}" for j in range(args.cols)]
        stride = ((args.cols + 31) // 32) * 32

        def run(tables):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = ingest.ingest_columns(tables, cols, "cuda", True, stride=stride)
            torch.cuda.synchronize()
            return time.perf_counter() - t0, out

        ingest.reset_ingest_stats()
        first, out = run(views)
        st = ingest.ingest_stats()
        steady = min(run(views)[0] for _ in range(args.repeat))
        pageable = min(run(host_tables)[0] for _ in range(max(1, args.repeat // 2)))
        # correctness spot check
        ref = torch.from_numpy(np.stack([views[0].column(c).to_numpy()[:1000] for c in cols], 1)).to(torch.bfloat16)
        ok = bool(torch.equal(out[:1000, :args.cols].cpu(), ref))
        gb = nbytes / 1e9
        print(json.dumps({
            "metric": "object store -> HBM ingest (Arrow f64 columns -> bf16 training matrix)",
            "rows": per * args.blocks, "cols": args.cols, "blocks": args.blocks, "arrow_gb": round(gb, 3),
            "first_call_s": round(first, 4), "first_call_gb_per_s": round(gb / first, 2),
            "steady_s": round(steady, 4), "steady_gb_per_s": round(gb / steady, 2),
            "pageable_s": round(pageable, 4), "pageable_gb_per_s": round(gb / pageable, 2),
            "pcie_gen5_x16_bound_gb_per_s": 63.0, "steady_fraction_of_pcie": round(gb / steady / 63.0, 3),
            "stats_first_call": st, "exact": ok}), flush=True)
    finally:
        store.destroy()


if __name__ == "__main__":
    main()
