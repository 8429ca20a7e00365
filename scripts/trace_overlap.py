"""Copy/kernel overlap summary of a rocprofv3 ``--kernel-trace --memory-copy-trace`` CSV run.

    python scripts/trace_overlap.py gpurun_out/prof/ingest [--kernel arrow_ingest]

For every kernel whose name contains ``--kernel``, reports how much of its execution overlaps
an in-flight host->device copy (and on which copy stream), plus per-stream busy time. Used to
check that the object-store->HBM DMA (copy stream) runs under the ingest decode kernel
(compute stream) instead of ahead of it.
"""
import argparse
import csv
import json


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Total length of the intersection of two merged interval lists."""
    i = j = tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="rocprofv3 output prefix, e.g. gpurun_out/prof/ingest")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    ks = [r for r in _rows(a.prefix + "_kernel_trace.csv") if a.kernel in r["Kernel_Name"]]
    cs = [r for r in _rows(a.prefix + "_memory_copy_trace.csv") if "HOST_TO_DEVICE" in r["Direction"]]
    kiv = _merge([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks])
    civ = _merge([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in cs])
    k_busy = sum(e - s for s, e in kiv)
    c_busy = sum(e - s for s, e in civ)
    ov = _overlap(kiv, civ)
    streams = sorted({r["Stream_Id"] for r in cs})
    kstreams = sorted({r["Stream_Id"] for r in ks})
    print(json.dumps({
        "kernels": len(ks), "kernel_streams": kstreams, "kernel_busy_us": round(k_busy / 1e3, 1),
        "h2d_copies": len(cs), "copy_streams": streams, "h2d_busy_us": round(c_busy / 1e3, 1),
        "kernel_time_under_copy_us": round(ov / 1e3, 1),
        "kernel_time_under_copy_frac": round(ov / k_busy, 3) if k_busy else None,
    }))


if __name__ == "__main__":
    main()
