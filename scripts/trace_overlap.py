"""Copy/kernel or kernel/kernel overlap summary of a rocprofv3 CSV run.

    python scripts/trace_overlap.py gpurun_out/prof/ingest [--kernel arrow_ingest]
    python scripts/trace_overlap.py gpurun_out/prof/ddp_overlap --kernel lin_ --with xg_allreduce

The second form (``--with``) reports, per process, how much of the ``--with`` kernels' time
runs concurrently with ``--kernel`` kernels on another stream: the DDP gradient buckets on the
comm stream under the backward GEMMs.

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


def kernel_pair(prefix, kernel, other):
    rows = _rows(prefix + "_kernel_trace.csv")
    out = {}
    pids = sorted({r.get("Process_Id", "0") for r in rows})
    for pid in pids:
        mine = [r for r in rows if r.get("Process_Id", "0") == pid]
        a = [r for r in mine if kernel in r["Kernel_Name"]]
        b = [r for r in mine if other in r["Kernel_Name"]]
        if not a or not b:
            continue
        aiv = _merge([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in a])
        biv = _merge([(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in b])
        b_busy = sum(e - s for s, e in biv)
        ov = _overlap(aiv, biv)
        out[pid] = {"kernel": kernel, "kernel_streams": sorted({r["Stream_Id"] for r in a}),
                    "with": other, "with_streams": sorted({r["Stream_Id"] for r in b}),
                    "with_launches": len(b), "with_busy_us": round(b_busy / 1e3, 1),
                    "with_time_under_kernel_us": round(ov / 1e3, 1),
                    "with_time_under_kernel_frac": round(ov / b_busy, 3) if b_busy else None}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix", help="rocprofv3 output prefix, e.g. gpurun_out/prof/ingest")
    ap.add_argument("--kernel", default="")
    ap.add_argument("--with", dest="other", default=None,
                    help="kernel/kernel mode: overlap of these kernels with --kernel ones")
    a = ap.parse_args()
    if a.other:
        print(json.dumps(kernel_pair(a.prefix, a.kernel, a.other), indent=1))
        return
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
