"""Device telemetry for benches and training runs: power, HBM use and GFX
activity of the node's GPUs sampled through AMD SMI while a region runs, plus a step-time
histogram helper for device-timed steps.

The sampler runs in a CHILD process (``python -m raydp_amd.utils.devmon``), started before the
region and stopped after it: the region's host path (Python ETL, dispatch) is what the
headline bench is bound by, and a sampling thread in the same process would compete for its
GIL. The child touches no HIP context (AMD SMI reads the kernel driver), so starting it from a
process that already initialised the GPU is a plain fork+exec of a new program in the child.

    with DeviceMonitor(interval_s=0.005) as mon:
        ...timed region...
    mon.summary()   # {"samples", "power_w_mean", "power_w_max", "vram_used_mib_max", ...}

Reference: RayDP has no device telemetry (CPU-only CI); Ray's dashboard reports node GPU
utilisation through its own agent, which this replaces for the single-node benches.
"""
import json
import os
import signal
import subprocess
import sys
import tempfile
import time
from typing import Dict, List, Optional

import numpy as np


def _sample_loop(out_path: str, interval_s: float, devices: Optional[List[int]]):
    import amdsmi
    amdsmi.amdsmi_init()
    handles = amdsmi.amdsmi_get_processor_handles()
    if devices:
        handles = [h for i, h in enumerate(handles) if i in devices]
    stop = {"v": False}

    def _stop(*_):
        stop["v"] = True
    signal.signal(signal.SIGTERM, _stop)
    signal.signal(signal.SIGINT, _stop)
    with open(out_path, "w") as f:
        f.write(json.dumps({"ready": True, "gpus": len(handles)}) + "\n")
        f.flush()
        while not stop["v"]:
            t = time.time()
            rows = []
            for h in handles:
                row = {}
                try:
                    p = amdsmi.amdsmi_get_power_info(h)
                    w = p.get("current_socket_power")
                    if w in (None, "N/A") or (isinstance(w, (int, float)) and w <= 0):
                        w = p.get("average_socket_power")
                    row["power_w"] = float(w) if isinstance(w, (int, float)) else None
                except Exception:  # noqa: BLE001
                    row["power_w"] = None
                try:
                    v = amdsmi.amdsmi_get_gpu_vram_usage(h)
                    row["vram_used_mib"] = float(v.get("vram_used"))
                    row["vram_total_mib"] = float(v.get("vram_total"))
                except Exception:  # noqa: BLE001
                    pass
                try:
                    a = amdsmi.amdsmi_get_gpu_activity(h)
                    g = a.get("gfx_activity")
                    row["gfx_pct"] = float(g) if isinstance(g, (int, float)) else None
                    u = a.get("umc_activity")
                    row["umc_pct"] = float(u) if isinstance(u, (int, float)) else None
                except Exception:  # noqa: BLE001
                    pass
                rows.append(row)
            f.write(json.dumps({"t": t, "gpus": rows}) + "\n")
            f.flush()
            time.sleep(max(0.0, interval_s - (time.time() - t)))
    amdsmi.amdsmi_shut_down()


class DeviceMonitor:
    """Sample AMD SMI telemetry in a child process while the ``with`` block runs. Never
    raises: without a driver / AMD SMI the summary says so and the region runs unaffected."""

    def __init__(self, interval_s: float = 0.01, devices: Optional[List[int]] = None,
                 ready_timeout_s: float = 5.0):
        self.interval_s, self.devices = interval_s, devices
        self.ready_timeout_s = ready_timeout_s
        self.proc = None
        self.path = None
        self.error = None
        self.records: List[dict] = []
        self.t0 = self.t1 = None

    def __enter__(self):
        try:
            fd, self.path = tempfile.mkstemp(prefix="raydp_devmon_", suffix=".jsonl")
            os.close(fd)
            args = [sys.executable, "-m", "raydp_amd.utils.devmon", self.path, str(self.interval_s)]
            if self.devices:
                args.append(",".join(str(d) for d in self.devices))
            env = dict(os.environ)
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
            self.proc = subprocess.Popen(args, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
            deadline = time.time() + self.ready_timeout_s
            while time.time() < deadline:       # wait until the sampler is live
                if self.proc.poll() is not None:
                    self.error = (self.proc.stderr.read() or b"").decode(errors="replace").strip()[-300:] \
                        or "sampler exited"
                    self.proc = None
                    break
                if os.path.getsize(self.path) > 0:
                    break
                time.sleep(0.01)
        except Exception as e:  # noqa: BLE001
            self.error, self.proc = repr(e), None
        self.t0 = time.time()
        return self

    def __exit__(self, *exc):
        self.t1 = time.time()
        if self.proc is not None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(timeout=5)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        if self.path and os.path.exists(self.path):
            with open(self.path) as f:
                for line in f:
                    try:
                        r = json.loads(line)
                    except ValueError:
                        continue
                    if "t" in r:
                        self.records.append(r)
            os.unlink(self.path)
        return False

    def summary(self) -> Dict[str, object]:
        if self.error and not self.records:
            return {"available": False, "reason": self.error}
        recs = [r for r in self.records if self.t0 is None or self.t0 - self.interval_s <= r["t"] <= (self.t1 or 1e30)]
        recs = recs or self.records
        if not recs:
            return {"available": False, "reason": "no samples (region shorter than the sampling interval)"}

        def col(k):
            v = [g.get(k) for r in recs for g in r["gpus"] if g.get(k) is not None]
            return np.asarray(v, dtype=np.float64)
        out = {"available": True, "samples": len(recs), "interval_s": self.interval_s,
               "gpus": len(recs[0]["gpus"])}
        for k, unit in (("power_w", "power_w"), ("gfx_pct", "gfx_activity_pct"), ("umc_pct", "umc_activity_pct")):
            v = col(k)
            if v.size:
                out[f"{unit}_mean"] = round(float(v.mean()), 1)
                out[f"{unit}_max"] = round(float(v.max()), 1)
        v = col("vram_used_mib")
        if v.size:
            out["vram_used_mib_max"] = round(float(v.max()), 1)
        v = col("vram_total_mib")
        if v.size:
            out["vram_total_mib"] = round(float(v.max()), 1)
        return out


def step_time_histogram(step_us, edges=(5, 10, 20, 30, 40, 60, 80, 120, 200, 500, 1000, 5000)) -> Dict[str, object]:
    """Percentiles and a fixed-edge histogram (microseconds) of per-step device times."""
    a = np.sort(np.asarray(step_us, dtype=np.float64).reshape(-1))
    if a.size == 0:
        return {}
    edges = list(edges)
    # one sort; percentiles by linear interpolation (numpy's default), bins by searchsorted --
    # this runs after every epoch, on the fit's critical path
    pos = np.searchsorted(a, edges, side="left")
    counts = np.diff(np.concatenate(([0], pos, [a.size])))
    labels = [f"<{edges[0]}"] + [f"{lo}-{hi}" for lo, hi in zip(edges[:-1], edges[1:])] + [f">={edges[-1]}"]

    def pct(q):
        x = (a.size - 1) * q / 100.0
        lo = int(x)
        hi = min(lo + 1, a.size - 1)
        return float(a[lo] + (a[hi] - a[lo]) * (x - lo))
    return {"steps": int(a.size), "p10": round(pct(10), 2), "p50": round(pct(50), 2), "p90": round(pct(90), 2),
            "p99": round(pct(99), 2), "max": round(float(a[-1]), 2), "mean": round(float(a.mean()), 2),
            "hist_us": {lab: int(c) for lab, c in zip(labels, counts) if c}}


if __name__ == "__main__":
    devs = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 and sys.argv[3] else None
    _sample_loop(sys.argv[1], float(sys.argv[2]), devs)
