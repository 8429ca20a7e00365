"""Price of one grid barrier of the multi-workgroup form (csrc/hip/mlp_core.h mw_barrier) on the
MI355X, by grid size: G workgroups pass N barriers in one launch; (t(N) - t(0)) / N per barrier,
median of several launches timed with HIP events. This is the number that decides how many
grid-wide phases a persistent kernel (the multi-workgroup NYC step, a whole DLRM step) can afford
against a kernel boundary (MI355X_MICROARCH.md price list: boundary ~1.1-1.5 us in a graph).
"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from raydp_amd.ops import _hip


def main():
    L = _hip.lib()
    L.rx_mw_barrier_probe.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    L.rx_mw_barrier_probe.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    ctl = torch.zeros(int(L.rx_mw_ctl_words()), dtype=torch.int32, device=dev)
    s = _hip.stream_ptr(dev)
    iters = int(os.environ.get("BARRIERS", "200"))
    out = {}

    def run(G, n, reps=7):
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            _hip.check(L.rx_mw_barrier_probe(ctypes.c_void_p(ctl.data_ptr()), G, n, 2.0, s), "rx_mw_barrier_probe")
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        if int(ctl[2].item()) != 0:
            raise RuntimeError(f"barrier timed out at G={G}")
        return statistics.median(ts)

    for G in (8, 16, 32, 64, 128, 256):
        t0 = run(G, 0)
        tn = run(G, iters)
        out[G] = {"launch_us": round(t0, 2), "per_barrier_us": round((tn - t0) / iters, 3)}
    print(json.dumps({"bench": "grid barrier (mw_barrier form)", "barriers_per_launch": iters,
                      "by_workgroups": out}), flush=True)


if __name__ == "__main__":
    main()
