"""Actor call round trip on this host: a no-op call and a 100 KB echo through the runtime's
Unix-socket transport (raydp_amd/runtime/actor_worker.py), each after a short idle gap (the
callee sleeping in recv) and back to back."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import raydp_amd.runtime as rt  # noqa: E402


def main():
    rt.init(num_cpus=4)

    @rt.remote
    class A:
        def echo(self, x=None):
            return x
    a = A.remote()
    rt.get(a.echo.remote())
    out = {}
    for name, arg, gap in (("noop", None, 0.0), ("noop_after_5ms_idle", None, 0.005),
                           ("noop_after_5ms_busy", None, -0.005),
                           ("echo_100KB", b"x" * 100_000, 0.0)):
        ts = []
        for _ in range(300):
            if gap > 0:
                time.sleep(gap)
            elif gap < 0:                 # busy idle: the caller never sleeps
                e = time.perf_counter() - gap
                while time.perf_counter() < e:
                    pass
            t = time.perf_counter()
            rt.get(a.echo.remote(arg))
            ts.append(time.perf_counter() - t)
        ts.sort()
        out[name] = {"p10_us": round(ts[30] * 1e6, 1), "p50_us": round(ts[150] * 1e6, 1),
                     "p90_us": round(ts[270] * 1e6, 1)}
    print(json.dumps(out))
    rt.shutdown()


if __name__ == "__main__":
    main()
