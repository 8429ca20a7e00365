"""Python garbage-collector time inside a region (observability).

The driver of a Spark-on-Ray job holds a large heap (torch, pyarrow, the engine's plans): one
full (generation-2) collection of it costs tens of milliseconds -- 89 ms measured in the middle
of the DLRM notebook preprocessing on this container, a third of that pipeline's wall time.
:class:`GcMeter` records how much of a region the collector took, so a benchmark can report it
next to its wall time instead of it showing up as unexplained jitter, and
:func:`freeze_long_lived` moves the long-lived state of a process (imported modules, built
engines) out of the collector's reach.
"""
import gc
import time
from typing import Dict, List


class GcMeter:
    """``with GcMeter() as m: ...`` then ``m.summary()`` -> collector ms and collections per
    generation inside the block (``gc.callbacks``; the collector itself is not changed)."""

    def __init__(self):
        self._start: Dict[int, float] = {}
        self.ms = 0.0
        self.max_ms = 0.0
        self.collections: List[int] = [0, 0, 0]

    def _cb(self, phase, info):
        g = info.get("generation", 0)
        if phase == "start":
            self._start[g] = time.perf_counter()
        else:
            t0 = self._start.pop(g, None)
            if t0 is not None:
                dt = (time.perf_counter() - t0) * 1e3
                self.ms += dt
                self.max_ms = max(self.max_ms, dt)
                if 0 <= g < 3:
                    self.collections[g] += 1

    def __enter__(self):
        gc.callbacks.append(self._cb)
        return self

    def __exit__(self, *exc):
        try:
            gc.callbacks.remove(self._cb)
        except ValueError:
            pass
        return False

    def summary(self) -> Dict[str, object]:
        return {"gc_ms": round(self.ms, 3), "gc_max_ms": round(self.max_ms, 3),
                "collections_by_generation": list(self.collections)}


def freeze_long_lived() -> int:
    """Move every object alive now to the permanent generation (``gc.freeze``): later
    collections -- the full ones included -- no longer walk it. No ``gc.collect()`` first: on the
    MI355X box a collect+freeze made the next pipeline slower than a plain freeze (the freed
    memory is faulted in again). Returns the number of objects frozen."""
    gc.freeze()
    return gc.get_freeze_count()
