"""Tracing: named spans as Chrome-trace events and (optionally) roctx ranges.

The reference has no tracing of its own (it relies on Ray's dashboard and the
Spark UI). Here every phase of the data + training path is a span — ETL stage, executor task,
Spark->dataset conversion, HBM ingest, train / eval epoch, checkpoint — so one timeline shows
where an end-to-end second goes:

* ``spark.ray.mi355x.trace=<path>`` (env ``RAYDP_TRACE``): each process appends its spans to
  ``<path>.<pid>.jsonl``; the native services (supervisor, app master, shuffle service) write
  their events to the same place (``csrc/common/trace.h``). :func:`merge` folds all of them
  into one JSON for chrome://tracing or Perfetto.
* ``spark.ray.mi355x.roctx=1`` (env ``RAYDP_ROCTX``): every span is also a roctx range, so
  ``rocprofv3 --marker-trace`` shows the phases around the kernels.

Spans cost one ``time.time_ns()`` pair when disabled checks are off; when neither is set they
are a no-op context manager.
"""
import contextlib
import ctypes
import glob
import json
import os
import threading
import time
from typing import Dict, Iterator, List, Optional

_lock = threading.Lock()
_file = None
_file_pid = None
_roctx = None
_roctx_tried = False


def _path() -> Optional[str]:
    return os.environ.get("RAYDP_TRACE") or None


def enabled() -> bool:
    return bool(_path()) or _roctx_enabled()


def _roctx_enabled() -> bool:
    return os.environ.get("RAYDP_ROCTX", "0") not in ("0", "", "false", "False")


def _roctx_lib():
    global _roctx, _roctx_tried
    if not _roctx_tried:
        _roctx_tried = True
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except OSError:
                continue
    return _roctx


def _sink():
    global _file, _file_pid
    p = _path()
    if not p:
        return None
    if _file is None or _file_pid != os.getpid():
        d = os.path.dirname(os.path.abspath(p))
        os.makedirs(d, exist_ok=True)
        _file = open(f"{p}.{os.getpid()}.jsonl", "a", buffering=1)
        _file_pid = os.getpid()
    return _file


def _emit(ev: Dict):
    with _lock:
        f = _sink()
        if f is not None:
            f.write(json.dumps(ev, default=str) + "\n")


def set_trace_path(path: Optional[str]):
    """Enable (or with None disable) the Chrome-trace sink for this process and its children."""
    global _file
    if path:
        os.environ["RAYDP_TRACE"] = path
    else:
        os.environ.pop("RAYDP_TRACE", None)
    with _lock:
        if _file is not None:
            _file.close()
        _file = None


@contextlib.contextmanager
def span(name: str, cat: str = "raydp", **args) -> Iterator[None]:
    if not (_path() or _roctx_enabled()):
        yield
        return
    rl = _roctx_lib() if _roctx_enabled() else None
    if rl is not None:
        rl.roctxRangePushA(f"{cat}:{name}".encode())
    t0 = time.time_ns()
    try:
        yield
    finally:
        t1 = time.time_ns()
        if rl is not None:
            rl.roctxRangePop()
        if _path():
            _emit({"name": name, "cat": cat, "ph": "X", "ts": t0 / 1000.0, "dur": (t1 - t0) / 1000.0,
                   "pid": os.getpid(), "tid": threading.get_ident() % 100000, "args": args})


def complete(name: str, t0_ns: int, cat: str = "raydp", t1_ns: Optional[int] = None, tid: Optional[int] = None,
             **args):
    """Record a span that started at ``t0_ns`` (``time.time_ns()``) and ends at ``t1_ns``
    (default: now), on thread row ``tid`` (default: the calling thread)."""
    if _path():
        t1 = time.time_ns() if t1_ns is None else t1_ns
        _emit({"name": name, "cat": cat, "ph": "X", "ts": t0_ns / 1000.0, "dur": (t1 - t0_ns) / 1000.0,
               "pid": os.getpid(), "tid": threading.get_ident() % 100000 if tid is None else tid, "args": args})


def instant(name: str, cat: str = "raydp", **args):
    if _roctx_enabled():
        rl = _roctx_lib()
        if rl is not None:
            rl.roctxMarkA(f"{cat}:{name}".encode())
    if _path():
        _emit({"name": name, "cat": cat, "ph": "i", "s": "p", "ts": time.time_ns() / 1000.0,
               "pid": os.getpid(), "tid": threading.get_ident() % 100000, "args": args})


def merge(path: Optional[str] = None, out: Optional[str] = None) -> str:
    """Fold every ``<path>.<pid>.jsonl`` (Python and native) into ``out`` (default
    ``<path>.json``) with process-name metadata; returns the output path."""
    path = path or _path()
    if not path:
        raise ValueError("no trace path")
    with _lock:
        if _file is not None:
            _file.flush()
    events: List[Dict] = []
    for fn in sorted(glob.glob(f"{glob.escape(path)}.*.jsonl")):
        with open(fn) as f:
            for line in f:
                line = line.strip()
                if line:
                    try:
                        events.append(json.loads(line))
                    except ValueError:
                        continue
    names = {}
    for e in events:
        pid = e.get("pid")
        if pid not in names:
            names[pid] = e.get("cat", "process")
    meta = [{"name": "process_name", "ph": "M", "pid": pid, "args": {"name": f"{n} ({pid})"}}
            for pid, n in names.items()]
    out = out or path + ".json"
    with open(out, "w") as f:
        json.dump({"traceEvents": meta + sorted(events, key=lambda e: e.get("ts", 0)),
                   "displayTimeUnit": "ms"}, f)
    return out
