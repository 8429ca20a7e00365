"""Named executor actors (``raydp-executor-<id>``) registered by the cluster backend."""
import threading

_lock = threading.RLock()
_executors = {}


def register_executor(name, handle):
    with _lock:
        _executors[name] = handle


def unregister_executor(name):
    with _lock:
        _executors.pop(name, None)


def lookup_executor(name):
    with _lock:
        return _executors.get(name)
