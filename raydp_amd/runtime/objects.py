"""Object references and the object-store front end (``put`` / ``get`` / ``free``).

Objects live in the node's shared-memory store (``csrc/runtime/objstore.cc`` via
``raydp_amd.runtime.store``) when a runtime node is up; Arrow tables are stored as Arrow IPC
so every process reads them zero-copy from the mapped arena. Without a running node the
objects stay in this process (driver-only use, unit tests).

An ``ObjectRef`` may carry *lineage* — the task that produced it — so a lost object
(its node was removed, or the store entry was evicted) is transparently re-created on
``get`` (parity: ``@ray.remote(max_retries=-1)`` fetch tasks in
``python/raydp/spark/dataset.py:54``).
"""
import threading
import uuid
from typing import Any, Callable, Dict, Optional

_local_lock = threading.RLock()
_local: Dict[str, Any] = {}


class ObjectLostError(RuntimeError):
    pass


class ObjectRef:
    __slots__ = ("id", "owner", "node_id", "_lineage", "__weakref__")

    def __init__(self, oid: Optional[str] = None, owner: str = "driver",
                 node_id: Optional[str] = None, lineage: Optional[Callable[[], Any]] = None):
        self.id = oid or uuid.uuid4().hex
        self.owner = owner
        self.node_id = node_id
        self._lineage = lineage

    def hex(self):
        return self.id

    def binary(self):
        return bytes.fromhex(self.id)

    def task_id(self):
        return self.id[:16]

    def __repr__(self):
        return f"ObjectRef({self.id})"

    def __hash__(self):
        return hash(self.id)

    def __eq__(self, other):
        return isinstance(other, ObjectRef) and other.id == self.id

    def __reduce__(self):
        # lineage closures stay with the owner; a deserialized ref resolves by id
        return (ObjectRef, (self.id, self.owner, self.node_id, None))

    def future(self):
        import concurrent.futures
        f = concurrent.futures.Future()
        f.set_result(get(self))
        return f


def _store():
    from raydp_amd.runtime import core
    node = core.current_node_store()
    return node


def put(value: Any, _owner: str = "driver", _lineage=None) -> ObjectRef:
    ref = ObjectRef(owner=_owner, lineage=_lineage)
    store = _store()
    if store is not None:
        store.put(ref.id, value)
        ref.node_id = store.node_id
    else:
        with _local_lock:
            _local[ref.id] = value
    return ref


def put_with_id(oid: str, value: Any, node_id: Optional[str] = None):
    from raydp_amd.runtime.core import store_for
    store = store_for(node_id) if node_id is not None else _store()
    if store is None:
        store = _store()
    if store is not None:
        store.put(oid, value)
    else:
        with _local_lock:
            _local[oid] = value


def contains(ref: ObjectRef) -> bool:
    from raydp_amd.runtime.core import store_for
    store = store_for(ref.node_id) if ref.node_id is not None else _store()
    if store is not None and store.contains(ref.id):
        return True
    with _local_lock:
        return ref.id in _local


_GET_SPIN = []


def _spin_until_done(fut):
    """Poll a pending call's future for up to ``RAYDP_ACTOR_SPIN_US`` before blocking on it: the
    reply is set by the connection's reader thread, and a getter asleep on the future's
    condition pays a second wake-up (csrc/runtime/spin.cc). ``time.sleep(0)`` hands the GIL
    over on every turn, so the reader thread is never kept from setting the result."""
    if not _GET_SPIN:
        import os
        try:
            _GET_SPIN.append(float(os.environ.get("RAYDP_ACTOR_SPIN_US", "0") or 0) * 1e-6)
        except ValueError:
            _GET_SPIN.append(0.0)
    window = _GET_SPIN[0]
    if window <= 0:
        return
    import time
    end = time.perf_counter() + window
    while not fut.done() and time.perf_counter() < end:
        time.sleep(0)


def get(ref, timeout: Optional[float] = None):
    if isinstance(ref, (list, tuple)):
        return [get(r, timeout) for r in ref]
    if not isinstance(ref, ObjectRef):
        return ref
    from raydp_amd.runtime import core
    pending = core.pending_result(ref)
    if pending is not None:
        if not pending.done():
            _spin_until_done(pending)
        return pending.result(timeout)
    from raydp_amd.runtime.core import store_for
    store = store_for(ref.node_id) if ref.node_id is not None else _store()
    if store is not None:
        found, value = store.get(ref.id)
        if found:
            return value
    with _local_lock:
        if ref.id in _local:
            return _local[ref.id]
    if ref._lineage is None and store is not None and getattr(core.current_node(), "gcs", None) is not None:
        # an attached driver holds refs other processes produce: the object may still be in
        # flight (Ray's get blocks until it is sealed) -- poll the arena for a bounded time
        value = _poll_store(store, ref.id, timeout)
        if value is not _MISSING:
            return value
    if ref._lineage is not None:
        # reconstruct from lineage (re-run the producing task) and re-seal under the same id
        value = ref._lineage()
        put_with_id(ref.id, value)
        st = _store()
        ref.node_id = st.node_id if st is not None else None
        return value
    raise ObjectLostError(f"object {ref.id} is lost and has no lineage to reconstruct it")


_MISSING = object()


def _poll_store(store, oid: str, timeout: Optional[float]):
    import os
    import time
    limit = float(timeout if timeout is not None else os.environ.get("RAYDP_GET_TIMEOUT_S", "60"))
    end = time.monotonic() + limit
    delay = 0.0005
    while time.monotonic() < end:
        time.sleep(delay)
        delay = min(delay * 2, 0.05)
        found, value = store.get(oid)
        if found:
            return value
    return _MISSING


def free(refs):
    if isinstance(refs, ObjectRef):
        refs = [refs]
    from raydp_amd.runtime.core import store_for
    for r in refs:
        store = store_for(r.node_id) if r.node_id is not None else _store()
        if store is not None:
            store.delete(r.id)
        with _local_lock:
            _local.pop(r.id, None)
