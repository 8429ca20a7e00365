"""Cross-process serialization with Arrow data passed through the shared-memory store.

``dumps`` is cloudpickle with a ``reducer_override``: every ``pyarrow.Table``/``RecordBatch``
above a small threshold is written once into the node's object store (Arrow IPC straight into
the arena) and pickled as a 32-byte id; ``loads`` maps it back zero-copy. Tables that were
themselves read from the store are passed by their existing id without a copy. This is how
task closures (plans holding materialised partitions), task results and actor-call arguments
move between the driver and actor processes (Ray does the same with plasma-backed
``ObjectRef`` arguments; reference: Arrow blocks in ``python/raydp/spark/dataset.py:54-84``).

Ownership: ``transfer=True`` objects are deleted by the (single) consumer right after it maps
them (the mapping pins the memory, so the bytes stay valid for as long as the table lives);
with ``transfer=False`` the producer keeps the ids (``Payload.oids``) and frees them after
all consumers are done (broadcast of one stage closure to many executors).
"""
import collections
import io
import sys
import threading
import types
import uuid
import weakref
from typing import Any, List, Optional, Tuple

import cloudpickle
import pyarrow as pa

THRESHOLD = 64 * 1024


# cloudpickle looks for imported submodules of every by-value function's module globals by
# scanning all of sys.modules (``_find_imported_submodules``): with torch loaded that is ~1,000
# names per function, and a stage closure holds ~40 functions (5 ms per stage payload). Same
# result from an index of sys.modules by parent package, rebuilt when sys.modules changes.
_sub_index = (None, {})


def _find_imported_submodules(code, top_level_dependencies):
    global _sub_index
    mods = sys.modules
    key = (len(mods), next(reversed(mods)) if mods else None)
    if _sub_index[0] != key:
        idx = collections.defaultdict(list)
        for name in list(mods):
            if name is None:
                continue
            parts = name.split(".")
            for i in range(1, len(parts)):
                idx[".".join(parts[:i])].append(name)
        _sub_index = (key, idx)
    idx = _sub_index[1]
    names = set(code.co_names)
    out = []
    for x in top_level_dependencies:
        if isinstance(x, types.ModuleType) and getattr(x, "__package__", None):
            prefix = x.__name__
            for name in idx.get(prefix, ()):
                if not set(name[len(prefix) + 1:].split(".")) - names and name in mods:
                    out.append(mods[name])
    return out


cloudpickle.cloudpickle._find_imported_submodules = _find_imported_submodules
_views_lock = threading.Lock()
_views = {}   # id(table) -> (weakref(table), oid): tables mapped from the store


def remember_view(table, oid: str):
    try:
        r = weakref.ref(table, lambda _r, k=id(table): _forget(k))
    except TypeError:
        return
    with _views_lock:
        _views[id(table)] = (r, oid)


def _forget(k):
    with _views_lock:
        _views.pop(k, None)


def _view_oid(table) -> Optional[str]:
    with _views_lock:
        e = _views.get(id(table))
    if e is not None and e[0]() is table:
        return e[1]
    return None


def _store():
    from raydp_amd.runtime import core
    return core.current_node_store()


def _store_of(node_id: str, path: str):
    from raydp_amd.runtime import core
    st = core.store_for(node_id, path)
    if st is None:
        from raydp_amd.runtime.objects import ObjectLostError
        raise ObjectLostError(f"object store of node {node_id} is gone")
    return st


def _adopt(st, v, node_id: str, path: str, oid: str):
    """Make ``v`` (a view of store object ``oid``) its owner: the object is deleted when the
    view is collected (deferred by the store while other processes still pin it)."""
    remember_view(v, (node_id, path, oid))
    weakref.finalize(v, _delete_quietly, st, oid)
    return v


def _delete_quietly(st, oid):
    try:
        if st._h is not None:
            st.delete(oid)
    except Exception:  # noqa: BLE001
        pass


def _load_owned(node_id: str, path: str, oid: str):
    """Consumer side of a transferred table: map zero-copy and take ownership of the entry."""
    st = _store_of(node_id, path)
    found, v = st.get(oid)
    if not found:
        raise RuntimeError(f"transferred object {oid} missing from the store")
    if isinstance(v, pa.Table):
        return _adopt(st, v, node_id, path, oid)
    st.delete(oid)
    return v


def share_table(t: pa.Table) -> pa.Table:
    """Copy ``t`` into the node's store once and return the owning zero-copy view: later
    pickles of the view travel as a reference (used for driver-side source tables)."""
    st = _store()
    if st is None or not isinstance(t, pa.Table) or _view_oid(t) is not None:
        return t
    oid = uuid.uuid4().hex
    st.put(oid, t)
    found, v = st.get(oid)
    return _adopt(st, v, st.node_id, st.path, oid)


def _load_shared(node_id: str, path: str, oid: str):
    st = _store_of(node_id, path)
    found, v = st.get(oid)
    if not found:
        raise RuntimeError(f"shared object {oid} missing from the store")
    remember_view(v, (node_id, path, oid))
    return v


_FLAT_DISPATCH = [None, -1]


def _flat_dispatch():
    """cloudpickle's dispatch table is a ChainMap over copyreg's: the C pickler then looks every
    object's type up through Python-level ``ChainMap.__getitem__`` / ``__missing__`` (~2 us
    each, 40 % of a model payload's pickling). The same mapping as one dict, rebuilt when
    copyreg gains entries."""
    import copyreg
    n = len(copyreg.dispatch_table)
    if _FLAT_DISPATCH[0] is None or _FLAT_DISPATCH[1] != n:
        _FLAT_DISPATCH[0] = dict(cloudpickle.CloudPickler.dispatch_table)
        _FLAT_DISPATCH[1] = n
    return _FLAT_DISPATCH[0]


class _Pickler(cloudpickle.CloudPickler):
    def __init__(self, f, transfer: bool):
        # the C pickler reads dispatch_table once, in __init__: set it on the class first
        _Pickler.dispatch_table = _flat_dispatch()
        super().__init__(f, protocol=5)
        self.transfer = transfer
        self.oids: List[str] = []
        self.store = _store()

    def reducer_override(self, obj):
        # every object of the stream passes through here (a model + optimizer payload: ~300
        # modules, dicts and tensors): decide by type once per type, not by a chain of checks
        kind = _KIND.get(type(obj))
        if kind is None:
            kind = _classify(type(obj))
        if kind == _PLAIN:
            # an instance of an ordinary class: cloudpickle's reducer_override returns
            # NotImplemented for those too (it rewrites classes and functions only)
            return NotImplemented
        if kind == _CLOUD:
            return super().reducer_override(obj)
        if kind == _TENSOR:
            red = _reduce_cpu_tensor(self, obj)
            if red is not None:
                return red
            return super().reducer_override(obj)
        if isinstance(obj, pa.Schema):
            # one IPC message instead of pyarrow's field-by-field reduction (plans cache their
            # output schema on every node: ~25 fields x 20 nodes per stage closure)
            return _schema_from_ipc, (obj.serialize().to_pybytes(),)
        if isinstance(obj, (pa.Table, pa.RecordBatch)) and (self.store is None or obj.nbytes < THRESHOLD):
            # small tables travel inline as Arrow IPC: unlike Arrow's own pickling, IPC writes
            # only the sliced range of each buffer (a slice must not drag its parent along)
            return _from_ipc, (_to_ipc(obj), isinstance(obj, pa.RecordBatch))
        if type(obj).__name__ == "MapPlan" and getattr(obj, "rel", None) is not None:
            # a chain of fusible operators ships as a cached structure + its source
            from raydp_amd.spark import exprc
            red = exprc.chain_reduce(obj)
            if red is not None:
                return red
        if self.store is not None and isinstance(obj, (pa.Table, pa.RecordBatch)) and obj.nbytes >= THRESHOLD:
            existing = _view_oid(obj)
            if existing is not None:
                return _load_shared, existing
            oid = uuid.uuid4().hex
            self.store.put(oid, obj)
            key = (self.store.node_id, self.store.path, oid)
            if self.transfer:
                return _load_owned, key
            self.oids.append(oid)
            return _load_shared, key
        return super().reducer_override(obj)


_PLAIN, _TENSOR, _CHECK, _CLOUD = 0, 1, 2, 3
_KIND = {}      # type -> how reducer_override treats its instances


def _classify(tp) -> int:
    """_TENSOR for torch.Tensor itself, _CHECK for the Arrow / plan types reducer_override
    rewrites (and their subclasses), _PLAIN for everything else (cloudpickle's own rules)."""
    t = _torch_tensor_type()
    if t is not None and tp is t:
        kind = _TENSOR
    elif issubclass(tp, (pa.Schema, pa.Table, pa.RecordBatch)) or tp.__name__ == "MapPlan":
        kind = _CHECK
    elif issubclass(tp, type) or issubclass(tp, types.FunctionType):
        kind = _CLOUD          # classes and functions: cloudpickle decides by value / reference
    else:
        kind = _PLAIN
    if t is not None or kind != _PLAIN:
        # before torch is imported, a plain verdict might be torch.Tensor's own later: not cached
        _KIND[tp] = kind
    return kind


def _torch_tensor_type():
    """torch.Tensor when torch is already imported (never imports it)."""
    m = sys.modules.get("torch")
    return getattr(m, "Tensor", None) if m is not None else None


class _StorageBox:
    """One CPU storage's bytes in a pickle stream, pickled once however many tensors view it
    (the pickler memoises the box): torch's own tensor pickling runs a whole ``torch.save``
    per storage, ~60 us each -- a model + optimizer payload pays that per parameter."""
    __slots__ = ("st",)

    def __init__(self, st):
        self.st = st

    def __reduce__(self):
        import numpy as np
        n = self.st.nbytes()
        import torch
        raw = torch.empty(0, dtype=torch.uint8).set_(self.st, 0, (n,), (1,)).numpy() if n else np.zeros(0, np.uint8)
        return _storage_from_bytes, (raw,)


def _storage_from_bytes(raw):
    import torch
    return torch.from_numpy(raw.copy() if not raw.flags.writeable else raw).untyped_storage()


def _reduce_cpu_tensor(pickler, obj):
    if obj.device.type != "cpu" or obj.layout.__repr__() != "torch.strided" or obj.is_quantized or \
            obj.is_conj() or obj.is_neg() or obj.requires_grad and obj.grad_fn is not None or \
            obj._backward_hooks:
        return None
    st = obj.untyped_storage()
    boxes = pickler.__dict__.setdefault("_storages", {})
    key = (st.data_ptr(), st.nbytes())
    box = boxes.get(key)
    if box is None:
        box = boxes[key] = _StorageBox(st)
    return _tensor_from_storage, (box, str(obj.dtype).split(".")[-1], obj.storage_offset(), tuple(obj.size()),
                                  tuple(obj.stride()), bool(obj.requires_grad))


def _tensor_from_storage(st, dtype: str, offset: int, size, stride, requires_grad: bool):
    import torch
    t = torch.empty(0, dtype=getattr(torch, dtype)).set_(st, offset, size, stride)
    if requires_grad:
        t.requires_grad_(True)
    return t


def _schema_from_ipc(data: bytes) -> pa.Schema:
    return pa.ipc.read_schema(pa.py_buffer(data))


def _to_ipc(obj) -> bytes:
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, obj.schema) as w:
        if isinstance(obj, pa.RecordBatch):
            w.write_batch(obj)
        else:
            w.write_table(obj)
    return sink.getvalue().to_pybytes()


def _from_ipc(data: bytes, batch: bool = False):
    t = pa.ipc.open_stream(pa.py_buffer(data)).read_all()
    if batch:
        return t.combine_chunks().to_batches()[0] if t.num_rows else pa.RecordBatch.from_pylist([], t.schema)
    return t


class Payload:
    __slots__ = ("data", "oids")

    def __init__(self, data: bytes, oids: List[str]):
        self.data, self.oids = data, oids

    def free(self):
        st = _store()
        if st is not None:
            for o in self.oids:
                st.delete(o)
        self.oids = []


def dumps(obj: Any, transfer: bool = True) -> bytes:
    f = io.BytesIO()
    p = _Pickler(f, transfer)
    p.dump(obj)
    if not transfer and p.oids:
        raise ValueError("use dumps_shared() for broadcast payloads")
    return f.getvalue()


def dumps_shared(obj: Any) -> Payload:
    f = io.BytesIO()
    p = _Pickler(f, transfer=False)
    p.dump(obj)
    return Payload(f.getvalue(), p.oids)


def loads(data) -> Any:
    return cloudpickle.loads(data)


_ = Tuple
