"""Checkpoint writer for state dicts whose layout repeats from save to save.

``torch.save`` spends most of its time pickling: its ``persistent_id`` hook runs in Python for
every object of the state dict (about 600 calls for the 48k-parameter NYC model, ~1 ms), while
writing the tensor bytes is a handful of C++ calls. The pickle (``data.pkl``) depends only on
the keys and on every tensor's dtype / shape / stride / storage offset / storage identity --
not on the values -- and a training job saves the same layout at every epoch and every fit.

``save_state_dict`` therefore keeps the pickle of each layout it has seen (taken from one
``torch.save`` of that layout, so it is torch's own bytes) and writes later checkpoints of the
same layout as that pickle plus the storages, through torch's zip writer, record for record
what ``torch.serialization._save`` writes. The first fast write of a layout is read back with
``torch.load(weights_only=True)`` and compared bit for bit with the state dict; any difference
or error sends that layout back to ``torch.save`` for good. The file is a regular ``model.pt``.
"""
import io
import sys
import threading
import zipfile
from collections import OrderedDict
from typing import Dict, Optional, Tuple

import torch

_lock = threading.Lock()
_layouts: Dict[tuple, Optional[bytes]] = {}   # layout -> data.pkl (None: use torch.save)
_verified: set = set()


def _layout(sd) -> Optional[Tuple[tuple, list]]:
    """(layout key, storages in torch's first-encounter key order) or None if unsupported."""
    if not isinstance(sd, (dict, OrderedDict)):
        return None
    ids: Dict[int, int] = {}
    storages = []
    # the pickle also carries the dict's type and the state dict's per-module ``_metadata``
    key = [type(sd).__name__, repr(getattr(sd, "_metadata", None))]
    for k, v in sd.items():
        if not isinstance(k, str) or type(v) is not torch.Tensor or v.device.type != "cpu" \
                or v.requires_grad or v.is_sparse or v.is_quantized:
            return None
        st = v.untyped_storage()
        ptr = st.data_ptr()
        sid = ids.get(ptr)
        if sid is None:
            sid = ids[ptr] = len(storages)
            storages.append((st, v.dtype))
        key.append((k, v.dtype, tuple(v.shape), v.stride(), v.storage_offset(), sid, st.nbytes()))
    return tuple(key), storages


def _pickle_of(sd) -> bytes:
    buf = io.BytesIO()
    torch.save(sd, buf)
    with zipfile.ZipFile(io.BytesIO(buf.getvalue())) as z:
        name = next(n for n in z.namelist() if n.endswith("/data.pkl"))
        return z.read(name)


def _write(path: str, pkl: bytes, storages) -> None:
    from torch import serialization as S
    with S._open_zipfile_writer(path) as f:       # __enter__ yields the PyTorchFileWriter
        f.write_record("data.pkl", pkl, len(pkl))
        f.write_record(".format_version", "1", 1)
        align = str(S._get_storage_alignment())
        f.write_record(".storage_alignment", align, len(align))
        f.write_record("byteorder", sys.byteorder, len(sys.byteorder))
        for i, (st, _dt) in enumerate(storages):
            f.write_record(f"data/{i}", st, st.nbytes())


def _bytes(t):
    return t.contiguous().reshape(-1).view(torch.uint8)


def _same(a, b) -> bool:
    if list(a.keys()) != list(b.keys()):
        return False
    for k in a:
        x, y = a[k], b[k]
        if x.dtype != y.dtype or x.shape != y.shape or x.stride() != y.stride():
            return False
        if not torch.equal(_bytes(x), _bytes(y)):     # bitwise: NaN payloads included
            return False
    return True


def save_state_dict(sd, path: str) -> bool:
    """Write ``sd`` to ``path`` as ``torch.save`` would; returns True when the cached-pickle
    path wrote it, False when it fell back to ``torch.save``."""
    lay = _layout(sd)
    if lay is None:
        torch.save(sd, path)
        return False
    key, storages = lay
    with _lock:
        known = key in _layouts
        pkl = _layouts.get(key)
    if known and pkl is None:
        torch.save(sd, path)
        return False
    if not known:
        try:
            pkl = _pickle_of(sd)
        except Exception:  # noqa: BLE001
            pkl = None
        with _lock:
            if len(_layouts) >= 256:        # bounded: layouts of long-gone models drop out
                _layouts.clear()
                _verified.clear()
            _layouts[key] = pkl
        if pkl is None:
            torch.save(sd, path)
            return False
    try:
        _write(path, pkl, storages)
        if key not in _verified:
            ok = _same(sd, torch.load(path, map_location="cpu", weights_only=True))
            if not ok:
                raise ValueError("read-back mismatch")
            with _lock:
                _verified.add(key)
    except Exception:  # noqa: BLE001 - torch internals moved: this layout uses torch.save
        with _lock:
            _layouts[key] = None
        torch.save(sd, path)
        return False
    return True
