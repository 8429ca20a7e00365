"""Legacy ``Dataset.to_torch`` iterable: ``(features, label)`` mini-batches as torch tensors.

Feature layout rules (Ray Data 1.x contract the reference estimator relies on,
``python/raydp/torch/estimator.py:300-330``): ``feature_columns`` as a list of names ->
one ``[B, F]`` tensor (one dtype); a list of lists -> a list of ``[B, F_i]`` tensors; a dict
name -> list -> a dict of tensors. Columns are converted with one numpy stack per batch; the
label is ``[B, 1]`` when ``unsqueeze_label_tensor``.

On a GPU device (``to_torch(..., device="cuda")``) the iterable is device-resident instead: the
first iteration ingests the whole shard into HBM once (pinned DMA + the ``arrow_ingest`` HIP
kernel, ``raydp_amd.ops.ingest``) and every batch of every epoch is a slice view of those
tensors -- no per-batch host conversion, no per-batch H2D copy.
"""
from typing import Any, List, Optional

import numpy as np


def _np_dtype(tdt):
    import torch
    if tdt is None:
        return np.float32
    return torch.empty((), dtype=tdt).numpy().dtype


class TorchBatchIterable:
    def __init__(self, ds, label_column, feature_columns, label_dtype, feature_dtypes, batch_size, drop_last,
                 unsqueeze_label, device="cpu"):
        self.ds = ds
        self.label_column = label_column
        self.feature_columns = feature_columns
        self.label_dtype = label_dtype
        self.feature_dtypes = feature_dtypes
        self.batch_size = int(batch_size)
        self.drop_last = drop_last
        self.unsqueeze_label = unsqueeze_label
        self.device = device

    def _cols(self, t, names: List[str], dtype) -> Any:
        import torch
        if isinstance(t, list):     # device path: the whole shard (list of tables) at once
            from raydp_amd.ops.ingest import ingest_columns
            dt = dtype or torch.float32
            ints = not dt.is_floating_point and dt != torch.bool
            m = ingest_columns(t, list(names), self.device, False, out_i64=ints)
            return m if m.dtype == dt else m.to(dt)
        nd = _np_dtype(dtype)
        arr = np.stack([t.column(c).to_numpy(zero_copy_only=False).astype(nd, copy=False) for c in names], axis=1)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(self.device)

    def _features(self, t):
        fc = self.feature_columns
        if fc is None:
            fc = [c for c in t.column_names if c != self.label_column]
        fd = self.feature_dtypes
        if isinstance(fc, dict):
            return {k: self._cols(t, v if isinstance(v, list) else [v], fd.get(k) if isinstance(fd, dict) else fd)
                    for k, v in fc.items()}
        if fc and isinstance(fc[0], (list, tuple)):
            dts = fd if isinstance(fd, (list, tuple)) else [fd] * len(fc)
            return [self._cols(t, list(names), dt) for names, dt in zip(fc, dts)]
        if isinstance(fd, (list, tuple)):
            # Ray Data semantics: a flat list of names is ONE [B, F] tensor; per-column dtypes are
            # applied first and the columns concatenated with type promotion
            if len({d for d in fd}) <= 1:
                return self._cols(t, list(fc), fd[0] if fd else None)
            import torch
            return torch.cat([self._cols(t, [c], dt) for c, dt in zip(fc, fd)], dim=1)
        return self._cols(t, list(fc), fd)

    def _on_gpu(self) -> bool:
        import torch
        try:
            return torch.device(self.device).type == "cuda"
        except (RuntimeError, TypeError):
            return False

    def _resident_tensors(self):
        res = getattr(self, "_resident", None)
        if res is None:
            tables = [t for t in self.ds._get_tables() if t.num_rows]
            n = int(sum(t.num_rows for t in tables))
            if self.feature_columns is None and tables:
                self.feature_columns = [c for c in tables[0].column_names if c != self.label_column]
            feats = self._features(tables)
            label = None
            if self.label_column is not None:
                label = self._cols(tables, [self.label_column], self.label_dtype)
                if not self.unsqueeze_label:
                    label = label.view(-1)
            res = self._resident = (n, feats, label)
        return res

    def _iter_device(self):
        n, feats, label = self._resident_tensors()
        b = self.batch_size
        stop = n - n % b if self.drop_last else n

        def cut(x, s):
            if isinstance(x, dict):
                return {k: v[s:s + b] for k, v in x.items()}
            if isinstance(x, list):
                return [v[s:s + b] for v in x]
            return x[s:s + b]
        for s in range(0, stop, b):
            yield cut(feats, s), (label[s:s + b] if label is not None else None)

    def __iter__(self):
        import torch
        if self._on_gpu():
            yield from self._iter_device()
            return
        for t in self.ds.iter_batches(self.batch_size, "pyarrow", self.drop_last):
            feats = self._features(t)
            label: Optional[torch.Tensor] = None
            if self.label_column is not None:
                nd = _np_dtype(self.label_dtype)
                lab = t.column(self.label_column).to_numpy(zero_copy_only=False).astype(nd, copy=False)
                label = torch.from_numpy(np.ascontiguousarray(lab)).to(self.device)
                if self.unsqueeze_label:
                    label = label.unsqueeze(1)
            yield feats, label

    def __len__(self):
        n = self.ds.count()
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)
