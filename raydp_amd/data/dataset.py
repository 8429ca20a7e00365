"""Distributed Arrow ``Dataset`` (the Ray Data surface RayDP relies on).

Blocks are Arrow tables held in the object store (``ObjectRef``) or inline. Reference call
sites: ``ray.data.from_arrow_refs`` (``python/raydp/spark/dataset.py:222``),
``Dataset.random_shuffle`` (``torch/estimator.py:335-338``), ``session.get_dataset_shard(...)
.to_torch(...)`` (``torch/estimator.py:226-241``), ``iter_internal_ref_bundles`` /
``to_spark`` (``tests/test_spark_cluster.py:169-216``).

MI355X path: ``to_device_tensors`` packs the requested columns of every block of a shard into
ONE pinned host staging buffer and moves it to HBM with one DMA, then the HIP ``arrow_ingest``
kernel decodes/casts/null-fills in HBM (``raydp_amd/ops/ingest.py``); epochs then run from
device-resident tensors with a device-side shuffle permutation.
"""
import builtins
import math
from typing import Any, Callable, Dict, Iterator, List, Optional, Union

import numpy as np
import pyarrow as pa

from raydp_amd.runtime.objects import ObjectRef, get as _get, put as _put


class BlockMetadata:
    def __init__(self, num_rows, size_bytes, schema):
        self.num_rows, self.size_bytes, self.schema = num_rows, size_bytes, schema


class RefBundle:
    def __init__(self, blocks):
        self.blocks = blocks


class BlockSlice:
    """Rows [offset, offset + length) of a block held in the object store: an equal shard of a
    dataset references its rows where they already are (a few ids when pickled to a worker,
    resolved zero-copy from the node's store there), instead of a concatenated copy of them."""
    __slots__ = ("ref", "offset", "length")

    def __init__(self, ref, offset: int, length: int):
        self.ref, self.offset, self.length = ref, int(offset), int(length)

    def __getstate__(self):
        return (self.ref, self.offset, self.length)

    def __setstate__(self, st):
        self.ref, self.offset, self.length = st


class BlockGather:
    """The rows ``index`` (global row numbers over the concatenation of ``refs``) of object-store
    blocks, in that order: a shuffled dataset is a permutation over the blocks where they already
    are, so a shard of it pickles to a few ids plus its row numbers and each worker gathers its
    own rows (in parallel, zero-copy reads of the store) instead of the driver shuffling and
    shipping copies of every row."""
    __slots__ = ("refs", "index")

    def __init__(self, refs, index):
        self.refs, self.index = tuple(refs), np.asarray(index, dtype=np.int64)

    def __getstate__(self):
        return (self.refs, self.index)

    def __setstate__(self, st):
        self.refs, self.index = st

    def __len__(self):
        return int(self.index.size)


def _resolve(b) -> pa.Table:
    if isinstance(b, BlockSlice):
        return _resolve(b.ref).slice(b.offset, b.length)
    if isinstance(b, BlockGather):
        ts = [_resolve(r) for r in b.refs]
        t = ts[0] if len(ts) == 1 else pa.concat_tables(ts, promote_options="permissive")
        return t.take(pa.array(b.index))
    if isinstance(b, ObjectRef):
        b = _get(b)
    if isinstance(b, (bytes, bytearray, memoryview)):
        b = pa.ipc.open_stream(pa.py_buffer(b)).read_all()
    if isinstance(b, pa.RecordBatch):
        b = pa.Table.from_batches([b])
    return b


class DeferredDatasetError(RuntimeError):
    """The computation behind a deferred Dataset failed; ``original`` is its exception. Trainers
    pass it through untouched (no worker-group restart: rerunning the workers cannot fix the
    input) and ``fit_on_spark`` re-raises ``original``."""

    def __init__(self, original: BaseException):
        super().__init__(f"dataset computation failed: {original!r}")
        self.original = original


class _Then:
    """Future-like: ``fn(parent)`` of a deferred parent Dataset, computed once, on the first
    ``result()`` (a failure of the parent's own computation is re-raised as itself)."""

    def __init__(self, parent, fn):
        import threading
        self.parent, self.fn = parent, fn
        self._lock = threading.Lock()
        self._done, self._val, self._exc = False, None, None

    def result(self):
        with self._lock:
            if not self._done:
                try:
                    _ = self.parent._blocks          # resolve the parent first
                    self._val = self.fn(self.parent)
                except DeferredDatasetError as e:
                    self._exc = e.original
                except BaseException as e:  # noqa: BLE001
                    self._exc = e
                self._done = True
        if self._exc is not None:
            raise self._exc
        return self._val


class Dataset:
    def __init__(self, blocks: List[Union[ObjectRef, pa.Table]], schema: Optional[pa.Schema] = None):
        import threading
        self._lock = threading.Lock()     # resolves a deferred dataset once, whoever asks first
        self._pending = None
        self._blocks_ = list(blocks)
        self._schema_ = schema
        self._tables: Optional[List[pa.Table]] = None

    @classmethod
    def deferred(cls, future) -> "Dataset":
        """A Dataset whose blocks are still being produced: ``future`` (``concurrent.futures``)
        yields a ``Dataset``. Ray Data datasets are lazy the same way; the estimators use it to
        build the training engine while the Spark stage that fills the blocks runs on the
        executors. Anything touching blocks or schema waits for the future."""
        ds = cls([], None)
        ds._pending = future
        return ds

    def _wait(self):
        with self._lock:
            fut = self._pending
            if fut is None:               # another thread resolved it meanwhile
                return
            try:
                done = fut.result()
            except BaseException as e:  # noqa: BLE001 - every later access reports the same failure
                raise DeferredDatasetError(e) from e
            self._blocks_, self._schema_ = done._blocks, done._schema
            self._pending = None

    @property
    def _blocks(self):
        if self._pending is not None:
            self._wait()
        return self._blocks_

    @_blocks.setter
    def _blocks(self, v):
        self._blocks_ = v

    @property
    def _schema(self):
        if self._pending is not None:
            self._wait()
        return self._schema_

    @_schema.setter
    def _schema(self, v):
        self._schema_ = v

    def __getstate__(self):
        # shipping a dataset to another process ships its resolved blocks
        _ = self._blocks
        d = dict(self.__dict__)
        d["_pending"] = None
        d.pop("_lock", None)
        return d

    def __setstate__(self, d):
        import threading
        self.__dict__.update(d)
        self._lock = threading.Lock()

    # ---------------------------------------------------------------- internals ----------
    def _get_tables(self) -> List[pa.Table]:
        if self._tables is None:
            self._tables = [_resolve(b) for b in self._blocks]
        return self._tables

    def _from_tables(self, tables):
        return Dataset(tables, self.schema())

    # ---------------------------------------------------------------- metadata -----------
    def schema(self) -> pa.Schema:
        if self._schema is None:
            ts = self._get_tables()
            self._schema = ts[0].schema if ts else pa.schema([])
        return self._schema

    def columns(self) -> List[str]:
        return list(self.schema().names)

    def _rows(self) -> List[int]:
        """Rows per block, without resolving gathers or slices (their sizes are known)."""
        if self._tables is None and all(isinstance(b, (BlockGather, BlockSlice)) for b in self._blocks):
            return [len(b) if isinstance(b, BlockGather) else b.length for b in self._blocks]
        return [t.num_rows for t in self._get_tables()]

    def count(self) -> int:
        return int(sum(self._rows()))

    def num_blocks(self) -> int:
        return len(self._blocks)

    def size_bytes(self) -> int:
        return int(sum(t.nbytes for t in self._get_tables()))

    def get_internal_block_refs(self) -> List[ObjectRef]:
        refs = []
        for i, b in enumerate(self._blocks):
            if not isinstance(b, ObjectRef):
                b = _put(_resolve(b) if isinstance(b, (BlockSlice, BlockGather)) else b)
                self._blocks[i] = b
            refs.append(b)
        return refs

    def iter_internal_ref_bundles(self):
        for r, t in zip(self.get_internal_block_refs(), self._get_tables()):
            yield RefBundle([(r, BlockMetadata(t.num_rows, t.nbytes, t.schema))])

    def materialize(self):
        self._get_tables()
        return self

    def stats(self) -> str:
        return f"Dataset(num_blocks={self.num_blocks()}, num_rows={self.count()})"

    def __repr__(self):
        return f"Dataset(num_blocks={self.num_blocks()}, schema={self.schema()})"

    # ---------------------------------------------------------------- consumption --------
    def to_arrow(self) -> pa.Table:
        ts = self._get_tables()
        if not ts:
            return self.schema().empty_table()
        return pa.concat_tables(ts, promote_options="permissive")

    def to_pandas(self, limit=None):
        t = self.to_arrow()
        return (t if limit is None else t.slice(0, limit)).to_pandas()

    def to_arrow_refs(self):
        return self.get_internal_block_refs()

    def take(self, limit: int = 20) -> List[Dict[str, Any]]:
        out = []
        for t in self._get_tables():
            if len(out) >= limit:
                break
            out.extend(t.slice(0, limit - len(out)).to_pylist())
        return out

    def take_all(self):
        return self.to_arrow().to_pylist()

    def show(self, limit=20):
        for r in self.take(limit):
            print(r)

    def iter_rows(self):
        for t in self._get_tables():
            yield from t.to_pylist()

    def iter_batches(self, batch_size: int = 256, batch_format: str = "numpy",
                     drop_last: bool = False) -> Iterator:
        carry = None
        for t in self._get_tables():
            if carry is not None and carry.num_rows:
                t = pa.concat_tables([carry, t])
            off = 0
            while t.num_rows - off >= batch_size:
                yield _format_batch(t.slice(off, batch_size), batch_format)
                off += batch_size
            carry = t.slice(off)
        if carry is not None and carry.num_rows and not drop_last:
            yield _format_batch(carry, batch_format)

    def iter_torch_batches(self, batch_size=256, dtypes=None, device="cpu", drop_last=False):
        import torch
        for b in self.iter_batches(batch_size, "numpy", drop_last):
            yield {k: torch.as_tensor(v, dtype=(dtypes.get(k) if isinstance(dtypes, dict) else dtypes),
                                      device=device) for k, v in b.items()}

    def to_torch(self, *, label_column=None, feature_columns=None, label_column_dtype=None,
                 feature_column_dtypes=None, batch_size=1, prefetch_blocks=0, drop_last=False,
                 unsqueeze_label_tensor=True, unsqueeze_feature_tensors=True, device=None):
        """Legacy Ray-Data ``to_torch`` contract used by the reference estimator.

        Returns an iterable of ``(features, label)``. ``feature_columns`` as a list of names
        with one dtype → one ``[B, F]`` tensor; a list of lists → a list of tensors; a dict
        → a dict of tensors. ``device=None``: inside a GPU train worker the worker's GPU (the
        shard is ingested into HBM once and batches are slices of it -- a user loop's
        ``.to(device)`` is then a no-op), else the CPU.
        """
        from raydp_amd.data.torch_iter import TorchBatchIterable
        if device is None:
            device = _worker_device()
        return TorchBatchIterable(self, label_column, feature_columns, label_column_dtype,
                                  feature_column_dtypes, batch_size, drop_last,
                                  unsqueeze_label_tensor, device)

    # ---------------------------------------------------------------- transforms ---------
    def random_shuffle(self, seed: Optional[int] = None, num_blocks: Optional[int] = None):
        if self._pending is not None:
            # still being produced: the shuffle waits with it (lazy, like Ray Data's)
            return Dataset.deferred(_Then(self, lambda d: d.random_shuffle(seed=seed, num_blocks=num_blocks)))
        rng = np.random.default_rng(seed)
        n = num_blocks or max(1, self.num_blocks())
        blocks = self._blocks
        if blocks and all(isinstance(b, ObjectRef) for b in blocks):
            # store-resident blocks stay where they are: the result is n gathers over them (the
            # same rows, order and block sizes as the materialised shuffle below)
            total = int(sum(t.num_rows for t in self._get_tables()))
            perm = rng.permutation(total)
            bounds = _split_bounds(total, n)
            return Dataset([BlockGather(blocks, perm[a:b]) for a, b in bounds], self.schema())
        t = self.to_arrow()
        perm = rng.permutation(t.num_rows)
        t = t.take(pa.array(perm))
        return Dataset(_split(t, n), t.schema)

    def randomize_block_order(self, seed=None):
        rng = np.random.default_rng(seed)
        order = rng.permutation(self.num_blocks())
        return Dataset([self._blocks[i] for i in order], self._schema)

    def repartition(self, num_blocks: int, shuffle: bool = False):
        t = self.to_arrow()
        return Dataset(_split(t, num_blocks), t.schema)

    def split(self, n: int, equal: bool = False, locality_hints=None) -> List["Dataset"]:
        if equal:
            # shard i = global rows [i per, (i + 1) per) in block order, as slices of the blocks
            # themselves (object-store blocks stay where they are: a shard pickles to a few ids;
            # a gather's shard is the gather of its row numbers' slice)
            rows = self._rows()
            per = int(sum(rows)) // n
            schema = self.schema()
            starts = np.cumsum([0] + rows)
            out = []
            for i in builtins.range(n):
                lo, hi = i * per, (i + 1) * per
                parts = []
                for j in builtins.range(len(rows)):
                    a, b = max(lo, int(starts[j])), min(hi, int(starts[j + 1]))
                    if a >= b:
                        continue
                    blk = self._blocks[j]
                    off = a - int(starts[j])
                    if isinstance(blk, BlockGather):
                        parts.append(BlockGather(blk.refs, blk.index[off:off + b - a]))
                    elif isinstance(blk, (ObjectRef, BlockSlice)):
                        parts.append(BlockSlice(blk, off, b - a))
                    else:
                        parts.append(self._get_tables()[j].slice(off, b - a))
                out.append(Dataset(parts or [schema.empty_table()], schema))
            return out
        tables = self._get_tables()
        if len(tables) >= n:
            # keep blocks whole, balance rows greedily
            sizes = [(t.num_rows, i) for i, t in enumerate(tables)]
            sizes.sort(reverse=True)
            buckets = [[] for _ in builtins.range(n)]
            loads = [0] * n
            for rows, i in sizes:
                j = int(np.argmin(loads))
                buckets[j].append(i)
                loads[j] += rows
            return [Dataset([self._blocks[i] for i in sorted(b)], self._schema) for b in buckets]
        t = self.to_arrow()
        return [Dataset([p], t.schema) for p in _split(t, n)]

    def split_at_indices(self, indices: List[int]) -> List["Dataset"]:
        t = self.to_arrow()
        bounds = [0] + list(indices) + [t.num_rows]
        return [Dataset([t.slice(a, b - a)], t.schema) for a, b in zip(bounds[:-1], bounds[1:])]

    def train_test_split(self, test_size=0.25, shuffle=False, seed=None):
        ds = self.random_shuffle(seed) if shuffle else self
        n = ds.count()
        k = int(n * (1 - test_size)) if isinstance(test_size, float) else n - int(test_size)
        return ds.split_at_indices([k])

    def limit(self, n: int):
        return Dataset([self.to_arrow().slice(0, n)], self.schema())

    def union(self, *others):
        blocks = list(self._blocks)
        for o in others:
            blocks += o._blocks
        return Dataset(blocks, self._schema)

    def map_batches(self, fn: Callable, batch_size=None, batch_format="pandas", **kw):
        out = []
        for t in self._get_tables():
            res = fn(_format_batch(t, batch_format))
            out.append(_to_table(res))
        return Dataset(out)

    def map(self, fn: Callable):
        rows = [fn(r) for r in self.iter_rows()]
        return from_items(rows)

    def filter(self, fn: Callable):
        out = []
        for t in self._get_tables():
            mask = [bool(fn(r)) for r in t.to_pylist()]
            out.append(t.filter(pa.array(mask, pa.bool_())))
        return Dataset(out, self._schema)

    def add_column(self, name, fn):
        return Dataset([t.append_column(name, pa.array(fn(t.to_pandas()))) for t in self._get_tables()])

    def drop_columns(self, cols):
        return Dataset([t.drop(cols) for t in self._get_tables()])

    def select_columns(self, cols):
        return Dataset([t.select(cols) for t in self._get_tables()])

    def write_parquet(self, path: str):
        import os
        import pyarrow.parquet as pq
        path = path[len("file://"):] if path.startswith("file://") else path
        os.makedirs(path, exist_ok=True)
        for i, t in enumerate(self._get_tables()):
            pq.write_table(t, os.path.join(path, f"part-{i:05d}.parquet"))

    def to_spark(self, spark):
        from raydp_amd.spark.dataset import ray_dataset_to_spark_dataframe
        return ray_dataset_to_spark_dataframe(spark, self.schema(), self.get_internal_block_refs())

    # ---------------------------------------------------------------- device path -------
    def to_device_tensors(self, feature_columns, label_column, feature_dtype, label_dtype,
                          device):
        """Whole shard → HBM in one DMA + HIP decode (see ``raydp_amd.ops.ingest``)."""
        from raydp_amd.ops.ingest import ingest_tables
        return ingest_tables(self._get_tables(), feature_columns, label_column, feature_dtype,
                             label_dtype, device)


def _format_batch(t: pa.Table, fmt: str):
    if fmt in ("pandas",):
        return t.to_pandas()
    if fmt in ("pyarrow", "arrow"):
        return t
    return {n: c.to_numpy(zero_copy_only=False) for n, c in zip(t.column_names, t.columns)}


def _to_table(res) -> pa.Table:
    import pandas as pd
    if isinstance(res, pa.Table):
        return res
    if isinstance(res, pd.DataFrame):
        return pa.Table.from_pandas(res, preserve_index=False)
    if isinstance(res, dict):
        return pa.table({k: np.asarray(v) for k, v in res.items()})
    raise TypeError(type(res))


def _split_bounds(rows: int, n: int):
    n = max(1, int(n))
    b = np.linspace(0, rows, n + 1).astype(np.int64)
    return [(int(b[i]), int(b[i + 1])) for i in builtins.range(n)]


def _split(t: pa.Table, n: int) -> List[pa.Table]:
    return [t.slice(a, b - a) for a, b in _split_bounds(t.num_rows, n)]


# ------------------------------------------------------------------------------ creation --
def from_arrow(tables) -> Dataset:
    if isinstance(tables, (pa.Table, pa.RecordBatch)):
        tables = [tables]
    ts = [_resolve(t) for t in tables]
    return Dataset(ts, ts[0].schema if ts else None)


def from_arrow_refs(refs: List[ObjectRef]) -> Dataset:
    return Dataset(list(refs))


def from_pandas(dfs) -> Dataset:
    import pandas as pd
    if isinstance(dfs, pd.DataFrame):
        dfs = [dfs]
    return from_arrow([pa.Table.from_pandas(d, preserve_index=False) for d in dfs])


def from_pandas_refs(refs):
    return from_pandas([_get(r) for r in refs])


def from_items(items: List[Any], parallelism: int = 1) -> Dataset:
    if items and not isinstance(items[0], dict):
        items = [{"item": x} for x in items]
    t = pa.Table.from_pylist(items)
    return Dataset(_split(t, min(max(1, parallelism), max(1, t.num_rows))), t.schema)


def from_numpy(arr) -> Dataset:
    arr = np.asarray(arr)
    if arr.ndim == 1:
        return from_arrow(pa.table({"data": arr}))
    return from_arrow(pa.table({"data": pa.FixedSizeListArray.from_arrays(arr.ravel(), arr.shape[1])}))


def range(n: int, parallelism: int = 1) -> Dataset:  # noqa: A001
    t = pa.table({"id": np.arange(n, dtype=np.int64)})
    return Dataset(_split(t, parallelism), t.schema)


def read_parquet(paths, file_extensions=None, **kw) -> Dataset:
    from raydp_amd.spark.sources import ParquetSource
    src = ParquetSource(paths)
    files = src.files
    if file_extensions:
        files = [f for f in files if any(f.endswith("." + e) or f.endswith(e) for e in file_extensions)]
    import pyarrow.parquet as pq
    return Dataset([pq.read_table(f) for f in files])


def read_csv(paths, **kw) -> Dataset:
    from raydp_amd.spark.sources import CsvSource
    import builtins
    src = CsvSource(paths, header=True, infer_schema=True)
    return Dataset([src.load(i) for i in builtins.range(src.num_partitions())])


def from_spark(df, parallelism: Optional[int] = None) -> Dataset:
    """``ray.data.from_spark`` equivalent (recoverable conversion)."""
    from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
    return spark_dataframe_to_ray_dataset(df, parallelism)


def _worker_device():
    """The GPU of the train worker this runs in (raydp_amd.train.session), else "cpu"."""
    try:
        from raydp_amd.train import session
        dev = session.get_device()
    except Exception:  # noqa: BLE001 - not inside a train worker
        return "cpu"
    return dev if dev is not None and getattr(dev, "type", "cpu") == "cuda" else "cpu"
