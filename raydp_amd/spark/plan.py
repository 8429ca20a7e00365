"""Logical/physical plan of the Arrow-native DataFrame engine.

A plan is a DAG of partition-wise operators. Narrow operators (filter, project, sample,
explode, mapInPandas) are fused into one per-partition task chain; wide operators (repartition,
join, groupBy, orderBy, window, distinct) are stage boundaries whose shuffle output is
materialised once, bottom-up, before the consuming stage runs (Spark's ``ShuffleMapStage``
→ ``ResultStage`` split, ``RayAppMaster``/executor task model in the reference's L4).

Tasks run through a pluggable ``TaskScheduler``: in-process threads (Arrow kernels release
the GIL), or the executor actor processes of a Spark-on-runtime session
(``raydp_amd/spark/cluster.py``).
"""
import io
import math
import os
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Tuple, Callable, List, Optional, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

_tls = threading.local()


def current_partition_index() -> int:
    return getattr(_tls, "partition", 0)


class _PartitionScope:
    def __init__(self, i):
        self.i = i

    def __enter__(self):
        self.prev = getattr(_tls, "partition", 0)
        _tls.partition = self.i

    def __exit__(self, *a):
        _tls.partition = self.prev


# ------------------------------------------------------------------------------------------
# Scheduler
# ------------------------------------------------------------------------------------------
class TaskScheduler:
    """Runs ``fn(i)`` for a list of partition indices; subclasses may ship tasks elsewhere."""

    def __init__(self, parallelism: int = 1):
        self.parallelism = max(1, int(parallelism))
        self._pool = ThreadPoolExecutor(max_workers=self.parallelism,
                                        thread_name_prefix="raydp-task")

    def map(self, fn: Callable[[int], object], indices: Sequence[int]) -> List[object]:
        indices = list(indices)
        if len(indices) <= 1 or self.parallelism == 1:
            return [fn(i) for i in indices]
        return list(self._pool.map(fn, indices))

    def run_plan(self, plan: "Plan", indices=None) -> List[pa.Table]:
        prepare(plan, self)
        idx = range(plan.num_partitions()) if indices is None else indices
        return self.map(plan.compute, idx)

    def shutdown(self):
        self._pool.shutdown(wait=False, cancel_futures=True)


_default_scheduler: Optional[TaskScheduler] = None


def get_scheduler() -> TaskScheduler:
    global _default_scheduler
    from raydp_amd.spark import session as _s
    active = _s.SparkSession.getActiveSession()
    if active is not None and active._scheduler is not None:
        return active._scheduler
    if _default_scheduler is None:
        _default_scheduler = TaskScheduler(os.cpu_count() or 1)
    return _default_scheduler


# ------------------------------------------------------------------------------------------
# Plans
# ------------------------------------------------------------------------------------------
class Plan:
    _schema: Optional[pa.Schema] = None

    def children(self) -> List["Plan"]:
        return []

    def num_partitions(self) -> int:
        raise NotImplementedError

    def compute(self, i: int) -> pa.Table:
        raise NotImplementedError

    def empty(self) -> pa.Table:
        """Zero-row table with this plan's output schema (schema inference by execution)."""
        raise NotImplementedError

    @property
    def schema(self) -> pa.Schema:
        if self._schema is None:
            self._schema = self.empty().schema
        return self._schema

    def is_wide(self) -> bool:
        return False

    def materialize(self, scheduler: TaskScheduler):
        pass


def preferred_node(plan: Plan, i: int) -> Optional[str]:
    """Node holding the input of partition ``i``, following the narrow chain down to its source
    (``RayDatasetRDD.getPreferredLocations``, ``RayDatasetRDD.scala:35-57``); None if unknown."""
    p = plan
    while True:
        if isinstance(p, SourcePlan):
            f = getattr(p.source, "preferred_node", None)
            return f(i) if f is not None else None
        if isinstance(p, MapPlan):
            p = p.child
            continue
        if getattr(p, "_broadcast", None) is not None:   # narrow broadcast join: follow the left
            p = p.left
            continue
        return None


def prepare(plan: Plan, scheduler: TaskScheduler):
    """Materialise every wide operator below ``plan`` bottom-up (stage scheduling)."""
    for c in plan.children():
        prepare(c, scheduler)
    if plan.is_wide():
        plan.materialize(scheduler)


def _empty_like(schema: pa.Schema) -> pa.Table:
    return schema.empty_table()


class SourcePlan(Plan):
    def __init__(self, source):
        self.source = source

    def num_partitions(self):
        return self.source.num_partitions()

    def compute(self, i):
        with _PartitionScope(i):
            return self.source.load(i)

    def empty(self):
        return _empty_like(self.source.schema())


class MapPlan(Plan):
    """Narrow per-partition operator: ``fn(table, partition_index) -> table``."""

    def __init__(self, child: Plan, fn: Callable, desc: str = "map"):
        self.child, self.fn, self.desc = child, fn, desc

    def children(self):
        return [self.child]

    def num_partitions(self):
        return self.child.num_partitions()

    rel = None  # relational description (spark/exprc.py) when the operator is fusible

    def compute(self, i):
        if self.rel is not None:
            from raydp_amd.spark import exprc
            if exprc.enabled():
                # the whole chain of fusible operators below runs as one native program
                return exprc.compute_fused(self, i)
        t = self.child.compute(i)
        with _PartitionScope(i):
            return self.fn(t, i)

    def __getstate__(self):
        st = dict(self.__dict__)
        st.pop("_fused_segs", None)  # compiled programs are per process
        st.pop("_native_lowered", None)  # native stage handle (spark/native_exec.py)
        if st.pop("_schema_static", False):
            st.pop("_schema", None)  # re-derived statically where needed: not worth shipping
        return st

    @property
    def schema(self) -> pa.Schema:
        if self._schema is None and self.rel is not None:
            # type the operator statically when every expression's type is certain
            from raydp_amd.spark import exprc
            self._schema = exprc.static_schema(self)
            self._schema_static = self._schema is not None
        if self._schema is None:
            self._schema = self.empty().schema
        return self._schema

    def empty(self):
        with _PartitionScope(0):
            return self.fn(self.child.schema.empty_table(), 0)


class UnionPlan(Plan):
    def __init__(self, plans: List[Plan], by_name=False):
        self.plans, self.by_name = plans, by_name
        self._offsets = None

    def children(self):
        return list(self.plans)

    def _offs(self):
        if self._offsets is None:
            self._offsets = np.cumsum([0] + [p.num_partitions() for p in self.plans])
        return self._offsets

    def num_partitions(self):
        return int(self._offs()[-1])

    def _conform(self, t: pa.Table) -> pa.Table:
        target = self.plans[0].schema
        if self.by_name:
            t = t.select(target.names)
        else:
            t = t.rename_columns(target.names)
        if t.schema != target:
            t = t.cast(target, safe=False)
        return t

    def compute(self, i):
        offs = self._offs()
        k = int(np.searchsorted(offs, i, side="right") - 1)
        return self._conform(self.plans[k].compute(i - int(offs[k])))

    def empty(self):
        return self.plans[0].schema.empty_table()


class MaterializedPlan(Plan):
    """Already-computed partitions (a cached DataFrame or a finished shuffle)."""

    def __init__(self, tables: List[pa.Table], schema: pa.Schema):
        self.tables, self._schema = tables, schema

    def num_partitions(self):
        return len(self.tables)

    def compute(self, i):
        return self.tables[i]

    def empty(self):
        return _empty_like(self._schema)


class WidePlan(Plan):
    """Stage boundary: output partitions are produced by a shuffle of the children."""

    def __init__(self):
        self._out: Optional[List[pa.Table]] = None
        self._lock = threading.Lock()

    def is_wide(self):
        return True

    def __getstate__(self):
        st = dict(self.__dict__)
        st.pop("_lock", None)
        if self._out is not None:
            # a finished stage ships only its outputs: the lineage below it stays on the
            # driver (otherwise every later stage would re-ship every upstream result)
            st["_schema"] = self.schema
            for k, v in list(st.items()):
                if isinstance(v, Plan) or (isinstance(v, (list, tuple)) and v and isinstance(v[0], Plan)):
                    st[k] = None
            st["_cut"] = True
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._lock = threading.Lock()

    def empty(self):
        if getattr(self, "_cut", False):
            return self._schema.empty_table()
        return self._empty()

    def _empty(self):
        raise NotImplementedError

    def materialize(self, scheduler):
        with self._lock:
            if self._out is None:
                self._out = self.execute(scheduler)

    def execute(self, scheduler) -> List[pa.Table]:
        raise NotImplementedError

    def compute(self, i):
        if self._out is None:
            self.materialize(get_scheduler())
        return self._out[i]


# ------------------------------------------------------------------------------------------
# shuffle primitives
# ------------------------------------------------------------------------------------------
def hash_columns(t: pa.Table, keys: List[str]) -> np.ndarray:
    """64-bit row hash of the key columns, consistent across partitions/processes."""
    from raydp_amd.native import exec_kernels
    h = np.zeros(t.num_rows, dtype=np.uint64)
    for k in keys:
        h = exec_kernels.hash_combine(h, t.column(k))
    return h


class MapOutput:
    """One map task's shuffle output: its rows ordered by bucket plus the bucket offsets (the
    in-memory analogue of Spark's data file + index file). Behaves as the list of bucket
    tables, but travels as ONE table: a 200-bucket exchange of 4 map tasks moves 4 objects
    through the store instead of 800."""

    def __init__(self, table: pa.Table, offsets: np.ndarray):
        self.table, self.offsets = table, np.asarray(offsets, dtype=np.int64)

    def __len__(self):
        return len(self.offsets) - 1

    def __getitem__(self, j):
        if isinstance(j, slice):
            return [self[k] for k in range(*j.indices(len(self)))]
        if j < 0:
            j += len(self)
        a, b = int(self.offsets[j]), int(self.offsets[j + 1])
        return self.table.slice(a, b - a)

    def __iter__(self):
        return (self[j] for j in range(len(self)))

    def bucket_bytes(self) -> np.ndarray:
        """Approximate bytes per bucket (rows x average row width)."""
        rows = np.diff(self.offsets)
        width = self.table.nbytes / max(1, self.table.num_rows)
        return rows * width

    def __reduce__(self):
        return MapOutput, (self.table, self.offsets)


def hash_partition(t: pa.Table, keys: List[str], n: int):
    if n == 1:
        return [t]
    if t.num_rows == 0:
        return [t.slice(0, 0) for _ in range(n)]
    from raydp_amd.native import exec_kernels
    part = (hash_columns(t, keys) % np.uint64(n)).astype(np.int64)
    order, counts = exec_kernels.partition_order(part, n)
    st = t.take(pa.array(order))
    return MapOutput(st, np.concatenate([[0], np.cumsum(counts)]))


def concat(tables: List[pa.Table], schema: pa.Schema) -> pa.Table:
    tables = [t for t in tables if t is not None]
    if not tables:
        return _empty_like(schema)
    try:
        return pa.concat_tables(tables, promote_options="permissive").combine_chunks()
    except pa.ArrowInvalid:
        return pa.concat_tables([t.cast(schema, safe=False) for t in tables]).combine_chunks()


class RepartitionPlan(WidePlan):
    """``repartition(n)`` (round-robin) or ``repartition(n, *cols)`` (hash)."""

    def __init__(self, child: Plan, n: int, keys: Optional[List[str]] = None,
                 adaptive: Optional[Tuple[int, int]] = None):
        """``adaptive`` = (advisory partition bytes, minimum partitions): the partition count was
        not given by the user, so after the map side adjacent hash buckets are coalesced to
        about that size (Spark AQE ``coalescePartitions``; hash co-location is preserved)."""
        super().__init__()
        self.child, self.n, self.keys = child, max(1, int(n)), keys
        self.adaptive = adaptive

    def children(self):
        return [self.child]

    def num_partitions(self):
        if self._out is None:
            # someone sized itself on the requested count before the shuffle ran (a join, an
            # RDD view): keep that count, coalescing would change it under their feet
            self._n_observed = True
        return self.n

    def _empty(self):
        return self.child.schema.empty_table()

    def execute(self, scheduler):
        n = self.n
        keys = self.keys

        def split(i):
            t = self.child.compute(i)
            if keys:
                return hash_partition(t, keys, n)
            # round robin starting at a partition-dependent offset (Spark's distribution)
            if n == 1:
                return [t]
            assign = (np.arange(t.num_rows) + i) % n
            order = np.argsort(assign, kind="stable")
            counts = np.bincount(assign, minlength=n)
            st = t.take(pa.array(order))
            res, off = [], 0
            for c in counts:
                res.append(st.slice(off, int(c)))
                off += int(c)
            return res

        pieces = scheduler.map(split, range(self.child.num_partitions()))
        schema = self.child.schema
        groups = [[j] for j in range(n)]
        if self.adaptive is not None and keys and n > 1 and not getattr(self, "_n_observed", False):
            sizes = np.zeros(n)
            for p in pieces:
                sizes += p.bucket_bytes() if isinstance(p, MapOutput) else \
                    np.array([q.nbytes for q in p], dtype=np.float64)
            groups = coalesce_buckets(sizes.tolist(), *self.adaptive)
            self.n = len(groups)
        # reduce side runs as tasks too: executors read the map outputs from the store
        return scheduler.map(lambda g: concat([p[j] for j in groups[g] for p in pieces], schema),
                             range(len(groups)))


def coalesce_buckets(sizes: List[int], advisory: int, min_parts: int) -> List[List[int]]:
    """Greedy merge of adjacent shuffle buckets up to a target size (Spark's
    ``ShufflePartitionsUtil.coalescePartitions``): target = min(advisory, total / min_parts)."""
    total = int(sum(sizes))
    target = max(1, min(int(advisory), -(-total // max(1, int(min_parts)))))
    groups, cur, acc = [], [], 0
    for j, s in enumerate(sizes):
        if cur and acc + s > target:
            groups.append(cur)
            cur, acc = [], 0
        cur.append(j)
        acc += s
    if cur:
        groups.append(cur)
    return groups


class CoalescePlan(Plan):
    """Narrow merge of adjacent partitions (``coalesce(n)``)."""

    def __init__(self, child: Plan, n: int):
        self.child = child
        m = child.num_partitions()
        self.n = max(1, min(int(n), m)) if m else 1
        self.groups = np.array_split(np.arange(m), self.n) if m else [np.arange(0)]

    def children(self):
        return [self.child]

    def num_partitions(self):
        return self.n

    def compute(self, i):
        return concat([self.child.compute(int(j)) for j in self.groups[i]], self.child.schema)

    def empty(self):
        return self.child.schema.empty_table()


class SortPlan(WidePlan):
    def __init__(self, child: Plan, sort_keys, n_out: Optional[int] = None):
        super().__init__()
        self.child, self.sort_keys = child, sort_keys  # list of (expr, ascending, nulls_first)
        self.n_out = n_out or child.num_partitions()

    def children(self):
        return [self.child]

    def num_partitions(self):
        return max(1, self.n_out)

    def _empty(self):
        return self.child.schema.empty_table()

    def execute(self, scheduler):
        parts = scheduler.map(self.child.compute, range(self.child.num_partitions()))
        t = concat(parts, self.child.schema)
        t = sort_table(t, self.sort_keys)
        n = self.num_partitions()
        rows = t.num_rows
        bounds = np.linspace(0, rows, n + 1).astype(np.int64)
        return [t.slice(int(bounds[j]), int(bounds[j + 1] - bounds[j])) for j in range(n)]


def sort_table(t: pa.Table, sort_keys) -> pa.Table:
    if t.num_rows == 0:
        return t
    tmp = t
    keys = []
    for j, (e, asc, nulls_first) in enumerate(sort_keys):
        name = f"__sk{j}"
        from raydp_amd.spark.column import as_array
        tmp = tmp.append_column(name, as_array(e.eval(t), t.num_rows))
        # Spark default: nulls first for ascending, last for descending
        nf = asc if nulls_first is None else nulls_first
        keys.append((name, "ascending" if asc else "descending", "at_start" if nf else "at_end"))
    idx = pc.sort_indices(tmp, sort_keys=keys)
    return t.take(idx)
