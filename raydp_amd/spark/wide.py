"""Shuffle-based operators: hash join, hash aggregate, window ranking, distinct.

Each is a stage boundary: the children are hash-partitioned on the key columns into the same
number of buckets, then bucket ``j`` of every child is combined with Arrow's C++ hash join /
hash aggregate. A join whose build side is below ``spark.sql.autoBroadcastJoinThreshold``
(10 MB) skips the shuffle and broadcasts that side to every probe partition.
"""
from typing import List, Optional, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from raydp_amd.spark.column import AggExpr, Expr, as_array
from raydp_amd.spark.plan import Plan, WidePlan, concat, hash_partition, sort_table
from raydp_amd.spark.shuffle import exchange

_BROADCAST_BYTES = 10 * 1024 * 1024

_JOIN_TYPES = {
    "inner": "inner", "cross": "inner", "outer": "full outer", "full": "full outer",
    "fullouter": "full outer", "full_outer": "full outer", "left": "left outer",
    "leftouter": "left outer", "left_outer": "left outer", "right": "right outer",
    "rightouter": "right outer", "right_outer": "right outer", "semi": "left semi",
    "leftsemi": "left semi", "left_semi": "left semi", "anti": "left anti",
    "leftanti": "left anti", "left_anti": "left anti",
}


class JoinPlan(WidePlan):
    def __init__(self, left: Plan, right: Plan, left_keys: List[str], right_keys: List[str],
                 how: str = "inner", n_out: Optional[int] = None):
        super().__init__()
        self.left, self.right = left, right
        self.lk, self.rk = left_keys, right_keys
        self.how = _JOIN_TYPES[how.lower()]
        self.n = n_out or max(left.num_partitions(), right.num_partitions(), 1)
        self._broadcast = None

    def children(self):
        return [self.left, self.right]

    def num_partitions(self):
        return self.n

    def _join(self, lt: pa.Table, rt: pa.Table) -> pa.Table:
        same = self.lk == self.rk
        if self.how in ("left semi", "left anti"):
            return lt.join(rt.select(self.rk), keys=self.lk, right_keys=self.rk,
                           join_type=self.how, use_threads=True)
        # disambiguate non-key duplicate names like Spark (right side suffix is dropped by
        # select later; keep both columns)
        overlap = (set(lt.column_names) & set(rt.column_names)) - (set(self.lk) if same else set())
        rk = self.rk
        if overlap:
            rt = rt.rename_columns([c + "#r" if c in overlap else c for c in rt.column_names])
            rk = [c + "#r" if c in overlap else c for c in rk]    # a right key may be renamed too
        out = lt.join(rt, keys=self.lk, right_keys=rk, join_type=self.how,
                      use_threads=True, coalesce_keys=same)
        if overlap:
            out = out.rename_columns([c[:-2] if c.endswith("#r") else c for c in out.column_names])
        return out

    def _empty(self):
        st = self.static_schema()
        if st is not None:
            return st.empty_table()
        return self._join(self.left.schema.empty_table(), self.right.schema.empty_table())

    def static_schema(self) -> Optional[pa.Schema]:
        """Output schema without running a join (inner / left outer / semi / anti: left fields,
        then the right side's, minus the keys when both sides name them alike, which Arrow
        coalesces); None for the join types whose column order Arrow arranges differently."""
        ls, rs = self.left.schema, self.right.schema
        if self.how in ("left semi", "left anti"):
            return ls
        if self.how not in ("inner", "left outer"):
            return None
        same = self.lk == self.rk
        return pa.schema(list(ls) + [f for f in rs if not (same and f.name in self.rk)])

    # Broadcast hash join is a NARROW operator (Spark's BroadcastHashJoinExec inside whole-stage
    # codegen): only the small side is materialised; each left partition is joined against it
    # inside whatever task computes that partition, so a chain of dimension joins (the DLRM
    # notebook's 26 categorical-model joins) runs in one pass per partition instead of one
    # materialised stage per join.
    def materialize(self, scheduler):
        with self._lock:
            if self._out is not None or self._broadcast is not None:
                return
            rparts = scheduler.map(self.right.compute, range(self.right.num_partitions()))
            rsize = sum(t.nbytes for t in rparts)
            if rsize <= _BROADCAST_BYTES and self.how in ("inner", "left outer", "left semi", "left anti"):
                self._broadcast = concat(rparts, self.right.schema)
                self.n = self.left.num_partitions()
                return
            self._out = self._shuffle_join(scheduler, rparts)

    def compute(self, i):
        if self._out is None and self._broadcast is None:
            from raydp_amd.spark.plan import get_scheduler
            self.materialize(get_scheduler())
        if self._broadcast is not None:
            return self._broadcast_join(self.left.compute(i))
        return self._out[i]

    def _broadcast_join(self, lt: pa.Table) -> pa.Table:
        """Join one left partition against the broadcast table. A single-key inner / left
        join whose build keys are unique (a dimension table, e.g. the DLRM value->id models) is
        a hash LOOKUP: one ``index_in`` over the build keys and a ``take`` of its columns,
        preserving the left rows' order; anything else runs Arrow's hash join."""
        rt = self._broadcast
        ok = self.__dict__.get("_lookup_ok")
        if ok is None:
            ok = self._can_lookup(rt)
            self.__dict__["_lookup_ok"] = ok
        if not ok:
            return self._join(lt, rt)
        key_l = lt.column(self.lk[0])
        if key_l.type != rt.schema.field(self.rk[0]).type:
            return self._join(lt, rt)
        vs = self.__dict__.get("_lookup_vs")
        if vs is None:
            vs = rt.column(self.rk[0]).combine_chunks()
            self.__dict__["_lookup_vs"] = vs
        idx = pc.index_in(key_l, options=pc.SetLookupOptions(value_set=vs, skip_nulls=True))
        if self.how == "inner":
            keep = pc.is_valid(idx)
            lt, idx = lt.filter(keep), idx.filter(keep)
        same = self.lk == self.rk
        rnames = [c for c in rt.column_names if not (same and c in self.rk)]
        taken = rt.select(rnames).take(idx)
        out = lt
        for c in rnames:
            out = out.append_column(c, taken.column(c))
        return out

    def _can_lookup(self, rt: pa.Table) -> bool:
        if len(self.lk) != 1 or self.how not in ("inner", "left outer"):
            return False
        overlap = (set(rt.column_names) & set(self.left.schema.names)) - \
            (set(self.lk) if self.lk == self.rk else set())
        if overlap:
            return False
        k = rt.column(self.rk[0])
        valid = len(k) - k.null_count
        return valid == len(k) and pc.count_distinct(k, mode="only_valid").as_py() == valid

    def __getstate__(self):
        if self._broadcast is not None:
            # ships the left lineage (computed per task) and the broadcast table, not the right
            st = dict(self.__dict__)
            st.pop("_lock", None)
            st["_schema"] = self.schema
            st["right"] = None
            st["_cut"] = True
            st.pop("_lookup_vs", None)
            return st
        return super().__getstate__()

    def execute(self, scheduler):
        rparts = scheduler.map(self.right.compute, range(self.right.num_partitions()))
        return self._shuffle_join(scheduler, rparts)

    def _shuffle_join(self, scheduler, rparts):
        n = self.n
        ls, rs = self.left.schema, self.right.schema
        lsh = exchange(scheduler, self.left.compute, self.left.num_partitions(), self.lk, n, ls)
        rbuck = [hash_partition(t, self.rk, n) for t in rparts]

        def one(j):
            return self._join(lsh.bucket(j), concat([p[j] for p in rbuck], rs))
        return _reduce(scheduler, one, n, lsh)


_AGG_MAP = {"sum": "sum", "avg": "mean", "min": "min", "max": "max", "count": "count",
            "first": "first", "last": "last", "stddev": "stddev", "variance": "variance",
            "collect_list": "list", "collect_set": "distinct"}


def aggregate_table(t: pa.Table, keys: List[str], aggs: List[Tuple[AggExpr, str]]) -> pa.Table:
    """Group ``t`` by ``keys`` and compute ``aggs`` ([(AggExpr, output_name)])."""
    n = t.num_rows
    work = t.select(keys) if keys else pa.table({"__one": pa.array(np.zeros(n, np.int8))})
    specs, names = [], []
    for j, (a, out_name) in enumerate(aggs):
        cname = f"__a{j}"
        if a.child is None:
            work = work.append_column(cname, pa.array(np.ones(n, dtype=np.int8)))
        else:
            v = as_array(a.child.eval(t), n)
            if a.fn in ("avg", "stddev", "variance") and pa.types.is_integer(v.type):
                v = pc.cast(v, pa.float64())
            work = work.append_column(cname, v)
        fn = _AGG_MAP[a.fn]
        opts = None
        if a.fn == "count":
            if a.distinct:
                fn = "count_distinct"
            opts = pc.CountOptions(mode="only_valid")
        elif a.fn in ("stddev", "variance"):
            opts = pc.VarianceOptions(ddof=1)
        elif a.fn in ("first", "last"):
            opts = pc.ScalarAggregateOptions(skip_nulls=False)
        specs.append((cname, fn, opts) if opts is not None else (cname, fn))
        names.append(out_name)
    gkeys = keys if keys else ["__one"]
    res = work.group_by(gkeys, use_threads=False).aggregate(specs)
    # group_by output: aggregate columns first ("<col>_<fn>"), then keys
    out_cols, out_names = [], []
    for k in keys:
        out_cols.append(res.column(k))
        out_names.append(k)
    for j, (spec, name) in enumerate(zip(specs, names)):
        col = res.column(f"{spec[0]}_{spec[1]}")
        a = aggs[j][0]
        if a.fn == "count":
            col = pc.cast(col, pa.int64())
        if a.fn == "sum" and pa.types.is_integer(col.type):
            col = pc.cast(col, pa.int64())
        out_cols.append(col)
        out_names.append(name)
    if not keys and n == 0:
        # global aggregate over empty input still yields one row (count=0, others null)
        vals = []
        for (a, _), c in zip(aggs, out_cols):
            vals.append(pa.array([0 if a.fn == "count" else None], type=c.type))
        return pa.table(vals, names=out_names)
    return pa.table(out_cols, names=out_names)


class AggregatePlan(WidePlan):
    def __init__(self, child: Plan, keys: List[str], aggs, n_out: Optional[int] = None):
        super().__init__()
        self.child, self.keys, self.aggs = child, keys, aggs
        self.n = (n_out or max(1, child.num_partitions())) if keys else 1

    def children(self):
        return [self.child]

    def num_partitions(self):
        return self.n

    def _empty(self):
        t = aggregate_table(self.child.schema.empty_table(), self.keys, self.aggs)
        return t.slice(0, 0)

    def execute(self, scheduler):
        n, keys = self.n, self.keys
        schema = self.child.schema
        if not keys:
            parts = scheduler.map(self.child.compute, range(self.child.num_partitions()))
            return [aggregate_table(concat(parts, schema), [], self.aggs)]
        sh = exchange(scheduler, self.child.compute, self.child.num_partitions(), keys, n, schema)
        return _reduce(scheduler, lambda j: aggregate_table(sh.bucket(j), keys, self.aggs), n, sh)


class DistinctPlan(WidePlan):
    def __init__(self, child: Plan, subset: Optional[List[str]] = None):
        super().__init__()
        self.child, self.subset = child, subset
        self.n = max(1, child.num_partitions())

    def children(self):
        return [self.child]

    def num_partitions(self):
        return self.n

    def _empty(self):
        return self.child.schema.empty_table()

    def _dedup(self, t: pa.Table) -> pa.Table:
        keys = self.subset or t.column_names
        if t.num_rows == 0:
            return t
        idx = pa.table({"__i": pa.array(np.arange(t.num_rows))})
        for k in keys:
            idx = idx.append_column(k, t.column(k))
        first = idx.group_by(keys, use_threads=False).aggregate([("__i", "min")])
        take = np.sort(first.column("__i_min").to_numpy())
        return t.take(pa.array(take))

    def execute(self, scheduler):
        keys = self.subset or self.child.schema.names
        n = self.n
        schema = self.child.schema
        sh = exchange(scheduler, self.child.compute, self.child.num_partitions(), keys, n, schema)
        return _reduce(scheduler, lambda j: self._dedup(sh.bucket(j)), n, sh)


class WindowPlan(WidePlan):
    """Adds one window-expression column: ranking (row_number/rank/dense_rank) or an
    aggregate over ``Window.partitionBy(...).orderBy(...)``."""

    def __init__(self, child: Plan, out_name: str, fn: str, args: List[Expr], window):
        super().__init__()
        self.child, self.out_name, self.fn, self.args, self.window = child, out_name, fn, args, window
        self.n = max(1, child.num_partitions())

    def children(self):
        return [self.child]

    def num_partitions(self):
        return self.n

    def _apply(self, t: pa.Table) -> pa.Table:
        w = self.window
        keys = w.partition_cols
        n = t.num_rows
        sort_keys = [(e, True, True) for e in [_col(k) for k in keys]] + list(w.order_keys)
        st = sort_table(t, sort_keys) if n and sort_keys else t
        if self.fn.startswith("agg:"):
            fn = self.fn[4:]
            from raydp_amd.spark.column import AggExpr as _A
            agg = aggregate_table(st, keys, [(_A(fn, self.args[0] if self.args else None), "__w")])
            res = st.join(agg, keys=keys, join_type="left outer") if keys else \
                st.append_column("__w", pa.repeat(agg.column("__w")[0], n))
            return res.rename_columns([self.out_name if c == "__w" else c for c in res.column_names])
        # group boundaries
        if n == 0:
            vals = pa.array([], pa.int32())
        else:
            starts = np.zeros(n, dtype=bool)
            starts[0] = True
            for k in keys:
                v = st.column(k).to_numpy(zero_copy_only=False)
                starts[1:] |= v[1:] != v[:-1]
            gid = np.cumsum(starts) - 1
            first_pos = np.flatnonzero(starts)
            pos = np.arange(n) - first_pos[gid]
            if self.fn == "row_number":
                vals = pos + 1
            else:
                ties = np.zeros(n, dtype=bool)
                ties[0] = True
                for e, _, _ in w.order_keys:
                    v = as_array(e.eval(st), n).to_numpy(zero_copy_only=False)
                    ties[1:] |= v[1:] != v[:-1]
                ties |= starts
                if self.fn == "rank":
                    last_change = np.maximum.accumulate(np.where(ties, np.arange(n), 0))
                    vals = last_change - first_pos[gid] + 1
                else:  # dense_rank
                    c = np.cumsum(ties)
                    vals = c - c[first_pos[gid]] + 1
            vals = pa.array(vals.astype(np.int32))
        return st.append_column(self.out_name, vals)

    def _empty(self):
        return self._apply(self.child.schema.empty_table())

    def execute(self, scheduler):
        keys = self.window.partition_cols
        schema = self.child.schema
        if not keys:
            parts = scheduler.map(self.child.compute, range(self.child.num_partitions()))
            self.n = 1
            return [self._apply(concat(parts, schema))]
        n = self.n
        sh = exchange(scheduler, self.child.compute, self.child.num_partitions(), keys, n, schema)
        return _reduce(scheduler, lambda j: self._apply(sh.bucket(j)), n, sh)


def _reduce(scheduler, fn, n, sh):
    """Reduce stage of a shuffle; the map outputs are dropped once it has run."""
    try:
        return scheduler.map(fn, range(n))
    finally:
        sh.release()


def _col(name):
    from raydp_amd.spark.column import ColRef
    return ColRef(name)
