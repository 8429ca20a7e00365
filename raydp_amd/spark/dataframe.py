"""Lazy, partitioned, Arrow-native ``DataFrame`` with the PySpark DataFrame surface.

Parity target: the subset of ``pyspark.sql.DataFrame`` exercised by the reference's examples,
tests and notebooks (``examples/data_process.py``, ``pytorch_dlrm.ipynb``,
``python/raydp/tests/*``): select/withColumn/filter/drop, joins, groupBy/agg, orderBy,
window functions, randomSplit, repartition, cache/persist, collect/take/count/toPandas and the
parquet/csv writers. Every operator builds a ``Plan`` node (``plan.py``/``wide.py``); nothing
executes until an action.
"""
import functools
import json
import os
import uuid
from typing import Dict, List, Optional, Union

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from raydp_amd.spark import plan as P
from raydp_amd.spark import wide as W
from raydp_amd.spark.column import (AggExpr, Alias, BinOp, ColRef, Column, Expr, Func, Lit, SortOrder,
                                    WindowExpr, _to_expr, as_array, map_children)
from raydp_amd.spark.row import Row
from raydp_amd.spark.types import StructType, from_arrow_schema


class StorageLevel:
    def __init__(self, useDisk, useMemory, useOffHeap, deserialized, replication=1):
        self.useDisk, self.useMemory, self.useOffHeap = useDisk, useMemory, useOffHeap
        self.deserialized, self.replication = deserialized, replication

    def __repr__(self):
        return (f"StorageLevel({self.useDisk}, {self.useMemory}, {self.useOffHeap}, "
                f"{self.deserialized}, {self.replication})")


StorageLevel.DISK_ONLY = StorageLevel(True, False, False, False)
StorageLevel.MEMORY_ONLY = StorageLevel(False, True, False, False)
StorageLevel.MEMORY_AND_DISK = StorageLevel(True, True, False, False)
StorageLevel.MEMORY_AND_DISK_DESER = StorageLevel(True, True, False, True)
StorageLevel.OFF_HEAP = StorageLevel(True, True, True, False)


def _names_of(cols):
    out = []
    for c in cols:
        if isinstance(c, (list, tuple)):
            out.extend(_names_of(c))
        else:
            out.append(c)
    return out


# ------------------------------------------------------------------------------------------
# relational narrow operators: module-level appliers bound with functools.partial, so a plan
# pickles as data (expression trees) instead of one closure code object per operator, and the
# same ``rel`` tuple drives both this per-operator path and the fused VM (spark/exprc.py)
# ------------------------------------------------------------------------------------------
def _count_rows(t: pa.Table, i) -> pa.Table:
    return pa.table({"n": [t.num_rows]})


def _apply_with(col_name, e, t: pa.Table, i) -> pa.Table:
    v = as_array(e.eval(t), t.num_rows)
    if col_name in t.column_names:
        return t.set_column(t.column_names.index(col_name), col_name, v)
    return t.append_column(col_name, v)


def _apply_filter(preds, t: pa.Table, i) -> pa.Table:
    mask = None
    for e in preds:
        m = e.eval(t)
        if isinstance(m, pa.Scalar):
            if not m.as_py():
                return t.slice(0, 0)
            continue
        mask = m if mask is None else pc.and_kleene(mask, m)
    if mask is None:
        return t
    return t.filter(mask, null_selection_behavior="drop")


def _apply_drop(names, t: pa.Table, i) -> pa.Table:
    return t.drop([c for c in t.column_names if c in names])


def _apply_project(exprs, t: pa.Table, i) -> pa.Table:
    return _eval_projection(t, exprs)


def _rel_node(src: "P.Plan", rel: tuple, desc: str) -> "P.MapPlan":
    kind = rel[0]
    if kind == "with":
        fn = functools.partial(_apply_with, rel[1], rel[2])
    elif kind == "filter":
        fn = functools.partial(_apply_filter, rel[1])
    elif kind == "drop":
        fn = functools.partial(_apply_drop, rel[1])
    else:
        fn = functools.partial(_apply_project, rel[1])
    node = P.MapPlan(src, fn, desc)
    node.rel = rel
    return node


def _eval_projection(t: pa.Table, exprs) -> pa.Table:
    """Evaluate a list of (Expr, name) into a table; handles explode/posexplode generators."""
    n = t.num_rows
    gen = [(i, e) for i, (e, _) in enumerate(exprs)
           if isinstance(e, Func) and e.fname in ("__explode__", "__posexplode__")
           or isinstance(e, Alias) and isinstance(e.child, Func)
           and e.child.fname in ("__explode__", "__posexplode__")]
    if len(gen) > 1:
        raise ValueError("Only one generator allowed per select clause")
    if not gen:
        cols, names = [], []
        for e, name in exprs:
            cols.append(as_array(e.eval(t), n))
            names.append(name)
        return pa.Table.from_arrays(cols, names=names)
    gi, ge = gen[0]
    f = ge.child if isinstance(ge, Alias) else ge
    lst = as_array(f.args[0].eval(t), n)
    if isinstance(lst, pa.ChunkedArray):
        lst = lst.combine_chunks()
    parents = pc.list_parent_indices(lst)
    values = pc.list_flatten(lst)
    pos = None
    if f.fname == "__posexplode__":
        offs = lst.offsets.to_numpy()
        pidx = parents.to_numpy()
        pos = pa.array((np.arange(len(pidx)) - (offs[pidx] - offs[0])).astype(np.int32))
    cols, names = [], []
    for i, (e, name) in enumerate(exprs):
        if i == gi:
            if pos is not None:
                cols += [pos, values]
                names += ["pos", "col"]
            else:
                cols.append(values)
                names.append(name if isinstance(ge, Alias) else "col")
        else:
            cols.append(as_array(e.eval(t), n).take(parents))
            names.append(name)
    return pa.Table.from_arrays(cols, names=names)


class GroupedData:
    def __init__(self, df: "DataFrame", keys: List[str]):
        self._df, self._keys = df, keys

    def agg(self, *exprs):
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            from raydp_amd.spark import functions as F
            exprs = [getattr(F, fn if fn != "mean" else "avg")(c) for c, fn in exprs[0].items()]
        aggs, post, hidden = [], [], {}

        def lift(e):
            # an aggregate inside a larger expression (round(avg(x), 2), sum(a) / count(b)):
            # aggregate it under a hidden name, evaluate the expression on the grouped rows
            if isinstance(e, AggExpr):
                nm = e.name()
                if nm not in hidden:
                    hidden[nm] = f"__agg{len(hidden)}"
                    aggs.append((e, hidden[nm]))
                return ColRef(hidden[nm])
            return map_children(e, lift)
        for c in exprs:
            e = c._expr
            name = e.name()
            if isinstance(e, Alias):
                e = e.child
            if isinstance(e, AggExpr):
                aggs.append((e, name))
                post.append(name)
            elif e.is_aggregate():
                post.append(Column(Alias(lift(e), name)))
            else:
                raise ValueError(f"{name} is not an aggregate expression")
        out = DataFrame(W.AggregatePlan(self._df._plan, self._keys, aggs), self._df._session)
        if hidden:
            out = out.select(*self._keys, *post)
        return out

    def _simple(self, fn, cols):
        from raydp_amd.spark import functions as F
        if not cols:
            num = [f.name for f in self._df._plan.schema
                   if (pa.types.is_integer(f.type) or pa.types.is_floating(f.type))
                   and f.name not in self._keys]
            cols = num
        return self.agg(*[getattr(F, fn)(c) for c in cols])

    def count(self):
        from raydp_amd.spark import functions as F
        return self.agg(F.count("*").alias("count"))

    def sum(self, *cols): return self._simple("sum", cols)
    def avg(self, *cols): return self._simple("avg", cols)
    mean = avg
    def min(self, *cols): return self._simple("min", cols)
    def max(self, *cols): return self._simple("max", cols)


def _pad_to(target, src, t, i=None):
    """The unmatched rows ``t`` of an outer join with a residual condition in the joined layout
    ``target``: column j is ``t``'s column ``src[j]``, or typed nulls where ``src[j]`` is -1
    (positional: a join keeps both sides' same-named columns)."""
    cols = [t.column(k).cast(f.type) if k >= 0 else pa.nulls(t.num_rows, f.type) for f, k in zip(target, src)]
    return pa.Table.from_arrays(cols, schema=target)


def _rewrite_refs(e, fn):
    """Copy of expression ``e`` with every ColRef replaced by ``fn(ref)``."""
    if isinstance(e, ColRef):
        return fn(e)
    return map_children(e, lambda c: _rewrite_refs(c, fn))


class DataFrameNaFunctions:
    def __init__(self, df):
        self.df = df

    def fill(self, value, subset=None):
        return self.df.fillna(value, subset)

    def drop(self, how="any", thresh=None, subset=None):
        return self.df.dropna(how, thresh, subset)


class DataFrame:
    def __init__(self, plan: P.Plan, session):
        self._plan = plan
        self._session = session
        self._cached: Optional[P.MaterializedPlan] = None
        self._storage_level = None
        self._id_ = None

    @property
    def _id(self) -> str:
        # drawn on first use (persist / conversion): a chain of transformations builds dozens
        # of intermediate DataFrames that never need one
        if self._id_ is None:
            self._id_ = uuid.uuid4().hex
        return self._id_

    # ------------------------------------------------------------------ metadata ---------
    @property
    def sparkSession(self):
        return self._session

    @property
    def sql_ctx(self):
        return self._session

    @property
    def schema(self) -> StructType:
        return from_arrow_schema(self._plan.schema)

    @property
    def arrow_schema(self) -> pa.Schema:
        return self._plan.schema

    @property
    def columns(self) -> List[str]:
        return list(self._plan.schema.names)

    @property
    def dtypes(self):
        return [(f.name, f.dataType.simpleString()) for f in self.schema]

    def printSchema(self):
        print("root")
        for f in self.schema:
            print(f" |-- {f.name}: {f.dataType.simpleString()} (nullable = {str(f.nullable).lower()})")

    @property
    def na(self):
        return DataFrameNaFunctions(self)

    @property
    def rdd(self):
        return _df_rdd(self)

    @property
    def write(self):
        from raydp_amd.spark.io import DataFrameWriter
        return DataFrameWriter(self)

    @property
    def storageLevel(self):
        return self._storage_level

    @property
    def is_cached(self):
        return self._cached is not None

    def __getitem__(self, item):
        if isinstance(item, str):
            return Column(self._ref(item))
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        raise TypeError(item)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        if name in self.columns:
            return Column(self._ref(name))
        raise AttributeError(f"'DataFrame' object has no attribute '{name}'")

    def _ref(self, name):
        r = ColRef(name)
        r.origin = id(self)       # which side of a join condition it belongs to (_join_side)
        return r

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{n}: {t}" for n, t in self.dtypes) + "]"

    # --------------------------------------------------------------- plan helpers --------
    def _src(self) -> P.Plan:
        return self._cached if self._cached is not None else self._plan

    def _with(self, plan: P.Plan) -> "DataFrame":
        return DataFrame(plan, self._session)

    def _map(self, fn, desc):
        return self._with(P.MapPlan(self._src(), fn, desc))

    # -------------------------------------------------------------- transformations ------
    def select(self, *cols):
        cols = _names_of(cols)
        exprs = []
        for c in cols:
            if isinstance(c, str) and c == "*":
                exprs += [(ColRef(n), n) for n in self.columns]
                continue
            e = _to_expr(c, name_is_col=True)
            if isinstance(e, ColRef) and e.col_name.endswith(".*"):
                exprs += [(ColRef(n), n) for n in self.columns]
                continue
            if isinstance(e, WindowExpr):
                tmp = f"__win_{uuid.uuid4().hex[:8]}"
                return self.withColumn(tmp, Column(e)).select(
                    *[x if not (x is c) else Column(Alias(ColRef(tmp), e.name())) for x in cols])
            if e.is_aggregate():
                return self.agg(*cols)
            exprs.append((e, e.name()))
        if not any(isinstance(x, Func) and x.fname in ("__explode__", "__posexplode__") or
                   isinstance(x, Alias) and isinstance(x.child, Func)
                   and x.child.fname in ("__explode__", "__posexplode__") for x, _ in exprs):
            return self._with(_rel_node(self._src(), ("project", list(exprs)), "project"))
        return self._map(functools.partial(_apply_project, exprs), "project")

    def selectExpr(self, *exprs):
        from raydp_amd.spark.functions import expr
        out = []
        for e in exprs:
            e = e.strip()
            out.append(e if e == "*" or e.replace("_", "").isalnum() else expr(e))
        return self.select(*out)

    def where(self, condition):
        return self.filter(condition)

    def withColumn(self, colName: str, col: Column):
        e = col._expr
        if isinstance(e, WindowExpr):
            return self._with(W.WindowPlan(self._src(), colName, e.fn, e.args, e.window))
        e, hoisted = _hoist_windows(e)
        if hoisted:
            # window functions nested in an expression (e.g. row_number().over(w) - 1): compute
            # each as a temporary column first, then the outer expression, then drop them
            df = self
            for tmp, we in hoisted:
                df = df._with(W.WindowPlan(df._src(), tmp, we.fn, we.args, we.window))
            return df.withColumn(colName, Column(e)).drop(*[t for t, _ in hoisted])
        self.columns   # resolves the input schema (analysis errors surface here, as in Spark)
        return self._with(_rel_node(self._src(), ("with", colName, e), f"withColumn({colName})"))

    def withColumns(self, colsMap: Dict[str, Column]):
        df = self
        for k, v in colsMap.items():
            df = df.withColumn(k, v)
        return df

    def withColumnRenamed(self, existing: str, new: str):
        return self._map(lambda t, i: t.rename_columns(
            [new if c == existing else c for c in t.column_names]), "rename")

    def toDF(self, *names):
        return self._map(lambda t, i: t.rename_columns(list(names)), "toDF")

    def alias(self, name):
        return self

    def drop(self, *cols):
        names = set()
        for c in cols:
            names.add(c if isinstance(c, str) else c._expr.name())
        return self._with(_rel_node(self._src(), ("drop", frozenset(names)), "drop"))

    def filter(self, condition):
        if isinstance(condition, str):
            from raydp_amd.spark.sqlexpr import parse
            condition = parse(condition)
        src = self._src()
        preds = [condition._expr]
        # CombineFilters: consecutive filters become one pass with an AND-ed predicate
        if isinstance(src, P.MapPlan) and getattr(src, "filter_preds", None) is not None:
            preds = src.filter_preds + preds
            src = src.child

        node = _rel_node(src, ("filter", list(preds)), "filter")
        node.filter_preds = preds
        return self._with(node)

    where = filter

    def limit(self, num: int):
        num = int(num)
        src = self._src()

        class _Limit(P.WidePlan):
            def children(self_):
                return [src]

            def num_partitions(self_):
                return 1

            def empty(self_):
                return src.schema.empty_table()

            def execute(self_, scheduler):
                out, have = [], 0
                for i in range(src.num_partitions()):
                    if have >= num:
                        break
                    t = src.compute(i)
                    t = t.slice(0, num - have)
                    have += t.num_rows
                    out.append(t)
                return [P.concat(out, src.schema)]
        return self._with(_Limit())

    def distinct(self):
        return self._with(W.DistinctPlan(self._src()))

    def dropDuplicates(self, subset=None):
        return self._with(W.DistinctPlan(self._src(), list(subset) if subset else None))

    drop_duplicates = dropDuplicates

    def _sort_keys(self, cols, ascending):
        cols = _names_of(cols)
        if isinstance(ascending, bool):
            ascending = [ascending] * len(cols)
        keys = []
        for c, asc in zip(cols, ascending):
            e = _to_expr(c, name_is_col=True)
            if isinstance(e, SortOrder):
                keys.append((e.child, e.ascending, e.nulls_first))
            else:
                keys.append((e, bool(asc), bool(asc)))
        return keys

    def orderBy(self, *cols, ascending=True):
        return self._with(P.SortPlan(self._src(), self._sort_keys(cols, ascending)))

    sort = orderBy

    def sortWithinPartitions(self, *cols, ascending=True):
        keys = self._sort_keys(cols, ascending)
        return self._map(lambda t, i: P.sort_table(t, keys), "sortWithinPartitions")

    def groupBy(self, *cols):
        keys, df = [], self
        for c in _names_of(cols):
            if isinstance(c, str):
                keys.append(c)
                continue
            e = c._expr
            inner = e.child if isinstance(e, Alias) else e
            if isinstance(inner, ColRef) and not isinstance(e, Alias):
                keys.append(inner.col_name)
            else:     # an expression key: materialise it under its name first
                df = df.withColumn(e.name(), c)
                keys.append(e.name())
        return GroupedData(df, keys)

    groupby = groupBy

    def agg(self, *exprs):
        return GroupedData(self, []).agg(*exprs)

    def join(self, other: "DataFrame", on=None, how: str = "inner"):
        """Spark's ``DataFrame.join``: ``on`` is a column name, a list of names, or a condition
        (``a.k == b.k``, conjunctions with ``&``, a list of conditions). Equalities between a left
        and a right column become the hash-join keys; every other conjunct is a residual condition
        that decides which key-matched pairs match (``a.k == b.k & (a.x < b.y)``), also for outer,
        semi and anti joins (reference: any join is Spark SQL's, ``doc/spark_on_ray.md:187-201``)."""
        how = how or "inner"
        if on is None:
            return self.crossJoin(other)
        if isinstance(on, str):
            lk = rk = [on]
        elif isinstance(on, (list, tuple)) and all(isinstance(x, str) for x in on):
            lk = rk = list(on)
        else:
            conds = on if isinstance(on, (list, tuple)) else [on]
            conj, stack = [], [c._expr for c in reversed(conds)]
            while stack:
                e = stack.pop()
                if isinstance(e, BinOp) and e.op == "&":
                    stack += [e.right, e.left]
                else:
                    conj.append(e)
            lk, rk, residual = [], [], []
            for e in conj:
                if isinstance(e, BinOp) and e.op == "==" and isinstance(e.left, ColRef) \
                        and isinstance(e.right, ColRef):
                    sa, sb = self._join_side(e.left, other), self._join_side(e.right, other)
                    if (sa, sb) in (("L", "R"), ("R", "L")):
                        a, b = (e.left, e.right) if sa == "L" else (e.right, e.left)
                        lk.append(a.col_name)
                        rk.append(b.col_name)
                        continue
                residual.append(e)
            if residual:
                return self._join_residual(other, lk, rk, residual, how)
            if not lk:
                raise NotImplementedError("a join condition needs an equality between a left and a "
                                          "right column (or use crossJoin + filter)")
        return self._with(W.JoinPlan(self._src(), other._src(), lk, rk, how))

    def _join_side(self, ref, other) -> Optional[str]:
        """'L' / 'R' for a column reference of a join condition: the DataFrame it was taken
        from (``a["x"]`` / ``a.x``), else the side that has the name (None if both or neither)."""
        o = getattr(ref, "origin", None)
        if o is not None and o == id(self) and ref.col_name in self.columns:
            return "L"
        if o is not None and o == id(other) and ref.col_name in other.columns:
            return "R"
        inl, inr = ref.col_name in self.columns, ref.col_name in other.columns
        return "L" if inl and not inr else "R" if inr and not inl else None

    def _join_residual(self, other, lk, rk, residual, how):
        """Join with non-equality conditions: the right side's columns the residual reads are
        renamed apart first (so ``a.x < b.x`` reads both), the key-matched pairs are filtered, and
        outer / semi / anti joins are rebuilt from the matched pairs by row ids."""
        from raydp_amd.spark import functions as F
        from raydp_amd.spark.wide import _JOIN_TYPES
        jt = _JOIN_TYPES[how.lower()]
        tag = f"__j{id(self) & 0xffff:x}"
        ren = {}

        def ref(e):
            side = self._join_side(e, other)
            if side is None:
                raise ValueError(f"join condition column {e.col_name!r} is ambiguous or unknown; "
                                 "take it from one DataFrame (a['x'])")
            if side == "R":
                ren.setdefault(e.col_name, f"{tag}_r_{e.col_name}")
                return ColRef(ren[e.col_name])
            if e.col_name in other.columns:      # the joined rows carry both sides' copies
                lren.setdefault(e.col_name, f"{tag}_l_{e.col_name}")
                return ColRef(lren[e.col_name])
            return ColRef(e.col_name)
        lren = {}
        res = [_rewrite_refs(e, ref) for e in residual]
        cond = Column(res[0])
        for e in res[1:]:
            cond = cond & Column(e)
        # row ids are materialised once (localCheckpoint): the matched pairs and the unmatched rows
        # must see the same id for a row, whichever stage later evaluates the side
        left = self.withColumn(tag + "_lid", F.monotonically_increasing_id()).localCheckpoint() \
            if jt in ("left outer", "full outer", "left semi", "left anti") else self
        for c, t in lren.items():
            left = left.withColumn(t, F.col(c))
        right = other
        for c, t in ren.items():
            right = right.withColumn(t, F.col(c))
        if jt in ("right outer", "full outer"):
            right = right.withColumn(tag + "_rid", F.monotonically_increasing_id()).localCheckpoint()
        if lk:
            matched = left._with(W.JoinPlan(left._src(), right._src(), lk, rk, "inner")).filter(cond)
        else:
            matched = left.crossJoin(right).filter(cond)
        helper = list(ren.values()) + list(lren.values())
        if jt == "inner":
            return matched.drop(*helper)
        if jt in ("left semi", "left anti"):
            ids = matched.select(tag + "_lid").distinct()
            return left.join(ids, tag + "_lid", "left_semi" if jt == "left semi" else "left_anti") \
                .drop(*([tag + "_lid"] + list(lren.values())))
        target = matched.arrow_schema
        lc, rc = left.columns, right.columns
        same = lk == rk and bool(lk)
        kept = [j for j, c in enumerate(rc) if not (same and c in rk)]
        if len(target) != len(lc) + len(kept):
            raise NotImplementedError("outer join with a residual condition: unexpected joined layout")
        parts = [matched]
        if jt in ("left outer", "full outer"):
            src = list(range(len(lc))) + [-1] * len(kept)
            lost = left.join(matched.select(tag + "_lid"), tag + "_lid", "left_anti")
            parts.append(lost._map(functools.partial(_pad_to, target, src), "join pad"))
        if jt in ("right outer", "full outer"):
            src = [rc.index(rk[lk.index(c)]) if same and c in lk else -1 for c in lc] + kept
            lost = right.join(matched.select(tag + "_rid"), tag + "_rid", "left_anti")
            parts.append(lost._map(functools.partial(_pad_to, target, src), "join pad"))
        out = parts[0]
        for p_ in parts[1:]:
            out = out.union(p_)
        return out.drop(*(helper + [c for c in (tag + "_lid", tag + "_rid") if c in target.names]))

    def crossJoin(self, other):
        from raydp_amd.spark import functions as F
        a = self.withColumn("__cj", F.lit(0))
        b = other.withColumn("__cj", F.lit(0))
        return a.join(b, "__cj").drop("__cj")

    def union(self, other):
        return self._with(P.UnionPlan([self._src(), other._src()]))

    unionAll = union

    def unionByName(self, other, allowMissingColumns=False):
        return self._with(P.UnionPlan([self._src(), other._src()], by_name=True))

    def repartition(self, numPartitions, *cols):
        adaptive = None
        if isinstance(numPartitions, (str, Column)):
            cols = (numPartitions,) + cols
            numPartitions = self._session.conf.get("spark.sql.shuffle.partitions", "200")
            conf = self._session.conf
            if str(conf.get("spark.sql.adaptive.enabled", "true")).lower() == "true" and \
                    str(conf.get("spark.sql.adaptive.coalescePartitions.enabled", "true")).lower() == "true":
                from raydp_amd.utils import parse_memory_size
                advisory = parse_memory_size(str(conf.get("spark.sql.adaptive.advisoryPartitionSizeInBytes", "64m")))
                min_parts = int(conf.get("spark.sql.adaptive.coalescePartitions.minPartitionNum",
                                         str(self._session._default_parallelism())))
                adaptive = (advisory, min_parts)
        keys = [c if isinstance(c, str) else c._expr.name() for c in _names_of(cols)] or None
        return self._with(P.RepartitionPlan(self._src(), int(numPartitions), keys, adaptive=adaptive))

    def coalesce(self, numPartitions):
        return self._with(P.CoalescePlan(self._src(), numPartitions))

    def randomSplit(self, weights, seed=None):
        w = np.asarray(weights, dtype=np.float64)
        if (w < 0).any():
            raise ValueError("Weights must be positive")
        w = w / w.sum()
        edges = np.concatenate([[0.0], np.cumsum(w)])
        edges[-1] = 1.0 + 1e-12
        seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
        src = self._src()
        out = []
        for k in range(len(w)):
            lo, hi = edges[k], edges[k + 1]

            def fn(t, i, lo=lo, hi=hi):
                r = np.random.default_rng([seed, i]).random(t.num_rows)
                return t.filter(pa.array((r >= lo) & (r < hi)))
            out.append(self._with(P.MapPlan(src, fn, f"randomSplit[{k}]")))
        return out

    def sample(self, withReplacement=None, fraction=None, seed=None):
        if isinstance(withReplacement, float):
            withReplacement, fraction, seed = False, withReplacement, fraction
        seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))

        def fn(t, i):
            rng = np.random.default_rng([seed, i, 7])
            if withReplacement:
                k = rng.poisson(fraction, t.num_rows)
                return t.take(pa.array(np.repeat(np.arange(t.num_rows), k)))
            return t.filter(pa.array(rng.random(t.num_rows) < fraction))
        return self._map(fn, "sample")

    def fillna(self, value, subset=None):
        if isinstance(subset, str):
            subset = [subset]

        def fn(t, i):
            cols = []
            for name, c in zip(t.column_names, t.columns):
                v = value.get(name) if isinstance(value, dict) else value
                if v is None or (subset is not None and name not in subset) or c.null_count == 0:
                    cols.append(c)
                    continue
                ty = c.type
                ok = (isinstance(v, str) and pa.types.is_string(ty)) or \
                     (isinstance(v, bool) and pa.types.is_boolean(ty)) or \
                     (isinstance(v, (int, float)) and not isinstance(v, bool)
                      and (pa.types.is_integer(ty) or pa.types.is_floating(ty)))
                if ok:
                    c = pc.fill_null(c, pa.scalar(v).cast(ty, safe=False))
                cols.append(c)
            return pa.Table.from_arrays(cols, names=t.column_names)
        return self._map(fn, "fillna")

    def dropna(self, how="any", thresh=None, subset=None):
        if isinstance(subset, str):
            subset = [subset]

        def fn(t, i):
            names = subset or t.column_names
            valid = np.zeros(t.num_rows, dtype=np.int64)
            for nme in names:
                valid += pc.is_valid(t.column(nme)).to_numpy(zero_copy_only=False).astype(np.int64)
            if thresh is not None:
                keep = valid >= thresh
            elif how == "all":
                keep = valid > 0
            else:
                keep = valid == len(names)
            return t.filter(pa.array(keep))
        return self._map(fn, "dropna")

    def replace(self, to_replace, value=None, subset=None):
        mapping = to_replace if isinstance(to_replace, dict) else {to_replace: value}

        def fn(t, i):
            cols = []
            for name, c in zip(t.column_names, t.columns):
                if subset and name not in subset:
                    cols.append(c)
                    continue
                for a, b in mapping.items():
                    try:
                        c = pc.if_else(pc.equal(c, pa.scalar(a).cast(c.type)), pa.scalar(b).cast(c.type), c)
                    except (pa.ArrowInvalid, pa.ArrowNotImplementedError, TypeError):
                        pass
                cols.append(c)
            return pa.Table.from_arrays(cols, names=t.column_names)
        return self._map(fn, "replace")

    def mapInPandas(self, func, schema):
        from raydp_amd.spark.session import _to_arrow_schema
        target = _to_arrow_schema(schema)

        def fn(t, i):
            pdfs = list(func(iter([t.to_pandas()])))
            if not pdfs:
                return target.empty_table()
            tables = [pa.Table.from_pandas(p, schema=target, preserve_index=False) for p in pdfs]
            return pa.concat_tables(tables)
        return self._map(fn, "mapInPandas")

    def mapInArrow(self, func, schema):
        from raydp_amd.spark.session import _to_arrow_schema
        target = _to_arrow_schema(schema)

        def fn(t, i):
            batches = list(func(iter(t.to_batches())))
            if not batches:
                return target.empty_table()
            return pa.Table.from_batches(batches).cast(target)
        return self._map(fn, "mapInArrow")

    # ------------------------------------------------------------------ caching ----------
    def persist(self, storageLevel=StorageLevel.MEMORY_AND_DISK):
        self._storage_level = storageLevel
        if self._cached is None:
            tables = self._session._run(self._plan)
            self._cached = P.MaterializedPlan(tables, self._plan.schema)
        return self

    def cache(self):
        return self.persist(StorageLevel.MEMORY_AND_DISK)

    def unpersist(self, blocking=False):
        self._cached = None
        self._storage_level = None
        return self

    def localCheckpoint(self, eager=True):
        return self._with(P.MaterializedPlan(self._session._run(self._src()), self._plan.schema))

    checkpoint = localCheckpoint

    # ------------------------------------------------------------------- actions ----------
    def _partitions(self) -> List[pa.Table]:
        return self._session._run(self._src())

    def toArrow(self) -> pa.Table:
        return P.concat(self._partitions(), self._plan.schema)

    def count(self) -> int:
        src = self._src()
        parts = self._session._run(P.MapPlan(src, _count_rows, "count"))
        return int(sum(t.column(0)[0].as_py() for t in parts))

    def collect(self) -> List[Row]:
        t = self.toArrow()
        names = t.column_names
        cols = [c.to_pylist() for c in t.columns]
        return [Row._make(names, vals) for vals in zip(*cols)] if cols else []

    def take(self, num):
        return self.limit(num).collect()

    def head(self, n=None):
        if n is None:
            rows = self.take(1)
            return rows[0] if rows else None
        return self.take(n)

    def first(self):
        return self.head()

    def isEmpty(self):
        return len(self.take(1)) == 0

    def toLocalIterator(self, prefetchPartitions=False):
        src = self._src()
        P.prepare(src, self._session._scheduler_or_default())
        for i in range(src.num_partitions()):
            t = src.compute(i)
            names = t.column_names
            for vals in zip(*[c.to_pylist() for c in t.columns]):
                yield Row._make(names, vals)

    def toPandas(self):
        return self.toArrow().to_pandas()

    def to_pandas_on_spark(self, index_col=None):
        from raydp_amd.spark import pandas as ps
        return ps.DataFrame(self)

    pandas_api = to_pandas_on_spark

    def show(self, n=20, truncate=True, vertical=False):
        rows = self.take(n)
        names = self.columns
        width = 20 if truncate is True else (int(truncate) if truncate else 10 ** 9)

        def fmt(v):
            s = "null" if v is None else str(v)
            return s if len(s) <= width else s[:width - 3] + "..."
        cells = [[fmt(v) for v in r] for r in rows]
        w = [max([len(nm)] + [len(r[j]) for r in cells]) for j, nm in enumerate(names)]
        sep = "+" + "+".join("-" * x for x in w) + "+"
        print(sep)
        print("|" + "|".join(nm.rjust(w[j]) for j, nm in enumerate(names)) + "|")
        print(sep)
        for r in cells:
            print("|" + "|".join(v.rjust(w[j]) for j, v in enumerate(r)) + "|")
        print(sep)
        if len(rows) == n:
            print(f"only showing top {n} rows")

    def describe(self, *cols):
        from raydp_amd.spark import functions as F
        cols = _names_of(cols) or [f.name for f in self._plan.schema
                                   if pa.types.is_integer(f.type) or pa.types.is_floating(f.type)]
        stats = {}
        for fn in ("count", "avg", "stddev", "min", "max"):
            r = self.agg(*[getattr(F, fn)(c).alias(c) for c in cols]).collect()[0]
            stats[fn if fn != "avg" else "mean"] = [str(r[c]) for c in cols]
        rows = [(k,) + tuple(v) for k, v in stats.items()]
        return self._session.createDataFrame(rows, ["summary"] + cols)

    def createOrReplaceTempView(self, name):
        self._session._catalog[name] = self

    createTempView = createOrReplaceTempView
    registerTempTable = createOrReplaceTempView

    def explain(self, extended=False):
        def walk(p, d=0):
            print("  " * d + type(p).__name__ + (f"({p.desc})" if hasattr(p, "desc") else ""))
            for c in p.children():
                walk(c, d + 1)
        walk(self._plan)

    def toJSON(self):
        return [json.dumps(r.asDict(), default=str) for r in self.collect()]

    def __len__(self):
        return self.count()


def _df_rdd(df: "DataFrame"):
    """``df.rdd``: an RDD of Row objects whose partitions are the DataFrame's partitions."""
    from raydp_amd.spark.rdd import RDD
    plan = df._src()
    P.prepare(plan, df._session._scheduler_or_default())
    names = plan.schema.names

    def rows(i):
        t = plan.compute(i)
        cols = [c.to_pylist() for c in t.columns]
        return [Row._make(names, vals) for vals in zip(*cols)] if cols else []
    r = RDD(df._session, plan.num_partitions(), rows, "dataframe", prefs=lambda i: P.preferred_node(plan, i))
    r._id_str = df._id
    return r


def _hoist_windows(e):
    """Replace every nested WindowExpr in ``e`` by a temporary column reference."""
    import copy
    import uuid
    found = []

    def walk(x):
        if isinstance(x, WindowExpr):
            name = f"__win_{uuid.uuid4().hex[:8]}"
            found.append((name, x))
            return ColRef(name)
        if isinstance(x, Expr):
            y = copy.copy(x)
            for k, v in vars(x).items():
                nv = walk(v) if isinstance(v, (Expr, list, tuple)) else v
                if nv is not v:
                    setattr(y, k, nv)
            return y
        if isinstance(x, (list, tuple)):
            out = [walk(v) if isinstance(v, (Expr, list, tuple)) else v for v in x]
            if any(a is not b for a, b in zip(out, x)):
                return type(x)(out) if isinstance(x, tuple) else out
            return x
        return x
    if isinstance(e, WindowExpr) or not _has_window(e):
        return e, []
    ne = walk(e)
    return (ne, found) if found else (e, [])


def _has_window(x) -> bool:
    # explicit stack: every withColumn of a plan build asks this (the recursive generator form
    # was ~a tenth of the NYC plan build)
    stack = [x]
    while stack:
        y = stack.pop()
        if isinstance(y, WindowExpr):
            return True
        if isinstance(y, Expr):
            vals = y.__dict__.values()
        elif isinstance(y, (list, tuple)):
            vals = y
        else:
            continue
        for v in vals:
            if isinstance(v, (Expr, list, tuple)):
                stack.append(v)
    return False
