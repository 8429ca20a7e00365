"""Column expressions evaluated on Arrow record batches with Arrow compute kernels.

A ``Column`` wraps an expression tree (``Expr``). Every node evaluates against one
partition (``pa.Table``) and returns an Arrow array or scalar; all arithmetic, comparison,
datetime and string work runs in Arrow's C++ compute kernels (the GIL is released), so a
partition task only touches Python at plan nodes, not per row (Python UDFs excepted, see
``udf.py``). Spark semantics kept: ``/`` always yields double, comparisons with null are
null and ``filter`` drops null predicates, ``dayofweek`` counts 1=Sunday..7=Saturday.
"""
from typing import Any, Callable, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from raydp_amd.spark.types import DataType, parse_type_string


# ------------------------------------------------------------------------------------------
# helpers
# ------------------------------------------------------------------------------------------
def as_array(v, n: int):
    """Broadcast a scalar result to a length-n array; pass arrays through."""
    if isinstance(v, pa.ChunkedArray):
        return v.combine_chunks() if v.num_chunks != 1 else v.chunk(0)
    if isinstance(v, pa.Array):
        return v
    if isinstance(v, pa.Scalar):
        if not v.is_valid:
            return pa.nulls(n, type=v.type if v.type != pa.null() else pa.null())
        return pa.repeat(v, n)
    return pa.repeat(pa.scalar(v), n) if v is not None else pa.nulls(n)


def _is_str(t):
    return pa.types.is_string(t) or pa.types.is_large_string(t)


def _num_type(v):
    return v.type


def _to_double(v):
    t = v.type
    if pa.types.is_floating(t) and t != pa.float64() or pa.types.is_integer(t) or \
            pa.types.is_boolean(t) or pa.types.is_decimal(t):
        return pc.cast(v, pa.float64())
    if _is_str(t):
        return pc.cast(v, pa.float64(), safe=False)
    return v


_TS_FORMATS = ["%Y-%m-%d %H:%M:%S", "%Y-%m-%dT%H:%M:%S", "%Y-%m-%d %H:%M", "%Y-%m-%d"]


def to_timestamp(v, fmt: Optional[str] = None):
    """Cast strings/dates to a timestamp the way Spark's implicit cast does.

    The session time zone is UTC, so timestamps are kept zone-naive (wall time == UTC);
    this avoids depending on a tz database for field extraction."""
    t = v.type
    if pa.types.is_timestamp(t):
        if t.tz is not None:
            return pc.cast(v, pa.timestamp(t.unit))
        return v
    if pa.types.is_date(t):
        return pc.cast(v, pa.timestamp("s"))
    if _is_str(t):
        chunks = v.chunks if isinstance(v, pa.ChunkedArray) else [v]
        key = (tuple((c.buffers()[2].address if c.buffers()[2] is not None else 0, c.offset, len(c))
                     for c in chunks), fmt)
        hit = _ts_cache_get(key, v)
        if hit is not None:
            return hit
        out = _parse_ts(v, fmt)
        _ts_cache_put(key, v, out)
        return out
    raise TypeError(f"cannot cast {t} to timestamp")


# One parsed-timestamp cache entry per thread: the NYC ETL calls 7 datetime functions on the
# same string column of a partition; parse it once (common-subexpression elimination).
import threading as _threading  # noqa: E402

_ts_tls = _threading.local()


def _ts_cache_get(key, v):
    # the entry holds a reference to the source array, so its buffer addresses stay valid
    ent = getattr(_ts_tls, "ent", None)
    if ent is not None and ent[0] == key:
        return ent[2]
    return None


def _ts_cache_put(key, v, out):
    _ts_tls.ent = (key, v, out)


def _parse_ts(v, fmt):
    if fmt is None:
        # fast path: "YYYY-MM-DD HH:MM:SS[ UTC]" — parse the first 19 code units directly
        blen = pc.binary_length(v)
        shape_ok = pc.or_(pc.equal(blen, 19), pc.and_(pc.equal(blen, 23), pc.ends_with(v, " UTC")))
        if pc.all(pc.fill_null(shape_ok, True)).as_py():
            try:
                # Arrow's ISO-8601 cast: ~10x faster than strptime on this shape
                return pc.utf8_slice_codeunits(v, 0, 19).cast(pa.timestamp("s"))
            except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
                pass
    if True:
        s = pc.utf8_trim_whitespace(v)
        # strip a trailing zone id (" UTC", "Z", "+00:00"): the session time zone is UTC
        s = pc.replace_substring_regex(s, pattern=r"(\s*UTC|Z|\+00:?00)$", replacement="")
        s = pc.replace_substring_regex(s, pattern=r"\.\d+$", replacement="")
        formats = [fmt] if fmt else _TS_FORMATS
        out = None
        for f in formats:
            parsed = pc.strptime(s, format=f, unit="s", error_is_null=True)
            out = parsed if out is None else pc.coalesce(out, parsed)
        return out


def _spark_type_coerce(a, b):
    """Unify operand types the way Spark's analyzer does for binary arithmetic/compare."""
    ta = a.type if hasattr(a, "type") else None
    tb = b.type if hasattr(b, "type") else None
    if ta is not None and tb is not None:
        if _is_str(ta) and (pa.types.is_integer(tb) or pa.types.is_floating(tb)):
            a = pc.cast(_numeric_or_null(a) if not isinstance(a, pa.Scalar) else a, pa.float64(), safe=False)
        elif _is_str(tb) and (pa.types.is_integer(ta) or pa.types.is_floating(ta)):
            b = pc.cast(_numeric_or_null(b) if not isinstance(b, pa.Scalar) else b, pa.float64(), safe=False)
        elif pa.types.is_timestamp(ta) and _is_str(tb):
            b = to_timestamp(b if isinstance(b, (pa.Array, pa.ChunkedArray)) else pa.array([b.as_py()]))[0] \
                if isinstance(b, pa.Scalar) else to_timestamp(b)
    return a, b


# ------------------------------------------------------------------------------------------
# expression nodes
# ------------------------------------------------------------------------------------------
class Expr:
    def eval(self, batch: pa.Table):
        raise NotImplementedError

    def name(self) -> str:
        raise NotImplementedError

    def children(self) -> List["Expr"]:
        return []

    def references(self) -> set:
        out = set()
        for c in self.children():
            out |= c.references()
        return out

    def is_aggregate(self) -> bool:
        return any(c.is_aggregate() for c in self.children())

    def __repr__(self):
        return f"Column<'{self.name()}'>"


class ColRef(Expr):
    qualifier = None      # ``alias`` of an SQL ``alias.col`` reference (set by the SQL parser)

    def __init__(self, col_name: str):
        self.col_name = col_name

    def eval(self, batch):
        if self.col_name == "*":
            raise ValueError("'*' is only valid in select")
        try:
            return batch.column(self.col_name)
        except KeyError:
            # case-insensitive resolution like Spark's default analyzer
            for n in batch.column_names:
                if n.lower() == self.col_name.lower():
                    return batch.column(n)
            raise KeyError(f"cannot resolve column '{self.col_name}' given input columns "
                           f"{batch.column_names}")

    def name(self):
        return self.col_name

    def references(self):
        return {self.col_name}


class Lit(Expr):
    def __init__(self, value):
        self.value = value

    def eval(self, batch):
        v = self.value
        if isinstance(v, pa.Scalar):
            return v
        return pa.scalar(v)

    def name(self):
        v = self.value
        if isinstance(v, str):
            return v
        if v is None:
            return "NULL"
        if isinstance(v, bool):
            return str(v).lower()
        return str(v)


_ARITH = {"+": pc.add, "-": pc.subtract, "*": pc.multiply}
_CMP = {"<": pc.less, "<=": pc.less_equal, ">": pc.greater, ">=": pc.greater_equal,
        "==": pc.equal, "!=": pc.not_equal}


class BinOp(Expr):
    def __init__(self, op: str, left: Expr, right: Expr):
        self.op, self.left, self.right = op, left, right

    def children(self):
        return [self.left, self.right]

    def eval(self, batch):
        a, b = self.left.eval(batch), self.right.eval(batch)
        op = self.op
        if op in _ARITH:
            a, b = _spark_type_coerce(a, b)
            return _ARITH[op](a, b)
        if op == "/":
            return pc.divide(_to_double(a), _to_double(b))
        if op == "%":
            a, b = _spark_type_coerce(a, b)
            if pa.types.is_integer(a.type) and pa.types.is_integer(b.type):
                # Java/Spark remainder takes the sign of the dividend
                q = pc.divide(a, b)
                return pc.subtract(a, pc.multiply(q, b))
            ad, bd = _to_double(a), _to_double(b)
            return pc.subtract(ad, pc.multiply(pc.trunc(pc.divide(ad, bd)), bd))
        if op == "**":
            return pc.power(_to_double(a), _to_double(b))
        if op in _CMP:
            a, b = _spark_type_coerce(a, b)
            return _CMP[op](a, b)
        if op == "&":
            return pc.and_kleene(a, b)
        if op == "|":
            return pc.or_kleene(a, b)
        if op == "<=>":
            eq = pc.equal(a, b)
            both_null = pc.and_(pc.is_null(a), pc.is_null(b))
            return pc.or_(pc.fill_null(eq, False), both_null)
        raise ValueError(op)

    def name(self):
        op = {"==": "=", "&": "AND", "|": "OR"}.get(self.op, self.op)
        return f"({self.left.name()} {op} {self.right.name()})"


class UnaryOp(Expr):
    def __init__(self, op: str, child: Expr):
        self.op, self.child = op, child

    def children(self):
        return [self.child]

    def eval(self, batch):
        v = self.child.eval(batch)
        if self.op == "-":
            return pc.negate(v)
        if self.op == "~":
            return pc.invert(v)
        if self.op == "isnull":
            return pc.is_null(v) if not isinstance(v, pa.Scalar) else pa.scalar(not v.is_valid)
        if self.op == "isnotnull":
            return pc.is_valid(v) if not isinstance(v, pa.Scalar) else pa.scalar(v.is_valid)
        if self.op == "isnan":
            return pc.is_nan(_to_double(v))
        raise ValueError(self.op)

    def name(self):
        if self.op == "-":
            return f"(- {self.child.name()})"
        if self.op == "~":
            return f"(NOT {self.child.name()})"
        return f"({self.child.name()} IS {'NOT ' if self.op == 'isnotnull' else ''}NULL)" \
            if self.op != "isnan" else f"isnan({self.child.name()})"


class Func(Expr):
    """A built-in SQL function: ``impl(list_of_evaluated_args, batch) -> array/scalar``."""

    native = None  # opcode tag when the fused expression VM implements this function

    def __init__(self, fname: str, args: List[Expr], impl: Callable, display: Optional[str] = None):
        self.fname, self.args, self.impl, self.display = fname, args, impl, display

    def children(self):
        return list(self.args)

    def eval(self, batch):
        return self.impl([a.eval(batch) for a in self.args], batch)

    def name(self):
        if self.display:
            return self.display
        return f"{self.fname}({', '.join(a.name() for a in self.args)})"


class UDFExpr(Expr):
    def __init__(self, udf, args: List[Expr]):
        self.udf, self.args = udf, args

    def children(self):
        return list(self.args)

    def eval(self, batch):
        n = batch.num_rows
        arrays = [as_array(a.eval(batch), n) for a in self.args]
        return self.udf.evaluate(arrays, n)

    def name(self):
        return f"{self.udf.__name__}({', '.join(a.name() for a in self.args)})"


class Alias(Expr):
    def __init__(self, child: Expr, alias: str):
        self.child, self.alias = child, alias

    def children(self):
        return [self.child]

    def eval(self, batch):
        return self.child.eval(batch)

    def name(self):
        return self.alias


_NUMERIC_RE = r"^\s*[-+]?((\d+\.?\d*|\.\d+)([eE][-+]?\d+)?|[Nn]a[Nn]|[Ii]nf(inity)?)\s*$"


def _numeric_or_null(v):
    """String array with every non-numeric entry replaced by NULL (trimmed)."""
    try:
        pc.cast(v, pa.float64())
        return v
    except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
        ok = pc.match_substring_regex(v, _NUMERIC_RE)
        return pc.utf8_trim_whitespace(pc.if_else(ok, v, pa.scalar(None, v.type)))


class Cast(Expr):
    def __init__(self, child: Expr, to: DataType):
        self.child, self.to = child, to

    def children(self):
        return [self.child]

    def eval(self, batch):
        v = self.child.eval(batch)
        t = self.to.to_arrow()
        if pa.types.is_timestamp(t):
            return to_timestamp(v if not isinstance(v, pa.Scalar) else pa.array([v.as_py()]))
        if pa.types.is_integer(t) and hasattr(v, "type") and pa.types.is_floating(v.type):
            return pc.cast(pc.trunc(v), t, safe=False)
        if hasattr(v, "type") and _is_str(v.type) and (pa.types.is_integer(t) or pa.types.is_floating(t)
                                                        or pa.types.is_decimal(t)):
            # Spark (non-ANSI) casts unparsable strings to NULL instead of failing
            v = _numeric_or_null(v)
            if pa.types.is_integer(t):
                return pc.cast(pc.trunc(pc.cast(v, pa.float64(), safe=False)), t, safe=False)
            return pc.cast(v, t, safe=False)
        if _is_str(t) and hasattr(v, "type") and pa.types.is_boolean(v.type):
            return pc.if_else(v, "true", "false")
        return pc.cast(v, t, safe=False)

    def name(self):
        return f"CAST({self.child.name()} AS {self.to.simpleString().upper()})"


class CaseWhen(Expr):
    def __init__(self, branches, otherwise: Optional[Expr] = None):
        self.branches, self.otherwise = list(branches), otherwise

    def children(self):
        out = []
        for c, v in self.branches:
            out += [c, v]
        if self.otherwise is not None:
            out.append(self.otherwise)
        return out

    def eval(self, batch):
        n = batch.num_rows
        vals = [as_array(v.eval(batch), n) for _, v in self.branches]
        other = as_array(self.otherwise.eval(batch), n) if self.otherwise is not None else None
        # common result type
        target = None
        for v in vals + ([other] if other is not None else []):
            if v.type != pa.null():
                target = v.type if target is None else _wider(target, v.type)
        target = target or pa.null()
        out = pc.cast(other, target) if other is not None else pa.nulls(n, type=target)
        for (c, _), v in reversed(list(zip(self.branches, vals))):
            cond = pc.fill_null(as_array(c.eval(batch), n), False)
            out = pc.if_else(cond, pc.cast(v, target), out)
        return out

    def when(self, cond, value):
        return CaseWhen(self.branches + [(_to_expr(cond), _to_expr(value))], self.otherwise)

    def name(self):
        s = "CASE " + " ".join(f"WHEN {c.name()} THEN {v.name()}" for c, v in self.branches)
        if self.otherwise is not None:
            s += f" ELSE {self.otherwise.name()}"
        return s + " END"


def _wider(a: pa.DataType, b: pa.DataType) -> pa.DataType:
    if a == b:
        return a
    if pa.types.is_floating(a) or pa.types.is_floating(b):
        return pa.float64()
    if pa.types.is_integer(a) and pa.types.is_integer(b):
        return pa.int64()
    return pa.string()


class SortOrder(Expr):
    def __init__(self, child: Expr, ascending=True, nulls_first=None):
        self.child, self.ascending = child, ascending
        self.nulls_first = ascending if nulls_first is None else nulls_first

    def children(self):
        return [self.child]

    def eval(self, batch):
        return self.child.eval(batch)

    def name(self):
        return self.child.name()


class AggExpr(Expr):
    """Aggregate function (evaluated by the groupBy/agg operator, not per row)."""

    def __init__(self, fn: str, child: Optional[Expr], distinct=False):
        self.fn, self.child, self.distinct = fn, child, distinct

    def children(self):
        return [self.child] if self.child is not None else []

    def is_aggregate(self):
        return True

    def eval(self, batch):
        raise ValueError(f"aggregate {self.fn} used outside groupBy/agg")

    def name(self):
        inner = self.child.name() if self.child is not None else "1"
        if self.distinct:
            inner = "DISTINCT " + inner
        return f"{self.fn}({inner})"


class WindowExpr(Expr):
    """``fn().over(window)`` — ranking functions and aggregates over a partitioned window."""

    def __init__(self, fn: str, args: List[Expr], window):
        self.fn, self.args, self.window = fn, args, window

    def children(self):
        return list(self.args)

    def eval(self, batch):
        raise ValueError("window expressions are evaluated by the Window operator")

    def name(self):
        return f"{self.fn}() OVER (...)"


def map_children(e: Expr, fn) -> Expr:
    """A shallow copy of ``e`` whose child expressions are replaced by ``fn(child)`` (every
    Expr-valued attribute, list element and tuple element; other state is shared)."""
    import copy

    def conv(v):
        if isinstance(v, Expr):
            return fn(v)
        if isinstance(v, list):
            return [conv(x) for x in v]
        if isinstance(v, tuple):
            return tuple(conv(x) for x in v)
        return v
    out = copy.copy(e)
    for k, v in list(vars(out).items()):
        if isinstance(v, (Expr, list, tuple)):
            setattr(out, k, conv(v))
    return out


def _to_expr(v, name_is_col=False) -> Expr:
    if isinstance(v, Column):
        return v._expr
    if isinstance(v, Expr):
        return v
    if name_is_col and isinstance(v, str):
        return ColRef(v)
    return Lit(v)


# ------------------------------------------------------------------------------------------
# Column (user facing)
# ------------------------------------------------------------------------------------------
class Column:
    def __init__(self, expr: Expr):
        self._expr = expr

    # arithmetic
    def _bin(self, op, other, reverse=False):
        o = _to_expr(other)
        return Column(BinOp(op, o, self._expr) if reverse else BinOp(op, self._expr, o))

    def __add__(self, o): return self._bin("+", o)
    def __radd__(self, o): return self._bin("+", o, True)
    def __sub__(self, o): return self._bin("-", o)
    def __rsub__(self, o): return self._bin("-", o, True)
    def __mul__(self, o): return self._bin("*", o)
    def __rmul__(self, o): return self._bin("*", o, True)
    def __truediv__(self, o): return self._bin("/", o)
    def __rtruediv__(self, o): return self._bin("/", o, True)
    def __mod__(self, o): return self._bin("%", o)
    def __rmod__(self, o): return self._bin("%", o, True)
    def __pow__(self, o): return self._bin("**", o)
    def __neg__(self): return Column(UnaryOp("-", self._expr))

    # comparison
    def __lt__(self, o): return self._bin("<", o)
    def __le__(self, o): return self._bin("<=", o)
    def __gt__(self, o): return self._bin(">", o)
    def __ge__(self, o): return self._bin(">=", o)
    def __eq__(self, o): return self._bin("==", o)  # noqa: E711 - Spark semantics
    def __ne__(self, o): return self._bin("!=", o)
    def eqNullSafe(self, o): return self._bin("<=>", o)

    # boolean
    def __and__(self, o): return self._bin("&", o)
    def __rand__(self, o): return self._bin("&", o, True)
    def __or__(self, o): return self._bin("|", o)
    def __ror__(self, o): return self._bin("|", o, True)
    def __invert__(self): return Column(UnaryOp("~", self._expr))

    def __bool__(self):
        raise ValueError("Cannot convert column into bool: please use '&' for 'and', '|' for "
                         "'or', '~' for 'not' when building DataFrame boolean expressions.")

    __hash__ = object.__hash__

    def __getitem__(self, k):
        from raydp_amd.spark import functions as F
        return F.element_at(self, k + 1) if isinstance(k, int) else F.col(f"{self._expr.name()}.{k}")

    # misc
    def alias(self, *names, **kw):
        return Column(Alias(self._expr, names[0]))

    name = alias

    def cast(self, dataType):
        return Column(Cast(self._expr, parse_type_string(dataType)))

    astype = cast

    def isNull(self): return Column(UnaryOp("isnull", self._expr))
    def isNotNull(self): return Column(UnaryOp("isnotnull", self._expr))

    def isin(self, *values):
        if len(values) == 1 and isinstance(values[0], (list, tuple, set)):
            values = tuple(values[0])
        vs = list(values)

        def impl(args, batch):
            v = as_array(args[0], batch.num_rows)
            return pc.is_in(v, value_set=pa.array(vs, type=v.type if vs else None))
        return Column(Func("in", [self._expr], impl,
                           display=f"({self._expr.name()} IN ({', '.join(map(str, vs))}))"))

    def between(self, lower, upper):
        return (self >= lower) & (self <= upper)

    def when(self, cond, value):
        if not isinstance(self._expr, CaseWhen):
            raise ValueError("when() can only be applied on a Column previously generated by when()")
        return Column(self._expr.when(cond, value))

    def otherwise(self, value):
        if not isinstance(self._expr, CaseWhen):
            raise ValueError("otherwise() can only be applied on a Column generated by when()")
        return Column(CaseWhen(self._expr.branches, _to_expr(value)))

    def asc(self): return Column(SortOrder(self._expr, True))
    def desc(self): return Column(SortOrder(self._expr, False))
    def asc_nulls_first(self): return Column(SortOrder(self._expr, True, True))
    def asc_nulls_last(self): return Column(SortOrder(self._expr, True, False))
    def desc_nulls_first(self): return Column(SortOrder(self._expr, False, True))
    def desc_nulls_last(self): return Column(SortOrder(self._expr, False, False))

    def over(self, window):
        e = self._expr
        if isinstance(e, WindowExpr):
            return Column(WindowExpr(e.fn, e.args, window))
        if isinstance(e, AggExpr):
            return Column(WindowExpr("agg:" + e.fn, [e.child] if e.child else [], window))
        raise ValueError("over() needs a ranking or aggregate function")

    def startswith(self, s):
        return Column(Func("startswith", [self._expr],
                           lambda a, b: pc.starts_with(a[0], pattern=s)))

    def endswith(self, s):
        return Column(Func("endswith", [self._expr], lambda a, b: pc.ends_with(a[0], pattern=s)))

    def contains(self, s):
        return Column(Func("contains", [self._expr],
                           lambda a, b: pc.match_substring(a[0], pattern=s)))

    def like(self, pattern):
        return Column(Func("like", [self._expr], lambda a, b: pc.match_like(a[0], pattern=pattern)))

    def rlike(self, pattern):
        return Column(Func("rlike", [self._expr],
                           lambda a, b: pc.match_substring_regex(a[0], pattern=pattern)))

    def substr(self, startPos, length):
        def impl(a, b):
            return pc.utf8_slice_codeunits(a[0], start=startPos - 1, stop=startPos - 1 + length)
        return Column(Func("substring", [self._expr], impl))

    def getItem(self, key):
        return self[key]

    def __repr__(self):
        return f"Column<'{self._expr.name()}'>"

    def _name(self):
        return self._expr.name()
