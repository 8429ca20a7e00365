"""``pyspark.sql.functions``-compatible built-ins, implemented with Arrow compute kernels.

Covers what the reference examples and notebooks use (``examples/data_process.py``: ``hour``,
``quarter``, ``month``, ``year``, ``dayofweek``, ``dayofmonth``, ``weekofyear``, ``col``,
``lit``, ``udf``, ``abs``; DLRM notebook: ``log``, ``rand``, ``row_number``, ``desc``,
``monotonically_increasing_id``, ``array``/``posexplode``, ``count``) plus the common
aggregates and math/string helpers.
"""
import functools
import math

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from raydp_amd.spark.column import (AggExpr, CaseWhen, Column, ColRef, Func, Lit, SortOrder,
                                    WindowExpr, _to_double, _to_expr, as_array)
from raydp_amd.spark.column import to_timestamp as _to_ts
from raydp_amd.spark.udf import pandas_udf, udf  # noqa: F401  (re-exported)


def col(name: str) -> Column:
    return Column(ColRef(name))


column = col


def lit(value) -> Column:
    if isinstance(value, Column):
        return value
    return Column(Lit(value))


def expr(s: str) -> Column:
    """Parse a Spark SQL expression string (raydp_amd.spark.sqlexpr)."""
    s = s.strip()
    if s.replace("_", "").isalnum():
        return col(s)
    from raydp_amd.spark.sqlexpr import parse
    return parse(s)


def _fn(name, cols, impl, display=None, native=None):
    e = Func(name, [_to_expr(c, name_is_col=True) for c in cols], impl, display)
    e.native = native  # opcode tag for the fused expression VM (spark/exprc.py), None = host only
    return Column(e)


def _unary_impl(f, a, b):
    return f(a[0])


def _unary(name, f, native=None):
    # module-level impl bound with partial: pickles by reference when ``f`` does (pc.abs, ...)
    def builder(c):
        return _fn(name, [c], functools.partial(_unary_impl, f), native=native)
    builder.__name__ = name
    return builder


# ---------------------------------------------------------------------------- math ---------
abs = _unary("abs", pc.abs, native=("abs",))  # noqa: A001 - Spark name
sqrt = _unary("SQRT", lambda v: pc.sqrt(_to_double(v)), native=("sqrt",))
exp = _unary("EXP", lambda v: pc.exp(_to_double(v)))
floor = _unary("FLOOR", lambda v: pc.cast(pc.floor(_to_double(v)), pa.int64()))
ceil = _unary("CEIL", lambda v: pc.cast(pc.ceil(_to_double(v)), pa.int64()))
sin = _unary("SIN", lambda v: pc.sin(_to_double(v)))
cos = _unary("COS", lambda v: pc.cos(_to_double(v)))
tan = _unary("TAN", lambda v: pc.tan(_to_double(v)))
signum = _unary("SIGNUM", lambda v: pc.cast(pc.sign(_to_double(v)), pa.float64()))
log10 = _unary("LOG10", lambda v: _nan_to_null(pc.log10(_to_double(v))))
log2 = _unary("LOG2", lambda v: _nan_to_null(pc.log2(_to_double(v))))
log1p = _unary("LOG1P", lambda v: _nan_to_null(pc.log1p(_to_double(v))))
isnan = _unary("isnan", lambda v: pc.is_nan(_to_double(v)), native=("isnan",))
isnull = _unary("isnull", pc.is_null)


def _nan_to_null(v):
    # Spark's log of a non-positive number is null, Arrow's is nan/-inf
    return pc.if_else(pc.or_(pc.is_nan(v), pc.is_inf(v)), pa.scalar(None, v.type), v)


def log(arg1, arg2=None):
    if arg2 is None:
        return _fn("ln", [arg1], lambda a, b: _nan_to_null(pc.ln(_to_double(a[0]))))
    base = float(arg1)
    return _fn("LOG", [arg2], lambda a, b: _nan_to_null(
        pc.divide(pc.ln(_to_double(a[0])), math.log(base))), display=None)


def pow(c1, c2):  # noqa: A001
    return _fn("POWER", [c1, c2], lambda a, b: pc.power(_to_double(a[0]), _to_double(a[1])))


power = pow


def round(c, scale=0):  # noqa: A001
    # Spark rounds HALF_UP
    return _fn("round", [c], lambda a, b: pc.round(a[0], ndigits=scale, round_mode="half_up")
               if pa.types.is_floating(a[0].type) else a[0])


def bround(c, scale=0):
    return _fn("bround", [c], lambda a, b: pc.round(a[0], ndigits=scale, round_mode="half_to_even"))


def greatest(*cols):
    return _fn("greatest", cols, lambda a, b: pc.max_element_wise(*a, skip_nulls=True))


def least(*cols):
    return _fn("least", cols, lambda a, b: pc.min_element_wise(*a, skip_nulls=True))


def coalesce(*cols):
    return _fn("coalesce", cols, lambda a, b: pc.coalesce(*a))


def nanvl(c1, c2):
    return _fn("nanvl", [c1, c2], lambda a, b: pc.if_else(pc.is_nan(_to_double(a[0])), a[1], a[0]))


def when(condition, value) -> Column:
    return Column(CaseWhen([(_to_expr(condition), _to_expr(value))]))


def rand(seed=None):
    state = {"seed": seed}

    def impl(a, batch):
        rng = np.random.default_rng(state["seed"])
        return pa.array(rng.random(batch.num_rows))
    return Column(Func("rand", [], impl, display=f"rand({seed})"))


def randn(seed=None):
    def impl(a, batch):
        return pa.array(np.random.default_rng(seed).standard_normal(batch.num_rows))
    return Column(Func("randn", [], impl, display=f"randn({seed})"))


def monotonically_increasing_id():
    """Partition index in the upper 31 bits, row position in the lower 33 (Spark layout)."""
    def impl(a, batch):
        from raydp_amd.spark.plan import current_partition_index
        base = current_partition_index() << 33
        return pa.array(np.arange(batch.num_rows, dtype=np.int64) + base)
    return Column(Func("monotonically_increasing_id", [], impl))


def spark_partition_id():
    def impl(a, batch):
        from raydp_amd.spark.plan import current_partition_index
        return pa.repeat(pa.scalar(current_partition_index(), pa.int32()), batch.num_rows)
    return Column(Func("SPARK_PARTITION_ID", [], impl))


# ---------------------------------------------------------------------- datetime ---------
def _dt_impl(f, a, b):
    return pc.cast(f(_to_ts(a[0] if not isinstance(a[0], pa.Scalar) else as_array(a[0], b.num_rows))),
                   pa.int32())


def _spark_dayofweek(t):
    # Spark: 1 = Sunday ... 7 = Saturday
    return pc.add(pc.day_of_week(t, count_from_zero=False, week_start=7), 0)


def _dt(name, f):
    def builder(c):
        return _fn(name, [c], functools.partial(_dt_impl, f), native=("dt", name))
    builder.__name__ = name
    return builder


hour = _dt("hour", pc.hour)
minute = _dt("minute", pc.minute)
second = _dt("second", pc.second)
dayofmonth = _dt("dayofmonth", pc.day)
month = _dt("month", pc.month)
year = _dt("year", pc.year)
quarter = _dt("quarter", pc.quarter)
weekofyear = _dt("weekofyear", pc.iso_week)
dayofyear = _dt("dayofyear", pc.day_of_year)
# Spark: 1 = Sunday ... 7 = Saturday; Arrow (count_from_zero, week_start=Monday): Monday=0
dayofweek = _dt("dayofweek", _spark_dayofweek)


def to_date(c, format=None):  # noqa: A002
    return _fn("to_date", [c], lambda a, b: pc.cast(
        _to_ts(as_array(a[0], b.num_rows), _java_fmt(format)), pa.date32()))


def to_timestamp_(c, format=None):  # noqa: A002
    return _fn("to_timestamp", [c], lambda a, b: _to_ts(as_array(a[0], b.num_rows),
                                                              _java_fmt(format)))


to_timestamp = to_timestamp_


def unix_timestamp(c=None, format=None):  # noqa: A002
    return _fn("unix_timestamp", [c], lambda a, b: pc.cast(pc.cast(
        _to_ts(as_array(a[0], b.num_rows), _java_fmt(format)), pa.timestamp("s")), pa.int64()))


def date_format(c, format):  # noqa: A002
    return _fn("date_format", [c], lambda a, b: pc.strftime(
        _to_ts(as_array(a[0], b.num_rows)), format=_java_fmt(format)))


def datediff(end, start):
    def impl(a, b):
        e = pc.cast(_to_ts(as_array(a[0], b.num_rows)), pa.date32())
        s = pc.cast(_to_ts(as_array(a[1], b.num_rows)), pa.date32())
        return pc.cast(pc.days_between(s, e), pa.int32())
    return _fn("datediff", [end, start], impl)


def _java_fmt(f):
    if f is None:
        return None
    rep = [("yyyy", "%Y"), ("MM", "%m"), ("dd", "%d"), ("HH", "%H"), ("mm", "%M"), ("ss", "%S")]
    for a, b in rep:
        f = f.replace(a, b)
    return f


# ------------------------------------------------------------------------- string ---------
lower = _unary("lower", pc.utf8_lower)
upper = _unary("upper", pc.utf8_upper)
trim = _unary("trim", pc.utf8_trim_whitespace)
ltrim = _unary("ltrim", pc.utf8_ltrim_whitespace)
rtrim = _unary("rtrim", pc.utf8_rtrim_whitespace)
length = _unary("length", lambda v: pc.cast(pc.utf8_length(v), pa.int32()))


def concat(*cols):
    return _fn("concat", cols, lambda a, b: pc.binary_join_element_wise(
        *[pc.cast(as_array(x, b.num_rows), pa.string()) for x in a], ""))


def concat_ws(sep, *cols):
    return _fn("concat_ws", cols, lambda a, b: pc.binary_join_element_wise(
        *[pc.cast(as_array(x, b.num_rows), pa.string()) for x in a], sep))


def substring(c, pos, length_):
    return Column(_to_expr(c, True)).substr(pos, length_) if not isinstance(c, Column) \
        else c.substr(pos, length_)


def regexp_replace(c, pattern, replacement):
    return _fn("regexp_replace", [c], lambda a, b: pc.replace_substring_regex(
        a[0], pattern=pattern, replacement=replacement))


def split(c, pattern, limit=-1):
    return _fn("split", [c], lambda a, b: pc.split_pattern_regex(
        a[0], pattern=pattern, max_splits=None if limit <= 0 else limit - 1))


# -------------------------------------------------------------------- collections ---------
def array(*cols):
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = cols[0]

    def impl(a, batch):
        n = batch.num_rows
        arrs = [as_array(x, n) for x in a]
        t = arrs[0].type
        arrs = [pc.cast(x, t) for x in arrs]
        k = len(arrs)
        values = pa.concat_arrays(arrs).take(
            pa.array((np.arange(n)[:, None] + np.arange(k)[None, :] * n).ravel()))
        return pa.ListArray.from_arrays(pa.array(np.arange(0, n * k + 1, k, dtype=np.int32)), values)
    return _fn("array", cols, impl)


def size(c):
    return _fn("size", [c], lambda a, b: pc.cast(pc.list_value_length(a[0]), pa.int32()))


def element_at(c, idx):
    return _fn("element_at", [c], lambda a, b: pc.list_element(a[0], idx - 1))


def explode(c):
    f = _fn("explode", [c], None)
    f._expr.fname = "__explode__"
    return f


def posexplode(c):
    f = _fn("posexplode", [c], None)
    f._expr.fname = "__posexplode__"
    return f


# ---------------------------------------------------------------------- ordering ---------
def asc(c):
    return Column(SortOrder(_to_expr(c, True), True))


def desc(c):
    return Column(SortOrder(_to_expr(c, True), False))


def asc_nulls_last(c):
    return Column(SortOrder(_to_expr(c, True), True, False))


def desc_nulls_first(c):
    return Column(SortOrder(_to_expr(c, True), False, True))


# -------------------------------------------------------------------- aggregates ---------
def _agg(fn, c, distinct=False):
    child = None if c is None else _to_expr(c, name_is_col=True)
    if isinstance(child, ColRef) and child.col_name == "*":
        child = None
    return Column(AggExpr(fn, child, distinct))


def count(c="*"):
    return _agg("count", c)


def countDistinct(c, *cols):
    return _agg("count", c, distinct=True)


count_distinct = countDistinct


def sum(c):  # noqa: A001
    return _agg("sum", c)


def avg(c):
    return _agg("avg", c)


mean = avg


def min(c):  # noqa: A001
    return _agg("min", c)


def max(c):  # noqa: A001
    return _agg("max", c)


def first(c, ignorenulls=False):
    return _agg("first", c)


def last(c, ignorenulls=False):
    return _agg("last", c)


def stddev(c):
    return _agg("stddev", c)


stddev_samp = stddev


def variance(c):
    return _agg("variance", c)


var_samp = variance


def collect_list(c):
    return _agg("collect_list", c)


def collect_set(c):
    return _agg("collect_set", c)


def approx_count_distinct(c, rsd=0.05):
    return _agg("count", c, distinct=True)


# ------------------------------------------------------------------------ window ---------
def row_number():
    return Column(WindowExpr("row_number", [], None))


def rank():
    return Column(WindowExpr("rank", [], None))


def dense_rank():
    return Column(WindowExpr("dense_rank", [], None))


def broadcast(df):
    return df
