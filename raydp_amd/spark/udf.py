"""Python UDFs: AST vectorizer with a verified per-row fallback.

Row UDFs sit on the measured ETL path of the reference workloads (``night``,
``late_night`` and ``manhattan`` in ``examples/data_process.py:35-56``). Spark runs them one
row at a time in a Python worker. Here each UDF is first *compiled*: its source AST is
rewritten into whole-column numpy code (chained comparisons → ``&``, ``and``/``or`` in a
condition → ``logical_and``/``logical_or``, ``if/else`` returns → ``np.where``, ``int()``
/``float()`` → ``astype``). The compiled form is accepted only after it reproduces the
per-row results exactly on a sample of the partition; otherwise, and whenever an input has
nulls, the UDF runs row by row with Spark's null semantics (``None`` in, ``None`` out).
"""
import ast
import builtins
import inspect
import math
import textwrap
from typing import Callable, List, Optional

import numpy as np
import pyarrow as pa

from raydp_amd.spark.types import DataType, parse_type_string

_VERIFY_ROWS = 64
_REVERIFY_ROWS = 8


def _argmin(a):
    return int(np.nanargmin(a)) if a.dtype.kind == "f" else int(np.argmin(a))


def _argmax(a):
    return int(np.nanargmax(a)) if a.dtype.kind == "f" else int(np.argmax(a))


class _Unsupported(Exception):
    pass


_NP_MATH = {
    "sqrt": np.sqrt, "exp": np.exp, "log": np.log, "log10": np.log10, "log2": np.log2,
    "sin": np.sin, "cos": np.cos, "tan": np.tan, "fabs": np.abs, "floor": np.floor,
    "ceil": np.ceil, "pow": np.power, "atan2": np.arctan2, "asin": np.arcsin,
    "acos": np.arccos, "atan": np.arctan, "hypot": np.hypot, "radians": np.radians,
    "degrees": np.degrees,
}


class _Vectorizer:
    """Compiles a restricted Python function body into numpy array code."""

    def __init__(self, fn: Callable):
        self.fn = fn
        src = textwrap.dedent(inspect.getsource(fn))
        tree = ast.parse(src)
        fdef = tree.body[0]
        if not isinstance(fdef, (ast.FunctionDef,)):
            raise _Unsupported("not a def")
        self.fdef = fdef
        self.arg_names = [a.arg for a in fdef.args.args]
        if fdef.args.vararg or fdef.args.kwarg or fdef.args.kwonlyargs:
            raise _Unsupported("varargs")
        self.globals = dict(fn.__globals__)
        if fn.__closure__:
            for name, cell in zip(fn.__code__.co_freevars, fn.__closure__):
                self.globals[name] = cell.cell_contents

    # -- public -----------------------------------------------------------------------------
    def __call__(self, arrays: List[np.ndarray], n: int):
        env = dict(zip(self.arg_names, arrays))
        out = self._block(self.fdef.body, env)
        if out is None:
            raise _Unsupported("no return")
        return out

    # -- statements -------------------------------------------------------------------------
    def _block(self, stmts, env):
        for i, st in enumerate(stmts):
            if isinstance(st, ast.Return):
                return self._expr(st.value, env) if st.value is not None else None
            if isinstance(st, ast.Expr) and isinstance(st.value, ast.Constant):
                continue  # docstring
            if isinstance(st, ast.Assign) and len(st.targets) == 1 and isinstance(st.targets[0], ast.Name):
                env[st.targets[0].id] = self._expr(st.value, env)
                continue
            if isinstance(st, ast.If):
                cond = self._cond(st.test, env)
                then_v = self._block(st.body, dict(env))
                rest = st.orelse if st.orelse else stmts[i + 1:]
                else_v = self._block(rest, dict(env))
                if then_v is None or else_v is None:
                    raise _Unsupported("branch without return")
                return np.where(cond, then_v, else_v)
            raise _Unsupported(type(st).__name__)
        return None

    # -- expressions ------------------------------------------------------------------------
    def _cond(self, node, env):
        if isinstance(node, ast.BoolOp):
            parts = [self._cond(v, env) for v in node.values]
            op = np.logical_and if isinstance(node.op, ast.And) else np.logical_or
            out = parts[0]
            for p in parts[1:]:
                out = op(out, p)
            return out
        if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.Not):
            return np.logical_not(self._cond(node.operand, env))
        v = self._expr(node, env)
        return np.asarray(v).astype(bool)

    def _expr(self, node, env):
        if isinstance(node, ast.Constant):
            if isinstance(node.value, (int, float, bool)) or node.value is None:
                return node.value
            raise _Unsupported("constant type")
        if isinstance(node, ast.Name):
            if node.id in env:
                return env[node.id]
            if node.id in self.globals:
                v = self.globals[node.id]
                if isinstance(v, (int, float, bool, np.number)):
                    return v
            raise _Unsupported(f"name {node.id}")
        if isinstance(node, ast.Tuple):
            return tuple(self._expr(e, env) for e in node.elts)
        if isinstance(node, ast.Subscript):
            base = self._expr(node.value, env)
            if isinstance(base, tuple):
                idx = self._expr(node.slice, env)
                if isinstance(idx, int):
                    return base[idx]
            raise _Unsupported("subscript")
        if isinstance(node, ast.BinOp):
            a, b = self._expr(node.left, env), self._expr(node.right, env)
            ops = {ast.Add: np.add, ast.Sub: np.subtract, ast.Mult: np.multiply,
                   ast.Div: np.true_divide, ast.FloorDiv: np.floor_divide, ast.Mod: np.mod,
                   ast.Pow: np.power}
            f = ops.get(type(node.op))
            if f is None:
                raise _Unsupported("binop")
            return f(a, b)
        if isinstance(node, ast.UnaryOp):
            v = self._expr(node.operand, env)
            if isinstance(node.op, ast.USub):
                return np.negative(v)
            if isinstance(node.op, ast.UAdd):
                return v
            if isinstance(node.op, ast.Not):
                return np.logical_not(v)
            raise _Unsupported("unary")
        if isinstance(node, ast.Compare):
            left = self._expr(node.left, env)
            out = None
            cmp = {ast.Lt: np.less, ast.LtE: np.less_equal, ast.Gt: np.greater,
                   ast.GtE: np.greater_equal, ast.Eq: np.equal, ast.NotEq: np.not_equal}
            for op, rnode in zip(node.ops, node.comparators):
                f = cmp.get(type(op))
                if f is None:
                    raise _Unsupported("compare op")
                right = self._expr(rnode, env)
                r = f(left, right)
                out = r if out is None else np.logical_and(out, r)
                left = right
            return out
        if isinstance(node, ast.BoolOp):
            # value semantics of `and`/`or` only match when operands are booleans
            return self._cond(node, env)
        if isinstance(node, ast.IfExp):
            return np.where(self._cond(node.test, env), self._expr(node.body, env),
                            self._expr(node.orelse, env))
        if isinstance(node, ast.Call):
            if node.keywords:
                raise _Unsupported("kwargs")
            fn = self._resolve_callable(node.func)
            args = [self._expr(a, env) for a in node.args]
            return fn(*args)
        raise _Unsupported(type(node).__name__)

    def _resolve_callable(self, fnode):
        if isinstance(fnode, ast.Name):
            name = fnode.id
            obj = self.globals.get(name, getattr(builtins, name, None))
            if obj is builtins.int:
                return _py_int
            if obj is builtins.float:
                return lambda x: np.asarray(x, dtype=np.float64)
            if obj is builtins.abs:
                return np.abs
            if obj is builtins.bool:
                return lambda x: np.asarray(x).astype(bool)
            if obj is builtins.min:      # Python's fold: keep the running value unless y < it
                return lambda *a: _reduce(lambda x, y: np.where(np.less(y, x), y, x), a)
            if obj is builtins.max:
                return lambda *a: _reduce(lambda x, y: np.where(np.greater(y, x), y, x), a)
            if obj is builtins.round:
                return lambda x, d=0: np.round(x, d)
            if isinstance(obj, np.ufunc):
                return obj
            if obj is not None and getattr(obj, "__module__", None) == "math":
                f = _NP_MATH.get(obj.__name__)
                if f is not None:
                    return f
            raise _Unsupported(f"call {name}")
        if isinstance(fnode, ast.Attribute) and isinstance(fnode.value, ast.Name):
            mod = self.globals.get(fnode.value.id)
            if mod is np:
                f = getattr(np, fnode.attr, None)
                if isinstance(f, np.ufunc) or fnode.attr in ("where", "clip", "round", "abs"):
                    return f
            if mod is math:
                f = _NP_MATH.get(fnode.attr)
                if f is not None:
                    return f
        raise _Unsupported("callable")


def _py_int(x):
    x = np.asarray(x)
    return (np.trunc(x) if x.dtype.kind == "f" else x).astype(np.int64)


def _reduce(f, args):
    out = args[0]
    for a in args[1:]:
        out = f(out, a)
    return out


def _np_dtype_for(rt: DataType):
    t = rt.to_arrow()
    if pa.types.is_integer(t) or pa.types.is_floating(t) or pa.types.is_boolean(t):
        return t.to_pandas_dtype()
    return None


class UserDefinedFunction:
    """A Spark-style Python row UDF (``@udf("int")``)."""

    def __init__(self, func: Callable, returnType="string", name: Optional[str] = None):
        self.func = func
        self.returnType = parse_type_string(returnType)
        self.__name__ = name or getattr(func, "__name__", "udf")
        self._vec = None
        self._vec_state = "untried"  # untried | ok | failed

    def __getstate__(self):
        # per-process caches stay behind: the vectoriser holds the function's module globals,
        # the structural key (spark/exprc.py) may hold process-local ids
        st = dict(self.__dict__)
        st.pop("_rx_key", None)
        st["_vec"] = None
        return st

    def __call__(self, *cols):
        from raydp_amd.spark.column import Column, UDFExpr, _to_expr
        return Column(UDFExpr(self, [_to_expr(c, name_is_col=True) for c in cols]))

    # -- evaluation -------------------------------------------------------------------------
    def evaluate(self, arrays: List[pa.Array], n: int) -> pa.Array:
        out_type = self.returnType.to_arrow()
        arrays = [a.combine_chunks() if isinstance(a, pa.ChunkedArray) else a for a in arrays]
        if n == 0:
            return pa.array([], type=out_type)
        has_nulls = any(a.null_count for a in arrays)
        np_dtype = _np_dtype_for(self.returnType)
        if not has_nulls and np_dtype is not None and self._vec_state != "failed" and \
                all(_numeric(a) for a in arrays):
            res = self._try_vectorized(arrays, n, np_dtype)
            if res is not None:
                return pa.array(res, type=out_type)
        return self._row_by_row(arrays, n, out_type)

    def _try_vectorized(self, arrays, n, np_dtype):
        try:
            if self._vec is None:
                self._vec = _Vectorizer(self.func)
            nps = [a.to_numpy(zero_copy_only=False) for a in arrays]
            # numpy returns inf/nan (or a warning) where Python raises -- a zero divisor, 0/0,
            # an invalid power: such a batch runs per row, with Python's semantics
            with np.errstate(divide="raise", invalid="raise", over="raise"):
                res = self._vec(nps, n)
            res = np.broadcast_to(np.asarray(res), (n,)).astype(np_dtype)
        except FloatingPointError:
            return None                    # this batch only: the UDF stays vectorised
        except Exception:  # noqa: BLE001 - any failure means "not vectorizable"
            self._vec_state = "failed"
            return None
        # verify against the exact per-row semantics on EVERY batch: the first one on a 64-row
        # sample, later ones on 8 spread rows, always adding each argument's minimum and maximum
        # row, so a branch that a new value range takes is checked when that range first shows up
        first = self._vec_state == "untried" or n <= _VERIFY_ROWS
        idx = np.linspace(0, n - 1, min(n, _VERIFY_ROWS if first else _REVERIFY_ROWS)).astype(np.int64)
        ext = [f(a) for a in nps if a.size and a.dtype.kind in "biuf" and not np.isnan(a.astype(np.float64)).all()
               for f in (_argmin, _argmax)]
        if ext:
            idx = np.unique(np.concatenate([idx, np.asarray(ext, dtype=np.int64)]))
        rows = [[a[i].as_py() for a in arrays] for i in idx]
        try:
            expect = np.array([self.func(*r) for r in rows]).astype(np_dtype)
        except Exception:  # noqa: BLE001
            self._vec_state = "failed"
            return None
        got = res[idx]
        if np.dtype(np_dtype).kind == "f":
            ok = np.allclose(got, expect, rtol=1e-6, atol=1e-9, equal_nan=True)
        else:
            ok = np.array_equal(got, expect)
        if not ok:
            self._vec_state = "failed"
            return None
        self._vec_state = "ok"
        return res

    def _row_by_row(self, arrays, n, out_type):
        cols = [a.to_pylist() for a in arrays]
        f = self.func
        out = [f(*row) for row in zip(*cols)] if cols else [f() for _ in range(n)]
        if pa.types.is_floating(out_type):
            # a Python int returned for a floating column converts like float(x) (Arrow refuses
            # ints beyond 2**53 that the vectorised paths cast without complaint)
            out = [float(v) if isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)) else v
                   for v in out]
        return pa.array(out, type=out_type, from_pandas=False)

    @property
    def vectorized(self) -> bool:
        return self._vec_state == "ok"


def _numeric(a: pa.Array) -> bool:
    t = a.type
    return pa.types.is_integer(t) or pa.types.is_floating(t) or pa.types.is_boolean(t)


def udf(f=None, returnType="string"):
    """``udf(func, "int")``, ``@udf("int")``, ``@udf(returnType=IntegerType())`` or ``@udf``."""
    if f is None:
        return lambda fn: UserDefinedFunction(fn, returnType)
    if isinstance(f, (str, DataType)):
        rt = f
        return lambda fn: UserDefinedFunction(fn, rt)
    return UserDefinedFunction(f, returnType)


def pandas_udf(f=None, returnType=None, functionType=None):
    """Vectorised UDF over pandas Series (Series-to-Series form)."""
    def wrap(fn, rt):
        u = UserDefinedFunction(fn, rt)

        def evaluate(arrays, n):
            import pandas as pd
            series = [a.to_pandas() if hasattr(a, "to_pandas") else pd.Series(a) for a in arrays]
            res = fn(*series)
            return pa.array(res, type=u.returnType.to_arrow(), from_pandas=True)
        u.evaluate = evaluate
        return u
    if f is None or isinstance(f, (str, DataType)):
        rt = returnType if f is None else f
        return lambda fn: wrap(fn, rt)
    return wrap(f, returnType)
