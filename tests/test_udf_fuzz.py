"""Fuzz of the Python-UDF -> expression-VM translator (raydp_amd/spark/exprc.py).

Random UDF bodies from the supported AST subset (arithmetic incl. / // % **, unary minus,
abs / min / max / float / int / math.sqrt, comparisons, chained comparisons, boolean
operators, conditional expressions, if/else statements with assignments) run over adversarial
columns (zeros, negatives, NaN, +-inf, int64 extremes) through the fused VM path, and the
result of every partition must equal the exact per-row Python path (RAYDP_FUSED_ETL=0): the
same values, or the same failure. The VM itself is fuzzed natively by
csrc/tests/expr_vm_fuzz.cc; this checks the translation and its guards (zero divisors,
fractional powers of negatives, int() of NaN, int64 overflow) and verification."""
import importlib.util
import math
import os
import random
import sys

import numpy as np
import pyarrow as pa
import pytest

from raydp_amd.spark import exprc
from raydp_amd.spark.functions import udf

N_UDFS = int(os.environ.get("RAYDP_UDF_FUZZ_N", "120"))


class _Gen:
    def __init__(self, rng: random.Random):
        self.r = rng

    def const(self):
        return self.r.choice(["0", "1", "2", "-3", "7", "0.5", "2.5", "-1.25", "1e-3", "3.0"])

    def atom(self, names):
        return self.r.choice(names) if self.r.random() < 0.7 else self.const()

    def expr(self, names, d=0):
        r = self.r.random()
        if d >= 3 or r < 0.25:
            return self.atom(names)
        if r < 0.62:
            op = self.r.choice(["+", "-", "*", "/", "//", "%", "+", "-", "*"])
            return f"({self.expr(names, d + 1)} {op} {self.expr(names, d + 1)})"
        if r < 0.68:
            return f"({self.expr(names, d + 1)} ** {self.r.choice(['2', '3', '0.5', '-1', '2.0'])})"
        if r < 0.73:
            return f"(-{self.expr(names, d + 1)})"
        if r < 0.80:
            f = self.r.choice(["abs", "float", "math.fabs", "np.abs", "math.sqrt", "np.sqrt", "int"])
            return f"{f}({self.expr(names, d + 1)})"
        if r < 0.87:
            f = self.r.choice(["min", "max", "np.minimum", "np.maximum"])
            return f"{f}({self.expr(names, d + 1)}, {self.expr(names, d + 1)})"
        return f"({self.expr(names, d + 1)} if {self.cond(names, d + 1)} else {self.expr(names, d + 1)})"

    def cond(self, names, d=0):
        r = self.r.random()
        cmp = self.r.choice(["<", "<=", ">", ">=", "==", "!="])
        if r < 0.6 or d >= 3:
            return f"{self.expr(names, d + 1)} {cmp} {self.expr(names, d + 1)}"
        if r < 0.75:
            return f"{self.atom(names)} < {self.atom(names)} <= {self.atom(names)}"
        if r < 0.9:
            j = self.r.choice(["and", "or"])
            return f"({self.cond(names, d + 1)}) {j} ({self.cond(names, d + 1)})"
        return f"not ({self.cond(names, d + 1)})"

    def body(self, names):
        lines = []
        env = list(names)
        for k in range(self.r.randint(0, 2)):
            v = f"t{k}"
            lines.append(f"    {v} = {self.expr(env)}")
            env.append(v)
        if self.r.random() < 0.4:
            lines.append(f"    if {self.cond(env)}:")
            lines.append(f"        return {self.expr(env)}")
            if self.r.random() < 0.5:
                lines.append("    else:")
                lines.append(f"        return {self.expr(env)}")
            else:
                lines.append(f"    return {self.expr(env)}")
        else:
            lines.append(f"    return {self.expr(env)}")
        return lines


def _module(tmp_path, n, seed):
    rng = random.Random(seed)
    g = _Gen(rng)
    src = ["import math", "import numpy as np", ""]
    for i in range(n):
        src.append(f"def f{i}(a, b, c):")
        src += g.body(["a", "b", "c"])
        src.append("")
    path = tmp_path / f"udf_fuzz_{seed}.py"
    path.write_text("\n".join(src))
    spec = importlib.util.spec_from_file_location(f"udf_fuzz_{seed}", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return mod


def _partitions(seed):
    rng = np.random.default_rng(seed)
    out = []
    for p in range(3):
        n = 64
        a = rng.normal(scale=[1.0, 50.0, 1e6][p], size=n)
        a[rng.random(n) < 0.08] = 0.0
        if p == 1:
            a[rng.integers(0, n, 3)] = [np.nan, np.inf, -np.inf]
        b = np.round(rng.normal(scale=3.0, size=n))           # many small integers incl. 0
        c = rng.integers(-5, 6, n).astype(np.int64)
        if p == 2:
            c[rng.integers(0, n, 2)] = [2 ** 62, -2 ** 62]      # int64 edges: Python ints do not wrap
        out.append(pa.table({"a": pa.array(a), "b": pa.array(b), "c": pa.array(c)}))
    return out


def _run(spark, t, u, fused, monkeypatch):
    monkeypatch.setenv("RAYDP_FUSED_ETL", "1" if fused else "0")
    df = spark.createDataFrame(t).withColumn("r", u("a", "b", "c"))
    try:
        parts = [df._plan.compute(i) for i in range(df._plan.num_partitions())]
        return "ok", pa.concat_tables(parts).column("r").combine_chunks()
    except Exception as e:  # noqa: BLE001 - Python raised on some row: both paths must
        return "error", type(e).__name__


def _same_values(x: pa.Array, y: pa.Array) -> bool:
    if x.type != y.type or not x.is_null().equals(y.is_null()):
        return False
    a = x.fill_null(0).to_numpy(zero_copy_only=False).astype(np.float64)
    b = y.fill_null(0).to_numpy(zero_copy_only=False).astype(np.float64)
    with np.errstate(invalid="ignore"):
        close = (a == b) | (np.isnan(a) & np.isnan(b)) | (np.abs(a - b) <= 1e-12 * np.maximum(np.abs(a), np.abs(b)))
    return bool(close.all())


@pytest.fixture
def spark(spark_session):
    spark_session.conf.set("spark.sql.session.timeZone", "UTC")
    return spark_session


def _oracle(fn, t):
    """Pure per-row Python (Spark's semantics for a row UDF): values, or the failure."""
    cols = [t.column(c).to_pylist() for c in ("a", "b", "c")]
    try:
        out = [fn(*row) for row in zip(*cols)]
        out = [float(v) if isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)) else v
               for v in out]      # a double UDF returning an int
        return "ok", pa.array(out, type=pa.float64(), from_pandas=False)
    except Exception as e:  # noqa: BLE001
        return "error", type(e).__name__


@pytest.mark.parametrize("seed", [1, 2])
def test_udf_translator_fuzz_matches_per_row_python(spark, monkeypatch, tmp_path, seed):
    """Both vectorised UDF paths -- the expression-VM inlining (RAYDP_FUSED_ETL=1) and the numpy
    vectoriser of the per-operator path (=0) -- against pure per-row Python."""
    mod = _module(tmp_path, N_UDFS // 2, seed)
    parts = _partitions(seed)
    compiled = 0
    mismatches = []
    for i in range(N_UDFS // 2):
        fn = getattr(mod, f"f{i}")
        before = exprc.STATS["fused_partitions"]
        for t in parts:
            want = _oracle(fn, t)
            for fused in (True, False):
                got = _run(spark, t, udf(fn, "double"), fused, monkeypatch)
                if want[0] != got[0] or (want[0] == "ok" and not _same_values(want[1], got[1])):
                    mismatches.append((f"f{i}", "vm" if fused else "numpy", want, got))
        compiled += exprc.STATS["fused_partitions"] > before
    import inspect
    assert not mismatches, "\n".join(
        f"{m[0]} [{m[1]}]: {inspect.getsource(getattr(mod, m[0]))} want={m[2][0]} got={m[3][0]}"
        for m in mismatches[:5])
    # the fuzz must actually exercise the translator, not only the fallback
    assert compiled >= N_UDFS // 8, compiled


_ = math
