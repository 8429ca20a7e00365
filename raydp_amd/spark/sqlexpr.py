"""Spark SQL expression strings -> Column (``F.expr``, ``df.filter("...")``,
``df.selectExpr``, ``df.where``).

A small Pratt parser for the expression subset data-prep code uses (the reference's DLRM
preprocessing filters with strings like ``'data is not null'`` and ``'column_id == 3'``):
column references (plain or back-quoted), numeric / string / boolean / NULL literals,
``+ - * / %``, comparisons (``= == != <> < <= > >=``), ``AND OR NOT``, ``IS [NOT] NULL``,
``[NOT] IN (...)``, ``[NOT] BETWEEN a AND b``, ``[NOT] LIKE``, ``CASE WHEN ... THEN ... ELSE ...
END``, ``CAST(x AS type)``, function calls resolved against ``raydp_amd.spark.functions``
(``count(*)`` included) and ``expr AS alias``.
"""
import re
from typing import List, Optional, Tuple

_TOKEN = re.compile(r"""
    \s*(?:
      (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?[LlDd]?)
     |(?P<str>'(?:[^'\\]|\\.|'')*'|"(?:[^"\\]|\\.)*")
     |(?P<bq>`[^`]+`)
     |(?P<op>==|!=|<>|<=|>=|\|\||[-+*/%(),<>=.])
     |(?P<id>[A-Za-z_][A-Za-z0-9_]*)
    )""", re.VERBOSE)

_KEYWORDS = {"and", "or", "not", "is", "null", "in", "between", "like", "rlike", "case", "when", "then", "else",
             "end", "cast", "as", "true", "false", "distinct"}


def _tokenize(s: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    s = s.rstrip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise ValueError(f"cannot parse SQL expression near {s[pos:pos + 20]!r}")
        pos = m.end()
        kind = m.lastgroup
        val = m.group(kind)
        if kind == "id" and val.lower() in _KEYWORDS:
            kind, val = "kw", val.lower()
        out.append((kind, val))
    out.append(("eof", ""))
    return out


class _Parser:
    # binding powers
    _BP = {"or": 1, "and": 2, "not": 3, "cmp": 4, "||": 5, "+": 6, "-": 6, "*": 7, "/": 7, "%": 7}

    def __init__(self, s: str):
        self.toks = _tokenize(s)
        self.i = 0

    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, kind, val=None):
        t = self.next()
        if t[0] != kind or (val is not None and t[1] != val):
            raise ValueError(f"expected {val or kind}, got {t[1]!r}")
        return t

    def accept(self, kind, val=None) -> bool:
        t = self.peek()
        if t[0] == kind and (val is None or t[1] == val):
            self.i += 1
            return True
        return False

    # ------------------------------------------------------------------------------
    def parse_top(self):
        from raydp_amd.spark import functions as F
        e = self.expr(0)
        if self.accept("kw", "as"):
            name = self.next()[1].strip("`")
            e = e.alias(name)
        elif self.peek()[0] in ("id", "bq"):
            e = e.alias(self.next()[1].strip("`"))
        if self.peek()[0] != "eof":
            raise ValueError(f"unexpected {self.peek()[1]!r}")
        _ = F
        return e

    def expr(self, rbp):
        left = self.prefix()
        while True:
            t = self.peek()
            op = self._infix_op(t)
            if op is None:
                break
            bp = self._BP["cmp"] if op in ("cmp", "is", "in", "between", "like", "notin", "notbetween",
                                           "notlike") else self._BP[op]
            if bp <= rbp:
                break
            left = self.infix(op, left, bp)
        return left

    def _infix_op(self, t):
        kind, v = t
        if kind == "op" and v in ("==", "=", "!=", "<>", "<", "<=", ">", ">="):
            return "cmp"
        if kind == "op" and v in ("+", "-", "*", "/", "%", "||"):
            return v
        if kind == "kw" and v in ("and", "or", "is", "in", "between", "like", "rlike"):
            return {"rlike": "like"}.get(v, v)
        if kind == "kw" and v == "not":
            nxt = self.peek(1)
            if nxt[0] == "kw" and nxt[1] in ("in", "between", "like", "rlike"):
                return "not" + {"rlike": "like"}.get(nxt[1], nxt[1])
        return None

    def infix(self, op, left, bp):
        from raydp_amd.spark import functions as F
        t = self.next()
        if op == "cmp":
            right = self.expr(bp)
            v = t[1]
            return {"==": left == right, "=": left == right, "!=": left != right, "<>": left != right,
                    "<": left < right, "<=": left <= right, ">": left > right, ">=": left >= right}[v]
        if op in ("+", "-", "*", "/", "%"):
            right = self.expr(bp)
            return {"+": left + right, "-": left - right, "*": left * right, "/": left / right,
                    "%": left % right}[op]
        if op == "||":
            return F.concat(left, self.expr(bp))
        if op == "and":
            return left & self.expr(bp)
        if op == "or":
            return left | self.expr(bp)
        if op == "is":
            neg = self.accept("kw", "not")
            self.expect("kw", "null")
            return left.isNotNull() if neg else left.isNull()
        if op.startswith("not"):
            self.next()   # the in / between / like keyword after NOT
            return ~self._rest(op[3:], left, bp)
        return self._rest(op, left, bp)

    def _rest(self, op, left, bp):
        if op == "in":
            self.expect("op", "(")
            vals = []
            if not self.accept("op", ")"):
                while True:
                    vals.append(self._literal_value(self.expr(0)))
                    if self.accept("op", ")"):
                        break
                    self.expect("op", ",")
            return left.isin(vals)
        if op == "between":
            lo = self.expr(self._BP["cmp"])
            self.expect("kw", "and")
            hi = self.expr(self._BP["cmp"])
            return (left >= lo) & (left <= hi)
        if op == "like":
            pat = self.expr(bp)
            return left.like(self._literal_value(pat))
        raise ValueError(op)

    @staticmethod
    def _literal_value(c):
        from raydp_amd.spark.column import Lit
        e = c._expr
        if isinstance(e, Lit):
            return e.value
        raise ValueError("IN / LIKE arguments must be literals")

    def prefix(self):
        from raydp_amd.spark import functions as F
        kind, v = self.next()
        if kind == "num":
            s = v.rstrip("LlDd")
            val = float(s) if any(ch in s for ch in ".eE") or v[-1:] in "Dd" else int(s)
            return F.lit(val)
        if kind == "str":
            q = v[0]
            body = v[1:-1].replace("''", "'") if q == "'" else v[1:-1]
            return F.lit(bytes(body, "utf-8").decode("unicode_escape") if "\\" in body else body)
        if kind == "bq":
            return F.col(v.strip("`"))
        if kind == "op" and v == "(":
            e = self.expr(0)
            self.expect("op", ")")
            return e
        if kind == "op" and v == "-":
            return -self.expr(self._BP["*"])
        if kind == "op" and v == "+":
            return self.expr(self._BP["*"])
        if kind == "op" and v == "*":
            return F.lit(1)
        if kind == "kw":
            if v == "not":
                return ~self.expr(self._BP["not"])
            if v == "null":
                return F.lit(None)
            if v in ("true", "false"):
                return F.lit(v == "true")
            if v == "case":
                return self._case()
            if v == "cast":
                self.expect("op", "(")
                e = self.expr(0)
                self.expect("kw", "as")
                ty = self._type_name()
                self.expect("op", ")")
                return e.cast(ty)
            raise ValueError(f"unexpected keyword {v!r}")
        if kind == "id":
            if self.accept("op", "("):
                return self._call(v)
            parts = [v]
            while self.peek() == ("op", "."):
                self.next()
                parts.append(self.next()[1].strip("`"))
            c = F.col(parts[-1])
            if len(parts) > 1:
                # ``t.c``: the column is ``c``; the qualifier names the relation it comes from
                # (JOIN ... ON resolves each side by it)
                c._expr.qualifier = parts[-2]
            return c
        raise ValueError(f"unexpected token {v!r}")

    def _type_name(self):
        parts = [self.next()[1]]
        if self.accept("op", "("):
            args = []
            while not self.accept("op", ")"):
                args.append(self.next()[1])
            parts.append("(" + "".join(args) + ")")
        return "".join(parts)

    def _case(self):
        from raydp_amd.spark import functions as F
        subject = None
        if not (self.peek() == ("kw", "when")):
            subject = self.expr(0)
        out: Optional[object] = None
        while self.accept("kw", "when"):
            cond = self.expr(0)
            if subject is not None:
                cond = subject == cond
            self.expect("kw", "then")
            val = self.expr(0)
            out = F.when(cond, val) if out is None else out.when(cond, val)
        if self.accept("kw", "else"):
            out = out.otherwise(self.expr(0))
        self.expect("kw", "end")
        return out

    def _call(self, name):
        from raydp_amd.spark import functions as F
        low = name.lower()
        distinct = self.accept("kw", "distinct")
        args = []
        if self.accept("op", "*"):
            args.append("*")
            self.expect("op", ")")
        elif not self.accept("op", ")"):
            while True:
                args.append(self.expr(0))
                if self.accept("op", ")"):
                    break
                self.expect("op", ",")
        if low == "count":
            if distinct:
                return F.countDistinct(*args)
            return F.count(F.lit(1) if args == ["*"] else args[0])
        alias = {"ln": "log", "power": "pow", "ifnull": "coalesce", "nvl": "coalesce", "mean": "avg",
                 "std": "stddev", "substr": "substring", "lcase": "lower", "ucase": "upper"}.get(low, low)
        fn = getattr(F, alias, None) or getattr(F, name, None)
        if fn is None:
            raise ValueError(f"unknown SQL function {name}")
        # SQL passes every argument as an expression; the Python API takes some as plain
        # values (round's scale, substring's positions, a date format, ...)
        scalar_at = _SCALAR_ARGS.get(alias)
        if scalar_at is not None:
            args = [self._literal_value(a) if (i in scalar_at or (-1 in scalar_at and i > 0))
                    and hasattr(a, "_expr") else a for i, a in enumerate(args)]
        return fn(*args)


# argument positions the Python function API takes as values, not Columns (-1: every argument
# after the first)
_SCALAR_ARGS = {
    "round": {-1}, "bround": {-1}, "substring": {-1}, "left": {-1}, "right": {-1}, "lpad": {1, 2},
    "rpad": {1, 2}, "repeat": {-1}, "split": {-1}, "regexp_replace": {-1}, "regexp_extract": {-1},
    "date_format": {-1}, "date_add": {-1}, "date_sub": {-1}, "add_months": {-1}, "format_number": {-1},
    "locate": {0, 2}, "instr": {-1}, "translate": {-1}, "trunc": {-1}, "date_trunc": {0},
    "from_unixtime": {-1}, "to_date": {-1}, "to_timestamp": {-1}, "unix_timestamp": {-1}, "sha2": {-1},
    "conv": {-1}, "concat_ws": {0}, "percentile_approx": {-1}, "ntile": {0},
}


def parse(s: str):
    """Parse one SQL expression (optionally ``... AS alias``) into a Column."""
    return _Parser(s).parse_top()
