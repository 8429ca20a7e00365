"""Spark SQL statements over the engine's catalog (``SparkSession.sql``).

Reference: RayDP hands ``spark.sql(...)`` to Spark, and its docs show Hive tables queried from
Spark-on-Ray (``doc/spark_on_ray.md:187-201``: ``enableHiveSupport`` + ``spark.sql("select *
from db.xxx")``; ``python/raydp/spark/ray_cluster.py:198``). Here statements are parsed into
the engine's own DataFrame plans (so a query runs exactly like the equivalent DataFrame code:
fused narrow operators, shuffles, broadcast joins):

* queries -- ``[WITH name AS (query), ...] SELECT [DISTINCT] items FROM source [JOIN ...]
  [WHERE ...] [GROUP BY ...] [HAVING ...] [UNION [ALL] ...] [ORDER BY ...] [LIMIT n]``; a source
  is a table / view name (``db.name`` too) or a parenthesised subquery, optionally aliased;
  joins are ``[INNER | LEFT [OUTER] | RIGHT [OUTER] | FULL [OUTER] | LEFT SEMI | LEFT ANTI |
  CROSS] JOIN ... ON <equalities> [AND <residual filter>] | USING (cols)``; select items are
  expressions of ``raydp_amd.spark.sqlexpr`` (``*``, ``t.*``, aliases, aggregates, CASE, CAST,
  functions); HAVING and ORDER BY may use aggregates that are not selected;
* DDL / catalog -- ``CREATE [OR REPLACE] [TEMP[ORARY]] VIEW v AS query``, ``CREATE TABLE
  [IF NOT EXISTS] t [USING parquet] AS query`` (persisted to the warehouse directory,
  ``spark.sql.warehouse.dir``), ``INSERT INTO|OVERWRITE [TABLE] t query``, ``CREATE
  DATABASE|SCHEMA [IF NOT EXISTS] d``, ``USE d``, ``DROP TABLE|VIEW [IF EXISTS] t``, ``DROP
  DATABASE [IF EXISTS] d``, ``SHOW TABLES [IN d]``, ``SHOW DATABASES``, ``DESCRIBE [TABLE] t``.
"""
import os
import re
import shutil
from typing import List, Optional, Tuple

from raydp_amd.spark.sqlexpr import _TOKEN

_CLAUSE = {"select", "from", "where", "group", "having", "order", "limit", "join", "inner", "left", "right",
           "full", "cross", "on", "using", "union", "semi", "anti", "outer", "as", "with", "distinct", "by",
           "all", "asc", "desc", "nulls", "first", "last", "intersect", "except"}


class SqlError(ValueError):
    pass


def _tokens(s: str) -> List[Tuple[str, str, int, int]]:
    """(kind, value, start, end) of every token; kind in num/str/bq/op/id."""
    out, pos = [], 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise SqlError(f"cannot parse SQL near {s[pos:pos + 30]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind), m.start(kind), m.end(kind)))
        pos = m.end()
    return out


class _Stmt:
    def __init__(self, session, text: str, ctes=None):
        self.session, self.text = session, text
        self.t = _tokens(text)
        self.i = 0
        self.ctes = dict(ctes or {})
        self.qualifiers = {}

    # ------------------------------------------------------------------ token helpers
    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else ("eof", "", len(self.text), len(self.text))

    def kw(self, k=0) -> str:
        tok = self.peek(k)
        return tok[1].lower() if tok[0] == "id" else ""

    def accept_kw(self, *words) -> bool:
        for j, w in enumerate(words):
            if self.kw(j) != w:
                return False
        self.i += len(words)
        return True

    def expect_kw(self, *words):
        if not self.accept_kw(*words):
            raise SqlError(f"expected {' '.join(words).upper()} near {self.rest()[:40]!r}")

    def accept_op(self, v) -> bool:
        tok = self.peek()
        if tok[0] == "op" and tok[1] == v:
            self.i += 1
            return True
        return False

    def expect_op(self, v):
        if not self.accept_op(v):
            raise SqlError(f"expected {v!r} near {self.rest()[:40]!r}")

    def rest(self) -> str:
        return self.text[self.peek()[2]:]

    def name(self) -> str:
        tok = self.peek()
        if tok[0] not in ("id", "bq"):
            raise SqlError(f"expected a name near {self.rest()[:40]!r}")
        self.i += 1
        parts = [tok[1].strip("`")]
        while self.peek()[0] == "op" and self.peek()[1] == "." and self.peek(1)[0] in ("id", "bq"):
            self.i += 1
            parts.append(self.peek()[1].strip("`"))
            self.i += 1
        return ".".join(parts)

    def span(self, stop_words, stop_ops=(",", ")")) -> str:
        """Source text of the expression starting here, up to a top-level clause keyword /
        comma / closing paren."""
        depth, start = 0, self.peek()[2]
        end = start
        while True:
            tok = self.peek()
            if tok[0] == "eof":
                break
            if tok[0] == "op" and tok[1] == "(":
                depth += 1
            elif tok[0] == "op" and tok[1] == ")":
                if depth == 0:
                    break
                depth -= 1
            elif depth == 0 and tok[0] == "op" and tok[1] in stop_ops:
                break
            elif depth == 0 and tok[0] == "id" and tok[1].lower() in stop_words:
                break
            end = tok[3]
            self.i += 1
        s = self.text[start:end].strip()
        if not s:
            raise SqlError(f"expected an expression near {self.text[start:start + 40]!r}")
        return s

    # ------------------------------------------------------------------ statements
    def statement(self):
        if self.kw() in ("select", "with") or (self.peek()[0] == "op" and self.peek()[1] == "("):
            df = self.query()
            self._end()
            return df
        if self.accept_kw("create"):
            return self._create()
        if self.accept_kw("insert"):
            return self._insert()
        if self.accept_kw("drop"):
            return self._drop()
        if self.accept_kw("use"):
            db = self.name()
            self._end()
            _catalog(self.session).use(db)
            return _empty(self.session)
        if self.accept_kw("show"):
            return self._show()
        if self.accept_kw("describe") or self.accept_kw("desc"):
            self.accept_kw("table")
            df = _catalog(self.session).lookup(self.name(), self.ctes)
            self._end()
            return self.session.createDataFrame([(f.name, f.dataType.simpleString(), None) for f in df.schema],
                                                ["col_name", "data_type", "comment"])
        raise SqlError(f"unsupported SQL statement: {self.text[:60]!r}")

    def _end(self):
        self.accept_op(";")
        if self.peek()[0] != "eof":
            raise SqlError(f"unexpected {self.rest()[:40]!r}")

    def _create(self):
        cat = _catalog(self.session)
        replace = self.accept_kw("or", "replace")
        self.accept_kw("global")
        temp = self.accept_kw("temporary") or self.accept_kw("temp")
        if self.accept_kw("view"):
            if_not = self.accept_kw("if", "not", "exists")
            name = self.name()
            self.expect_kw("as")
            df = self.query()
            self._end()
            if if_not and cat.exists(name):
                return _empty(self.session)
            if not replace and name in self.session._catalog and not if_not:
                raise SqlError(f"view {name} already exists")
            df.createOrReplaceTempView(name)
            return _empty(self.session)
        if self.accept_kw("database") or self.accept_kw("schema"):
            if_not = self.accept_kw("if", "not", "exists")
            cat.create_database(self.name(), if_not)
            self._end()
            return _empty(self.session)
        if self.accept_kw("table"):
            if_not = self.accept_kw("if", "not", "exists")
            name = self.name()
            if self.accept_kw("using"):
                fmt = self.name().lower()
                if fmt != "parquet":
                    raise SqlError("CREATE TABLE ... USING supports parquet")
            self.expect_kw("as")
            df = self.query()
            self._end()
            if cat.exists(name) and not temp:
                if if_not:
                    return _empty(self.session)
                if not replace:
                    raise SqlError(f"table {name} already exists")
            cat.save(name, df, "overwrite")
            return _empty(self.session)
        raise SqlError(f"unsupported CREATE statement: {self.text[:60]!r}")

    def _insert(self):
        mode = "append"
        if self.accept_kw("overwrite"):
            mode = "overwrite"
        else:
            self.expect_kw("into")
        self.accept_kw("table")
        name = self.name()
        df = self.query()
        self._end()
        cat = _catalog(self.session)
        if not cat.exists(name):
            raise SqlError(f"table {name} not found")
        cat.save(name, df, mode)
        return _empty(self.session)

    def _drop(self):
        cat = _catalog(self.session)
        if self.accept_kw("database") or self.accept_kw("schema"):
            if_exists = self.accept_kw("if", "exists")
            cat.drop_database(self.name(), if_exists)
            self.accept_kw("cascade")
            self._end()
            return _empty(self.session)
        if not (self.accept_kw("table") or self.accept_kw("view")):
            raise SqlError("expected TABLE or VIEW after DROP")
        if_exists = self.accept_kw("if", "exists")
        name = self.name()
        self._end()
        if not cat.drop(name) and not if_exists:
            raise SqlError(f"table or view {name} not found")
        return _empty(self.session)

    def _show(self):
        cat = _catalog(self.session)
        if self.accept_kw("databases") or self.accept_kw("schemas"):
            self._end()
            return self.session.createDataFrame([(d,) for d in cat.databases()], ["namespace"])
        self.expect_kw("tables")
        db = None
        if self.accept_kw("in") or self.accept_kw("from"):
            db = self.name()
        self._end()
        rows = cat.tables(db)
        return self.session.createDataFrame(rows, ["namespace", "tableName", "isTemporary"]) if rows else \
            _empty(self.session, ["namespace", "tableName", "isTemporary"])

    # ------------------------------------------------------------------ queries
    def query(self):
        if self.accept_kw("with"):
            while True:
                name = self.name()
                self.expect_kw("as")
                self.expect_op("(")
                sub = _Stmt(self.session, self.text, self.ctes)
                sub.t, sub.i = self.t, self.i
                self.ctes[name] = sub.query()
                self.i = sub.i
                self.expect_op(")")
                if not self.accept_op(","):
                    break
        df = self._select()
        while self.kw() in ("union", "intersect", "except"):
            op = self.kw()
            self.i += 1
            dist = not self.accept_kw("all")
            self.accept_kw("distinct")
            rhs = self._select()
            if op == "union":
                df = df.union(rhs)
                if dist:
                    df = df.distinct()
            else:
                key = list(df.columns)
                rhs = rhs.toDF(*key)
                df = df.join(rhs, key, "left_semi" if op == "intersect" else "left_anti")
                if dist:
                    df = df.distinct()
        df = self._order_limit(df, None)
        return df

    def _select(self):
        if self.accept_op("("):
            df = self.query()
            self.expect_op(")")
            return df
        self.expect_kw("select")
        distinct = self.accept_kw("distinct")
        self.accept_kw("all")
        items = []
        while True:
            items.append(self._select_item())
            if not self.accept_op(","):
                break
        src = None
        if self.accept_kw("from"):
            src = self._from()
        else:
            src = self.session.createDataFrame([(0,)], ["__one"])
        if self.accept_kw("where"):
            src = src.filter(self._expr(self.span(_CLAUSE - {"as", "asc", "desc", "all", "by", "first", "last"})))
        group = None
        if self.accept_kw("group"):
            self.expect_kw("by")
            group = []
            while True:
                group.append(self.span(_CLAUSE - {"as", "asc", "desc", "all", "by", "first", "last"}))
                if not self.accept_op(","):
                    break
        having = None
        if self.accept_kw("having"):
            having = self.span(_CLAUSE - {"as", "asc", "desc", "all", "by", "first", "last"})
        return self._project(src, items, group, having, distinct)

    def _select_item(self):
        tok = self.peek()
        if tok[0] == "op" and tok[1] == "*":
            self.i += 1
            return ("*", None)
        if tok[0] in ("id", "bq") and self.peek(1)[:2] == ("op", ".") and self.peek(2)[:2] == ("op", "*"):
            self.i += 3
            return ("*", tok[1].strip("`"))
        text = self.span({"from", "where", "group", "having", "order", "limit", "union", "intersect", "except"})
        return ("expr", text)

    def _from(self):
        df, lquals = self._source()
        while True:
            how = None
            if self.accept_kw("join") or self.accept_kw("inner", "join"):
                how = "inner"
            elif self.accept_kw("cross", "join"):
                how = "cross"
            elif self.kw() in ("left", "right", "full"):
                side = self.kw()
                self.i += 1
                if self.accept_kw("semi"):
                    how = "left_semi"
                elif self.accept_kw("anti"):
                    how = "left_anti"
                else:
                    self.accept_kw("outer")
                    how = {"left": "left", "right": "right", "full": "outer"}[side]
                self.expect_kw("join")
            elif self.accept_op(","):
                how = "cross"
            else:
                break
            rhs, rquals = self._source()
            if how == "cross":
                df = df.crossJoin(rhs)
                lquals |= rquals
                continue
            if self.accept_kw("using"):
                self.expect_op("(")
                cols = []
                while True:
                    cols.append(self.name().split(".")[-1])
                    if not self.accept_op(","):
                        break
                self.expect_op(")")
                df = df.join(rhs, cols, how)
                lquals |= rquals
                continue
            self.expect_kw("on")
            cond = self._expr(self.span(_CLAUSE - {"as", "asc", "desc", "all", "by", "first", "last"}))
            df = _join_on(df, rhs, cond, how, lquals, rquals)
            lquals |= rquals
        return df

    def _source(self):
        tname = None
        if self.accept_op("("):
            df = self.query()
            self.expect_op(")")
        else:
            tname = self.name()
            df = _catalog(self.session).lookup(tname, self.ctes)
        alias = None
        if self.accept_kw("as"):
            alias = self.name()
        elif self.peek()[0] in ("id", "bq") and self.kw() not in _CLAUSE | {"join", "on", "using", "left", "right",
                                                                            "full", "inner", "cross", "where"}:
            alias = self.name()
        # qualifier -> its columns, for ``alias.*`` in the select list; the set of names that
        # refer to this source, for ``alias.col`` in JOIN ... ON
        quals = set()
        for q in (alias, tname, tname.split(".")[-1] if tname else None):
            if q:
                self.qualifiers[q] = list(df.columns)
                quals.add(q)
        if alias:      # an alias hides the table's own name (Spark: t AS a -> only a.col)
            quals = {alias}
        return df, quals

    def _expr(self, text):
        from raydp_amd.spark.sqlexpr import parse
        return parse(text)

    def _project(self, df, items, group, having, distinct):
        from raydp_amd.spark.column import AggExpr, Alias, Column
        cols = []     # (Column, output name)
        star = False
        for kind, v in items:
            if kind == "*":
                star = True
                have = set(df.columns)
                names = self.qualifiers.get(v, df.columns) if v else df.columns
                cols += [(None, c) for c in names if c in have and (None, c) not in cols]
                continue
            c = self._expr(v)
            e = c._expr
            cols.append((c, e.name()))
        exprs = [c for c, _ in cols if c is not None]
        has_agg = any(c._expr.is_aggregate() for c in exprs)
        self._agg_ctx = None
        hv = self._expr(having) if having else None
        if group is None and not has_agg and hv is None:
            if star and all(c is None for c, _ in cols):
                out = df
            else:
                out = df.select(*[c if c is not None else n for c, n in cols])
            return out.distinct() if distinct else out
        keys = [self._expr(g) for g in group or []]
        key_names = []
        pre = df
        for k in keys:   # grouping by an expression: materialise it first under its name
            e = k._expr
            from raydp_amd.spark.column import ColRef
            if isinstance(e, ColRef):
                key_names.append(e.col_name)
            else:
                nm = e.name()
                pre = pre.withColumn(nm, k)
                key_names.append(nm)
        aggs, hidden = [], {}

        def lift(e):
            """Replace every aggregate sub-expression by a reference to its output column."""
            from raydp_amd.spark.column import ColRef, map_children
            if isinstance(e, AggExpr):
                nm = e.name()
                if nm not in hidden:
                    hidden[nm] = f"__agg{len(hidden)}"
                    aggs.append(Column(Alias(e, hidden[nm])))
                return ColRef(hidden[nm])
            return map_children(e, lift)
        post = []
        for c, n in cols:
            if c is None:
                post.append((None, n))
                continue
            e = c._expr
            inner = e.child if isinstance(e, Alias) else e
            if e.is_aggregate():
                post.append((Column(Alias(lift(inner), n)), n))
            else:
                post.append((Column(Alias(lift_keys(inner, keys, key_names), n)), n))
        hcol = Column(lift(hv._expr)) if hv is not None else None
        self._agg_ctx = ctx = dict(pre=pre, key_names=key_names, keys=keys, aggs=aggs, lift=lift, having=hcol,
                                   post=post)
        out = self._grouped_projection(ctx)
        return out.distinct() if distinct else out

    @staticmethod
    def _grouped(ctx):
        """The grouped frame: keys + every aggregate lifted so far (select, HAVING, ORDER BY),
        HAVING applied when it only needs those columns."""
        pre, key_names, aggs, hcol = ctx["pre"], ctx["key_names"], ctx["aggs"], ctx["having"]
        grouped = pre.groupBy(*key_names).agg(*aggs) if aggs else pre.select(*key_names).distinct()
        late = None
        if hcol is not None:
            if hcol._expr.references() <= set(grouped.columns):
                grouped = grouped.filter(hcol)
            else:
                late = hcol         # refers to select aliases: filter the projection
        return grouped, late

    def _grouped_projection(self, ctx, extra=()):
        grouped, late = self._grouped(ctx)
        proj = [c if c is not None else n for c, n in ctx["post"]]
        out = grouped.select(*(proj + [c.alias(nm) for nm, c in extra]))
        if late is not None:
            out = out.filter(late)
        return out

    def _order_limit(self, df, _):
        if self.accept_kw("order"):
            self.expect_kw("by")
            keys = []
            while True:
                text = self.span(_CLAUSE - {"as", "all", "by", "first", "last"} | {"asc", "desc", "nulls"})
                asc = True
                if self.accept_kw("desc"):
                    asc = False
                else:
                    self.accept_kw("asc")
                nulls_first = None
                if self.accept_kw("nulls"):
                    nulls_first = self.accept_kw("first")
                    if not nulls_first:
                        self.expect_kw("last")
                keys.append((text, asc, nulls_first))
                if not self.accept_op(","):
                    break
            df = self._sort(df, keys)
        if self.accept_kw("limit"):
            tok = self.peek()
            if tok[0] != "num":
                raise SqlError("LIMIT takes a number")
            self.i += 1
            df = df.limit(int(tok[1]))
        return df

    def _sort(self, df, keys):
        from raydp_amd.spark.column import Column, SortOrder
        cols = set(df.columns)
        orders, extra = [], []
        ctx = getattr(self, "_agg_ctx", None)
        for text, asc, nf in keys:
            c = self._expr(text)
            e = c._expr
            if re.fullmatch(r"\d+", text):          # ORDER BY 2: the second output column
                nm = df.columns[int(text) - 1]
                orders.append(SortOrder(_colref(nm), asc, nf))
                continue
            if e.references() <= cols and not e.is_aggregate():
                orders.append(SortOrder(e, asc, nf))
                continue
            if ctx is None:
                raise SqlError(f"cannot resolve ORDER BY {text!r}")
            # an aggregate / key expression that is not in the output: lift it into the
            # grouping (a new hidden aggregate if needed), sort, then project it away
            nm = f"__ord{len(extra)}"
            extra.append((nm, Column(lift_keys(ctx["lift"](e), ctx["keys"], ctx["key_names"]))))
            orders.append(SortOrder(_colref(nm), asc, nf))
        if not extra:
            return df.orderBy(*[Column(o) for o in orders])
        full = self._grouped_projection(ctx, extra)
        return full.orderBy(*[Column(o) for o in orders]).select(*[n for _, n in ctx["post"]])


def _colref(name):
    from raydp_amd.spark.column import ColRef
    return ColRef(name)


def lift_keys(e, keys, key_names):
    """Rewrite occurrences of a grouping expression by a reference to its key column."""
    from raydp_amd.spark.column import ColRef, map_children
    names = {k._expr.name(): n for k, n in zip(keys, key_names)}
    if not isinstance(e, ColRef) and e.name() in names:
        return ColRef(names[e.name()])
    return map_children(e, lambda c: lift_keys(c, keys, key_names))


def _side(ref, lcols, rcols, lquals, rquals):
    """Which join input a column reference of an ON condition reads: "L", "R" or None (neither).
    A qualified ``alias.col`` goes by its qualifier; a bare name must exist on exactly one side
    (Spark's analyzer rejects an ambiguous reference instead of guessing)."""
    q, c = ref.qualifier, ref.col_name
    if q is not None:
        if q in rquals and c in rcols:
            return "R"
        if q in lquals and c in lcols:
            return "L"
        if q not in rquals and q not in lquals:
            raise SqlError(f"unknown qualifier {q!r} in JOIN ... ON")
        raise SqlError(f"cannot resolve column {q}.{c} in JOIN ... ON")
    inl, inr = c in lcols, c in rcols
    if inl and inr:
        raise SqlError(f"reference {c!r} in JOIN ... ON is ambiguous (both sides have it); qualify it")
    return "L" if inl else "R" if inr else None


def _join_on(left, right, cond, how, lquals=frozenset(), rquals=frozenset()):
    """Equi-join on every ``a = b`` conjunct between a left and a right column; other conjuncts
    filter the joined rows (inner joins only). Each side of an equality is resolved by its
    qualifier (``ON b.k = a.j`` joins a.j with b.k whatever the order of the operands)."""
    from raydp_amd.spark import wide as W
    from raydp_amd.spark.column import BinOp, ColRef, Column
    conj, stack = [], [cond._expr]
    while stack:
        e = stack.pop()
        if isinstance(e, BinOp) and e.op == "&":
            stack += [e.right, e.left]
        else:
            conj.append(e)
    lk, rk, residual = [], [], []
    lcols, rcols = set(left.columns), set(right.columns)
    for e in conj:
        if isinstance(e, BinOp) and e.op == "==" and isinstance(e.left, ColRef) and isinstance(e.right, ColRef):
            sa = _side(e.left, lcols, rcols, lquals, rquals)
            sb = _side(e.right, lcols, rcols, lquals, rquals)
            a, b = e.left.col_name, e.right.col_name
            if (sa, sb) == ("L", "R"):
                lk.append(a)
                rk.append(b)
                continue
            if (sa, sb) == ("R", "L"):
                lk.append(b)
                rk.append(a)
                continue
        residual.append(e)
    if not lk and how not in ("inner", "cross"):
        raise SqlError("JOIN ... ON needs at least one equality between a left and a right column")
    if residual:
        # every column of the residual resolved to its side here (qualifiers), then the
        # DataFrame join's residual machinery (outer / semi / anti too)
        from raydp_amd.spark.column import map_children

        def tag(e):
            if isinstance(e, ColRef):
                side = _side(e, lcols, rcols, lquals, rquals)
                r = ColRef(e.col_name)
                if side is not None:
                    r.origin = id(left) if side == "L" else id(right)
                return r
            return map_children(e, tag)
        return left._join_residual(right, lk, rk, [tag(e) for e in residual], how)
    if any(a != b for a, b in zip(lk, rk)):
        # the keys are resolved already: build the join on them directly (DataFrame.join would
        # guess the sides again by name, which a self-join cannot disambiguate)
        return left._with(W.JoinPlan(left._src(), right._src(), lk, rk, how))
    return left.join(right, lk, how)


def _empty(session, names=None):
    import pyarrow as pa
    names = names or []
    return session.createDataFrame(pa.table({n: pa.array([], pa.string()) for n in names}))


# ---------------------------------------------------------------------- catalog ------------
class _Catalog:
    """Temp views (the session's in-memory catalog) over persistent parquet tables under the
    warehouse directory: ``<warehouse>/<table>`` for the default database, ``<warehouse>/<db>.db/
    <table>`` otherwise (Spark's layout)."""

    def __init__(self, session):
        self.session = session
        self.current = "default"

    @property
    def warehouse(self) -> str:
        d = self.session.conf.get("spark.sql.warehouse.dir") or os.path.join(os.getcwd(), "spark-warehouse")
        if d.startswith("file://"):
            d = d[len("file://"):]
        return d

    def _db_dir(self, db: str) -> str:
        return self.warehouse if db == "default" else os.path.join(self.warehouse, f"{db}.db")

    def _split(self, name: str):
        parts = name.split(".")
        if len(parts) == 1:
            return self.current, parts[0]
        return parts[-2], parts[-1]

    def path(self, name: str) -> str:
        db, t = self._split(name)
        return os.path.join(self._db_dir(db), t.lower())

    def exists(self, name: str) -> bool:
        return name in self.session._catalog or os.path.isdir(self.path(name))

    def lookup(self, name: str, ctes=None):
        if ctes and name in ctes:
            return ctes[name]
        views = self.session._catalog
        if name in views:
            return views[name]
        low = {k.lower(): v for k, v in views.items()}
        if name.lower() in low:
            return low[name.lower()]
        p = self.path(name)
        if os.path.isdir(p):
            return self.session.read.parquet(p)
        raise SqlError(f"Table or view not found: {name}")

    def save(self, name: str, df, mode: str):
        db, _ = self._split(name)
        if db != "default" and not os.path.isdir(self._db_dir(db)):
            raise SqlError(f"Database '{db}' not found")
        p = self.path(name)
        if mode == "append" and os.path.isdir(p):
            df.write.mode("append").parquet(p)
            return
        if os.path.isdir(p):
            # the new content may read the old table (INSERT OVERWRITE t SELECT ... FROM t):
            # materialise first, then replace
            df = df.localCheckpoint()
            shutil.rmtree(p)
        df.write.mode("overwrite").parquet(p)

    def drop(self, name: str) -> bool:
        if name in self.session._catalog:
            del self.session._catalog[name]
            return True
        p = self.path(name)
        if os.path.isdir(p):
            shutil.rmtree(p)
            return True
        return False

    def create_database(self, db: str, if_not_exists: bool):
        d = self._db_dir(db)
        if os.path.isdir(d) and db != "default":
            if if_not_exists:
                return
            raise SqlError(f"Database '{db}' already exists")
        os.makedirs(d, exist_ok=True)

    def drop_database(self, db: str, if_exists: bool):
        d = self._db_dir(db)
        if db == "default":
            raise SqlError("cannot drop the default database")
        if not os.path.isdir(d):
            if if_exists:
                return
            raise SqlError(f"Database '{db}' not found")
        shutil.rmtree(d)
        if self.current == db:
            self.current = "default"

    def use(self, db: str):
        if db != "default" and not os.path.isdir(self._db_dir(db)):
            raise SqlError(f"Database '{db}' not found")
        self.current = db

    def databases(self) -> List[str]:
        out = ["default"]
        if os.path.isdir(self.warehouse):
            out += sorted(n[:-3] for n in os.listdir(self.warehouse) if n.endswith(".db"))
        return out

    def tables(self, db: Optional[str] = None):
        db = db or self.current
        rows = []
        d = self._db_dir(db)
        if os.path.isdir(d):
            for n in sorted(os.listdir(d)):
                if os.path.isdir(os.path.join(d, n)) and not n.endswith(".db"):
                    rows.append((db, n, False))
        rows += [("", n, True) for n in sorted(self.session._catalog)]
        return rows


def _catalog(session) -> _Catalog:
    cat = getattr(session, "_sql_catalog", None)
    if cat is None:
        cat = session._sql_catalog = _Catalog(session)
    return cat


def execute(session, query: str):
    """Run one SQL statement; returns a DataFrame (empty for DDL)."""
    q = query.strip().rstrip(";").rstrip()
    if not q:
        raise SqlError("empty SQL statement")
    return _Stmt(session, q).statement()


def save_as_table(session, name: str, df, mode: str = "errorifexists"):
    """``DataFrameWriter.saveAsTable``: persist ``df`` as a parquet table of the warehouse."""
    cat = _catalog(session)
    mode = (mode or "errorifexists").lower()
    if cat.exists(name) and name not in session._catalog:
        if mode in ("error", "errorifexists"):
            raise SqlError(f"Table {name} already exists")
        if mode == "ignore":
            return
    cat.save(name, df, "append" if mode == "append" else "overwrite")
