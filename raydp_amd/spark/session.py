"""``SparkSession`` of the Arrow-native engine.

``raydp.init_spark`` returns one of these (reference: ``python/raydp/context.py:142-150`` →
``SparkSession.builder...master("ray://...").getOrCreate()``). The session owns the task
scheduler: executor actor processes when created through ``init_spark`` (the cluster
backend), or an in-process thread pool for ``SparkSession.builder.master("local[n]")``.
"""
import datetime
import decimal
import threading
import time
import uuid
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from raydp_amd.spark import plan as P
from raydp_amd.spark.dataframe import DataFrame
from raydp_amd.spark.row import Row
from raydp_amd.spark.sources import RangeSource, TableSource, split_table
from raydp_amd.spark.types import DataType, StructType, parse_type_string

_active_lock = threading.RLock()
_active_session: Optional["SparkSession"] = None


class RuntimeConfig:
    def __init__(self, conf: Dict[str, str]):
        self._conf = conf

    def set(self, key, value):
        self._conf[key] = str(value) if not isinstance(value, str) else value

    def get(self, key, default=None):
        return self._conf.get(key, default)

    def unset(self, key):
        self._conf.pop(key, None)

    def getAll(self):
        return dict(self._conf)

    def isModifiable(self, key):
        return True


class SparkConf:
    def __init__(self, conf: Optional[Dict[str, str]] = None):
        self._conf = dict(conf or {})

    def get(self, key, defaultValue=None):
        return self._conf.get(key, defaultValue)

    def set(self, key, value):
        self._conf[key] = str(value)
        return self

    def getAll(self):
        return list(self._conf.items())

    def contains(self, key):
        return key in self._conf


class SparkContext:
    def __init__(self, session: "SparkSession"):
        self._session = session
        self.applicationId = f"app-{time.strftime('%Y%m%d%H%M%S')}{int(time.time() * 1000) % 1000:03d}"
        self.startTime = int(time.time() * 1000)

    @property
    def appName(self):
        return self._session.conf.get("spark.app.name", "raydp")

    @property
    def master(self):
        return self._session.conf.get("spark.master", "local[*]")

    @property
    def defaultParallelism(self):
        return self._session._default_parallelism()

    def getConf(self):
        return SparkConf(self._session.conf.getAll())

    def setLogLevel(self, level):
        pass

    def stop(self):
        self._session.stop()

    def parallelize(self, data, numSlices=None):
        from raydp_amd.spark.rdd import RDD
        data = list(data)
        n = max(1, int(numSlices or self.defaultParallelism))
        n = min(n, max(1, len(data)))
        bounds = [len(data) * k // n for k in range(n + 1)]
        parts = [data[bounds[k]:bounds[k + 1]] for k in range(n)]
        return RDD(self._session, n, lambda i: parts[i], "parallelize")

    def range(self, start, end=None, step=1, numSlices=None):
        if end is None:
            start, end = 0, start
        return self.parallelize(range(start, end, step), numSlices)

    def emptyRDD(self):
        from raydp_amd.spark.rdd import RDD
        return RDD(self._session, 1, lambda i: [], "empty")


def _to_arrow_schema(schema) -> pa.Schema:
    if isinstance(schema, pa.Schema):
        return schema
    if isinstance(schema, StructType):
        return schema.to_arrow()
    if isinstance(schema, str):
        fields = []
        for part in _split_ddl(schema):
            name, ty = part.strip().split(None, 1) if " " in part.strip() else part.strip().split(":", 1)
            fields.append(pa.field(name.strip(), parse_type_string(ty.strip()).to_arrow()))
        return pa.schema(fields)
    raise TypeError(f"unsupported schema {schema!r}")


def _split_ddl(s):
    depth, cur, out = 0, "", []
    for ch in s:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def _infer_value_type(v) -> Optional[pa.DataType]:
    if v is None:
        return None
    if isinstance(v, bool):
        return pa.bool_()
    if isinstance(v, (int, np.integer)):
        return pa.int64()
    if isinstance(v, (float, np.floating)):
        return pa.float64()
    if isinstance(v, str):
        return pa.string()
    if isinstance(v, datetime.datetime):
        return pa.timestamp("us")
    if isinstance(v, datetime.date):
        return pa.date32()
    if isinstance(v, decimal.Decimal):
        return pa.decimal128(38, 18)
    if isinstance(v, (bytes, bytearray)):
        return pa.binary()
    if isinstance(v, (list, tuple, np.ndarray)):
        for x in v:
            t = _infer_value_type(x)
            if t is not None:
                return pa.list_(t)
        return pa.list_(pa.null())
    return None


class Builder:
    _lock = threading.RLock()

    def __init__(self):
        self._options: Dict[str, str] = {}

    def master(self, m):
        self._options["spark.master"] = m
        return self

    def appName(self, name):
        self._options["spark.app.name"] = name
        return self

    def config(self, key=None, value=None, conf=None, map=None):  # noqa: A002
        if conf is not None:
            for k, v in conf.getAll():
                self._options[k] = v
        if map is not None:
            self._options.update({k: str(v) for k, v in map.items()})
        if key is not None:
            self._options[key] = str(value) if not isinstance(value, str) else value
        return self

    def enableHiveSupport(self):
        self._options["spark.sql.catalogImplementation"] = "hive"
        return self

    def getOrCreate(self) -> "SparkSession":
        global _active_session
        with _active_lock:
            if _active_session is not None and not _active_session._stopped:
                for k, v in self._options.items():
                    _active_session.conf.set(k, v)
                return _active_session
            opts = dict(_submit_conf())
            opts.update(self._options)
            master = opts.get("spark.master", "")
            if master == "ray" or master.startswith("ray://"):
                # "--master ray" (raydp-submit / RayCoarseGrainedSchedulerBackend.scala:81-117):
                # bring up the runtime and the executor cluster for this application
                from raydp_amd.context import init_spark
                return init_spark(opts.get("spark.app.name", "raydp-app"),
                                  int(opts.get("spark.executor.instances", "1")),
                                  int(opts.get("spark.executor.cores", "1")),
                                  opts.get("spark.executor.memory", "1g"),
                                  enable_hive=opts.get("spark.sql.catalogImplementation") == "hive",
                                  configs={k: v for k, v in opts.items() if k != "spark.master"})
            s = SparkSession(opts)
            _active_session = s
            return s


def _submit_conf() -> Dict[str, str]:
    """Spark confs handed over by ``raydp-submit`` (RAYDP_SUBMIT_CONF, JSON)."""
    import json
    import os
    raw = os.environ.get("RAYDP_SUBMIT_CONF")
    return json.loads(raw) if raw else {}


class SparkSession:
    builder = Builder()

    def __init__(self, conf: Dict[str, str], scheduler: Optional[P.TaskScheduler] = None,
                 cluster=None):
        conf.setdefault("spark.app.name", "raydp")
        conf.setdefault("spark.master", "local[*]")
        conf.setdefault("spark.sql.shuffle.partitions", "200")
        self.conf = RuntimeConfig(conf)
        self._cluster = cluster
        self._scheduler = scheduler
        self._stopped = False
        self._catalog: Dict[str, DataFrame] = {}
        self.sparkContext = SparkContext(self)
        self.version = "3.5.0-raydp-amd"

    # ------------------------------------------------------------------ plumbing ---------
    @classmethod
    def getActiveSession(cls) -> Optional["SparkSession"]:
        s = _active_session
        return s if s is not None and not s._stopped else None

    @classmethod
    def _set_active(cls, s: Optional["SparkSession"]):
        global _active_session
        with _active_lock:
            _active_session = s

    def _default_parallelism(self) -> int:
        v = self.conf.get("spark.default.parallelism")
        if v:
            return int(v)
        inst = self.conf.get("spark.executor.instances")
        cores = self.conf.get("spark.executor.cores")
        if inst and cores:
            return max(1, int(inst) * int(cores))
        m = self.conf.get("spark.master", "local[*]")
        if m.startswith("local["):
            inner = m[6:-1]
            if inner != "*":
                return max(1, int(inner))
        import os
        return os.cpu_count() or 1

    def _scheduler_or_default(self) -> P.TaskScheduler:
        if self._scheduler is None:
            self._scheduler = P.TaskScheduler(self._default_parallelism())
        return self._scheduler

    def _run(self, plan: P.Plan) -> List[pa.Table]:
        if self._stopped:
            raise RuntimeError("Cannot call methods on a stopped SparkSession")
        return self._scheduler_or_default().run_plan(plan)

    @property
    def read(self):
        from raydp_amd.spark.io import DataFrameReader
        return DataFrameReader(self)

    @property
    def udf(self):
        return _UDFRegistration()

    @property
    def catalog(self):
        return self

    def listTables(self):
        return list(self._catalog)

    def table(self, name):
        from raydp_amd.spark.sql import _catalog
        return _catalog(self).lookup(name)

    def tableExists(self, name) -> bool:
        from raydp_amd.spark.sql import _catalog
        return _catalog(self).exists(name)

    def dropTempView(self, name) -> bool:
        return self._catalog.pop(name, None) is not None

    def sql(self, query: str, args=None):
        """Run a Spark SQL statement (``raydp_amd/spark/sql.py``): queries over temp views and
        warehouse tables, views, CTAS / INSERT, databases."""
        from raydp_amd.spark.sql import execute
        if args:
            raise NotImplementedError("parameterised SQL (args=) is not supported")
        return execute(self, query)

    def newSession(self):
        return self

    def stop(self):
        if self._stopped:
            return
        self._stopped = True
        if self._scheduler is not None:
            self._scheduler.shutdown()
        if _active_session is self:
            SparkSession._set_active(None)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()

    # ------------------------------------------------------------------ creation --------
    def range(self, start, end=None, step=1, numPartitions=None) -> DataFrame:
        if end is None:
            start, end = 0, start
        n = numPartitions or self._default_parallelism()
        return DataFrame(P.SourcePlan(RangeSource(start, end, step, n)), self)

    def createDataFrame(self, data, schema=None, samplingRatio=None, verifySchema=True) -> DataFrame:
        from raydp_amd.spark.rdd import RDD, RDDSource
        if isinstance(data, RDD):
            src = RDDSource(data, schema, rows_to_table)
            src.schema()   # resolved on the driver, shipped with the plan
            return DataFrame(P.SourcePlan(src), self)
        table = self._to_table(data, schema)
        n = self._default_parallelism()
        n = max(1, min(n, table.num_rows)) if table.num_rows else 1
        parts = split_table(table, n)
        if getattr(self._scheduler, "remote", False):
            # executors are processes: place the source partitions in the object store once
            from raydp_amd.runtime.serialization import share_table
            parts = [share_table(t) for t in parts]
        return DataFrame(P.SourcePlan(TableSource(parts, table.schema)), self)

    def _to_table(self, data, schema) -> pa.Table:
        return rows_to_table(data, schema)


def rows_to_table(data, schema) -> pa.Table:
    """Python rows / dicts / Row objects / pandas frame -> Arrow table (createDataFrame)."""
    import pandas as pd
    if isinstance(data, pa.Table):
        return data if schema is None else data.cast(_to_arrow_schema(schema))
    if isinstance(data, pd.DataFrame):
        t = pa.Table.from_pandas(data, preserve_index=False)
        if schema is not None:
            target = _to_arrow_schema(schema) if not isinstance(schema, (list, tuple)) else None
            if target is not None:
                t = t.rename_columns(target.names).cast(target)
            else:
                t = t.rename_columns(list(schema))
        return t
    rows = list(data)
    names = None
    target = None
    if isinstance(schema, (list, tuple)):
        names = list(schema)
    elif schema is not None:
        target = _to_arrow_schema(schema)
        names = target.names
    if rows and isinstance(rows[0], dict):
        names = names or list(rows[0].keys())
        cols = {k: [r.get(k) for r in rows] for k in names}
    elif rows and isinstance(rows[0], Row) and rows[0].__fields__:
        names = names or list(rows[0].__fields__)
        cols = {k: [r[j] for r in rows] for j, k in enumerate(names)}
    else:
        rows = [r if isinstance(r, (tuple, list)) else (r,) for r in rows]
        width = len(rows[0]) if rows else (len(names) if names else 0)
        names = names or [f"_{j + 1}" for j in range(width)]
        cols = {k: [r[j] for r in rows] for j, k in enumerate(names)}
    if target is not None:
        arrays = [pa.array(cols[f.name], type=f.type) for f in target]
        return pa.Table.from_arrays(arrays, schema=target)
    arrays = []
    for k in names:
        vals = cols[k]
        ty = None
        for v in vals:
            ty = _infer_value_type(v)
            if ty is not None:
                break
        arrays.append(pa.array(vals, type=ty))
    return pa.Table.from_arrays(arrays, names=names)


class _UDFRegistration:
    def register(self, name, f, returnType=None):
        from raydp_amd.spark.udf import UserDefinedFunction
        return f if isinstance(f, UserDefinedFunction) else UserDefinedFunction(f, returnType or "string")
