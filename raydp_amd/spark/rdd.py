"""Resilient distributed datasets of Python objects (the subset of ``pyspark.RDD`` RayDP users
touch: ``sc.parallelize``, ``df.rdd``, ``map``/``flatMap``/``filter``/``mapPartitions``,
key-value shuffles, ``toDF`` / ``createDataFrame(rdd)``).

An RDD is a partition count plus a picklable ``compute(i) -> iterable`` function; narrow
transformations compose those functions, actions run them as tasks on the session's scheduler
(the executor actor processes of a Spark-on-runtime session, ``raydp_amd.spark.cluster``), so
the per-partition Python work happens in parallel outside the driver. Wide transformations
(``reduceByKey``, ``groupByKey``, ``distinct``, ``sortBy``, ``repartition``) run a map stage
that hash-buckets each partition, then a reduce stage whose tasks read their bucket of every
map output (through the object store when executors are processes).
"""
import itertools
import random as _random
from typing import Any, Callable, Iterable, List, Optional

import pyarrow as pa


def _portable_hash(x) -> int:
    if x is None:
        return 0
    if isinstance(x, (tuple, list)):
        h = 0x345678
        for e in x:
            h = (1000003 * h) ^ _portable_hash(e)
            h &= 0xFFFFFFFFFFFF
        return h
    if isinstance(x, str):
        import zlib
        return zlib.crc32(x.encode())
    if isinstance(x, bytes):
        import zlib
        return zlib.crc32(x)
    return hash(x)


class RDD:
    def __init__(self, session, num_partitions: int, compute: Callable[[int], Iterable], name: str = "rdd",
                 prefs: Optional[Callable[[int], Optional[str]]] = None):
        self._session = session
        self._n = max(1, int(num_partitions))
        self._compute = compute
        self._name = name
        self._prefs = prefs   # partition -> node holding its input (narrow lineage only)
        self._cached: Optional[List[list]] = None
        import uuid
        self._id = uuid.uuid4().int & 0x7FFFFFFF

    # ------------------------------------------------------------------ plumbing ---------
    @property
    def context(self):
        return self._session.sparkContext

    def id(self):
        return self._id

    def getNumPartitions(self) -> int:
        return self._n

    def _part_fn(self):
        if self._cached is not None:
            parts = self._cached
            return lambda i: parts[i]
        return self._compute

    def _run(self, fn: Callable[[int], Any]) -> list:
        sched = self._session._scheduler_or_default()
        if self._prefs is not None and self._cached is None and getattr(sched, "remote", False):
            return sched.map(fn, range(self._n), prefs={i: self._prefs(i) for i in range(self._n)})
        return sched.map(fn, range(self._n))

    def _derive(self, fn: Callable[[Iterable, int], Iterable], name: str, n: Optional[int] = None) -> "RDD":
        src = self._part_fn()
        keep = n is None or n == self._n
        return RDD(self._session, self._n if n is None else n, lambda i: fn(src(i), i), name,
                   prefs=self._prefs if keep and self._cached is None else None)

    # ------------------------------------------------------------------ narrow -----------
    def map(self, f, preservesPartitioning=False) -> "RDD":
        return self._derive(lambda it, i: [f(x) for x in it], "map")

    def flatMap(self, f, preservesPartitioning=False) -> "RDD":
        return self._derive(lambda it, i: [y for x in it for y in f(x)], "flatMap")

    def filter(self, f) -> "RDD":
        return self._derive(lambda it, i: [x for x in it if f(x)], "filter")

    def mapPartitions(self, f, preservesPartitioning=False) -> "RDD":
        return self._derive(lambda it, i: list(f(iter(it))), "mapPartitions")

    def mapPartitionsWithIndex(self, f, preservesPartitioning=False) -> "RDD":
        return self._derive(lambda it, i: list(f(i, iter(it))), "mapPartitionsWithIndex")

    def glom(self) -> "RDD":
        return self._derive(lambda it, i: [list(it)], "glom")

    def keys(self) -> "RDD":
        return self.map(lambda kv: kv[0])

    def values(self) -> "RDD":
        return self.map(lambda kv: kv[1])

    def mapValues(self, f) -> "RDD":
        return self.map(lambda kv: (kv[0], f(kv[1])))

    def flatMapValues(self, f) -> "RDD":
        return self.flatMap(lambda kv: [(kv[0], v) for v in f(kv[1])])

    def keyBy(self, f) -> "RDD":
        return self.map(lambda x: (f(x), x))

    def sample(self, withReplacement, fraction, seed=None) -> "RDD":
        seed = 17 if seed is None else seed

        def samp(it, i):
            r = _random.Random(seed * 7919 + i)
            if withReplacement:
                out = []
                for x in it:
                    k = 0
                    # Poisson(fraction) draws
                    import math
                    L, p = math.exp(-fraction), 1.0
                    while True:
                        p *= r.random()
                        if p <= L:
                            break
                        k += 1
                    out += [x] * k
                return out
            return [x for x in it if r.random() < fraction]
        return self._derive(samp, "sample")

    def union(self, other: "RDD") -> "RDD":
        a, b, na = self._part_fn(), other._part_fn(), self._n
        return RDD(self._session, self._n + other._n, lambda i: a(i) if i < na else b(i - na), "union")

    def zipWithIndex(self) -> "RDD":
        counts = self._run(lambda i, f=self._part_fn(): len(list(f(i))))
        offs = list(itertools.accumulate([0] + counts[:-1]))
        return self._derive(lambda it, i: [(x, offs[i] + j) for j, x in enumerate(it)], "zipWithIndex")

    def coalesce(self, numPartitions, shuffle=False) -> "RDD":
        if shuffle:
            return self.repartition(numPartitions)
        n = max(1, min(int(numPartitions), self._n))
        src, m = self._part_fn(), self._n
        groups = [list(range(m))[k::n] for k in range(n)]
        groups = [sorted(g) for g in groups]
        return RDD(self._session, n, lambda i: [x for j in groups[i] for x in src(j)], "coalesce")

    # ------------------------------------------------------------------ wide -------------
    def _shuffle(self, n: int, key: Callable[[Any], Any], combine=None) -> List[list]:
        """Map stage: bucket each partition by hash(key) into n lists (optionally combined)."""
        src = self._part_fn()

        def bucket(i):
            out = [[] for _ in range(n)]
            for x in src(i):
                out[_portable_hash(key(x)) % n].append(x)
            if combine is not None:
                out = [combine(b) for b in out]
            return out
        return self._run(bucket)

    def partitionBy(self, numPartitions, partitionFunc=_portable_hash) -> "RDD":
        pieces = self._shuffle(int(numPartitions), lambda kv: kv[0])
        return RDD(self._session, numPartitions, lambda j: [x for p in pieces for x in p[j]], "partitionBy")

    def repartition(self, numPartitions) -> "RDD":
        n = int(numPartitions)
        src = self._part_fn()
        pieces = self._run(lambda i: [[x for k, x in enumerate(src(i)) if (k + i) % n == j] for j in range(n)])
        return RDD(self._session, n, lambda j: [x for p in pieces for x in p[j]], "repartition")

    def reduceByKey(self, func, numPartitions=None) -> "RDD":
        n = int(numPartitions or self._n)

        def combine(b):
            acc = {}
            for k, v in b:
                acc[k] = func(acc[k], v) if k in acc else v
            return list(acc.items())
        pieces = self._shuffle(n, lambda kv: kv[0], combine)
        return RDD(self._session, n, lambda j: combine([x for p in pieces for x in p[j]]), "reduceByKey")

    def groupByKey(self, numPartitions=None) -> "RDD":
        n = int(numPartitions or self._n)
        pieces = self._shuffle(n, lambda kv: kv[0])

        def group(j):
            acc = {}
            for p in pieces:
                for k, v in p[j]:
                    acc.setdefault(k, []).append(v)
            return list(acc.items())
        return RDD(self._session, n, group, "groupByKey")

    def distinct(self, numPartitions=None) -> "RDD":
        n = int(numPartitions or self._n)
        pieces = self._shuffle(n, lambda x: x, lambda b: list(dict.fromkeys(b)))
        return RDD(self._session, n, lambda j: list(dict.fromkeys(x for p in pieces for x in p[j])), "distinct")

    def sortBy(self, keyfunc, ascending=True, numPartitions=None) -> "RDD":
        allx = sorted(self.collect(), key=keyfunc, reverse=not ascending)
        n = int(numPartitions or self._n)
        return self._session.sparkContext.parallelize(allx, n)

    def sortByKey(self, ascending=True, numPartitions=None, keyfunc=lambda k: k) -> "RDD":
        return self.sortBy(lambda kv: keyfunc(kv[0]), ascending, numPartitions)

    # ------------------------------------------------------------------ actions ----------
    def collect(self) -> list:
        f = self._part_fn()
        return [x for part in self._run(lambda i: list(f(i))) for x in part]

    def count(self) -> int:
        f = self._part_fn()
        return int(sum(self._run(lambda i: sum(1 for _ in f(i)))))

    def take(self, num: int) -> list:
        out = []
        f = self._part_fn()
        for i in range(self._n):
            if len(out) >= num:
                break
            out += list(itertools.islice(iter(f(i)), num - len(out)))
        return out

    def first(self):
        r = self.take(1)
        if not r:
            raise ValueError("RDD is empty")
        return r[0]

    def reduce(self, f):
        g = self._part_fn()

        def red(i):
            it = iter(g(i))
            try:
                acc = next(it)
            except StopIteration:
                return ("empty",)
            for x in it:
                acc = f(acc, x)
            return ("ok", acc)
        vals = [r[1] for r in self._run(red) if r[0] == "ok"]
        if not vals:
            raise ValueError("Can not reduce() empty RDD")
        acc = vals[0]
        for v in vals[1:]:
            acc = f(acc, v)
        return acc

    def fold(self, zeroValue, op):
        g = self._part_fn()

        def fo(i):
            acc = zeroValue
            for x in g(i):
                acc = op(acc, x)
            return acc
        acc = zeroValue
        for v in self._run(fo):
            acc = op(acc, v)
        return acc

    def sum(self):
        return self.fold(0, lambda a, b: a + b)

    def max(self):
        return self.reduce(lambda a, b: a if a >= b else b)

    def min(self):
        return self.reduce(lambda a, b: a if a <= b else b)

    def mean(self):
        s, c = self.map(lambda x: (x, 1)).reduce(lambda a, b: (a[0] + b[0], a[1] + b[1]))
        return s / c

    def foreach(self, f):
        g = self._part_fn()
        self._run(lambda i: [f(x) for x in g(i)] and None)

    def foreachPartition(self, f):
        g = self._part_fn()
        self._run(lambda i: f(iter(g(i))))

    def countByKey(self):
        return dict(self.map(lambda kv: (kv[0], 1)).reduceByKey(lambda a, b: a + b).collect())

    def collectAsMap(self):
        return dict(self.collect())

    def isEmpty(self):
        return len(self.take(1)) == 0

    # ------------------------------------------------------------------ caching ----------
    def persist(self, storageLevel=None) -> "RDD":
        if self._cached is None:
            f = self._compute
            self._cached = self._run(lambda i: list(f(i)))
        return self

    def cache(self) -> "RDD":
        return self.persist()

    def unpersist(self, blocking=False) -> "RDD":
        self._cached = None
        return self

    @property
    def is_cached(self):
        return self._cached is not None

    # ------------------------------------------------------------------ to DataFrame -----
    def toDF(self, schema=None, sampleRatio=None):
        return self._session.createDataFrame(self, schema)

    def __repr__(self):
        return f"{self._name} RDD[{self._id}] ({self._n} partitions)"

    def __getstate__(self):
        # tasks carry compute functions, never the driver's session
        st = dict(self.__dict__)
        st["_session"] = None
        return st


class RDDSource:
    """DataFrame source over an RDD of rows: each partition becomes one Arrow table."""

    def __init__(self, rdd: RDD, schema, to_table: Callable[[list, Any], pa.Table]):
        self.rdd = rdd
        self.n = rdd._n
        self.f = rdd._part_fn()
        self.to_table = to_table
        self.user_schema = schema
        self._schema: Optional[pa.Schema] = None

    def num_partitions(self):
        return self.n

    def __getstate__(self):
        st = dict(self.__dict__)
        st["rdd"] = None
        return st

    def load(self, i):
        rows = list(self.f(i))
        t = self.to_table(rows, self.user_schema if self._schema is None else self._schema)
        if self._schema is not None and t.schema != self._schema:
            t = t.cast(self._schema)
        return t

    def schema(self):
        if self._schema is None:
            sample = self.rdd.take(100)
            t = self.to_table(sample, self.user_schema)
            self._schema = t.schema
        return self._schema
