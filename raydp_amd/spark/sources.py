"""Partitioned data sources: in-memory Arrow, ``range``, CSV byte-splits, Parquet files.

CSV follows Spark's file-split model: each file is cut into ``spark.sql.files.maxPartitionBytes``
byte ranges aligned to line boundaries, and every split is parsed independently by Arrow's
multi-threaded C++ CSV reader with the schema inferred once from the head of the first file
(``inferSchema=true``) so all partitions agree on column types.
"""
import glob
import io
import os
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.parquet as pq

# pyarrow's read_csv installs a SignalStopHandler whose constructor, on Python 3.10, works
# around bpo-42248 with gc.get_referrers() -- a walk over the WHOLE heap on every call (3.3 ms
# per CSV block read with a 300k-object heap vs 0.27 ms without). The cycle it breaks is
# collected by the GC anyway, so the engine's CSV reads skip the walk.
if getattr(pa.lib, "have_signal_refcycle", False):
    pa.lib.have_signal_refcycle = False


class Source:
    def preferred_node(self, i: int):
        """Node id whose store holds partition ``i``'s input (locality hint), or None."""
        return None

    def num_partitions(self) -> int:
        raise NotImplementedError

    def load(self, i: int) -> pa.Table:
        raise NotImplementedError

    def schema(self) -> pa.Schema:
        raise NotImplementedError


class TableSource(Source):
    def __init__(self, tables: List[pa.Table], schema: Optional[pa.Schema] = None):
        self.tables = tables
        self._schema = schema if schema is not None else (tables[0].schema if tables else pa.schema([]))

    def num_partitions(self):
        return len(self.tables)

    def load(self, i):
        return self.tables[i]

    def schema(self):
        return self._schema


def split_table(t: pa.Table, n: int) -> List[pa.Table]:
    n = max(1, int(n))
    bounds = np.linspace(0, t.num_rows, n + 1).astype(np.int64)
    return [t.slice(int(bounds[j]), int(bounds[j + 1] - bounds[j])) for j in range(n)]


class RangeSource(Source):
    def __init__(self, start, end, step, num_partitions):
        self.start, self.end, self.step = int(start), int(end), int(step)
        self.n = max(1, int(num_partitions))
        total = max(0, -(-(self.end - self.start) // self.step)) if self.step > 0 else \
            max(0, -(-(self.start - self.end) // -self.step))
        self.total = total
        self.bounds = np.linspace(0, total, self.n + 1).astype(np.int64)

    def num_partitions(self):
        return self.n

    def load(self, i):
        lo, hi = int(self.bounds[i]), int(self.bounds[i + 1])
        ids = self.start + np.arange(lo, hi, dtype=np.int64) * self.step
        return pa.table({"id": pa.array(ids, type=pa.int64())})

    def schema(self):
        return pa.schema([pa.field("id", pa.int64(), False)])


def _expand_paths(path) -> List[str]:
    paths = [path] if isinstance(path, str) else list(path)
    out = []
    for p in paths:
        if p.startswith("file://"):
            p = p[len("file://"):]
        if os.path.isdir(p):
            for root, _, files in os.walk(p):
                for f in sorted(files):
                    if f.startswith(("_", ".")) or f.endswith(".crc"):
                        continue
                    out.append(os.path.join(root, f))
        elif any(ch in p for ch in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    if not out:
        raise FileNotFoundError(f"Path does not exist: {path}")
    return out


def _downcast_ints(t: pa.Table) -> pa.Table:
    """Spark's CSV inference picks int for values that fit 32 bits."""
    cols = []
    changed = False
    for name, c in zip(t.column_names, t.columns):
        if pa.types.is_int64(c.type) and len(c) > 0:
            import pyarrow.compute as pc
            mm = pc.min_max(c)
            lo, hi = mm["min"].as_py(), mm["max"].as_py()
            if lo is not None and -2 ** 31 <= lo and hi < 2 ** 31:
                c = c.cast(pa.int32())
                changed = True
        cols.append(c)
    return pa.table(cols, names=t.column_names) if changed else t


def _native_infer(head: bytes, sep: str) -> Optional[pa.Table]:
    try:
        from raydp_amd.spark import native_exec
        t = native_exec.read_csv_infer(head, sep)
    except Exception:  # noqa: BLE001 - the native reader is an optimisation: pyarrow reads
        return None
    if t is not None:
        native_exec.STATS["native_csv_reads"] += 1
    return t


class CsvSource(Source):
    def __init__(self, path, header=True, infer_schema=False, sep=",", schema=None,
                 max_partition_bytes=128 * 1024 * 1024, null_value=None, parallelism=1,
                 open_cost_bytes=4 * 1024 * 1024):
        self.files = _expand_paths(path)
        self.header, self.sep = header, sep
        self.null_value = null_value
        self.splits = []
        # Spark's FilePartition sizing: maxSplitBytes = min(maxPartitionBytes,
        # max(openCostInBytes, totalBytes / defaultParallelism))
        total = sum(os.path.getsize(f) + open_cost_bytes for f in self.files)
        split_bytes = min(max_partition_bytes, max(open_cost_bytes, total // max(1, parallelism)))
        for f in self.files:
            size = os.path.getsize(f)
            nsplit = max(1, int(np.ceil(size / split_bytes)))
            if nsplit > parallelism > 1:
                # whole waves: 10 splits on 4 cores run as 4 + 4 + 2 (the last wave half idle,
                # measured 2.09 s for 10 M NYC rows, profiles/r4_datascale_10M_e1_timeline.txt);
                # 12 smaller ones run as 4 + 4 + 4. Same rows, same order, smaller splits.
                nsplit = -(-nsplit // parallelism) * parallelism
            b = np.linspace(0, size, nsplit + 1).astype(np.int64)
            for j in range(nsplit):
                self.splits.append((f, int(b[j]), int(b[j + 1])))
        self._header_line = None
        # small-file fast path: when schema inference parsed a whole single-split file, that
        # parse IS the partition (same parser, same types, same null tokens), so the task
        # ships it instead of parsing the file a second time
        self._parsed: Dict[int, pa.Table] = {}
        if schema is not None:
            self._schema = schema
        else:
            self._schema = self._infer(infer_schema)

    def _read_opts(self, column_names=None, nbytes=None):
        # Arrow's threaded reader only pays off past a few blocks
        ro = pacsv.ReadOptions(column_names=column_names, autogenerate_column_names=not self.header
                               and column_names is None,
                               use_threads=nbytes is None or nbytes > (4 << 20))
        return ro

    def _infer(self, infer):
        f = self.files[0]
        with open(f, "rb") as fh:
            head = fh.read(1 << 20)
        cut = head.rfind(b"\n")
        if cut > 0 and len(head) == (1 << 20):
            head = head[:cut + 1]
        first_nl = head.find(b"\n")
        self._header_line = head[:first_nl + 1] if self.header else b""
        # Spark's CSV null token is the empty string only ("N/A", "NULL", ... stay values)
        nulls = [self.null_value] if self.null_value else [""]
        conv = pacsv.ConvertOptions(strings_can_be_null=True, null_values=nulls) if infer else \
            pacsv.ConvertOptions(column_types=None, null_values=nulls)
        t = None
        if infer and self.header and not self.null_value:
            # one native pass that returns exactly pyarrow's inferred table, or None when the
            # bytes hold anything it does not decide (csrc/exec/csv_infer.cc)
            t = _native_infer(head, self.sep)
        if t is None:
            t = pacsv.read_csv(pa.BufferReader(pa.py_buffer(head)), read_options=self._read_opts(nbytes=len(head)),
                               parse_options=pacsv.ParseOptions(delimiter=self.sep),
                               convert_options=conv)
        if not infer:
            return pa.schema([pa.field(n, pa.string()) for n in t.column_names])
        t = _downcast_ints(t)
        fields = []
        for fld in t.schema:
            ty = fld.type
            if pa.types.is_null(ty):
                ty = pa.string()
            fields.append(pa.field(fld.name, ty))
        schema = pa.schema(fields)
        whole = len(head) == os.path.getsize(f)
        if whole and len(self.splits) == 1 and self.splits[0] == (f, 0, len(head)) and \
                self.null_value is None and t.num_rows and \
                all(a == b for a, b in zip(t.schema.types, schema.types)):
            self._parsed[0] = t.replace_schema_metadata()
        return schema

    def num_partitions(self):
        return len(self.splits)

    def schema(self):
        return self._schema

    def load(self, i):
        hit = self._parsed.get(i)
        if hit is not None:
            return hit
        f, lo, hi = self.splits[i]
        with open(f, "rb") as fh:
            header = b""
            if self.header:
                header = fh.readline()
            if lo > 0:
                fh.seek(lo - 1)
                prev = fh.read(1)
                if prev != b"\n":
                    fh.readline()  # finish the line owned by the previous split
            start = max(fh.tell(), len(header))
            if start >= hi and lo > 0:
                return self._schema.empty_table()
            fh.seek(start)
            data = fh.read(max(0, hi - start))
            if data and not data.endswith(b"\n"):
                data += fh.readline()
        names = self._schema.names
        conv = pacsv.ConvertOptions(column_types={f.name: f.type for f in self._schema},
                                    strings_can_be_null=True,
                                    null_values=[self.null_value] if self.null_value else [""])
        if not data.strip():
            return self._schema.empty_table()
        t = pacsv.read_csv(pa.BufferReader(pa.py_buffer(data)),
                           read_options=pacsv.ReadOptions(column_names=names,
                                                          use_threads=len(data) > (4 << 20),
                                                          block_size=max(1 << 20, len(data) + 1)),
                           parse_options=pacsv.ParseOptions(delimiter=self.sep),
                           convert_options=conv)
        return t


class TextSource(Source):
    """``spark.read.text``: one string column ``value``, one row per line (without the line
    terminator; a trailing ``\r`` is dropped too, as Hadoop's LineRecordReader does). Files are cut
    into line-aligned byte splits like CSV files (``CsvSource``), in whole waves of the cores."""

    def __init__(self, path, max_partition_bytes=128 * 1024 * 1024, parallelism=1, wholetext=False):
        self.files = _expand_paths(path)
        self.wholetext = wholetext
        self.splits = []
        total = sum(os.path.getsize(f) for f in self.files)
        split_bytes = max(1, min(max_partition_bytes, max(4 << 20, total // max(1, parallelism))))
        for f in self.files:
            size = os.path.getsize(f)
            if wholetext:
                self.splits.append((f, 0, size))
                continue
            nsplit = max(1, int(np.ceil(size / split_bytes)))
            if nsplit > parallelism > 1:
                nsplit = -(-nsplit // parallelism) * parallelism
            b = np.linspace(0, size, nsplit + 1).astype(np.int64)
            for j in range(nsplit):
                self.splits.append((f, int(b[j]), int(b[j + 1])))
        self._schema = pa.schema([pa.field("value", pa.string())])

    def num_partitions(self):
        return len(self.splits)

    def schema(self):
        return self._schema

    def load(self, i):
        f, lo, hi = self.splits[i]
        with open(f, "rb") as fh:
            if self.wholetext:
                return pa.table({"value": pa.array([fh.read().decode("utf-8")], pa.string())})
            if lo > 0:
                fh.seek(lo - 1)
                if fh.read(1) != b"\n":
                    fh.readline()            # the line belongs to the previous split
            start = fh.tell() if lo > 0 else 0
            if start >= hi and lo > 0:
                return self._schema.empty_table()
            fh.seek(start)
            data = fh.read(max(0, hi - start))
            if data and not data.endswith(b"\n"):
                data += fh.readline()
        if not data:
            return self._schema.empty_table()
        lines = data.split(b"\n")
        if lines and lines[-1] == b"":
            lines.pop()
        arr = pa.array([ln[:-1] if ln.endswith(b"\r") else ln for ln in lines], pa.binary())
        return pa.table({"value": arr.cast(pa.string())})


class ParquetSource(Source):
    def __init__(self, path):
        self.files = [f for f in _expand_paths(path) if not os.path.basename(f).startswith(("_", "."))]
        self._schema = pq.read_schema(self.files[0])

    def num_partitions(self):
        return len(self.files)

    def load(self, i):
        return pq.read_table(self.files[i])

    def schema(self):
        return self._schema


class JsonSource(Source):
    def __init__(self, path):
        import pyarrow.json as pj
        self.files = _expand_paths(path)
        self._pj = pj
        self._schema = pj.read_json(self.files[0]).schema

    def num_partitions(self):
        return len(self.files)

    def load(self, i):
        return self._pj.read_json(self.files[i]).cast(self._schema)

    def schema(self):
        return self._schema
