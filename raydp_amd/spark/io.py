"""``DataFrameReader`` / ``DataFrameWriter`` (csv, parquet, json).

The writer produces Spark's directory layout (``part-00000-<uuid>.snappy.parquet`` files plus a
``_SUCCESS`` marker) so ``read_spark_parquet`` and other Spark-aware readers skip the marker
files (reference: ``python/raydp/spark/dataset.py:316-320``, ``tests/test_read_parquet.py``).
"""
import os
import shutil
import uuid

import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.parquet as pq

from raydp_amd.spark import plan as P
from raydp_amd.spark.sources import CsvSource, JsonSource, ParquetSource, TextSource


def _local(path: str) -> str:
    return path[len("file://"):] if path.startswith("file://") else path


class DataFrameReader:
    def __init__(self, session):
        self._session = session
        self._format = "parquet"
        self._options = {}
        self._schema = None

    def format(self, source):
        self._format = source.lower()
        return self

    def option(self, key, value):
        self._options[key.lower()] = value
        return self

    def options(self, **opts):
        for k, v in opts.items():
            self.option(k, v)
        return self

    def schema(self, schema):
        self._schema = schema
        return self

    def _flag(self, key, default=False):
        v = self._options.get(key, default)
        return v if isinstance(v, bool) else str(v).lower() == "true"

    def load(self, path=None, format=None, schema=None, **opts):  # noqa: A002
        if format:
            self._format = format.lower()
        if schema is not None:
            self._schema = schema
        for k, v in opts.items():
            self.option(k, v)
        fmt = self._format
        if fmt == "csv":
            return self.csv(path)
        if fmt == "parquet":
            return self.parquet(path)
        if fmt == "json":
            return self.json(path)
        if fmt == "text":
            return self.text(path)
        raise ValueError(f"unsupported format {fmt}")

    def csv(self, path, schema=None, sep=None, header=None, inferSchema=None, **kw):
        from raydp_amd.spark.dataframe import DataFrame
        from raydp_amd.spark.session import _to_arrow_schema
        if header is not None:
            self.option("header", header)
        if inferSchema is not None:
            self.option("inferschema", inferSchema)
        if sep is not None:
            self.option("sep", sep)
        schema = schema or self._schema
        mpb = int(self._session.conf.get("spark.sql.files.maxPartitionBytes", str(128 << 20)))
        src = CsvSource(path, header=self._flag("header"), infer_schema=self._flag("inferschema"),
                        sep=self._options.get("sep", self._options.get("delimiter", ",")),
                        schema=_to_arrow_schema(schema) if schema is not None else None,
                        max_partition_bytes=mpb, null_value=self._options.get("nullvalue"),
                        parallelism=self._session._default_parallelism(),
                        open_cost_bytes=int(self._session.conf.get(
                            "spark.sql.files.openCostInBytes", str(4 << 20))))
        return DataFrame(P.SourcePlan(src), self._session)

    def text(self, paths, wholetext: bool = False, lineSep=None):
        """``spark.read.text``: a DataFrame with one string column ``value``, one row per line
        (``wholetext=True``: one row per file)."""
        from raydp_amd.spark.dataframe import DataFrame
        if lineSep not in (None, "\n"):
            raise ValueError("text: only newline-separated lines are supported")
        mpb = int(self._session.conf.get("spark.sql.files.maxPartitionBytes", str(128 << 20)))
        src = TextSource(paths if isinstance(paths, (str, list, tuple)) else str(paths), max_partition_bytes=mpb,
                         parallelism=self._session._default_parallelism(), wholetext=wholetext)
        return DataFrame(P.SourcePlan(src), self._session)

    def parquet(self, *paths):
        from raydp_amd.spark.dataframe import DataFrame
        src = ParquetSource(list(paths) if len(paths) > 1 else paths[0])
        return DataFrame(P.SourcePlan(src), self._session)

    def json(self, path):
        from raydp_amd.spark.dataframe import DataFrame
        return DataFrame(P.SourcePlan(JsonSource(path)), self._session)


class DataFrameWriter:
    def __init__(self, df):
        self._df = df
        self._mode = "errorifexists"
        self._format = "parquet"
        self._options = {}
        self._partition_by = None

    def mode(self, saveMode):
        self._mode = (saveMode or "errorifexists").lower()
        return self

    def format(self, source):
        self._format = source.lower()
        return self

    def option(self, key, value):
        self._options[key.lower()] = value
        return self

    def options(self, **kw):
        for k, v in kw.items():
            self.option(k, v)
        return self

    def partitionBy(self, *cols):
        self._partition_by = list(cols)
        return self

    def _prepare_dir(self, path):
        path = _local(path)
        if os.path.exists(path):
            if self._mode in ("overwrite",):
                shutil.rmtree(path) if os.path.isdir(path) else os.remove(path)
            elif self._mode in ("ignore",):
                return None
            elif self._mode in ("append",):
                pass
            else:
                raise FileExistsError(f"path {path} already exists.")
        os.makedirs(path, exist_ok=True)
        return path

    def save(self, path, format=None, mode=None, **kw):  # noqa: A002
        if format:
            self._format = format
        if mode:
            self.mode(mode)
        getattr(self, self._format)(path, **kw)

    def parquet(self, path, mode=None, partitionBy=None, compression=None):
        if mode:
            self.mode(mode)
        d = self._prepare_dir(path)
        if d is None:
            return
        codec = compression or self._options.get("compression", "snappy")
        codec = "none" if codec in (None, "none", "uncompressed") else codec
        job = uuid.uuid4()
        session = self._df._session

        def write(t, i):
            ext = "" if codec == "none" else f".{codec}"
            pq.write_table(t, os.path.join(d, f"part-{i:05d}-{job}-c000{ext}.parquet"),
                           compression=codec)
            return pa.table({"n": [t.num_rows]})
        session._run(P.MapPlan(self._df._src(), write, "writeParquet"))
        open(os.path.join(d, "_SUCCESS"), "w").close()

    def csv(self, path, mode=None, header=None, sep=","):
        if mode:
            self.mode(mode)
        d = self._prepare_dir(path)
        if d is None:
            return
        hdr = header if header is not None else str(self._options.get("header", "false")).lower() == "true"
        job = uuid.uuid4()

        def write(t, i):
            pacsv.write_csv(t, os.path.join(d, f"part-{i:05d}-{job}-c000.csv"),
                            write_options=pacsv.WriteOptions(include_header=bool(hdr), delimiter=sep))
            return pa.table({"n": [t.num_rows]})
        self._df._session._run(P.MapPlan(self._df._src(), write, "writeCsv"))
        open(os.path.join(d, "_SUCCESS"), "w").close()

    def json(self, path, mode=None):
        if mode:
            self.mode(mode)
        d = self._prepare_dir(path)
        if d is None:
            return
        import json as _json
        job = uuid.uuid4()

        def write(t, i):
            with open(os.path.join(d, f"part-{i:05d}-{job}-c000.json"), "w") as fh:
                for row in t.to_pylist():
                    fh.write(_json.dumps(row, default=str) + "\n")
            return pa.table({"n": [t.num_rows]})
        self._df._session._run(P.MapPlan(self._df._src(), write, "writeJson"))
        open(os.path.join(d, "_SUCCESS"), "w").close()

    def saveAsTable(self, name, format=None, mode=None, **kw):  # noqa: A002
        """Persist as a parquet table of the session's warehouse (``spark.sql.warehouse.dir``);
        ``spark.table(name)`` / ``spark.sql("select ... from name")`` read it back, from this
        session or a later one."""
        from raydp_amd.spark.sql import save_as_table
        if format and format.lower() != "parquet":
            raise NotImplementedError("saveAsTable stores parquet tables")
        save_as_table(self._df._session, name, self._df, mode or self._mode)

    def insertInto(self, tableName, overwrite=False):
        from raydp_amd.spark.sql import _catalog
        _catalog(self._df._session).save(tableName, self._df, "overwrite" if overwrite else "append")
