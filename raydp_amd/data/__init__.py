"""Distributed Arrow datasets (Ray Data equivalent)."""
from raydp_amd.data.dataset import (Dataset, from_arrow, from_arrow_refs, from_items, from_numpy,
                                    from_pandas, from_pandas_refs, from_spark, range, read_csv,
                                    read_parquet)

__all__ = ["Dataset", "from_arrow", "from_arrow_refs", "from_items", "from_numpy", "from_pandas",
           "from_pandas_refs", "from_spark", "range", "read_csv", "read_parquet"]
