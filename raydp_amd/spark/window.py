"""``pyspark.sql.Window`` specification (partitionBy / orderBy)."""
from raydp_amd.spark.column import Column, SortOrder, _to_expr


class WindowSpec:
    def __init__(self, partition_cols=None, order_keys=None):
        self.partition_cols = list(partition_cols or [])
        self.order_keys = list(order_keys or [])

    def partitionBy(self, *cols):
        names = []
        for c in _flatten(cols):
            names.append(c if isinstance(c, str) else c._expr.name())
        return WindowSpec(names, self.order_keys)

    def orderBy(self, *cols):
        keys = []
        for c in _flatten(cols):
            e = _to_expr(c, name_is_col=True)
            if isinstance(e, SortOrder):
                keys.append((e.child, e.ascending, e.nulls_first))
            else:
                keys.append((e, True, True))
        return WindowSpec(self.partition_cols, keys)

    def rowsBetween(self, start, end):
        return self

    def rangeBetween(self, start, end):
        return self


def _flatten(cols):
    out = []
    for c in cols:
        if isinstance(c, (list, tuple)):
            out.extend(c)
        else:
            out.append(c)
    return out


class Window:
    unboundedPreceding = -(1 << 63)
    unboundedFollowing = (1 << 63) - 1
    currentRow = 0

    @staticmethod
    def partitionBy(*cols):
        return WindowSpec().partitionBy(*cols)

    @staticmethod
    def orderBy(*cols):
        return WindowSpec().orderBy(*cols)
