"""``pyspark.sql.Row``: a tuple with field-name access."""


class Row(tuple):
    def __new__(cls, *args, **kwargs):
        if args and kwargs:
            raise ValueError("Can not use both args and kwargs to create Row")
        if kwargs:
            row = tuple.__new__(cls, list(kwargs.values()))
            row.__fields__ = list(kwargs.keys())
            return row
        row = tuple.__new__(cls, args)
        row.__fields__ = None
        return row

    @classmethod
    def _make(cls, fields, values):
        row = tuple.__new__(cls, values)
        row.__fields__ = list(fields)
        return row

    def asDict(self, recursive=False):
        if self.__fields__ is None:
            raise TypeError("Cannot convert a Row class into dict")
        return dict(zip(self.__fields__, self))

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        try:
            idx = self.__fields__.index(item)
        except (ValueError, AttributeError, TypeError):
            raise AttributeError(item)
        return self[idx]

    def __getitem__(self, item):
        if isinstance(item, str):
            return tuple.__getitem__(self, self.__fields__.index(item))
        return tuple.__getitem__(self, item)

    def __contains__(self, item):
        return self.__fields__ is not None and item in self.__fields__

    def __reduce__(self):
        return (Row._make, (self.__fields__, tuple(self)))

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"
