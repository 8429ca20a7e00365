"""Spark SQL data types mapped 1:1 onto Arrow types.

The engine stores every column as Arrow; these classes exist so user code written against
``pyspark.sql.types`` (``StructType``, ``IntegerType()``, ``"int"`` type strings in ``@udf``)
keeps working. Parity: the reference builds ``StructType`` from Arrow schemas in
``python/raydp/spark/dataset.py:298-305`` (``from_arrow_type``).
"""
from typing import List, Optional

import pyarrow as pa


class DataType:
    arrow: pa.DataType = None
    simple: str = None

    def __eq__(self, other):
        return type(self) is type(other) and self.to_arrow() == other.to_arrow()

    def __hash__(self):
        return hash(str(self.to_arrow()))

    def __repr__(self):
        return f"{type(self).__name__}()"

    def to_arrow(self) -> pa.DataType:
        return self.arrow

    def simpleString(self) -> str:
        return self.simple

    def typeName(self) -> str:
        return self.simple


class NullType(DataType):
    arrow, simple = pa.null(), "void"


class StringType(DataType):
    arrow, simple = pa.string(), "string"


class BinaryType(DataType):
    arrow, simple = pa.binary(), "binary"


class BooleanType(DataType):
    arrow, simple = pa.bool_(), "boolean"


class ByteType(DataType):
    arrow, simple = pa.int8(), "tinyint"


class ShortType(DataType):
    arrow, simple = pa.int16(), "smallint"


class IntegerType(DataType):
    arrow, simple = pa.int32(), "int"


class LongType(DataType):
    arrow, simple = pa.int64(), "bigint"


class FloatType(DataType):
    arrow, simple = pa.float32(), "float"


class DoubleType(DataType):
    arrow, simple = pa.float64(), "double"


class DateType(DataType):
    arrow, simple = pa.date32(), "date"


class TimestampType(DataType):
    arrow, simple = pa.timestamp("us"), "timestamp"


class DecimalType(DataType):
    def __init__(self, precision=10, scale=0):
        self.precision, self.scale = precision, scale
        self.arrow = pa.decimal128(precision, scale)
        self.simple = f"decimal({precision},{scale})"


class ArrayType(DataType):
    def __init__(self, elementType: DataType, containsNull: bool = True):
        self.elementType = elementType
        self.containsNull = containsNull
        self.arrow = pa.list_(elementType.to_arrow())
        self.simple = f"array<{elementType.simpleString()}>"

    def __repr__(self):
        return f"ArrayType({self.elementType!r})"


class MapType(DataType):
    def __init__(self, keyType: DataType, valueType: DataType, valueContainsNull=True):
        self.keyType, self.valueType = keyType, valueType
        self.arrow = pa.map_(keyType.to_arrow(), valueType.to_arrow())
        self.simple = f"map<{keyType.simpleString()},{valueType.simpleString()}>"


class StructField:
    def __init__(self, name: str, dataType: DataType, nullable: bool = True, metadata=None):
        self.name, self.dataType, self.nullable = name, dataType, nullable
        self.metadata = metadata or {}

    def __repr__(self):
        return f"StructField('{self.name}', {self.dataType!r}, {self.nullable})"

    def __eq__(self, other):
        return (isinstance(other, StructField) and self.name == other.name
                and self.dataType == other.dataType and self.nullable == other.nullable)

    def simpleString(self):
        return f"{self.name}:{self.dataType.simpleString()}"


class StructType(DataType):
    def __init__(self, fields: Optional[List[StructField]] = None):
        self.fields: List[StructField] = list(fields or [])

    def add(self, field, data_type=None, nullable=True, metadata=None):
        if isinstance(field, StructField):
            self.fields.append(field)
        else:
            if isinstance(data_type, str):
                data_type = parse_type_string(data_type)
            self.fields.append(StructField(field, data_type, nullable, metadata))
        return self

    @property
    def names(self):
        return [f.name for f in self.fields]

    def fieldNames(self):
        return self.names

    def __iter__(self):
        return iter(self.fields)

    def __len__(self):
        return len(self.fields)

    def __getitem__(self, key):
        if isinstance(key, int):
            return self.fields[key]
        for f in self.fields:
            if f.name == key:
                return f
        raise KeyError(key)

    def __eq__(self, other):
        return isinstance(other, StructType) and self.fields == other.fields

    def __hash__(self):
        return hash(tuple(f.name for f in self.fields))

    def __repr__(self):
        return f"StructType([{', '.join(repr(f) for f in self.fields)}])"

    def to_arrow(self) -> pa.Schema:
        return pa.schema([pa.field(f.name, f.dataType.to_arrow(), f.nullable) for f in self.fields])

    def simpleString(self):
        return "struct<" + ",".join(f.simpleString() for f in self.fields) + ">"

    def json(self):
        import json
        return json.dumps({"type": "struct", "fields": [
            {"name": f.name, "type": f.dataType.simpleString(), "nullable": f.nullable,
             "metadata": f.metadata} for f in self.fields]})


_SIMPLE = {
    "string": StringType, "str": StringType, "varchar": StringType, "binary": BinaryType,
    "boolean": BooleanType, "bool": BooleanType, "tinyint": ByteType, "byte": ByteType,
    "smallint": ShortType, "short": ShortType, "int": IntegerType, "integer": IntegerType,
    "bigint": LongType, "long": LongType, "float": FloatType, "real": FloatType,
    "double": DoubleType, "date": DateType, "timestamp": TimestampType, "void": NullType,
}


def parse_type_string(s) -> DataType:
    """Parse a Spark DDL type string (``"int"``, ``"array<float>"``) or pass a DataType."""
    if isinstance(s, DataType):
        return s
    t = str(s).strip().lower()
    if t in _SIMPLE:
        return _SIMPLE[t]()
    if t.startswith("array<") and t.endswith(">"):
        return ArrayType(parse_type_string(t[6:-1]))
    if t.startswith("decimal"):
        inner = t[t.find("(") + 1:t.find(")")] if "(" in t else "10,0"
        p, sc = (int(x) for x in inner.split(","))
        return DecimalType(p, sc)
    raise ValueError(f"unsupported type string: {s!r}")


def from_arrow_type(t: pa.DataType) -> DataType:
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        return StringType()
    if pa.types.is_boolean(t):
        return BooleanType()
    if pa.types.is_int8(t):
        return ByteType()
    if pa.types.is_int16(t):
        return ShortType()
    if pa.types.is_int32(t) or pa.types.is_uint16(t) or pa.types.is_uint8(t):
        return IntegerType()
    if pa.types.is_integer(t):
        return LongType()
    if pa.types.is_float32(t) or pa.types.is_float16(t):
        return FloatType()
    if pa.types.is_float64(t):
        return DoubleType()
    if pa.types.is_date(t):
        return DateType()
    if pa.types.is_timestamp(t):
        return TimestampType()
    if pa.types.is_binary(t) or pa.types.is_large_binary(t):
        return BinaryType()
    if pa.types.is_decimal(t):
        return DecimalType(t.precision, t.scale)
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        return ArrayType(from_arrow_type(t.value_type))
    if pa.types.is_null(t):
        return NullType()
    if pa.types.is_map(t):
        return MapType(from_arrow_type(t.key_type), from_arrow_type(t.item_type))
    raise TypeError(f"unsupported arrow type {t}")


def from_arrow_schema(schema: pa.Schema) -> StructType:
    return StructType([StructField(f.name, from_arrow_type(f.type), f.nullable) for f in schema])


def to_arrow_type(dt) -> pa.DataType:
    return parse_type_string(dt).to_arrow()
