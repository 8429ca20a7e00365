"""Native small-file CSV inference (``csrc/exec/csv_infer.cc``): whenever it answers, the table
must equal pyarrow's ``read_csv`` with the engine's options (type inference, null token "" only)
-- schema, values, nulls and NaN bits -- over random files mixing ints, reals, text, quoting,
nulls and the values it must refuse (booleans, dates, timestamps, NaN words, hex, whitespace)."""
import random

import pyarrow as pa
import pyarrow.csv as pacsv
import pytest

from raydp_amd.spark import native_exec

pa.lib.have_signal_refcycle = False


def _arrow(data: bytes, sep=","):
    return pacsv.read_csv(pa.BufferReader(pa.py_buffer(data)),
                          read_options=pacsv.ReadOptions(use_threads=False),
                          parse_options=pacsv.ParseOptions(delimiter=sep),
                          convert_options=pacsv.ConvertOptions(strings_can_be_null=True, null_values=[""]))


def _same(a: pa.Table, b: pa.Table):
    assert a.schema == b.schema, (a.schema, b.schema)
    for x, y in zip(a.columns, b.columns):
        x, y = x.combine_chunks(), y.combine_chunks()
        if pa.types.is_floating(x.type):
            assert x.is_null().equals(y.is_null())
            xs = x.to_numpy(zero_copy_only=False)
            ys = y.to_numpy(zero_copy_only=False)
            assert xs.tobytes() == ys.tobytes()
        else:
            assert x.equals(y)


def _value(rng, kind):
    if kind == "int":
        return str(rng.choice([0, 7, -3, 123456789, -2 ** 40, 10 ** 17]) + rng.randint(-5, 5))
    if kind == "real":
        return rng.choice([repr(rng.uniform(-1e3, 1e3)), f"{rng.uniform(-5, 5):.3f}", "1e5", "-2.5E-3",
                           "0.1", "123.000", "-0.0", repr(rng.gauss(0, 1e-300))])
    if kind == "text":
        return rng.choice(["fake_key", "abc def", "2014-04-02 09:20:27 UTC", "N/A", "NULL", "x1", "hello-world",
                           "a:b", "1/2/2020", "e", "1e"])
    if kind == "odd":
        return rng.choice(["true", "False", "nan", "-inf", "2020-01-02", "2020-01-02 03:04:05", "12:30",
                           "0x1F", "+5", " 7", "8 ", "1.", ".5", "TRUE", "Infinity"])
    if kind == "null":
        return ""
    raise AssertionError(kind)


def _file(rng, ncol, nrow, kinds, quote_p=0.2, sep=","):
    names = [f"c{i}" for i in range(ncol)]
    lines = [sep.join(f'"{n}"' if rng.random() < 0.5 else n for n in names)]
    for _ in range(nrow):
        vals = []
        for c in range(ncol):
            k = kinds[c] if rng.random() > 0.1 else rng.choice(["null", kinds[c]])
            if kinds[c] == "mix" or k == "mix":
                k = rng.choice(["int", "real"])
            v = _value(rng, k)
            if v and rng.random() < quote_p:
                v = f'"{v}"'
            vals.append(v)
        lines.append(sep.join(vals))
    return ("\n".join(lines) + ("\n" if rng.random() < 0.8 else "")).encode()


@pytest.mark.parametrize("seed", range(40))
def test_native_csv_inference_matches_arrow(seed):
    rng = random.Random(seed)
    ncol = rng.randint(1, 6)
    kinds = [rng.choice(["int", "real", "text", "mix", "odd", "text"]) for _ in range(ncol)]
    sep = rng.choice([",", ",", "\t", ";"])
    data = _file(rng, ncol, rng.randint(1, 300), kinds, sep=sep)
    got = native_exec.read_csv_infer(data, sep)
    try:
        want = _arrow(data, sep)
    except pa.ArrowInvalid:
        assert got is None
        return
    if got is not None:
        _same(got, want)
    if "odd" not in kinds:
        assert got is not None or any(k == "text" for k in kinds), kinds


def test_nyc_shaped_file_is_read_natively(tmp_path):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    p = str(tmp_path / "n.csv")
    bench.make_csv(p, 1280, 3)
    data = open(p, "rb").read()
    got = native_exec.read_csv_infer(data)
    assert got is not None
    _same(got, _arrow(data))


@pytest.mark.parametrize("data", [
    b"a,b\n1,2\n3\n",                 # ragged
    b'a,b\n"1,2",3\n',                 # delimiter inside quotes (handled)
    b'a\n"x""y"\n',                    # escaped quote
    b"a,b\r\n1,2\r\n",                 # CRLF
    b"a\n\n\n",                        # header only (after empty lines)
    b"a,b\n,\n,\n",                    # all-null columns
    "a\ncafé\n".encode(),         # non-ASCII
    b"a\nabc\n\xff\xfe\n",            # invalid UTF-8 AFTER the first text value (Arrow: binary)
    "a,b\nabc,1\ncafé,2\n".encode(),  # valid non-ASCII after the first text value
])
def test_edge_inputs_fall_back_or_match(data):
    got = native_exec.read_csv_infer(data)
    try:
        want = _arrow(data)
    except pa.ArrowInvalid:
        assert got is None
        return
    if got is not None:
        _same(got, want)


def test_sources_use_the_native_reader(tmp_path):
    import pyarrow as pa
    from raydp_amd.spark import sources
    p = tmp_path / "x.csv"
    p.write_bytes(b"k,x,y,s\n1,2.5,3,a\n2,,4,\n3,1e3,-5,c\n")
    src = sources.CsvSource(str(p), header=True, infer_schema=True)
    assert src._schema.names == ["k", "x", "y", "s"]
    assert src._schema.field("k").type == pa.int32() and src._schema.field("x").type == pa.float64()
    assert src.load(0).column("x").to_pylist() == [2.5, None, 1000.0]
    assert native_exec.STATS["native_csv_reads"] >= 1


@pytest.mark.parametrize("seed", range(6))
def test_short_mantissa_reals_are_bit_exact(seed):
    """Reals the exact fast path decides (mantissa < 2^53, |decimal exponent| <= 22) and the
    ones just outside it (17-digit mantissas, 2^53 +- 1, exponents 22 / 23) -- bit for bit
    against Arrow's parser, on a file wide enough for the threaded column pass."""
    rng = random.Random(seed)
    pool = ["9007199254740992", "9007199254740993", "9007199254740991.5", "1e22", "1e23", "1.5e-22",
            "4.9e-23", "123456789012345678.5", "0.000000000000000000001", "-0.0", "0.30000000000000004"]

    def val():
        r = rng.random()
        if r < 0.25:
            return rng.choice(pool)
        if r < 0.6:
            return f"{rng.uniform(-1e4, 1e4):.{rng.randint(1, 9)}f}"
        if r < 0.8:
            return f"{rng.randint(1, 99999)}e{rng.choice(['-', ''])}{rng.randint(0, 25)}"
        return repr(rng.uniform(-180, 180))
    ncol, nrow = 8, 1500
    lines = [",".join(f"c{i}" for i in range(ncol))]
    lines += [",".join(val() for _ in range(ncol)) for _ in range(nrow)]
    data = ("\n".join(lines) + "\n").encode()
    got = native_exec.read_csv_infer(data)
    assert got is not None
    _same(got, _arrow(data))
