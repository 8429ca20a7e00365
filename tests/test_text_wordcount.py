"""``spark.read.text`` and the word count of BASELINE.json config 1 ("raydp.init_spark local
word_count + ray.data.from_spark on CPU"), against a plain Python count."""
import collections

import pytest

from raydp_amd.spark import functions as F


@pytest.fixture
def text_file(tmp_path):
    words = ["ray", "spark", "arrow", "mi355x", "xgmi", "hbm", "lds", "mfma"]
    lines = [" ".join(words[(i * 7 + j * 3) % len(words)] for j in range(1 + i % 9)) for i in range(5000)]
    p = tmp_path / "words.txt"
    p.write_text("\n".join(lines) + "\n")
    return str(p), lines


def test_read_text_lines(spark_session, text_file):
    path, lines = text_file
    df = spark_session.read.text(path)
    assert df.columns == ["value"]
    assert [r[0] for r in df.collect()] == lines
    assert spark_session.read.format("text").load(path).count() == len(lines)
    whole = spark_session.read.text(path, wholetext=True).collect()
    assert len(whole) == 1 and whole[0][0].count("\n") == len(lines)


def test_word_count_through_from_spark(spark_session, text_file):
    from raydp_amd.spark.dataset import spark_dataframe_to_ray_dataset
    path, lines = text_file
    spark_session.conf.set("spark.sql.files.maxPartitionBytes", "4096")   # several line-aligned splits
    df = spark_session.read.text(path)
    counts = df.select(F.explode(F.split(F.col("value"), " ")).alias("word")).groupBy("word").count()
    ds = spark_dataframe_to_ray_dataset(counts)
    got = {r["word"]: r["count"] for r in ds.take_all()}
    want = collections.Counter(w for ln in lines for w in ln.split(" "))
    assert got == dict(want)
