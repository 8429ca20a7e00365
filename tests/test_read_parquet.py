"""read_spark_parquet over a Spark-written directory (port of tests/test_read_parquet.py):
part files plus _SUCCESS / .crc side files must be skipped."""
from raydp.spark.dataset import read_spark_parquet


def test_read_spark_parquet(spark_on_ray_small, tmp_path):
    spark = spark_on_ray_small
    output_dir = str(tmp_path / "parquet_out")
    data = [("James", "", "Smith", "36636", "M", 3000), ("Michael", "Rose", "", "40288", "M", 4000),
            ("Robert", "", "Williams", "42114", "M", 4000), ("Maria", "Anne", "Jones", "39192", "F", 4000),
            ("Jen", "Mary", "Brown", "", "F", -1)]
    columns = ["firstname", "middlename", "lastname", "dob", "gender", "salary"]
    spark_df = spark.createDataFrame(data, schema=columns)
    spark_df.write.mode("overwrite").parquet(output_dir)
    import os
    open(os.path.join(output_dir, ".part-00000.crc"), "w").write("x")
    ds = read_spark_parquet(path=str(output_dir))
    assert ds.count() == len(data)
    assert sorted(r["firstname"] for r in ds.take(10)) == sorted(d[0] for d in data)
