"""Application submitted with ``--py-files test_pyfile.py``: executors import the shipped
module inside a task (reference: examples/test_pyfiles_main.py)."""
import sys

import raydp


def main():
    spark = raydp.init_spark("Test PyFiles", 1, 1, "500M")
    rdd = spark.sparkContext.parallelize([1, 2, 3, 4, 5], 2)

    def per_partition(it):
        from test_pyfile import compute_sum  # shipped by --py-files, imported on the executor
        return [compute_sum(list(it))]

    total = sum(rdd.mapPartitions(per_partition).collect())
    raydp.stop_spark()
    assert total == 15, total
    print(f"py-files OK: sum from executors = {total}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
