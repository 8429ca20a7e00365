import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def runtime_local():
    from raydp_amd import runtime
    runtime.shutdown()
    runtime.init(num_cpus=6)
    yield
    from raydp_amd import context
    context.stop_spark()
    runtime.shutdown()


@pytest.fixture
def spark_on_ray_small(runtime_local):
    import raydp_amd
    spark = raydp_amd.init_spark("test", 1, 1, "500M")
    yield spark
    raydp_amd.stop_spark()


@pytest.fixture
def spark_on_ray_2_executors(runtime_local):
    import raydp_amd
    spark = raydp_amd.init_spark("test2", 2, 1, "500M")
    yield spark
    raydp_amd.stop_spark()


@pytest.fixture
def spark_session():
    from raydp_amd.spark import SparkSession
    s = SparkSession.builder.master("local[2]").appName("RayDP test").getOrCreate()
    yield s
    s.stop()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False
