"""Typed configuration registry (raydp_amd/utils/config.py) and its C++ mirror
(csrc/common/config_keys.h). Key names follow SparkOnRayConfigs.java / SURVEY.md §5.6."""
import os
import re

import pytest

from raydp_amd.utils import config as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_types_and_defaults(monkeypatch):
    monkeypatch.delenv("RAYDP_ALLREDUCE", raising=False)
    assert C.get("spark.ray.mi355x.allreduce") == "auto"
    assert C.get("spark.executor.memory", {"spark.executor.memory": "2g"}) == 2 << 30
    assert C.get("spark.executor.cores", {"spark.executor.cores": "3"}) == 3
    assert C.get("spark.shuffle.service.enabled", {"spark.shuffle.service.enabled": "true"}) is True
    with pytest.raises(ValueError):
        C.get("spark.ray.mi355x.allreduce", {"spark.ray.mi355x.allreduce": "bogus"})
    with pytest.raises(KeyError):
        C.get("spark.ray.mi355x.no_such_key")


def test_precedence(monkeypatch):
    monkeypatch.setenv("RAYDP_ALLREDUCE", "rccl")
    assert C.get("spark.ray.mi355x.allreduce") == "rccl"                      # env over default
    assert C.get("spark.ray.mi355x.allreduce", {"spark.ray.mi355x.allreduce": "xgmi"}) == "xgmi"


def test_prefix_keys_and_jvm_only_keys():
    conf = {"spark.ray.raydp_spark_executor.actor.resource.cpu": "0.5",
            "spark.ray.raydp_spark_executor.actor.resource.GPU": "1",
            "spark.driver.extraJavaOptions": "-Xss4m", "spark.app.name": "x"}
    assert C.with_prefix("spark.ray.raydp_spark_executor.actor.resource.", conf) == {"cpu": 0.5, "GPU": 1.0}
    assert C.lookup("spark.ray.raydp_spark_master.resource.memory").key == \
        "spark.ray.raydp_spark_master.actor.resource."    # deprecated alias
    assert C.validate(conf) == ["spark.driver.extraJavaOptions"]


def test_env_for_workers_carries_session_settings():
    env = C.env_for_workers({"spark.ray.mi355x.allreduce": "rccl", "spark.ray.mi355x.hip_graphs": "false"})
    assert env["RAYDP_ALLREDUCE"] == "rccl" and env["RAYDP_TORCH_GRAPHS"] == "false"


def test_cpp_mirror_matches_registry():
    text = open(os.path.join(ROOT, "csrc", "common", "config_keys.h")).read()
    cpp = dict(re.findall(r'\{"(spark\.ray\.mi355x\.[^"]+)", "([A-Z_]+)"', text))
    py = {k.key: k.env for k in C.REGISTRY.values() if k.key.startswith("spark.ray.mi355x.")}
    assert cpp == py
    assert "spark.ray.mi355x.allreduce" in C.describe()
