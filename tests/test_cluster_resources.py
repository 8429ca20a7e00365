"""Executor placement check over the runtime's node table (raydp_amd/ray_cluster_resources.py;
reference role: python/raydp/ray_cluster_resources.py)."""
import pytest

from raydp_amd.ray_cluster_resources import NodeView, plan_executors


def _nodes():
    return [NodeView("a", "10.0.0.1", {"CPU": 4.0, "memory": 8e9}, {"CPU": 1.0, "memory": 8e9}),
            NodeView("b", "10.0.0.2", {"CPU": 2.0, "memory": 8e9, "spark_node": 1.0},
                     {"CPU": 2.0, "memory": 8e9, "spark_node": 1.0})]


def test_capacity_counts_totals_and_free_resources():
    plan = plan_executors(5, {"num_cpus": 2, "memory": 1e9}, nodes=_nodes())
    assert plan.request == {"CPU": 2.0, "memory": 1e9}
    assert plan.capacity_total == 3 and plan.capacity_free == 1
    assert plan.hosts() == ["a", "b"] and plan.hosts(free_only=True) == ["b"]


def test_custom_resource_limits_the_hosts():
    plan = plan_executors(1, {"CPU": 1, "spark_node": 0.5}, nodes=_nodes())
    assert plan.hosts() == ["b"] and plan.capacity_total == 2


def test_impossible_request_fails_fast_with_the_node_table():
    with pytest.raises(ValueError, match="no node can host"):
        plan_executors(1, {"CPU": 8}, nodes=_nodes())
    with pytest.raises(ValueError, match="10.0.0.2"):
        plan_executors(1, {"CPU": 1, "gpu_x": 1}, nodes=_nodes())


def test_init_spark_rejects_an_executor_no_node_can_host():
    import raydp_amd
    from raydp_amd import runtime
    runtime.shutdown()
    runtime.init(num_cpus=2)
    try:
        with pytest.raises(ValueError, match="no node can host"):
            raydp_amd.init_spark("too-big", 1, 1, "500M",
                                 configs={"spark.ray.raydp_spark_executor.actor.resource.not_here": "1"})
    finally:
        raydp_amd.stop_spark()
        runtime.shutdown()
