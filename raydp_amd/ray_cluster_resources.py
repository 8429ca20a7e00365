"""Per-node resource view with a short refresh interval
(reference: ``python/raydp/ray_cluster_resources.py:25-79``).

``satisfy(request)`` lists the node labels (``node:<ip>``-style resource keys) whose *total*
resources can host ``request``; used to decide where executors may go. Memory requests are
in bytes and compared in the runtime's memory units.
"""
import time
from typing import Dict, List

from raydp_amd.utils import MEMORY_RESOURCE_UNIT_BYTES


class ClusterResources:
    refresh_interval = 0.1
    latest_refresh_time = time.time() - refresh_interval
    node_to_resources: Dict[str, Dict[str, float]] = {}
    item_keys_mapping = {"num_cpus": "CPU", "num_gpus": "GPU"}
    label_name = "__ray_spark_node_label"

    @classmethod
    def total_alive_nodes(cls) -> int:
        cls._refresh()
        return len(cls.node_to_resources)

    @classmethod
    def satisfy(cls, request: Dict[str, float]) -> List[str]:
        cls._refresh()
        return [res[cls.label_name] for res in cls.node_to_resources.values()
                if cls._compare_two_dict(res, request)]

    @classmethod
    def _refresh(cls, force: bool = False):
        from raydp_amd.runtime import api
        if not force and (time.time() - cls.latest_refresh_time) < cls.refresh_interval:
            return
        fresh = {}
        for node in api.nodes():
            if not node["Alive"]:
                continue
            res = dict(node["Resources"])
            label = next((k for k in res if k.startswith("node:")), None)
            if label is None:
                label = f"node:{node['NodeManagerAddress']}"
                res[label] = 1.0
            res[cls.label_name] = label
            fresh[node["NodeID"]] = res
        cls.node_to_resources = fresh
        cls.latest_refresh_time = time.time()

    @classmethod
    def _compare_two_dict(cls, available: Dict[str, float], request: Dict[str, float]) -> bool:
        for k, v in request.items():
            k = cls.item_keys_mapping.get(k, k)
            if k not in available:
                return False
            if k == "memory":
                v = int(v / MEMORY_RESOURCE_UNIT_BYTES)
            if available[k] < v:
                return False
        return True
