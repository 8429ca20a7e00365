"""Spark master actor (reference: ``python/raydp/spark/ray_cluster_master.py`` —
``RayDPSparkMaster``: ``start_up``, ``get_master_url``, ``get_host``, ``add_objects``,
``get_spark_home``, ``stop``).

A process actor named ``<app>_SPARK_MASTER``. Besides identifying the application it is the
*owner* of converted partitions when the caller asks for it (``get_raydp_master_owner`` /
``stop_spark(cleanup_data=False)``): it holds references to those objects so they outlive the
executors (``add_objects`` in the reference pins Ray ObjectRefs the same way).
"""
import os
import time
from typing import Dict, List


class RayDPSparkMaster:
    def __init__(self, app_name: str, configs: Dict[str, str]):
        self.app_name = app_name
        self.configs = dict(configs)
        self._objects: Dict[str, List] = {}
        self._started = False
        self._url = None

    def start_up(self, resources: Dict[str, float] = None):
        from raydp_amd.utils import get_node_ip_address
        self._started = True
        self._url = f"ray://{self.app_name}@{get_node_ip_address()}:{os.getpid()}"
        self.resources = dict(resources or {})
        return self._url

    def get_master_url(self) -> str:
        return self._url

    def get_host(self) -> str:
        from raydp_amd.utils import get_node_ip_address
        return get_node_ip_address()

    def get_node_ip(self) -> str:
        return self.get_host()

    def get_spark_home(self) -> str:
        return os.environ.get("SPARK_HOME", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

    def add_objects(self, timestamp, objects) -> int:
        self._objects[str(timestamp)] = list(objects)
        return len(objects)

    def get_object(self, timestamp, idx):
        from raydp_amd.runtime.objects import get
        return get(self._objects[str(timestamp)][idx])

    def num_held_objects(self) -> int:
        return sum(len(v) for v in self._objects.values())

    def stop(self, cleanup_data=True):
        if cleanup_data:
            self._objects.clear()
        self._started = False
        return time.time()
