"""Cluster service ABCs (reference: ``python/raydp/services.py:22-107``).

``Cluster`` is what ``SparkCluster`` (``raydp_amd/spark/ray_cluster.py``) implements: set up a
master with a resource requirement, add workers, expose a URL, stop. ``ClusterMaster`` /
``ClusterWorker`` describe the processes behind it.
"""
from abc import ABC, abstractmethod
from typing import Any, Dict, NoReturn


class Cluster(ABC):
    """Base of a sub-cluster (Spark today) running on the runtime."""

    def __init__(self, master_resources_requirement):
        # the master lives with the driver; its resources are not counted as a node
        self._num_nodes = 0

    @abstractmethod
    def _set_up_master(self, resources: Dict[str, float], kwargs: Dict[Any, Any]):
        """Set up the master service."""

    def add_worker(self, resources_requirement: Dict[str, float], **kwargs: Dict[Any, Any]):
        """Add one worker; the cluster is stopped if that fails."""
        try:
            self._set_up_worker(resources_requirement, kwargs)
        except BaseException:
            self.stop()
            raise

    @abstractmethod
    def _set_up_worker(self, resources: Dict[str, float], kwargs: Dict[str, str]):
        """Set up one worker service."""

    @abstractmethod
    def get_cluster_url(self) -> str:
        """URL of the cluster master, e.g. ``ray://<host>:<port>``."""

    @abstractmethod
    def stop(self):
        """Stop the cluster."""


class ClusterMaster(ABC):
    @abstractmethod
    def start_up(self) -> NoReturn:
        pass

    @abstractmethod
    def get_master_url(self) -> str:
        pass

    @abstractmethod
    def get_host(self) -> str:
        pass

    @abstractmethod
    def stop(self):
        pass


class ClusterWorker(ABC):
    @abstractmethod
    def start_up(self) -> str:
        """Start the worker; return an error message or None on success."""

    @abstractmethod
    def get_host(self) -> str:
        pass

    @abstractmethod
    def stop(self):
        pass
