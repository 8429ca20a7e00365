"""Runtime core: node lifecycle, task futures, runtime context.

This module is the process-local entry point of the actor runtime (``raydp_amd.runtime``):
``init`` brings up a node (shared-memory object store + actor supervisor), ``shutdown``
tears it down. See ``raydp_amd/runtime/node.py`` for the node itself.
"""
import os
import threading
from concurrent.futures import Future
from typing import Dict, Optional

from raydp_amd.utils import get_node_ip_address

_lock = threading.RLock()
_node = None
_pending: Dict[str, Future] = {}


class RuntimeContext:
    def __init__(self, node):
        self.node = node

    @property
    def node_ip(self):
        return get_node_ip_address()

    @property
    def namespace(self):
        return self.node.namespace if self.node is not None else "default"

    def get_node_id(self):
        return self.node.node_id if self.node is not None else "local"

    def get_job_id(self):
        return self.node.job_id if self.node is not None else "01000000"

    def get_actor_id(self):
        return os.environ.get("RAYDP_ACTOR_ID")

    @property
    def gcs_address(self):
        return self.node.address if self.node is not None else None

    def get_assigned_resources(self):
        return {}

    @property
    def was_current_actor_reconstructed(self):
        return int(os.environ.get("RAYDP_ACTOR_RESTART_COUNT", "0")) > 0


def is_initialized() -> bool:
    return _node is not None


def address() -> Optional[str]:
    """Address other processes use to reach this node (None before ``init``)."""
    n = _node
    return None if n is None else getattr(n, "address", None)


def current_node():
    return _node


def current_node_store():
    n = _node
    return None if n is None else n.store


def init(address=None, num_cpus=None, num_gpus=None, resources=None, object_store_memory=None,
         namespace=None, include_dashboard=False, ignore_reinit_error=True, logging_level=None,
         job_config=None, **kwargs):
    global _node
    with _lock:
        if _node is not None:
            if ignore_reinit_error:
                return _node.info()
            raise RuntimeError("runtime already initialized")
        from raydp_amd.runtime.node import Node
        _node = Node.create(address=address, num_cpus=num_cpus, num_gpus=num_gpus,
                            resources=resources, object_store_memory=object_store_memory,
                            namespace=namespace)
        return _node.info()


def shutdown():
    global _node
    with _lock:
        n = _node
        _node = None
    if n is not None:
        n.shutdown()
    with _lock:
        _pending.clear()


def get_runtime_context() -> RuntimeContext:
    return RuntimeContext(_node)


def register_pending(ref_id: str, fut: Future):
    with _lock:
        _pending[ref_id] = fut


def pending_result(ref) -> Optional[Future]:
    with _lock:
        return _pending.get(ref.id)
