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


_stores_lock = threading.Lock()
_attached_stores: Dict[str, object] = {}


def store_for(node_id: Optional[str], path: Optional[str] = None):
    """Object store of ``node_id`` as seen from this process (attaching by path if needed).

    Returns None when that node's arena no longer exists (node removed)."""
    n = _node
    if n is None:
        return None
    if node_id is None or node_id == n.store.node_id:
        return n.store
    vn = n.cluster.nodes.get(node_id) if n.cluster is not None else None
    if vn is not None:
        return vn.store if vn.alive else None
    if not path and n.session_dir:
        f = os.path.join(n.session_dir, "nodes", node_id)
        if os.path.exists(f):
            with open(f) as fh:
                path = fh.read().strip()
    with _stores_lock:
        st = _attached_stores.get(node_id)
        if st is None and path:
            if not os.path.exists(path):
                return None
            from raydp_amd.runtime.store import attach_store
            try:
                st = attach_store(path, node_id)
            except OSError:
                return None
            _attached_stores[node_id] = st
        return st


def attach_from_env():
    """Worker-process mode: join the node described by ``RAYDP_*`` environment variables."""
    global _node
    with _lock:
        if _node is None:
            from raydp_amd.runtime.node import Node
            _node = Node.attach(os.environ["RAYDP_SESSION_DIR"], os.environ["RAYDP_STORE_PATH"],
                                os.environ["RAYDP_NODE_ID"], os.environ.get("RAYDP_NAMESPACE"))
        return _node


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
        if os.environ.get("RAYDP_SESSION_DIR") and os.environ.get("RAYDP_STORE_PATH"):
            # inside an actor process: join the existing node instead of starting one
            _node = Node.attach(os.environ["RAYDP_SESSION_DIR"], os.environ["RAYDP_STORE_PATH"],
                                os.environ["RAYDP_NODE_ID"], os.environ.get("RAYDP_NAMESPACE"))
            return _node.info()
        if address is None:
            address = os.environ.get("RAYDP_ADDRESS") or None
        if address not in (None, "", "local"):
            # another process's running node (raydp_amd/runtime/gcs.py): attach to it
            _node = Node.connect(address, namespace=namespace)
            return _node.info()
        _node = Node.create(address=address, num_cpus=num_cpus, num_gpus=num_gpus,
                            resources=resources, object_store_memory=object_store_memory,
                            namespace=namespace)
        return _node.info()


def shutdown():
    global _node
    import sys
    tr = sys.modules.get("raydp_amd.train.trainer")
    if tr is not None:      # warm training worker groups are actors of this node
        tr.release_worker_groups()
    with _lock:
        n = _node
        _node = None
    if n is not None:
        n.shutdown()
    with _lock:
        _pending.clear()
    with _stores_lock:
        for st in _attached_stores.values():
            st.close()
        _attached_stores.clear()


def get_runtime_context() -> RuntimeContext:
    return RuntimeContext(_node)


def register_pending(ref_id: str, fut: Future):
    with _lock:
        _pending[ref_id] = fut


def pending_result(ref) -> Optional[Future]:
    with _lock:
        return _pending.get(ref.id)
