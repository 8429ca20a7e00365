"""A runtime node: resource accounting, object store, actor supervisor.

One driver process hosts the *head*: the cluster resource table (one or more virtual nodes,
each with its own CPU/GPU/memory/custom resources and its own shared-memory object-store
arena — the analogue of ``ray.cluster_utils.Cluster`` used by the reference's multi-node
tests, ``python/raydp/tests/test_spark_cluster.py:90-110``), the named-actor registry and the
placement-group table. Actor processes are supervised natively (``csrc/runtime``).
"""
import os
import threading
import uuid
from typing import Dict, List, Optional

from raydp_amd.utils import get_node_ip_address, parse_memory_size


class ResourceError(RuntimeError):
    pass


class VirtualNode:
    def __init__(self, node_id: str, resources: Dict[str, float], store=None, ip: str = None):
        self.node_id = node_id
        self.total = dict(resources)
        self.available = dict(resources)
        self.store = store
        self.alive = True
        self.ip = ip or get_node_ip_address()

    def fits(self, req: Dict[str, float]) -> bool:
        return self.alive and all(self.available.get(k, 0.0) + 1e-9 >= v for k, v in req.items() if v)

    def acquire(self, req: Dict[str, float]):
        for k, v in req.items():
            if v:
                self.available[k] = self.available.get(k, 0.0) - v

    def release(self, req: Dict[str, float]):
        for k, v in req.items():
            if v:
                self.available[k] = min(self.total.get(k, 0.0), self.available.get(k, 0.0) + v)


class ClusterState:
    def __init__(self):
        self.lock = threading.RLock()
        self.nodes: Dict[str, VirtualNode] = {}
        self.order: List[str] = []

    def add(self, n: VirtualNode):
        with self.lock:
            self.nodes[n.node_id] = n
            self.order.append(n.node_id)

    def alive_nodes(self) -> List[VirtualNode]:
        with self.lock:
            return [self.nodes[i] for i in self.order if self.nodes[i].alive]

    def pick_node(self, req: Dict[str, float], prefer: Optional[str] = None) -> VirtualNode:
        with self.lock:
            if prefer and prefer in self.nodes and self.nodes[prefer].fits(req):
                return self.nodes[prefer]
            for n in self.alive_nodes():
                if n.fits(req):
                    return n
        raise ResourceError(f"no node can satisfy resource request {req}")

    def place_group(self, pg):
        with self.lock:
            nodes = self.alive_nodes()
            chosen: List[VirtualNode] = []
            snapshot = {n.node_id: dict(n.available) for n in nodes}
            try:
                for i, b in enumerate(pg.bundle_specs):
                    cand = nodes
                    if pg.strategy == "STRICT_PACK" and chosen:
                        cand = [chosen[0]]
                    elif pg.strategy == "STRICT_SPREAD":
                        cand = [n for n in nodes if n not in chosen]
                    elif pg.strategy == "SPREAD":
                        cand = sorted(nodes, key=lambda n: sum(1 for c in chosen if c is n))
                    elif pg.strategy == "PACK" and chosen:
                        cand = [chosen[-1]] + [n for n in nodes if n is not chosen[-1]]
                    node = next((n for n in cand if n.fits(b)), None)
                    if node is None:
                        raise ResourceError(f"cannot place bundle {i} {b} with strategy {pg.strategy}")
                    node.acquire(b)
                    chosen.append(node)
            except ResourceError:
                for n in nodes:
                    n.available = snapshot[n.node_id]
                raise
            pg.bundle_nodes = [n.node_id for n in chosen]
            # bundle reservations become the bundle's private pool
            pg.bundle_free = [dict(b) for b in pg.bundle_specs]

    def release_group(self, pg):
        with self.lock:
            for nid, b in zip(pg.bundle_nodes, pg.bundle_specs):
                n = self.nodes.get(nid)
                if n is not None:
                    n.release(b)


def _default_resources(num_cpus=None, num_gpus=None, memory=None, resources=None):
    if num_cpus is None:
        num_cpus = os.cpu_count() or 1
    if num_gpus is None:
        num_gpus = 0
        try:
            import torch
            num_gpus = torch.cuda.device_count()
        except Exception:  # noqa: BLE001
            pass
    if memory is None:
        try:
            import psutil
            memory = int(psutil.virtual_memory().total * 0.7)
        except Exception:  # noqa: BLE001
            memory = 8 << 30
    r = {"CPU": float(num_cpus), "GPU": float(num_gpus), "memory": float(memory)}
    r.update({k: float(v) for k, v in (resources or {}).items()})
    return r


class Node:
    def __init__(self, namespace=None):
        self.node_id = uuid.uuid4().hex[:16]
        self.namespace = namespace or "default"
        self.job_id = uuid.uuid4().hex[:8]
        self.address = f"{get_node_ip_address()}:0"
        self.cluster = ClusterState()
        self.session_dir = None
        self.store = None
        self.supervisor = None
        self.actors = None
        self.attached = False
        self.gcs = None            # driver attached through the head's control endpoint
        self.gcs_service = None    # head: the control endpoint it serves (raydp_amd/runtime/gcs.py)
        self.supervisor_sock = None

    @classmethod
    def attach(cls, session_dir: str, store_path: str, node_id: str, namespace=None) -> "Node":
        """A worker process's view of an existing node (its store arena, supervisor, session)."""
        from raydp_amd.runtime.actors import ActorManager
        from raydp_amd.runtime.store import attach_store
        n = cls(namespace)
        n.attached = True
        n.node_id = os.environ.get("RAYDP_HEAD_NODE_ID", node_id)
        n.session_dir = session_dir
        n.store = attach_store(store_path, node_id)
        import json
        res_file = os.path.join(session_dir, "node_resources.json")
        res = {"CPU": float(os.cpu_count() or 1)}
        if os.path.exists(res_file):
            with open(res_file) as f:
                res = json.load(f)
        n.cluster.add(VirtualNode(node_id, res, n.store))
        n.actors = ActorManager(n)
        return n

    @classmethod
    def create(cls, address=None, num_cpus=None, num_gpus=None, resources=None,
               object_store_memory=None, namespace=None, memory=None):
        import tempfile
        n = cls(namespace)
        n.session_dir = tempfile.mkdtemp(prefix=f"raydp_session_{n.node_id[:8]}_")
        os.makedirs(os.path.join(n.session_dir, "logs"), exist_ok=True)
        from raydp_amd.runtime.store import open_store
        n.store = open_store(n.node_id, object_store_memory, n.session_dir)
        head = VirtualNode(n.node_id, _default_resources(num_cpus, num_gpus, memory, resources),
                           n.store)
        n.cluster.add(head)
        n._record_store(n.store)
        import json
        with open(os.path.join(n.session_dir, "node_resources.json"), "w") as f:
            json.dump(head.total, f)
        from raydp_amd.runtime.actors import ActorManager
        n.actors = ActorManager(n)
        n._serve_control()
        return n

    def _serve_control(self):
        """Start the control endpoint other processes attach through (runtime.init(address=...))
        and record this head as the host's current node (address='auto')."""
        from raydp_amd.runtime import gcs
        from raydp_amd.utils.config import get as conf_get
        self.gcs_service = gcs.HeadService(self, int(conf_get("spark.ray.mi355x.runtime.port")),
                                           str(conf_get("spark.ray.mi355x.runtime.host")))
        self.address = self.gcs_service.address
        gcs.record_current(self.address)

    def attach_info(self) -> dict:
        """What a process attaching to this head needs (the control endpoint's ``info``)."""
        head = self.cluster.nodes.get(self.node_id)
        return {"node_id": self.node_id, "session_dir": self.session_dir, "store_path": self.store.path,
                "supervisor_sock": self.actors.supervisor.sock_path, "namespace": self.namespace,
                "job_id": self.job_id, "address": self.address, "ip": head.ip if head is not None else "",
                "resources": dict(head.total) if head is not None else {},
                "tcp_address": self.gcs_service.tcp_address if self.gcs_service is not None else None}

    @classmethod
    def connect(cls, address: str, namespace=None) -> "Node":
        """A driver process attached to a running head (``ray.init(address=...)``): the head's
        object store, supervisor, named actors and cluster table, reached through its control
        endpoint. Actors this process creates are placed by the head and die with this process
        unless created with ``lifetime="detached"``."""
        from raydp_amd.runtime import gcs
        from raydp_amd.runtime.actors import ActorManager
        from raydp_amd.runtime.store import attach_store
        client = gcs.GcsClient(address)
        info = client.call("info")
        n = cls(namespace or info.get("namespace"))
        n.attached = True
        n.gcs = client
        n.node_id = info["node_id"]
        n.session_dir = info["session_dir"]
        n.address = info["address"]
        n.supervisor_sock = info["supervisor_sock"]
        n.store = attach_store(info["store_path"], info["node_id"])
        n.cluster.add(VirtualNode(info["node_id"], info.get("resources") or {}, n.store, ip=info.get("ip") or None))
        n.actors = ActorManager(n)
        return n

    def add_virtual_node(self, num_cpus=1, num_gpus=0, resources=None, object_store_memory=None,
                         memory=None) -> VirtualNode:
        from raydp_amd.runtime.store import open_store
        nid = uuid.uuid4().hex[:16]
        store = open_store(nid, object_store_memory, self.session_dir)
        vn = VirtualNode(nid, _default_resources(num_cpus, num_gpus, memory or (2 << 30), resources), store)
        self.cluster.add(vn)
        self._record_store(store)
        return vn

    def _record_store(self, store):
        d = os.path.join(self.session_dir, "nodes")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, store.node_id), "w") as f:
            f.write(store.path)

    def remove_virtual_node(self, node_id: str):
        vn = self.cluster.nodes[node_id]
        vn.alive = False
        if self.actors is not None:
            self.actors.on_node_removed(node_id)
        if vn.store is not None and vn.store is not self.store:
            vn.store.destroy()
            try:
                os.unlink(os.path.join(self.session_dir, "nodes", node_id))
            except OSError:
                pass

    def info(self):
        return {"node_id": self.node_id, "address": self.address, "session_dir": self.session_dir,
                "namespace": self.namespace}

    def shutdown(self):
        if self.gcs is not None and self.actors is not None:
            # an attached driver's actors die with it (Ray's non-detached actors die with their job)
            self.actors.kill_owned()
        if self.actors is not None:
            self.actors.shutdown()
        if self.attached:
            self.store.close()
            if self.gcs is not None:
                self.gcs.close()
            return
        if self.gcs_service is not None:
            from raydp_amd.runtime import gcs
            gcs.clear_current(self.address)
            self.gcs_service.close()
        for vn in list(self.cluster.nodes.values()):
            if vn.store is not None:
                vn.store.destroy()
        from raydp_amd.runtime import pgroup as pg
        pg._reset()
        if self.session_dir and not os.environ.get("RAYDP_KEEP_SESSION_DIR"):
            import shutil
            shutil.rmtree(self.session_dir, ignore_errors=True)
