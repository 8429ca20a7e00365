"""Placement groups: atomic reservation of resource bundles on runtime nodes.

Reference use: ``ray.util.placement_group(bundles, strategy)`` in ``python/raydp/context.py:
119-140`` (one ``{CPU, memory}`` bundle per executor), ``STRICT_SPREAD`` peers in
``python/raydp/mpi/mpi_job.py:192-222`` and round-robin bundle assignment of executors in
``RayAppMaster.scala:341-349``. Strategies: PACK (fill one node first, fall back to others),
STRICT_PACK (all bundles on one node), SPREAD (round-robin nodes, best effort), STRICT_SPREAD
(every bundle on a distinct node).
"""
import threading
import uuid
from typing import Dict, List, Optional

_lock = threading.RLock()
_groups: Dict[str, "PlacementGroup"] = {}


class PlacementGroupID:
    def __init__(self, h: str):
        self._h = h

    def hex(self):
        return self._h

    def __repr__(self):
        return f"PlacementGroupID({self._h})"


class PlacementGroup:
    def __init__(self, bundles: List[Dict[str, float]], strategy: str, name: str = ""):
        self.id = PlacementGroupID(uuid.uuid4().hex[:28])
        self.bundle_specs = [dict(b) for b in bundles]
        self.strategy = strategy
        self.name = name
        self.bundle_nodes: List[str] = []
        self.state = "PENDING"

    @property
    def bundle_count(self):
        return len(self.bundle_specs)

    def ready(self):
        """Object that ``get`` resolves once the group is placed (placement is synchronous)."""
        from raydp_amd.runtime.objects import put
        return put(True)

    def wait(self, timeout_seconds: float = 30) -> bool:
        return self.state == "CREATED"

    def node_of(self, bundle_index: int) -> str:
        return self.bundle_nodes[bundle_index]


def placement_group(bundles: List[Dict[str, float]], strategy: str = "PACK", name: str = "",
                    lifetime: Optional[str] = None) -> PlacementGroup:
    from raydp_amd.runtime import core
    if strategy not in ("PACK", "STRICT_PACK", "SPREAD", "STRICT_SPREAD"):
        raise ValueError(f"invalid placement strategy {strategy}")
    if not core.is_initialized():
        core.init()
    pg = PlacementGroup(bundles, strategy, name)
    node = core.current_node()
    if getattr(node, "gcs", None) is not None:
        # an attached driver: the group lives in the head's table; this is its local mirror
        pid, nodes = node.gcs.call("pg_create", [dict(b) for b in bundles], strategy, name)
        pg.id = PlacementGroupID(pid)
        pg.bundle_nodes = list(nodes)
        pg.bundle_free = [dict(b) for b in pg.bundle_specs]
        pg.remote = True
    else:
        node.cluster.place_group(pg)
    pg.state = "CREATED"
    with _lock:
        _groups[pg.id.hex()] = pg
    return pg


def remove_placement_group(pg: PlacementGroup):
    from raydp_amd.runtime import core
    with _lock:
        g = _groups.get(pg.id.hex())
    if g is None or g.state == "REMOVED":
        return
    node = core.current_node()
    if getattr(g, "remote", False):
        if node is not None and node.gcs is not None:
            node.gcs.call("pg_remove", g.id.hex())
    elif node is not None:
        node.cluster.release_group(g)
    g.state = "REMOVED"


def get_placement_group(name: str) -> PlacementGroup:
    with _lock:
        for g in _groups.values():
            if g.name == name and g.state != "REMOVED":
                return g
    raise ValueError(f"placement group {name} not found")


def get_placement_group_by_id(pg_id: str) -> PlacementGroup:
    with _lock:
        g = _groups.get(pg_id)
    if g is None or g.state == "REMOVED":
        raise ValueError(f"placement group {pg_id} not found")
    return g


def placement_group_table(pg: Optional[PlacementGroup] = None):
    with _lock:
        items = {k: {"placement_group_id": k, "name": g.name, "strategy": g.strategy,
                     "state": g.state, "bundles": dict(enumerate(g.bundle_specs))}
                 for k, g in _groups.items()}
    if pg is not None:
        return items[pg.id.hex()]
    return items


def _reset():
    with _lock:
        _groups.clear()
