"""Executor placement check over the runtime's live node table.

Reference role: ``python/raydp/ray_cluster_resources.py`` keeps a 0.1 s-refreshed copy of
``ray.nodes()`` and answers which nodes could host a resource request. Here the node table is
the runtime's own (``raydp_amd.runtime``), so there is nothing to poll: :func:`plan_executors`
reads every alive node's total and available resources once, and the Spark cluster calls it
before launching its executors (``raydp_amd/spark/cluster.py``) to fail fast -- with the nodes
and their resources in the message -- when no node can ever host one executor of the requested
shape, instead of leaving the launch queued forever.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional

_ALIASES = {"num_cpus": "CPU", "num_gpus": "GPU", "cpu": "CPU", "gpu": "GPU"}


@dataclass
class NodeView:
    node_id: str
    address: str
    total: Dict[str, float]
    available: Dict[str, float]

    def capacity(self, request: Dict[str, float], free_only: bool = False) -> int:
        """How many bundles of ``request`` this node holds (its free resources with
        ``free_only``, else its totals)."""
        have = self.available if free_only else self.total
        n = None
        for k, v in request.items():
            if not v:
                continue
            fits = int(have.get(k, 0.0) // v + 1e-9) if have.get(k, 0.0) >= v else 0
            n = fits if n is None else min(n, fits)
        return 0 if n is None else n


@dataclass
class PlacementPlan:
    request: Dict[str, float]
    wanted: int
    nodes: List[NodeView] = field(default_factory=list)

    @property
    def capacity_total(self) -> int:
        return sum(nv.capacity(self.request) for nv in self.nodes)

    @property
    def capacity_free(self) -> int:
        return sum(nv.capacity(self.request, free_only=True) for nv in self.nodes)

    def hosts(self, free_only: bool = False) -> List[str]:
        """Node ids that can host at least one bundle."""
        return [nv.node_id for nv in self.nodes if nv.capacity(self.request, free_only) > 0]

    def describe(self) -> str:
        rows = [f"{nv.node_id}@{nv.address}: total {nv.total}, free {nv.available}" for nv in self.nodes]
        return "; ".join(rows) or "no alive nodes"


def normalise(request: Dict[str, float]) -> Dict[str, float]:
    return {_ALIASES.get(k, k): float(v) for k, v in request.items() if v}


def live_nodes() -> List[NodeView]:
    from raydp_amd.runtime import core
    node = core.current_node()
    if node is None:
        return []
    return [NodeView(v.node_id, v.ip, dict(v.total), dict(v.available)) for v in node.cluster.alive_nodes()]


def plan_executors(count: int, request: Dict[str, float], nodes: Optional[List[NodeView]] = None) -> PlacementPlan:
    """Check ``count`` executors of ``request`` (``{"CPU": 1, "memory": bytes, "<custom>": x}``)
    against the alive nodes. Raises ``ValueError`` when no node can host even one executor; the
    returned plan tells the caller how many fit in total and right now."""
    plan = PlacementPlan(normalise(request), int(count), list(nodes) if nodes is not None else live_nodes())
    if plan.nodes and plan.request and not plan.hosts():
        raise ValueError(f"no node can host an executor requesting {plan.request} "
                         f"(nodes: {plan.describe()})")
    return plan
