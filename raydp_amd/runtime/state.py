"""Actor state API (``ray.util.state.list_actors`` subset used by the reference's
``tests/test_spark_master_memory.py:49-55``)."""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


@dataclass
class ActorState:
    actor_id: str
    name: Optional[str]
    state: str
    pid: Optional[int]
    node_id: Optional[str]
    class_name: str = ""
    required_resources: Dict[str, float] = field(default_factory=dict)
    num_restarts: int = 0
    placement_group_id: Optional[str] = None


def list_actors(filters: Optional[Sequence[Tuple[str, str, str]]] = None, detail: bool = False,
                limit: int = 10000) -> List[ActorState]:
    from raydp_amd.runtime import core
    node = core.current_node()
    if node is None or node.actors is None:
        return []
    out = []
    for a in node.actors.list():
        cls = ""
        if a.opts is not None:
            cls = a.opts.get("_class_name", "")
        out.append(ActorState(actor_id=a.actor_id, name=a.name, state="DEAD" if a.dead else "ALIVE",
                              pid=getattr(a, "pid", None),
                              node_id=a.vnode.node_id if a.vnode is not None else None, class_name=cls,
                              required_resources={k: v for k, v in a.resources.items() if v},
                              num_restarts=a.restarts,
                              placement_group_id=a.pg.id.hex() if a.pg is not None else None))
    for key, op, val in filters or ():
        if op not in ("=", "!="):
            raise ValueError(f"unsupported filter predicate {op}")
        out = [s for s in out if (str(getattr(s, key)) == str(val)) == (op == "=")]
    return out[:limit]
