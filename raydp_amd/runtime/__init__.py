"""Actor runtime (Ray-core equivalent): nodes, object store, tasks, actors, placement groups."""
from raydp_amd.runtime.core import (get_runtime_context, init, is_initialized, shutdown)
from raydp_amd.runtime.objects import ObjectRef, free, get, put
from raydp_amd.runtime.api import get_actor, kill, remote, wait
from raydp_amd.runtime.pgroup import (placement_group, placement_group_table,
                                               remove_placement_group)

__all__ = ["init", "shutdown", "is_initialized", "get_runtime_context", "ObjectRef", "get", "put",
           "free", "remote", "get_actor", "kill", "wait", "placement_group", "remove_placement_group", "placement_group_table"]
