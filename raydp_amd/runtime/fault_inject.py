"""Fault injection for tests and chaos runs (the analogue of the reference's
``cluster.remove_node`` / forced-GC fault injection in tests/test_spark_cluster.py:262-333).

* :func:`kill_actor` — SIGKILL a named actor's process; the supervisor restarts it when its
  ``max_restarts`` allows (executors: forever), like a node-local crash.
* :func:`kill_executor` — the same for executor ``<id>`` of the active Spark application;
  returns the killed pid.
* :func:`wait_restarted` — block until the actor answers again from a new process.
* :func:`remove_node` — drop a virtual node (its object-store arena and actors) from a
  ``Cluster`` (``raydp_amd.runtime.cluster_utils``).
"""
import os
import signal
import time
from typing import Optional


def _handle(name: str, namespace: Optional[str] = None):
    from raydp_amd import runtime
    return runtime.get_actor(name, namespace=namespace) if namespace else runtime.get_actor(name)


def actor_pid(name: str) -> int:
    """Pid of the process serving actor ``name`` (actors expose ``info()`` with a ``pid``)."""
    from raydp_amd import runtime
    info = runtime.get(_handle(name).info.remote())
    if isinstance(info, dict) and "pid" in info:
        return int(info["pid"])
    raise RuntimeError(f"cannot determine the pid of actor {name!r}")


def kill_actor(name: str, sig: int = signal.SIGKILL) -> int:
    """Kill the process currently backing actor ``name``; returns its pid."""
    pid = actor_pid(name)
    os.kill(pid, sig)
    return pid


def kill_executor(executor_id: str = "0", sig: int = signal.SIGKILL) -> int:
    return kill_actor(f"raydp-executor-{executor_id}", sig)


def wait_restarted(name: str, old_pid: int, timeout: float = 30.0) -> int:
    """Wait until actor ``name`` is served by a process other than ``old_pid``."""
    deadline = time.time() + timeout
    last = None
    while time.time() < deadline:
        try:
            pid = actor_pid(name)
            if pid != old_pid:
                return pid
        except Exception as e:  # noqa: BLE001 - the actor is between processes
            last = e
        time.sleep(0.05)
    raise TimeoutError(f"actor {name!r} did not come back within {timeout}s ({last})")


def remove_node(cluster, node):
    """``Cluster.remove_node``: the node's arena and actors go away; lineage recovers objects."""
    cluster.remove_node(node)
