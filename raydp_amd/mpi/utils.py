"""Process helpers for MPI jobs (reference: ``python/raydp/mpi/utils.py``).

``run_cmd`` starts the launcher in its own session/process group so ``stop`` can signal the
whole tree by its exact group id, forwards its output line by line, and calls a failure
callback when it exits non-zero.
"""
import os
import socket
import subprocess
import sys
import threading
from typing import Callable, Dict, List, Optional, Tuple

import psutil

from raydp_amd.mpi.network import insecure_channel as create_insecure_channel  # noqa: F401


class RemoteFunctionError:
    """Carries a rank's exception back to the driver (which re-raises it)."""

    def __init__(self, rank: int, exc: BaseException, tb: str):
        self.rank, self.exc, self.tb = rank, exc, tb


class StoppableThread(threading.Thread):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self._stop_event = threading.Event()

    def stop(self):
        self._stop_event.set()

    def stopped(self) -> bool:
        return self._stop_event.is_set()


def run_cmd(cmd: List[str], env: Dict[str, str], failed_callback: Optional[Callable] = None,
            out=None) -> Tuple[subprocess.Popen, StoppableThread, StoppableThread]:
    out = out or sys.stdout
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            start_new_session=True)

    def forward():
        for line in iter(proc.stdout.readline, b""):
            if fwd.stopped():
                break
            try:
                out.write(line.decode(errors="replace"))
                out.flush()
            except ValueError:
                break

    def check():
        rc = proc.wait()
        if rc != 0 and not chk.stopped() and failed_callback is not None:
            failed_callback()

    fwd = StoppableThread(target=forward, name="mpi-output", daemon=True)
    chk = StoppableThread(target=check, name="mpi-check", daemon=True)
    fwd.start()
    chk.start()
    return proc, chk, fwd


def get_environ_value(key: str) -> str:
    assert key in os.environ, f"{key} should be set in the environ"
    return os.environ[key]


def local_addresses() -> List[str]:
    addrs = ["127.0.0.1"]
    for _, lst in psutil.net_if_addrs().items():
        for a in lst:
            if a.family == socket.AF_INET:
                addrs.append(a.address)
    return addrs


def get_node_ip_address(node_addresses: List[str]) -> Optional[str]:
    """The entry of ``node_addresses`` that belongs to this machine."""
    mine = set(local_addresses())
    for a in node_addresses:
        if a in mine:
            return a
    return None
