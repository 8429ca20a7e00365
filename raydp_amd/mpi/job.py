"""Driver half of an MPI job (reference: ``python/raydp/mpi/mpi_job.py``).

Lifecycle (``start``): reserve one bundle of ``num_cpus_per_process * ppn`` CPUs per node in a
``STRICT_SPREAD`` placement group (or use the caller's group/bundles), resolve the bundle
nodes' addresses, serve ``DriverService`` over gRPC, launch ``mpirun`` (or the built-in
launcher when ``mpirun`` is absent) running ``worker.py`` on every rank, wait until every rank
has registered twice (process up, then its ``WorkerService`` port), and connect to each
rank. ``run(fn)`` ships ``fn`` to all ranks and returns the per-rank results in rank order,
re-raising the first rank exception. ``stop`` tells every rank to exit, terminates the
launcher's process group and releases the placement group; a job can be started again.
"""
import logging
import os
import shutil
import sys
import threading
from enum import Enum, unique
from typing import Any, Callable, Dict, List, Optional

import cloudpickle

from raydp_amd.mpi import constants, network

logger = logging.getLogger(__name__)


@unique
class MPIType(Enum):
    OPEN_MPI = 0
    INTEL_MPI = 1
    MPICH = 2


_FLAVOUR_NAME = {MPIType.OPEN_MPI: "openmpi", MPIType.INTEL_MPI: "intel_mpi", MPIType.MPICH: "mpich"}


class MPIJobContext:
    """Handed to ``mpi_script_prepare_fn``: hosts, ranks per node and the launch environment."""

    def __init__(self, hosts: List[str], num_procs_per_node: int, env: Dict[str, str]):
        self._hosts = hosts
        self._num_procs_per_node = num_procs_per_node
        self._env = env

    @property
    def hosts(self) -> List[str]:
        return self._hosts

    @property
    def num_procs_per_node(self) -> int:
        return self._num_procs_per_node

    @property
    def env(self) -> Dict[str, str]:
        return self._env

    def add_env(self, key: str, value: str):
        self._env[key] = value

    def add_envs(self, envs: Dict[str, str]):
        self._env.update(envs)


class MPIWorkerMeta:
    def __init__(self, rank: int):
        self.rank = rank
        self.stub: Optional[network.Stub] = None
        self.worker_ip: Optional[str] = None
        self.worker_port: Optional[int] = None
        self.peer = None


class _Results:
    def __init__(self, func_id: int, n: int):
        self.func_id = func_id
        self.remaining = n
        self.results: List[Any] = [None] * n
        self.done = threading.Event()
        self.failed: Optional[str] = None


class _MPIPeer:
    """Per-node placeholder actor: pins the bundle and reports the node address."""

    def get_node_ip(self):
        from raydp_amd.utils import get_node_ip_address
        return get_node_ip_address()


class MPIJob:
    def __init__(self, mpi_type: MPIType, job_name: str = None, world_size: int = 1,
                 num_cpus_per_process: int = 1, num_processes_per_node: int = 1,
                 mpi_script_prepare_fn: Callable = None, timeout: int = 1,
                 placement_group=None, placement_group_bundle_indexes: List[int] = None):
        assert world_size % num_processes_per_node == 0, (
            f"world_size: {world_size} should be multiple of num_processes_per_node: {num_processes_per_node}")
        self.mpi_type = mpi_type
        self.job_name = job_name or "raydp-mpi"
        self.world_size = world_size
        self.num_cpus_per_process = num_cpus_per_process
        self.num_processes_per_node = num_processes_per_node
        self.mpi_script_prepare_fn = mpi_script_prepare_fn
        self.timeout = timeout
        self.placement_group = placement_group
        self.placement_group_bundle_indexes = placement_group_bundle_indexes
        self.server = None
        self.server_host = None
        self.server_port = None
        self.node_addresses: List[str] = []
        self.peers = None
        self.pg = None
        self.workers: List[Optional[MPIWorkerMeta]] = [None] * world_size
        self.mpirun_proc = None
        self.mpirun_check_thread = None
        self.mpirun_forward_thread = None
        self.lock = threading.RLock()
        self._registered = 0
        self._register_event = threading.Event()
        self.func_id = 0
        self.func_result: Optional[_Results] = None
        self.started = False
        self.launch_command: List[str] = []

    # --------------------------------------------------------------- DriverService ------
    def RegisterWorker(self, request, context):
        assert request.job_id == self.job_name, (request.job_id, self.job_name)
        with self.lock:
            self.workers[request.world_rank] = MPIWorkerMeta(request.world_rank)
            self._bump()
        return network.RegisterWorkerReply(node_addresses=self.node_addresses)

    def RegisterWorkerService(self, request, context):
        from raydp_amd.runtime import core
        with self.lock:
            w = self.workers[request.world_rank]
            w.worker_ip, w.worker_port = request.worker_ip, request.worker_port
            if self.peers and request.worker_ip in self.node_addresses:
                w.peer = self.peers[self.node_addresses.index(request.worker_ip)]
            self._bump()
        return network.RegisterWorkerServiceReply(ray_address=str(core.address() or ""))

    def RegisterFuncResult(self, request, context):
        res = self.func_result
        if res is None or res.func_id != request.func_id:
            return network.Empty()
        with self.lock:
            res.results[request.world_rank] = cloudpickle.loads(request.result)
            res.remaining -= 1
            if res.remaining == 0:
                res.done.set()
        return network.Empty()

    def _bump(self):
        self._registered += 1
        if self._registered == self.world_size:
            self._registered = 0
            self._register_event.set()

    def _wait_register(self):
        if not self._register_event.wait(self.timeout):
            raise TimeoutError(f"MPI job {self.job_name}: ranks did not register within {self.timeout}s")
        self._register_event.clear()

    # ----------------------------------------------------------------- lifecycle --------
    def start(self):
        if self.started:
            return
        try:
            self._start_network_service()
            self._start_mpirun()
            self._wait_register()
            with self.lock:
                for w in self.workers:
                    w.stub = network.Stub(network.insecure_channel(f"{w.worker_ip}:{w.worker_port}"),
                                          "WorkerService")
            self.started = True
        except BaseException:
            self._reset()
            raise

    def _start_peers(self) -> List[str]:
        from raydp_amd import runtime
        from raydp_amd.runtime import pgroup
        if not runtime.is_initialized():
            runtime.init()
        num_nodes = self.world_size // self.num_processes_per_node
        if self.placement_group is not None:
            idx = list(self.placement_group_bundle_indexes or range(num_nodes))
            assert len(idx) == num_nodes, (
                f"The length of placement_group_bundle_indexes({len(idx)}) should be equal with the "
                f"number of nodes({num_nodes})")
            pg = self.placement_group
        else:
            cpus = self.num_cpus_per_process * self.num_processes_per_node
            self.pg = pgroup.placement_group([{"CPU": cpus}] * num_nodes, strategy="STRICT_SPREAD",
                                             name=f"{self.job_name}_pg")
            assert self.pg.wait(self.timeout), pgroup.placement_group_table(self.pg)
            pg, idx = self.pg, list(range(num_nodes))
        cls = runtime.remote(_MPIPeer)
        self.peers = [cls.options(placement_group=pg, placement_group_bundle_index=i).remote() for i in idx]
        self.node_addresses = runtime.get([p.get_node_ip.remote() for p in self.peers])
        return self.node_addresses

    def _start_network_service(self):
        from raydp_amd.utils import get_node_ip_address
        self.server = network.make_server(max_workers=4)
        network.add_service(self.server, "DriverService", self)
        self.server_host = get_node_ip_address()
        self.server_port = self.server.add_insecure_port(f"{self.server_host}:0")
        self.server.start()

    def get_default_mpirun_script(self, context: MPIJobContext) -> List[str]:
        raise NotImplementedError

    def _launcher_command(self, script: List[str]) -> List[str]:
        """Swap ``mpirun`` for the built-in launcher when it is not installed."""
        prog = [sys.executable, "-u", constants.MPI_MAIN_CLASS_PATH]
        if script and os.path.basename(script[0]) == "mpirun" and shutil.which(script[0]) is None:
            return ([sys.executable, "-m", "raydp_amd.mpi.launcher", "--mpi-type", _FLAVOUR_NAME[self.mpi_type]]
                    + script[1:] + ["-n", str(self.world_size), "--"] + prog)
        return script + prog

    def _start_mpirun(self):
        from raydp_amd.mpi.utils import run_cmd
        hosts = self._start_peers()
        env = os.environ.copy()
        context = MPIJobContext(hosts, self.num_processes_per_node, env)
        if self.mpi_script_prepare_fn:
            script = self.mpi_script_prepare_fn(context)
            if isinstance(script, str):
                script = script.split()
            script = list(script)
        else:
            script = self.get_default_mpirun_script(context)
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
        context.add_envs({
            constants.MPI_TYPE: str(self.mpi_type.value),
            constants.MPI_JOB_ID: self.job_name,
            constants.MPI_DRIVER_HOST: str(self.server_host),
            constants.MPI_DRIVER_PORT: str(self.server_port),
            constants.MAXIMUM_WAIT_TIME_OUT: str(max(self.timeout, 5)),
            "PYTHONPATH": os.pathsep.join(p for p in (root, env.get("PYTHONPATH", "")) if p),
        })
        self.launch_command = self._launcher_command(script)
        logger.info("MPI job %s command: %s", self.job_name, self.launch_command)
        self.mpirun_proc, self.mpirun_check_thread, self.mpirun_forward_thread = run_cmd(
            self.launch_command, context.env, failed_callback=self._on_launcher_failed)
        self._wait_register()

    def _on_launcher_failed(self):
        res = self.func_result
        if res is not None:
            res.failed = f"MPI launcher exited with code {self.mpirun_proc.returncode}"
            res.done.set()

    # ----------------------------------------------------------------------- use --------
    def run(self, mpi_func: Callable) -> List[Any]:
        """Run ``mpi_func(WorkerContext)`` on every rank; results in rank order."""
        from raydp_amd.mpi.utils import RemoteFunctionError
        assert self.started, "MPI job is not started"
        req = network.Function(func_id=self.func_id, func=cloudpickle.dumps(mpi_func))
        with self.lock:
            self.func_result = res = _Results(self.func_id, self.world_size)
        for w in self.workers:
            w.stub.RunFunction(req)
        self.func_id += 1
        res.done.wait()
        with self.lock:
            self.func_result = None
        if res.failed:
            raise RuntimeError(f"function call failed: {res.failed}")
        for r in res.results:
            if isinstance(r, RemoteFunctionError):
                raise RuntimeError(f"MPI rank {r.rank} raised {r.exc!r}\n{r.tb}") from r.exc
        return res.results

    def apply_peers(self, fn: Callable):
        assert self.started
        return fn(self.workers)

    def get_rank_addresses(self) -> List[str]:
        assert self.started
        return [w.worker_ip for w in self.workers]

    def _reset(self):
        for w in self.workers or []:
            if w is not None and w.stub is not None:
                try:
                    w.stub.Stop(network.Empty(), timeout=2)
                except Exception:
                    pass
                w.stub.close()
        proc = self.mpirun_proc
        if self.mpirun_check_thread is not None:
            self.mpirun_check_thread.stop()
            if threading.current_thread() is not self.mpirun_check_thread:
                self.mpirun_check_thread.join(2)
            if proc is not None and proc.poll() is None:
                import signal
                try:
                    os.killpg(proc.pid, signal.SIGTERM)  # the launcher leads its own session
                except ProcessLookupError:
                    pass
                try:
                    proc.wait(5)
                except Exception:
                    pass
        if self.mpirun_forward_thread is not None:
            self.mpirun_forward_thread.stop()
        self.mpirun_proc = self.mpirun_check_thread = self.mpirun_forward_thread = None
        self.workers = [None] * self.world_size
        if self.server is not None:
            self.server.stop(None)
            self.server = None
        self.func_id = 0
        res = self.func_result
        if res is not None:
            res.failed = res.failed or "job stopped"
            res.done.set()
            self.func_result = None
        self.peers = None
        if self.pg is not None:
            from raydp_amd.runtime import pgroup
            pgroup.remove_placement_group(self.pg)
            self.pg = None
        self._registered = 0
        self._register_event.clear()
        self.started = False

    def stop(self):
        self._reset()

    def __del__(self):
        try:
            if self.started:
                self.stop()
        except Exception:
            pass

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.stop()


class OpenMPIJob(MPIJob):
    def get_default_mpirun_script(self, context: MPIJobContext) -> List[str]:
        return ["mpirun", "--tag-output", "-H", ",".join(context.hosts), "-N", f"{context.num_procs_per_node}"]


class IntelMPIJob(MPIJob):
    def get_default_mpirun_script(self, context: MPIJobContext) -> List[str]:
        return ["mpirun", "-prepend-rank", "-hosts", ",".join(context.hosts), "-ppn",
                f"{context.num_procs_per_node}"]


class MPICHJob(MPIJob):
    def get_default_mpirun_script(self, context: MPIJobContext) -> List[str]:
        return ["mpirun", "-prepend-rank", "-hosts", ",".join(context.hosts), "-ppn",
                f"{context.num_procs_per_node}"]
