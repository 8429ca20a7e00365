"""Rank-side half of an MPI job (reference: ``python/raydp/mpi/mpi_worker.py``).

Each rank started by ``mpirun`` (or the built-in launcher) runs this file: it registers with
the driver's gRPC ``DriverService``, serves a ``WorkerService`` on an ephemeral port, and
executes the cloudpickled functions the driver sends, strictly in ``func_id`` order, on a
single task thread. Results (or the raised exception, which the reference drops) go back via
``RegisterFuncResult``. The process exits when the driver calls ``Stop``.
"""
import os
import sys
import threading
import traceback
from queue import Queue

if __name__ == "__main__" and __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__)))))

import cloudpickle  # noqa: E402

from raydp_amd.mpi import constants, network  # noqa: E402
from raydp_amd.mpi.utils import RemoteFunctionError, get_environ_value, get_node_ip_address  # noqa: E402,F401

_RANK_ENV = {
    0: ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_LOCAL_RANK"),   # MPIType.OPEN_MPI
    1: ("PMI_RANK", "MPI_LOCALRANKID"),                          # MPIType.INTEL_MPI
    2: ("PMI_RANK", "MPI_LOCALRANKID"),                          # MPIType.MPICH
}


def get_rank(mpi_type) -> tuple:
    key = getattr(mpi_type, "value", mpi_type)
    if key not in _RANK_ENV:
        raise Exception(f"Not supported MPI type: {mpi_type}")
    rk, lrk = _RANK_ENV[key]
    return int(os.environ[rk]), int(os.environ[lrk])


class WorkerContext:
    """What a function sent with ``MPIJob.run`` receives."""

    def __init__(self, job_id: str, world_rank: int, local_rank: int, node_ip: str):
        self.job_id = job_id
        self.world_rank = world_rank
        self.local_rank = local_rank
        self.node_ip = node_ip

    def __repr__(self):
        return (f"WorkerContext(job_id={self.job_id!r}, world_rank={self.world_rank}, "
                f"local_rank={self.local_rank}, node_ip={self.node_ip!r})")


class MPIWorker:
    def __init__(self, job_id: str, driver_host: str, driver_port: int, world_rank: int, local_rank: int):
        self.job_id = job_id
        self.driver = network.Stub(network.insecure_channel(f"{driver_host}:{driver_port}"), "DriverService")
        self.world_rank, self.local_rank = world_rank, local_rank
        self.node_ip = None
        self.server = None
        self.stop_event = threading.Event()
        self.queue: Queue = Queue()
        self.failed = None

    # --- WorkerService ---
    def RunFunction(self, request, context):
        self.queue.put(request)
        return network.Empty()

    def Stop(self, request, context):
        self.stop_event.set()
        self.queue.put(None)
        return network.Empty()

    def _task_loop(self, ctx: WorkerContext):
        expected = 0
        while True:
            req = self.queue.get()
            if req is None:
                return
            if req.func_id != expected:
                self.failed = Exception(f"rank {self.world_rank}: expected function id {expected}, "
                                        f"got {req.func_id}")
                self.stop_event.set()
                return
            try:
                result = cloudpickle.loads(req.func)(ctx)
            except BaseException as e:  # noqa: BLE001 - shipped back to the driver
                result = RemoteFunctionError(self.world_rank, e, traceback.format_exc())
            try:
                payload = cloudpickle.dumps(result)
            except Exception as e:  # unpicklable result
                payload = cloudpickle.dumps(RemoteFunctionError(self.world_rank, RuntimeError(str(e)), ""))
            self.driver.RegisterFuncResult(network.FunctionResult(
                world_rank=self.world_rank, func_id=expected, result=payload))
            expected += 1

    def run(self, wait_timeout: float = 30.0) -> int:
        reply = self.driver.RegisterWorker(network.RegisterWorkerRequest(
            job_id=self.job_id, world_rank=self.world_rank), timeout=wait_timeout)
        addrs = list(reply.node_addresses)
        self.node_ip = get_node_ip_address(addrs) or (addrs[0] if addrs else "127.0.0.1")
        self.server = network.make_server(max_workers=2)
        network.add_service(self.server, "WorkerService", self)
        port = self.server.add_insecure_port(f"{self.node_ip}:0")
        self.server.start()
        rep = self.driver.RegisterWorkerService(network.RegisterWorkerServiceRequest(
            world_rank=self.world_rank, worker_ip=self.node_ip, worker_port=port), timeout=wait_timeout)
        if rep.ray_address:
            # join the job driver's runtime node before any function runs (the reference's rank
            # calls ray.init(address=reply.ray_address), python/raydp/mpi/mpi_worker.py:159-160):
            # rank functions reach its object store and (named) actors
            os.environ.setdefault("RAYDP_RUNTIME_ADDRESS", rep.ray_address)
            try:
                from raydp_amd import runtime
                runtime.init(address=rep.ray_address)
            except (ConnectionError, OSError, ValueError) as e:
                print(f"MPI worker {self.world_rank}: cannot attach to the runtime at "
                      f"{rep.ray_address!r}: {e}", file=sys.stderr)
        ctx = WorkerContext(self.job_id, self.world_rank, self.local_rank, self.node_ip)
        t = threading.Thread(target=self._task_loop, args=(ctx,), name="mpi-task-runner", daemon=True)
        t.start()
        self.stop_event.wait()
        self.server.stop(0.5)
        self.driver.close()
        try:
            from raydp_amd.runtime import core
            if core.is_initialized():
                core.shutdown()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass
        if self.failed is not None:
            print(f"MPI worker failed: {self.failed}", file=sys.stderr)
            return 1
        return 0


def main() -> int:
    mpi_type = int(get_environ_value(constants.MPI_TYPE))
    rank, local_rank = get_rank(mpi_type)
    w = MPIWorker(get_environ_value(constants.MPI_JOB_ID), get_environ_value(constants.MPI_DRIVER_HOST),
                  int(get_environ_value(constants.MPI_DRIVER_PORT)), rank, local_rank)
    return w.run(float(os.environ.get(constants.MAXIMUM_WAIT_TIME_OUT, "30")))


if __name__ == "__main__":
    sys.exit(main())
