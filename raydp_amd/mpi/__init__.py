"""MPI jobs on the runtime (reference: ``python/raydp/mpi/__init__.py``).

``create_mpi_job`` returns a job object for Open MPI, Intel MPI or MPICH; ranks are launched
by ``mpirun`` when installed, otherwise by :mod:`raydp_amd.mpi.launcher` with the same rank
environment variables.
"""
from typing import Callable, List, Optional

from raydp_amd.mpi.job import (IntelMPIJob, MPICHJob, MPIJob, MPIJobContext, MPIType,  # noqa: F401
                               OpenMPIJob)
from raydp_amd.mpi.worker import WorkerContext  # noqa: F401

_TYPES = {"openmpi": (MPIType.OPEN_MPI, OpenMPIJob), "intel_mpi": (MPIType.INTEL_MPI, IntelMPIJob),
          "mpich": (MPIType.MPICH, MPICHJob)}


def _get_mpi_type(mpi_type: str) -> Optional[MPIType]:
    t = _TYPES.get(mpi_type.strip().lower())
    return t[0] if t else None


def create_mpi_job(job_name: str, world_size: int, num_cpus_per_process: int, num_processes_per_node: int,
                   mpi_script_prepare_fn: Callable = None, timeout: int = 1, mpi_type: str = "intel_mpi",
                   placement_group=None, placement_group_bundle_indexes: List[int] = None) -> MPIJob:
    """Create (not start) an MPI job; see :class:`raydp_amd.mpi.job.MPIJob`."""
    t = _TYPES.get(mpi_type.strip().lower())
    if t is None:
        raise Exception(f"MPI type: {mpi_type} not supported now")
    mtype, cls = t
    return cls(mpi_type=mtype, job_name=job_name, world_size=world_size,
               num_cpus_per_process=num_cpus_per_process, num_processes_per_node=num_processes_per_node,
               mpi_script_prepare_fn=mpi_script_prepare_fn, timeout=timeout, placement_group=placement_group,
               placement_group_bundle_indexes=placement_group_bundle_indexes)


__all__ = ["create_mpi_job", "MPIJobContext", "WorkerContext", "MPIType", "MPIJob"]
