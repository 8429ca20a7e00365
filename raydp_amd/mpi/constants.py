"""Environment keys shared by the MPI job driver and its worker processes.

Same key names as the reference (``python/raydp/mpi/constants.py:18-28``) so scripts that
inspect them keep working.
"""
import os

MPI_TYPE = "raydp_mpi_type"
MPI_JOB_ID = "raydp_mpi_job_id"
MPI_DRIVER_HOST = "raydp_mpi_driver_host"
MPI_DRIVER_PORT = "raydp_mpi_driver_port"
MAXIMUM_WAIT_TIME_OUT = "raydp_maximum_wait_time_out"

MPI_MAIN_CLASS_PATH = os.path.join(os.path.dirname(os.path.realpath(__file__)), "worker.py")

MAX_MESSAGE_LENGTH = 64 * 1024 * 1024
