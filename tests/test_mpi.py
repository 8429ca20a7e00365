"""MPI job API (port of the reference's python/raydp/tests/test_mpi.py).

``mpirun`` is not installed in this image, so the jobs run through the built-in launcher
(raydp_amd/mpi/launcher.py), which exports the same per-flavour rank variables.
"""
import pytest

from raydp_amd import runtime
from raydp_amd.mpi import MPIJobContext, WorkerContext, create_mpi_job
from raydp_amd.runtime.pgroup import placement_group, remove_placement_group
from raydp_amd.utils import get_node_ip_address


@pytest.fixture
def rt():
    runtime.shutdown()
    runtime.init(num_cpus=4)
    yield
    runtime.shutdown()


@pytest.mark.timeout(60)
@pytest.mark.parametrize("mpi_type", ["mpich", "openmpi", "intel_mpi"])
def test_mpi_start(rt, mpi_type):
    job = create_mpi_job(job_name="test", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                         timeout=20, mpi_type=mpi_type)
    job.start()

    def func(context: WorkerContext):
        return context.job_id, context.world_rank, context.local_rank

    results = job.run(func)
    assert [r[0] for r in results] == ["test", "test"]
    assert [r[1] for r in results] == [0, 1]
    job.stop()
    # restart the same job object
    job.start()
    results = job.run(lambda ctx: ctx.job_id)
    assert results == ["test", "test"]
    assert job.run(lambda ctx: ctx.world_rank * 10) == [0, 10]  # function ids advance
    job.stop()


@pytest.mark.timeout(60)
def test_mpi_get_rank_address(rt):
    with create_mpi_job(job_name="test", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                        timeout=20, mpi_type="mpich") as job:
        addresses = job.get_rank_addresses()
        assert len(addresses) == 2
        assert get_node_ip_address() == addresses[0] == addresses[1]


@pytest.mark.timeout(60)
def test_mpi_with_script_prepare_fn(rt):
    def script_prepare_fn(context: MPIJobContext):
        context.add_env("is_test", "True")
        return ["mpirun", "-prepend-rank", "-hosts", ",".join(context.hosts), "-ppn",
                f"{context.num_procs_per_node}"]

    with create_mpi_job(job_name="test", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                        timeout=20, mpi_type="mpich", mpi_script_prepare_fn=script_prepare_fn) as job:
        def f(context: WorkerContext):
            import os
            return os.environ.get("is_test", None)
        assert job.run(f) == ["True", "True"]


@pytest.mark.timeout(60)
def test_mpi_with_pg(rt):
    pg = placement_group(bundles=[{"CPU": 2}], strategy="STRICT_SPREAD")
    with create_mpi_job(job_name="test", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                        timeout=20, mpi_type="mpich", placement_group=pg,
                        placement_group_bundle_indexes=[0]) as job:
        assert job.run(lambda c: c.job_id) == ["test", "test"]
    remove_placement_group(pg)


@pytest.mark.timeout(60)
def test_mpi_rank_exception_propagates(rt):
    with create_mpi_job(job_name="err", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                        timeout=20, mpi_type="mpich") as job:
        def bad(ctx):
            if ctx.world_rank == 1:
                raise ValueError("boom")
            return 1
        with pytest.raises(RuntimeError, match="boom"):
            job.run(bad)
        assert job.run(lambda c: c.world_rank) == [0, 1]  # job still usable


def test_launcher_parses_mpirun_flags():
    from raydp_amd.mpi.launcher import parse_mpirun
    hosts, ppn, np_, prefix, env, prog = parse_mpirun(
        ["-prepend-rank", "-hosts", "a,b", "-ppn", "2", "-genv", "K", "V", "python", "x.py"])
    assert hosts == ["a", "b"] and ppn == 2 and np_ is None and prefix and env == {"K": "V"}
    assert prog == ["python", "x.py"]
    hosts, ppn, *_ , prog = parse_mpirun(["--tag-output", "-H", "h1", "-N", "3", "--", "p"])
    assert hosts == ["h1"] and ppn == 3 and prog == ["p"]


def test_wire_messages_roundtrip():
    from raydp_amd.mpi import network
    m = network.RegisterWorkerServiceRequest(world_rank=3, worker_ip="1.2.3.4", worker_port=99)
    back = network.RegisterWorkerServiceRequest.FromString(m.SerializeToString())
    assert (back.world_rank, back.worker_ip, back.worker_port) == (3, "1.2.3.4", 99)
