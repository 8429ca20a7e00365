"""Other processes attaching to a running node (``raydp_amd/runtime/gcs.py``): the equivalent of
``ray.init(address=...)`` that the reference relies on for MPI ranks
(``python/raydp/mpi/mpi_worker.py:159-160``), ``raydp-submit`` against an existing cluster
(``doc/spark_on_ray.md:116-144``) and its client-address test fixtures
(``python/raydp/tests/conftest.py:77-84``)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

from raydp_amd import runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def head():
    runtime.shutdown()
    runtime.init(num_cpus=4)
    yield runtime.core.current_node()
    runtime.shutdown()


@runtime.remote
class Counter:
    def __init__(self, start):
        self.n = start

    def incr(self, k):
        self.n += k
        return self.n

    def pid(self):
        return os.getpid()


def _child(code: str, *args, env=None, timeout=120):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    for k in ("RAYDP_SESSION_DIR", "RAYDP_STORE_PATH", "RAYDP_ADDRESS"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", textwrap.dedent(code)] + list(args), stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=timeout, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_second_driver_gets_objects_and_calls_named_actor(head):
    ref = runtime.put({"payload": list(range(10))})
    c = Counter.options(name="shared_counter").remote(100)
    assert runtime.get(c.incr.remote(1)) == 101
    addr = runtime.core.address()
    assert addr.startswith("raydp://")
    before = runtime.api.available_resources()["CPU"]
    out = _child("""
        import json, sys
        from raydp_amd import runtime
        from raydp_amd.runtime.objects import ObjectRef
        runtime.init(address=sys.argv[1])
        obj = runtime.get(ObjectRef(sys.argv[2], node_id=sys.argv[3]))
        h = runtime.get_actor("shared_counter")
        v = runtime.get(h.incr.remote(10))
        mine = runtime.put("from the second driver")

        @runtime.remote
        class Echo:
            def hi(self):
                return "hi"
        e = Echo.options(name="child_echo", num_cpus=1).remote()
        hi = runtime.get(e.hi.remote())
        res = runtime.api.cluster_resources()
        avail = runtime.api.available_resources()
        print(json.dumps({"obj": obj, "v": v, "mine": [mine.id, mine.node_id], "hi": hi,
                          "cpu": res["CPU"], "avail_cpu": avail["CPU"],
                          "session": runtime.core.current_node().session_dir}))
        runtime.shutdown()
    """, addr, ref.id, ref.node_id)
    assert out["obj"] == {"payload": list(range(10))}
    assert out["v"] == 111 and runtime.get(c.incr.remote(0)) == 111     # same actor state
    assert out["hi"] == "hi"
    assert out["cpu"] == 4.0 and out["avail_cpu"] == before - 1          # placed by the head
    assert out["session"] == head.session_dir
    from raydp_amd.runtime.objects import ObjectRef
    assert runtime.get(ObjectRef(out["mine"][0], node_id=out["mine"][1])) == "from the second driver"
    # the child's (non-detached) actor died with it and its reservation came back
    with pytest.raises(ValueError):
        runtime.get_actor("child_echo")
    assert runtime.api.available_resources()["CPU"] == before


def test_auto_address_and_env(head):
    out = _child("""
        import json
        from raydp_amd import runtime
        runtime.init(address="auto")
        a = runtime.core.current_node().session_dir
        runtime.shutdown()
        print(json.dumps({"a": a}))
    """)
    assert out["a"] == head.session_dir
    out = _child("""
        import json
        from raydp_amd import runtime
        runtime.init()          # RAYDP_ADDRESS
        print(json.dumps({"a": runtime.core.current_node().session_dir}))
        runtime.shutdown()
    """, env={"RAYDP_ADDRESS": runtime.core.address()})
    assert out["a"] == head.session_dir


def test_tcp_endpoint_requires_token(monkeypatch):
    runtime.shutdown()
    monkeypatch.setenv("RAYDP_RUNTIME_PORT", "0")
    runtime.init(num_cpus=2)
    try:
        node = runtime.core.current_node()
        tcp = node.gcs_service.tcp_address
        assert tcp.startswith("127.0.0.1:")
        token = node.gcs_service.token
        from raydp_amd.runtime.gcs import GcsClient, GcsError
        with pytest.raises((ConnectionError, GcsError, OSError)):
            GcsClient(f"{tcp}?token=wrong").call("info")
        with pytest.raises(ConnectionError):
            GcsClient(tcp)              # no token at all
        c = GcsClient(f"{tcp}?token={token}")
        assert c.call("info")["session_dir"] == node.session_dir
        c.call("kv_put", "k", "v")
        assert c.call("kv_get", "k") == "v"
        c.close()
    finally:
        runtime.shutdown()


def test_attached_driver_placement_group(head):
    out = _child("""
        import json, sys
        from raydp_amd import runtime
        from raydp_amd.runtime.pgroup import placement_group, remove_placement_group
        runtime.init(address=sys.argv[1])
        pg = placement_group([{"CPU": 1}, {"CPU": 1}], strategy="PACK")
        mid = runtime.api.available_resources()["CPU"]

        @runtime.remote
        class A:
            def ok(self):
                return 1
        a = A.options(placement_group=pg, placement_group_bundle_index=1, num_cpus=1).remote()
        v = runtime.get(a.ok.remote())
        runtime.kill(a)
        remove_placement_group(pg)
        end = runtime.api.available_resources()["CPU"]
        runtime.shutdown()
        print(json.dumps({"mid": mid, "v": v, "end": end}))
    """, runtime.core.address())
    assert out == {"mid": 2.0, "v": 1, "end": 4.0}


@pytest.mark.timeout(90)
def test_mpi_rank_reads_stored_object(head):
    from raydp_amd.mpi import create_mpi_job
    ref = runtime.put([3, 1, 4, 1, 5])
    rid, nid = ref.id, ref.node_id

    def fn(ctx):
        from raydp_amd import runtime as rt
        from raydp_amd.runtime.objects import ObjectRef
        return sum(rt.get(ObjectRef(rid, node_id=nid))) + ctx.world_rank

    with create_mpi_job(job_name="attach", world_size=2, num_cpus_per_process=1, num_processes_per_node=2,
                        timeout=20, mpi_type="mpich") as job:
        assert job.run(fn) == [14, 15]


def test_submit_runs_against_callers_node(head, tmp_path):
    ref = runtime.put("head object")
    app = tmp_path / "app.py"
    app.write_text(textwrap.dedent(f"""
        import json
        from raydp_amd import runtime
        from raydp_amd.runtime.objects import ObjectRef
        node = runtime.core.current_node()
        print(json.dumps({{"session": node.session_dir, "obj": runtime.get(ObjectRef("{ref.id}", node_id="{ref.node_id}"))}}))
    """))
    conf = tmp_path / "ray.conf"
    conf.write_text(json.dumps({"ray": {"address": runtime.core.address()}}))
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-m", "raydp_amd.submit", "--ray-conf", str(conf), str(app)],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out == {"session": head.session_dir, "obj": "head object"}
    # the head node is still up and serving after the submitted application detached
    assert runtime.get(ref) == "head object"


def test_detached_actor_of_attached_driver_keeps_its_reservation(head):
    """A detached actor placed by an attached driver keeps its CPU after that driver exits (the
    head must not hand it to the next actor); the reservation comes back once the actor's
    process is gone."""
    import signal
    import time
    before = runtime.api.available_resources()["CPU"]
    out = _child("""
        import json, os, sys
        from raydp_amd import runtime
        runtime.init(address=sys.argv[1])

        @runtime.remote
        class D:
            def pid(self):
                return os.getpid()
        d = D.options(name="detached_d", lifetime="detached", num_cpus=1).remote()
        pid = runtime.get(d.pid.remote())
        print(json.dumps({"pid": pid}))
    """, runtime.core.address())
    pid = out["pid"]
    try:
        time.sleep(1.5)             # the head noticed the connection close
        alive = True
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            alive = False
        assert alive, "the detached actor died with its driver"
        assert runtime.api.available_resources()["CPU"] == before - 1
    finally:
        try:
            os.kill(pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    deadline = time.time() + 15
    while runtime.api.available_resources()["CPU"] != before and time.time() < deadline:
        time.sleep(0.2)
    assert runtime.api.available_resources()["CPU"] == before


def test_tcp_endpoint_rejects_oversized_hello(monkeypatch):
    """The pre-authentication frame's length is checked before anything is allocated."""
    import socket
    import struct
    runtime.shutdown()
    monkeypatch.setenv("RAYDP_RUNTIME_PORT", "0")
    runtime.init(num_cpus=2)
    try:
        node = runtime.core.current_node()
        host, port = node.gcs_service.tcp_address.split(":")
        s = socket.create_connection((host, int(port)), timeout=5)
        s.sendall(struct.pack("<Q", 1 << 40))
        s.settimeout(5)
        assert s.recv(16) == b""      # closed by the head
        s.close()
        from raydp_amd.runtime.gcs import GcsClient
        c = GcsClient(f"{node.gcs_service.tcp_address}?token={node.gcs_service.token}")
        assert c.call("info")["session_dir"] == node.session_dir
        c.close()
    finally:
        runtime.shutdown()
