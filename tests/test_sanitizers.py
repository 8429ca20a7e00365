"""Host C++ runtime under sanitizers (the reference has none).

* the object-store / frame stress test (csrc/tests/runtime_stress.cc) built with
  AddressSanitizer+UBSan and with ThreadSanitizer, run with several threads and processes;
* the fused expression VM driven by random well-typed programs (csrc/tests/expr_vm_fuzz.cc)
  under AddressSanitizer+UBSan (incl. float-cast-overflow);
* the supervisor, app master and shuffle service built with ASan+UBSan and driven through a
  protocol session (spawn / kill / restart, registration / restart remap / kill, map-output
  register / fd-passing fetch); their logs must hold no sanitizer report.
"""
import os
import signal
import subprocess
import tempfile
import time

import pyarrow as pa
import pytest

from raydp_amd.native import build

_DIRS = {}


def _built(kind):
    if kind not in _DIRS:
        d = tempfile.mkdtemp(prefix=f"raydp_{kind}_")
        build.build_sanitized(kind, d)
        _DIRS[kind] = d
    return _DIRS[kind]


@pytest.mark.parametrize("kind,args", [("asan", ["4", "3", "1500"]), ("tsan", ["4", "1", "800"])])
def test_runtime_stress_under_sanitizer(kind, args):
    exe = os.path.join(_built(kind), "runtime_stress")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "store errors 0" in r.stdout and "Sanitizer" not in r.stdout


def test_expression_vm_random_programs_under_asan_ubsan():
    """csrc/tests/expr_vm_fuzz.cc: well-typed random programs of every opcode over adversarial
    values (nulls, NaN/inf, INT_MIN, huge timestamps, zero divisors) and random filters; the
    32-bit calendar path is checked against the 64-bit one over its whole range."""
    exe = os.path.join(_built("asan"), "expr_vm_fuzz")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "250", "7"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "calendar mismatches 0" in r.stdout and "runtime error" not in r.stdout


def _no_reports(path):
    if not os.path.exists(path):
        return
    text = open(path, errors="replace").read()
    assert "AddressSanitizer" not in text and "runtime error:" not in text and "LeakSanitizer" not in text, text[-4000:]


def test_services_under_asan(monkeypatch):
    d = _built("asan")
    monkeypatch.setenv("RAYDP_NATIVE_BIN_DIR", d)
    monkeypatch.setenv("ASAN_OPTIONS", "detect_leaks=1")
    from raydp_amd.runtime.supervisor import SupervisorClient
    from raydp_amd.spark import shuffle as S
    from raydp_amd.spark.appmaster import AppMasterClient, ExecutorRegistration
    work = tempfile.mkdtemp(prefix="raydp_asan_session_")
    os.makedirs(os.path.join(work, "logs"), exist_ok=True)

    # supervisor: spawn, SIGKILL -> restart, kill without restart
    sup = SupervisorClient.launch(work)
    assert sup.proc.args[0].startswith(d)
    pid = sup.spawn("a1", ["sleep", "30"], {"RAYDP_JOB_ID": "j1"}, log=os.path.join(work, "logs", "a1.log"),
                    max_restarts=1)
    os.kill(pid, signal.SIGKILL)
    deadline = time.time() + 10
    while time.time() < deadline and sup.list().get("a1", {}).get("pid") in (None, pid):
        time.sleep(0.02)
    assert sup.kill("a1", no_restart=True)
    sup.shutdown()

    # app master + shuffle service
    m = AppMasterClient.launch(work)
    assert m.proc.args[0].startswith(d)
    m.register_app("asan", 2, 1, 128, 1.0, shuffle_service=True, local_dir=os.path.join(work, "shuffle"))
    r0 = ExecutorRegistration(m.sock_path, "0", "n0", restarted=False)
    r1 = ExecutorRegistration(m.sock_path, "1", "n0", restarted=False)
    t = pa.table({"x": list(range(100))})
    S.write_map_output(r0.shuffle_socket, "sa", 0, [t, t.slice(0, 0), t.slice(10, 5)])
    assert S.client(r0.shuffle_socket).fetch("sa", 0, 2).equals(t.slice(10, 5))
    r1.close()
    time.sleep(0.1)
    r1b = ExecutorRegistration(m.sock_path, "1", "n0", restarted=True)
    assert r1b.executor_id == "2"
    assert m.kill_executors(["0"]) == ["0"]
    m.app_info()
    m.unregister_app()
    r0.close()
    r1b.close()
    m.shutdown()
    time.sleep(0.3)  # shuffle service is SIGTERMed by the master on shutdown
    _no_reports(os.path.join(work, "logs", "appmaster.err"))
    _no_reports(os.path.join(work, "logs", "supervisor.err"))


@pytest.mark.parametrize("kind,mode", [("asan", "full"), ("tsan", "sync")])
def test_native_executor_core_under_sanitizer(kind, mode):
    """csrc/tests/executor_stress.cc: four driver threads submit CSV-split tasks of one stage to
    the native task loop and wait on them while another thread reads the block cache and the
    CSV inference reader. ASan+UBSan runs the whole data path; ThreadSanitizer runs the queue,
    waits and cache alone (Arrow's uninstrumented thread pool and allocator only add noise)."""
    exe = os.path.join(_built(kind), "executor_stress")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    args = ["4", "5", "3000"] + (["sync"] if mode == "sync" else [])
    r = subprocess.run([exe] + args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "failures 0" in r.stdout and "Sanitizer" not in r.stdout and "runtime error" not in r.stdout
