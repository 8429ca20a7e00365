"""Actor call transport (raydp_amd/runtime/actor_worker.py): frames of any size arrive whole
(one MSG_WAITALL receive, gathered header + payload send), and a sequential actor -- whose
calls now run on the connection's reader thread -- still runs one call at a time when several
driver threads call it at once."""
import socket
import threading
import time

import pytest

from raydp_amd.runtime.actor_worker import recv_frame, send_frame


@pytest.mark.parametrize("n", [0, 1, 4095, 4096, 100_000, 3_000_001])
def test_frames_round_trip_whole(n):
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_STREAM)
    lock = threading.Lock()
    data = bytes((i * 7) & 0xFF for i in range(min(n, 1000))) * (n // 1000 + 1)
    data = data[:n]
    t = threading.Thread(target=lambda: send_frame(b, threading.Lock(), bytes(recv_frame(b))))
    t.start()
    send_frame(a, lock, data)
    got = recv_frame(a)
    t.join()
    assert bytes(got) == data
    a.close()
    b.close()


def test_sequential_actor_never_overlaps_calls():
    import raydp_amd.runtime as rt
    owned = not rt.is_initialized()
    if owned:
        rt.init(num_cpus=2)
    try:
        @rt.remote
        class Seq:
            def __init__(self):
                self.active, self.max_active = 0, 0

            def work(self, x):
                self.active += 1
                self.max_active = max(self.max_active, self.active)
                time.sleep(0.002)
                self.active -= 1
                return x

            def peak(self):
                return self.max_active

        a = Seq.remote()
        out = []

        def caller(base):
            out.extend(rt.get([a.work.remote(base + i) for i in range(10)]))
        ts = [threading.Thread(target=caller, args=(100 * j,)) for j in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert sorted(out) == sorted(100 * j + i for j in range(4) for i in range(10))
        assert rt.get(a.peak.remote()) == 1
        big = b"z" * 2_000_000
        assert rt.get(a.work.remote(big)) == big
        rt.kill(a)
    finally:
        if owned:
            rt.shutdown()
