// Bounded busy-wait for a socket to become readable (raydp_amd/runtime/actor_worker.py
// wait_readable). An actor call is a request frame and a reply frame over a Unix socket; a
// thread that sleeps in recv() between calls is woken by the kernel when the frame lands, and
// on a host whose idle cores drop into deep idle states that wake-up -- not the copy, not the
// Python work -- dominates a small call (measured in the CPU container: a no-op round trip
// 169 us back to back, 850 us after 5 ms idle, scripts/dev/actor_rtt.py). Polling the socket
// for a bounded window before the blocking read keeps the receiving thread on its core for
// calls that arrive in quick succession (the stages and fits of a pipeline), at the price of
// that core for the window. Called through ctypes, so the GIL is released while it spins.
#include <errno.h>
#include <stdint.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <time.h>

namespace {
inline int64_t now_ns() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return static_cast<int64_t>(t.tv_sec) * 1000000000LL + t.tv_nsec;
}
}  // namespace

extern "C" {

// 1 when `fd` is readable (data or EOF or an error the blocking read will report), 0 when
// `max_ns` passed first.
int rt_spin_readable(int fd, int64_t max_ns) {
  const int64_t start = now_ns();
  char c;
  for (;;) {
    const ssize_t r = recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    if (r >= 0) return 1;
    if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) return 1;
    for (int k = 0; k < 64; ++k) __builtin_ia32_pause();
    if (now_ns() - start >= max_ns) return 0;
  }
}

}  // extern "C"
