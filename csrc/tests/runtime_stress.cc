// Host-side stress test of the native runtime, built under sanitizers
// (scripts/sanitize_runtime.sh, tests/test_sanitizers.py): ASan+UBSan and TSan variants.
//
// * object store (csrc/runtime/objstore.cc): T threads and P forked processes share one arena
//   and create / fill / seal / get / verify / release / delete objects of random sizes, so
//   allocator coalescing, the slot table, pinning and the robust process-shared mutex run
//   under contention; every read checks the object's fill pattern.
// * frames (csrc/common/frame.h): encode/decode round trips of random string lists, and a
//   decode of truncated payloads must fail cleanly.
// SURVEY.md §5.2 ("build the C++ runtime with -fsanitize=thread and
// -fsanitize=address,undefined CI variants").
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <random>
#include <string>
#include <vector>

#include "frame.h"

extern "C" {
void* rt_store_create(const char* path, uint64_t capacity, uint32_t nslots);
void* rt_store_open(const char* path);
void rt_store_close(void* hs);
int rt_store_unlink(const char* path);
uint8_t* rt_store_data(void* hs);
int64_t rt_obj_create(void* hs, const char* id, uint64_t size, int32_t kind, int64_t pid);
int rt_obj_seal(void* hs, const char* id);
int rt_obj_get(void* hs, const char* id, uint64_t* off, uint64_t* size, int32_t* kind);
int rt_obj_release(void* hs, const char* id);
int rt_obj_delete(void* hs, const char* id);
}

namespace {

std::atomic<long> g_errors{0};
std::string g_path;

struct Args {
  int worker;
  int iters;
};

void* store_worker(void* p) {
  Args* a = (Args*)p;
  void* s = rt_store_open(g_path.c_str());
  if (!s) {
    g_errors++;
    return nullptr;
  }
  std::mt19937_64 rng(1234 + a->worker);
  uint8_t* data = rt_store_data(s);
  for (int it = 0; it < a->iters; ++it) {
    char id[40];
    snprintf(id, sizeof(id), "w%02dp%05di%06d", a->worker, (int)getpid() % 100000, it);
    const uint64_t size = 1 + rng() % 65536;
    int64_t off = rt_obj_create(s, id, size, 1, getpid());
    if (off == -1) continue;  // arena full under contention: fine
    if (off < 0) {
      g_errors++;
      continue;
    }
    const uint8_t pat = (uint8_t)(it * 31 + a->worker);
    memset(data + off, pat, size);
    if (rt_obj_seal(s, id) != 0) g_errors++;
    uint64_t goff = 0, gsize = 0;
    int32_t kind = 0;
    if (rt_obj_get(s, id, &goff, &gsize, &kind) != 0 || gsize != size || kind != 1) {
      g_errors++;
      continue;
    }
    for (uint64_t k = 0; k < gsize; k += 977)
      if (data[goff + k] != pat) {
        g_errors++;
        break;
      }
    if (rt_obj_release(s, id) != 0) g_errors++;
    if (rng() % 4 != 0 && rt_obj_delete(s, id) != 0) g_errors++;
  }
  rt_store_close(s);
  return nullptr;
}

int frame_checks() {
  std::mt19937 rng(7);
  int bad = 0;
  for (int it = 0; it < 2000; ++it) {
    rx_frame::Msg m;
    m.op = rng();
    const int n = rng() % 12;
    for (int i = 0; i < n; ++i) {
      std::string x(rng() % 300, '\0');
      for (auto& c : x) c = (char)rng();
      m.s.push_back(x);
    }
    std::string enc = rx_frame::encode(m);
    rx_frame::Msg d;
    if (!rx_frame::decode(enc.substr(4), d) || d.op != m.op || d.s != m.s) ++bad;
    if (enc.size() > 13) {
      rx_frame::Msg t;
      // truncated payloads must be rejected, never read out of bounds
      if (rx_frame::decode(enc.substr(4, enc.size() - 4 - 1 - rng() % 4), t) && n > 0 && t.s == m.s) ++bad;
    }
  }
  return bad;
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  const int procs = argc > 2 ? atoi(argv[2]) : 2;
  const int iters = argc > 3 ? atoi(argv[3]) : 2000;
  g_path = "/dev/shm/raydp_stress_" + std::to_string(getpid());
  void* s = rt_store_create(g_path.c_str(), 64ull << 20, 4096);
  if (!s) {
    fprintf(stderr, "store create failed\n");
    return 2;
  }
  const int fb = frame_checks();
  std::vector<pid_t> kids;
  for (int p = 1; p < procs; ++p) {
    pid_t k = fork();
    if (k == 0) {
      std::vector<pthread_t> ts(threads);
      std::vector<Args> as(threads);
      for (int t = 0; t < threads; ++t) {
        as[t] = {100 * p + t, iters};
        pthread_create(&ts[t], nullptr, store_worker, &as[t]);
      }
      for (auto& t : ts) pthread_join(t, nullptr);
      _exit(g_errors.load() ? 1 : 0);
    }
    kids.push_back(k);
  }
  std::vector<pthread_t> ts(threads);
  std::vector<Args> as(threads);
  for (int t = 0; t < threads; ++t) {
    as[t] = {t, iters};
    pthread_create(&ts[t], nullptr, store_worker, &as[t]);
  }
  for (auto& t : ts) pthread_join(t, nullptr);
  int child_fail = 0;
  for (pid_t k : kids) {
    int st = 0;
    waitpid(k, &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) ++child_fail;
  }
  rt_store_close(s);
  rt_store_unlink(g_path.c_str());
  printf("runtime_stress: store errors %ld, child failures %d, frame errors %d\n", g_errors.load(), child_fail, fb);
  return (g_errors.load() || child_fail || fb) ? 1 : 0;
}
