// Native executor core under sanitizers: several driver threads submit CSV-split
// tasks of a pass-through stage to one task loop and wait for them, while other threads hammer
// the partition cache and the CSV inference reader. Every task's rows land in the object store
// as Arrow IPC; the row total must equal the file's.
//
//   executor_stress <threads> <tasks per thread> <rows> [sync]
//
// "sync": the tasks point at a missing file (each fails in the task loop before any Arrow code
// runs) and the CSV reader is not driven -- the task queue, waits and cache alone, for
// ThreadSanitizer (Arrow's uninstrumented thread pool and allocator would only add noise).
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* rt_store_create(const char* path, uint64_t capacity, uint32_t nslots);
void rt_store_close(void* hs);
int rt_store_unlink(const char* path);
int rt_obj_delete(void* hs, const char* id);
void* rx_exec_create(int threads);
void rx_exec_destroy(void* ex);
void* rx_stage_create(const uint8_t* spec, int64_t len, char* err, int errlen);
void rx_stage_destroy(void* st);
int64_t rx_exec_submit(void* ex, void* stage, const char* path, int64_t lo, int64_t hi, void* stream, void* store,
                       const char* oid, void* tap, void* user, char* err, int errlen);
int rx_exec_wait(void* ex, int64_t id, int64_t* rows, int64_t* bytes, int64_t* times, char* err, int errlen);
void rx_cache_put(void* ex, const char* rdd, int32_t idx, const char* oid, char* old);
int rx_cache_get(void* ex, const char* rdd, int32_t idx, char* oid);
int rx_cache_pop(void* ex, const char* rdd, int32_t idx, char* oid);
int rx_cache_list(void* ex, const char* rdd, int32_t* out, int max);
int rx_cache_unpersist(void* ex, const char* rdd, void* store);
int rx_csv_infer(const char* data, int64_t len, char delim, void* out);
}

namespace {

struct Spec {
  std::string b;
  void u8(uint8_t v) { b.push_back(static_cast<char>(v)); }
  void u32(uint32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }
  void i32(int32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }
  void s(const std::string& v) { u32(static_cast<uint32_t>(v.size())); b += v; }
};

// header + (a int64, b double, s string) columns; one segment, no VM code, all columns passed
std::string pass_through_stage() {
  Spec w;
  w.u32(0x31535852u);
  w.u8(1);
  w.u8(',');
  w.s("");
  const char* names[3] = {"a", "b", "s"};
  const char* types[3] = {"int64", "double", "string"};
  w.u32(3);
  for (int i = 0; i < 3; ++i) {
    w.s(names[i]);
    w.s(types[i]);
  }
  w.u32(1);   // segments
  w.u32(0);   // code
  w.u32(0);   // fconst
  w.u32(0);   // iconst
  w.u32(0);   // live
  w.i32(1);   // nslots
  w.u32(0);   // inputs
  w.u32(0);   // outputs
  w.u8(0);    // has_filter
  w.u8(0);    // taps
  w.u32(3);
  for (int i = 0; i < 3; ++i) {
    w.s(names[i]);
    w.u8(1);  // kind: input column
    w.i32(i);
  }
  return w.b;
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  const int per = argc > 2 ? atoi(argv[2]) : 8;
  const int rows = argc > 3 ? atoi(argv[3]) : 5000;
  const bool sync_only = argc > 4 && strcmp(argv[4], "sync") == 0;
  char csv[] = "/tmp/rx_exec_stress_XXXXXX";
  int fd = mkstemp(csv);
  if (fd < 0) return 2;
  std::string data = "a,b,s\n";
  for (int r = 0; r < rows; ++r) data += std::to_string(r) + "," + std::to_string(r * 0.25) + ",x" + std::to_string(r % 13) + "\n";
  if (write(fd, data.data(), data.size()) != static_cast<ssize_t>(data.size())) return 2;
  close(fd);
  const std::string store_path = std::string("/dev/shm/rx_exec_stress_") + std::to_string(getpid());
  void* store = rt_store_create(store_path.c_str(), 256ull << 20, 4096);
  if (!store) return 3;
  void* ex = rx_exec_create(4);
  char err[512];
  const std::string spec = pass_through_stage();
  void* stage = rx_stage_create(reinterpret_cast<const uint8_t*>(spec.data()), static_cast<int64_t>(spec.size()), err,
                                sizeof(err));
  if (!stage) {
    printf("stage error: %s\n", err);
    return 4;
  }
  const int64_t size = static_cast<int64_t>(data.size());
  std::atomic<int64_t> total{0}, failures{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&, t] {
      for (int round = 0; round < per; ++round) {
        // one pass over the whole file in `splits` byte ranges; ids unique per (t, round, split)
        const int splits = 1 + (t + round) % 5;
        std::vector<int64_t> ids;
        std::vector<std::string> oids;
        for (int k = 0; k < splits; ++k) {
          char oid[33];
          snprintf(oid, sizeof(oid), "t%02dr%03ds%02d%020d", t, round, k, 0);
          const int64_t lo = size * k / splits, hi = size * (k + 1) / splits;
          char e[256];
          ids.push_back(rx_exec_submit(ex, stage, sync_only ? "/nonexistent/rx.csv" : csv, lo, hi, nullptr, store, oid,
                                       nullptr, nullptr, e, sizeof(e)));
          oids.push_back(oid);
        }
        int64_t got = 0;
        for (size_t k = 0; k < ids.size(); ++k) {
          int64_t n = 0, b = 0, tm[3];
          char e[256];
          const int st = rx_exec_wait(ex, ids[k], &n, &b, tm, e, sizeof(e));
          if (sync_only) {
            if (st != -1) failures++;     // the missing file must surface as a task error
          } else if (st != 0) {
            failures++;
            printf("task error %d: %s\n", st, e);
          }
          got += n;
          char old[33];
          rx_cache_put(ex, "stress", static_cast<int32_t>(t * 1000 + round * 10 + static_cast<int>(k)),
                       oids[k].c_str(), old);
        }
        if (!sync_only && got != rows) failures++;
        total += sync_only ? rows : got;
      }
    });
  }
  // a burst submitter: hundreds of queued tasks (failing fast on a missing file) inserted while
  // the threads above wait on theirs -- the task map rehashes under a waiter that released the
  // executor lock for an inline run or a condition wait (the waiter must not keep an iterator)
  std::thread burst([&] {
    for (int round = 0; round < per; ++round) {
      std::vector<int64_t> ids;
      for (int k = 0; k < 256; ++k) {
        char oid[33], e[256];
        snprintf(oid, sizeof(oid), "burst%03d%04d%020d", round, k, 0);
        ids.push_back(rx_exec_submit(ex, stage, "/nonexistent/rx_burst.csv", 0, 1, nullptr, store, oid, nullptr, nullptr,
                                     e, sizeof(e)));
      }
      for (int64_t id : ids) {
        int64_t n = 0, b = 0, tm[3];
        char e[256];
        if (rx_exec_wait(ex, id, &n, &b, tm, e, sizeof(e)) != -1) failures++;
      }
    }
  });
  // concurrent cache readers and the CSV inference reader
  std::atomic<bool> stop{false};
  std::thread reader([&] {
    int32_t buf[256];
    char oid[33];
    while (!stop.load()) {
      rx_cache_list(ex, "stress", buf, 256);
      rx_cache_get(ex, "stress", 0, oid);
      unsigned char stream[64];
      if (!sync_only && rx_csv_infer(data.data(), static_cast<int64_t>(data.size()), ',', stream) == 1) {
        // release the exported stream (ArrowArrayStream.release is the 4th pointer)
        void (*release)(void*) = nullptr;
        memcpy(&release, stream + 3 * sizeof(void*), sizeof(release));
        if (release) release(stream);
      }
    }
  });
  for (auto& t : ts) t.join();
  burst.join();
  stop = true;
  reader.join();
  char oid[33];
  rx_cache_pop(ex, "stress", 0, oid);
  const int dropped = rx_cache_unpersist(ex, "stress", store);
  rx_stage_destroy(stage);
  rx_exec_destroy(ex);
  rt_store_close(store);
  rt_store_unlink(store_path.c_str());
  unlink(csv);
  printf("rows %lld expected %lld failures %lld dropped %d\n", static_cast<long long>(total.load()),
         static_cast<long long>(static_cast<int64_t>(rows) * threads * per), static_cast<long long>(failures.load()),
         dropped);
  return failures.load() == 0 && total.load() == static_cast<int64_t>(rows) * threads * per ? 0 : 1;
}
