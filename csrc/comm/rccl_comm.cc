// Gradient all-reduce for the fused trainer's native step loop, straight on RCCL.
//
// The fused NYC step (csrc/hip/fused_mlp.hip: rx_mlp_train_steps) enqueues kernel -> all-reduce
// -> optimizer for every step of an epoch from C++, so a multi-GPU epoch has no Python in the
// loop. This file provides that all-reduce: a communicator of its own over RCCL (over xGMI on
// MI355X), created from a unique id that rank 0 generates and the ranks exchange through
// torch.distributed. RCCL is resolved with dlopen so the library torch already loaded is
// reused (no second copy, no link-time dependency). The whole gradient vector is one bucket:
// the NYC model is 194 KB of fp32, far below any size where splitting into buckets pays.
//
// Reference role: the DDP/Horovod gradient all-reduce of the reference's training paths
// (python/raydp/torch/estimator.py:243 prepare_model -> DDP; examples/horovod_nyctaxi.py:133).
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <string.h>

namespace {

struct UniqueId {
  char internal[128];
};
typedef void* Comm;
typedef int (*GetUniqueIdFn)(UniqueId*);
typedef int (*CommInitRankFn)(Comm*, int, UniqueId, int);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef int (*BroadcastFn)(const void*, void*, size_t, int, int, Comm, hipStream_t);
typedef int (*CommDestroyFn)(Comm);
typedef const char* (*ErrStrFn)(int);

constexpr int kFloat32 = 7;  // ncclFloat32
constexpr int kSum = 0;      // ncclSum

struct Api {
  void* h = nullptr;
  GetUniqueIdFn get_uid = nullptr;
  CommInitRankFn init = nullptr;
  AllReduceFn allreduce = nullptr;
  BroadcastFn bcast = nullptr;
  CommDestroyFn destroy = nullptr;
  ErrStrFn err = nullptr;
};

Api g_api;

bool load_api() {
  if (g_api.h) return true;
  const char* names[] = {"librccl.so.1", "librccl.so"};
  for (const char* n : names) {
    g_api.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);  // the copy torch loaded
    if (g_api.h) break;
  }
  if (!g_api.h)
    for (const char* n : names) {
      g_api.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
      if (g_api.h) break;
    }
  if (!g_api.h) return false;
  g_api.get_uid = (GetUniqueIdFn)dlsym(g_api.h, "ncclGetUniqueId");
  g_api.init = (CommInitRankFn)dlsym(g_api.h, "ncclCommInitRank");
  g_api.allreduce = (AllReduceFn)dlsym(g_api.h, "ncclAllReduce");
  g_api.bcast = (BroadcastFn)dlsym(g_api.h, "ncclBroadcast");
  g_api.destroy = (CommDestroyFn)dlsym(g_api.h, "ncclCommDestroy");
  g_api.err = (ErrStrFn)dlsym(g_api.h, "ncclGetErrorString");
  return g_api.get_uid && g_api.init && g_api.allreduce && g_api.destroy;
}

struct Ctx {
  Comm comm;
  int nranks, rank;
};

}  // namespace

extern "C" {

int rx_comm_available() { return load_api() ? 1 : 0; }

int rx_comm_unique_id(char* out128) {
  if (!load_api()) return -1;
  UniqueId id;
  int rc = g_api.get_uid(&id);
  if (rc) return rc;
  memcpy(out128, id.internal, 128);
  return 0;
}

void* rx_comm_init(int nranks, int rank, const char* uid128, int device) {
  if (!load_api()) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  UniqueId id;
  memcpy(id.internal, uid128, 128);
  Ctx* c = new Ctx{nullptr, nranks, rank};
  int rc = g_api.init(&c->comm, nranks, id, rank);
  if (rc) {
    fprintf(stderr, "rx_comm_init: ncclCommInitRank failed: %s\n", g_api.err ? g_api.err(rc) : "?");
    delete c;
    return nullptr;
  }
  return c;
}

// rx_allreduce_fn signature used by rx_mlp_train_steps: in-place sum over all ranks.
int rx_comm_allreduce(float* buf, int n, void* ctx, hipStream_t stream) {
  Ctx* c = (Ctx*)ctx;
  if (c->nranks == 1) return 0;
  return g_api.allreduce(buf, buf, (size_t)n, kFloat32, kSum, c->comm, stream);
}

int rx_comm_broadcast(float* buf, int n, int root, void* ctx, hipStream_t stream) {
  Ctx* c = (Ctx*)ctx;
  if (c->nranks == 1) return 0;
  return g_api.bcast(buf, buf, (size_t)n, kFloat32, root, c->comm, stream);
}

int rx_comm_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return 0;
  int rc = g_api.destroy(c->comm);
  delete c;
  return rc;
}

}  // extern "C"
