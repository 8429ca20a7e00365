// Host side of the one-shot xGMI all-reduce (protocol: csrc/comm/xgmi.h) and its stand-alone
// reduce kernel.
//
// Setup (one communicator per process group, driven by raydp_amd/ops/comm.py XgmiComm):
//   rx_xg_create   -> allocate this rank's uncached exchange region, zero its flags
//   rx_xg_handle   -> 64-byte IPC handle of the region (exchanged over torch.distributed)
//   rx_xg_open     -> map every peer's region (hipIpcOpenMemHandle, lazy peer access)
// Use:
//   rx_xg_allreduce            -> in-place sum of a device fp32 buffer (copy into slot, one kernel)
//   rx_xg_devdesc/take_seq/slot -> the fused step loop (csrc/hip/fused_mlp.hip) reduces inside
//                                 its optimizer kernel instead
//   rx_xg_error                -> nonzero once any wait timed out (a peer never arrived)
//
// Reference role: the small-bucket gradient all-reduce of DDP / Horovod
// (python/raydp/torch/estimator.py:243; examples/horovod_nyctaxi.py:133-138), see SURVEY.md
// §2.11 K2 and §5.8 (one-shot P2P all-reduce for <= 1 MB buckets).
#include "comm/xgmi.h"

#include <stdio.h>
#include <string.h>

namespace {

struct XgHost {
  XgDev dev;
  void* base = nullptr;
  size_t bytes = 0;
  hipIpcMemHandle_t handle;
  unsigned seq = 0;
  int device = 0;
  bool opened[RX_XG_MAXR] = {false};
};

constexpr int kThreads = 256;
constexpr int kPerThread = 4;

__global__ __launch_bounds__(kThreads) void xg_reduce_kernel(XgDev x, float* __restrict__ out, int n, unsigned seq) {
  __shared__ int ok;
  if (threadIdx.x == 0) ok = rx_xg_rendezvous(x, seq) ? 1 : 0;
  __syncthreads();
  if (!ok) return;
  const int par = (int)(seq & 1u);
  const int base = blockIdx.x * kThreads * kPerThread + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kPerThread; ++k) {
    const int idx = base + k * kThreads;
    if (idx < n) out[idx] = rx_xg_sum(x, par, idx);
  }
}

}  // namespace

extern "C" {

int rx_xg_devdesc_size() { return (int)sizeof(XgDev); }

void* rx_xg_create(int world, int rank, int device, int n, double timeout_s) {
  if (world < 1 || world > RX_XG_MAXR || rank < 0 || rank >= world || n <= 0) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  XgHost* h = new XgHost();
  h->device = device;
  const int nf = (n + 63) & ~63;
  h->bytes = (2 * (size_t)nf + RX_XG_MAXR) * sizeof(float);
  if (hipExtMallocWithFlags(&h->base, h->bytes, hipDeviceMallocUncached) != hipSuccess) {
    delete h;
    return nullptr;
  }
  unsigned* err = nullptr;
  if (hipMalloc(&err, 64) != hipSuccess || hipMemset(err, 0, 64) != hipSuccess ||
      hipMemset(h->base, 0, h->bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipIpcGetMemHandle(&h->handle, h->base) != hipSuccess) {
    if (err) (void)hipFree(err);
    (void)hipFree(h->base);
    delete h;
    return nullptr;
  }
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  memset(&h->dev, 0, sizeof(h->dev));
  h->dev.world = world;
  h->dev.rank = rank;
  h->dev.nf = nf;
  h->dev.err = err;
  h->dev.spin_ticks = (unsigned long long)(timeout_s * khz * 1000.0);
  h->dev.region[rank] = (float*)h->base;
  return h;
}

int rx_xg_handle(void* ctx, char* out64) {
  XgHost* h = (XgHost*)ctx;
  static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle larger than 64 bytes");
  memset(out64, 0, 64);
  memcpy(out64, &h->handle, sizeof(hipIpcMemHandle_t));
  return 0;
}

// handles: world * 64 bytes, rank order (this rank's own entry is ignored)
int rx_xg_open(void* ctx, const char* handles) {
  XgHost* h = (XgHost*)ctx;
  if (hipSetDevice(h->device) != hipSuccess) return -1;
  for (int p = 0; p < h->dev.world; ++p) {
    if (p == h->dev.rank) continue;
    hipIpcMemHandle_t hp;
    memcpy(&hp, handles + 64 * p, sizeof(hp));
    void* ptr = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&ptr, hp, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
      fprintf(stderr, "rx_xg_open: rank %d cannot map rank %d's region: %s\n", h->dev.rank, p, hipGetErrorString(e));
      return (int)e;
    }
    h->dev.region[p] = (float*)ptr;
    h->opened[p] = true;
  }
  return 0;
}

const XgDev* rx_xg_devdesc(void* ctx) { return &((XgHost*)ctx)->dev; }

// Reserve n consecutive sequence numbers; returns the first. Slot parity of step k is
// (first + k) & 1.
unsigned rx_xg_take_seq(void* ctx, int n) {
  XgHost* h = (XgHost*)ctx;
  const unsigned first = h->seq + 1;
  h->seq += (unsigned)n;
  return first;
}

float* rx_xg_slot(void* ctx, int parity) {
  XgHost* h = (XgHost*)ctx;
  return (float*)h->base + (size_t)(parity & 1) * h->dev.nf;
}

// In-place all-reduce (sum) of n floats on `stream`.
int rx_xg_allreduce(float* buf, int n, void* ctx, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (n > h->dev.nf) return -2;
  if (h->dev.world == 1) return 0;
  const unsigned seq = rx_xg_take_seq(ctx, 1);
  float* slot = rx_xg_slot(ctx, (int)(seq & 1u));
  hipError_t e = hipMemcpyAsync(slot, buf, (size_t)n * sizeof(float), hipMemcpyDeviceToDevice, stream);
  if (e != hipSuccess) return (int)e;
  const int blocks = (n + kThreads * kPerThread - 1) / (kThreads * kPerThread);
  hipLaunchKernelGGL(xg_reduce_kernel, dim3(blocks), dim3(kThreads), 0, stream, h->dev, buf, n, seq);
  return (int)hipGetLastError();
}

int rx_xg_error(void* ctx) {
  XgHost* h = (XgHost*)ctx;
  unsigned v = 0;
  if (hipMemcpy(&v, h->dev.err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

int rx_xg_destroy(void* ctx) {
  XgHost* h = (XgHost*)ctx;
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < h->dev.world; ++p)
    if (h->opened[p]) (void)hipIpcCloseMemHandle(h->dev.region[p]);
  (void)hipFree(h->dev.err);
  (void)hipFree(h->base);
  delete h;
  return 0;
}

}  // extern "C"
