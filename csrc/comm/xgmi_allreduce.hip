// Host side of the one-shot xGMI all-reduce (protocol: csrc/comm/xgmi.h) and its stand-alone
// reduce kernel.
//
// Setup (one communicator per process group, driven by raydp_amd/ops/comm.py XgmiComm):
//   rx_xg_create   -> allocate this rank's uncached exchange region, zero its flags
//   rx_xg_handle   -> 64-byte IPC handle of the region (exchanged over torch.distributed)
//   rx_xg_open     -> map every peer's region (hipIpcOpenMemHandle, lazy peer access)
// Use:
//   rx_xg_allreduce            -> in-place sum of a device fp32 buffer: ONE kernel (copy into the
//                                 slot, one launch-wide rendezvous, 16-B peer reads, sum), with
//                                 its sequence number kept on the device: the launch is
//                                 identical every call, so a HIP graph can capture and replay it
//   rx_xg_devdesc/take_seq/slot -> the fused step loop (csrc/hip/fused_mlp.hip) reduces inside
//                                 its optimizer kernel instead (host-side sequence numbers)
//   rx_xg_allgather            -> every rank's n words side by side (device-sequenced too):
//                                 the replicated DLRM tables' sparse gradient rows and ids
//   rx_xg_alltoallv            -> variable-split all-to-all (device-sequenced): the sharded
//                                 DLRM tables' id and row exchanges
//   rx_xg_vote                 -> epoch-end agreement for the fused loop: every rank's error word
//                                 summed into a double the host reads with the epoch metrics
//   rx_xg_error                -> nonzero once any wait timed out (a peer never arrived)
//
// Reference role: the small-bucket gradient all-reduce of DDP / Horovod
// (python/raydp/torch/estimator.py:243; examples/horovod_nyctaxi.py:133-138), see SURVEY.md
// §2.11 K2 and §5.8 (one-shot P2P all-reduce for <= 1 MB buckets).
#include "comm/xgmi.h"

#include <stdint.h>
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
  bool host_seq = false;  // sequence numbers taken on the host (fused step loop) or on the device
  bool opened[RX_XG_MAXR] = {false};
  XgDev* ddev = nullptr;  // device copy of `dev` (in-launch tile exchange: csrc/comm/xgmi.h XgStep)
};

constexpr int kThreads = 256;
// Workgroups per launch: every one must be resident at once (the launch-wide rendezvous), also
// when several ranks share one device in a rehearsal, and the work is xGMI-link bound, not
// compute bound -- 128 x 256 threads keep ~2 MB of 16-B peer loads in flight.
constexpr int kMaxBlocks = 128;

// In-place all-reduce of n floats. VEC: buf is 16-B aligned (n / 4 float4 plus a scalar tail),
// otherwise scalar. Each element is owned by one thread in both phases (same grid-stride
// mapping), so the rank's own contribution is re-read from buf before the thread overwrites
// it with the sum.
// hseq: the host-chosen sequence number of a host-sequenced communicator, or 0 (device-sequenced:
// the number is ctl[kXgDevSeq] + 1 and this launch's last workgroup stores it back).
template <bool VEC>
__global__ __launch_bounds__(kThreads) void xg_allreduce_kernel(XgDev x, float* __restrict__ buf, int n,
                                                                unsigned hseq, float scale) {
  const unsigned seq =
      hseq ? hseq : __hip_atomic_load(x.ctl + kXgDevSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(seq & 1u);
  float* mine = x.region[x.rank] + (size_t)par * x.nf;
  const int stride = gridDim.x * kThreads;
  const int t = blockIdx.x * kThreads + threadIdx.x;
  if (VEC) {
    const int n4 = n >> 2;
    const int tail = n & 3;
    for (int i = t; i < n4; i += stride) reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(buf)[i];
    if (blockIdx.x == 0 && threadIdx.x < tail) mine[(n4 << 2) + threadIdx.x] = buf[(n4 << 2) + threadIdx.x];
    if (!rx_xg_grid_rendezvous(x, seq, gridDim.x)) return;
    for (int i = t; i < n4; i += stride) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int p = 0; p < x.world; ++p) {   // rank order: bit-identical sums on every rank
        const float4 v = p == x.rank ? reinterpret_cast<const float4*>(buf)[i]
                                     : rx_xg_load4(x.region[p] + (size_t)par * x.nf, (size_t)i);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
      s.x *= scale;
      s.y *= scale;
      s.z *= scale;
      s.w *= scale;
      reinterpret_cast<float4*>(buf)[i] = s;
    }
    if (blockIdx.x == 0 && threadIdx.x < tail) {
      const int i = (n4 << 2) + threadIdx.x;
      buf[i] = rx_xg_sum(x, par, i) * scale;
    }
  } else {
    for (int i = t; i < n; i += stride) mine[i] = buf[i];
    if (!rx_xg_grid_rendezvous(x, seq, gridDim.x)) return;
    for (int i = t; i < n; i += stride) buf[i] = rx_xg_sum(x, par, i) * scale;
  }
  // the launch's last workgroup advances the device sequence number for the next launch
  if (hseq) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(x.ctl + kXgDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.ctl + kXgDevSeq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Two-shot in-place all-reduce (all-pairs reduce-scatter, then all-gather) of n floats, n a
// multiple of 4 and buf 16-B aligned. The bucket is cut into `world` chunks of chunk4 float4s;
// rank r owns chunk r:
//   1. every rank publishes its whole bucket in its slot; launch-wide rendezvous (seq s0)
//   2. rank r reads chunk r of every peer's slot (S/N bytes over each link, all links at once),
//      sums in rank order, scales, writes the result into buf AND over chunk r of its own slot
//      (no peer reads that chunk of this slot: peer q reads chunk q); rendezvous (seq s0 + 1)
//   3. rank r copies every peer's reduced chunk p out of peer p's slot into buf.
// Per link 2S/N bytes against the one-shot kernel's S: the path for buckets large enough that
// link bandwidth, not the extra flag round, sets the time. Every element
// is reduced by one rank only, so all ranks hold bit-identical sums.
// Sequencing: one call consumes THREE sequence numbers (s0, s0 + 1, and s0 + 2 unused), so the
// next call's first number has the other parity and uses the other slot, exactly as after a
// one-shot call (which consumes one): slot reuse stays two calls apart whatever the mix.
__global__ __launch_bounds__(kThreads) void xg_allreduce2_kernel(XgDev x, float* __restrict__ buf, int n,
                                                                 int chunk4, float scale) {
  const unsigned s0 = __hip_atomic_load(x.ctl + kXgDevSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(s0 & 1u);
  float4* mine = reinterpret_cast<float4*>(x.region[x.rank] + (size_t)par * x.nf);
  float4* b4 = reinterpret_cast<float4*>(buf);
  const int n4 = n >> 2;
  const int stride = gridDim.x * kThreads;
  const int t = blockIdx.x * kThreads + threadIdx.x;
  for (int i = t; i < n4; i += stride) mine[i] = b4[i];
  if (!rx_xg_grid_rendezvous(x, s0, gridDim.x)) return;
  {
    const int c0 = x.rank * chunk4;
    const int c1 = min(n4, c0 + chunk4);
    for (int i = c0 + t; i < c1; i += stride) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int p = 0; p < x.world; ++p) {   // rank order: the same sum whichever rank owns it
        const float4 v = p == x.rank ? b4[i] : rx_xg_load4(x.region[p] + (size_t)par * x.nf, (size_t)i);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
      s.x *= scale;
      s.y *= scale;
      s.z *= scale;
      s.w *= scale;
      mine[i] = s;
      b4[i] = s;
    }
  }
  if (!rx_xg_grid_rendezvous(x, s0 + 1u, gridDim.x)) return;
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank) continue;
    const int c0 = p * chunk4;
    const int c1 = min(n4, c0 + chunk4);
    const float* from = x.region[p] + (size_t)par * x.nf;
    for (int i = c0 + t; i < c1; i += stride) b4[i] = rx_xg_load4(from, (size_t)i);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(x.ctl + kXgDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.ctl + kXgDevSeq, s0 + 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// All-gather of n floats (raw 4-byte words of any dtype) per rank: dst[p * n + i] = rank p's
// src[i]. Device-sequenced like the all-reduce (capturable); VEC: src and dst 16-B aligned and
// n a multiple of 4.
template <bool VEC>
__global__ __launch_bounds__(kThreads) void xg_allgather_kernel(XgDev x, const float* __restrict__ src,
                                                                float* __restrict__ dst, int n) {
  const unsigned seq = __hip_atomic_load(x.ctl + kXgDevSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(seq & 1u);
  float* mine = x.region[x.rank] + (size_t)par * x.nf;
  const int stride = gridDim.x * kThreads;
  const int t = blockIdx.x * kThreads + threadIdx.x;
  const int units = VEC ? n >> 2 : n;
  for (int i = t; i < units; i += stride) {
    if (VEC)
      reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(src)[i];
    else
      mine[i] = src[i];
  }
  if (!rx_xg_grid_rendezvous(x, seq, gridDim.x)) return;
  for (int p = 0; p < x.world; ++p) {
    const float* from = x.region[p] + (size_t)par * x.nf;
    for (int i = t; i < units; i += stride) {
      if (VEC) {
        const float4 v = p == x.rank ? reinterpret_cast<const float4*>(src)[i] : rx_xg_load4(from, (size_t)i);
        reinterpret_cast<float4*>(dst + (size_t)p * n)[i] = v;
      } else {
        dst[(size_t)p * n + i] = p == x.rank ? src[i]
                                             : __hip_atomic_load(from + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(x.ctl + kXgDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.ctl + kXgDevSeq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Variable-split all-to-all of raw 4-byte words (the sharded-embedding id and row exchanges,
// raydp_amd/parallel/embedding_mp.py): every rank publishes its whole send buffer (src_words) in
// its slot; after the rendezvous, rank r copies len[p] words starting at from_off[p] of rank p's
// buffer into dst + dst_off[p]. Device-sequenced like the all-reduce (capturable); VEC: every
// count / offset a multiple of 4 and src / dst 16-B aligned.
struct XgA2A {
  int src_words;
  int from_off[RX_XG_MAXR];
  int len[RX_XG_MAXR];
  int dst_off[RX_XG_MAXR];
};

template <bool VEC>
__global__ __launch_bounds__(kThreads) void xg_alltoallv_kernel(XgDev x, const float* __restrict__ src,
                                                                float* __restrict__ dst, XgA2A a) {
  const unsigned seq = __hip_atomic_load(x.ctl + kXgDevSeq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int par = (int)(seq & 1u);
  float* mine = x.region[x.rank] + (size_t)par * x.nf;
  const int stride = gridDim.x * kThreads;
  const int t = blockIdx.x * kThreads + threadIdx.x;
  const int su = VEC ? a.src_words >> 2 : a.src_words;
  for (int i = t; i < su; i += stride) {
    if (VEC)
      reinterpret_cast<float4*>(mine)[i] = reinterpret_cast<const float4*>(src)[i];
    else
      mine[i] = src[i];
  }
  if (!rx_xg_grid_rendezvous(x, seq, gridDim.x)) return;
  for (int p = 0; p < x.world; ++p) {
    const int units = VEC ? a.len[p] >> 2 : a.len[p];
    const int fo = VEC ? a.from_off[p] >> 2 : a.from_off[p];
    const int dof = VEC ? a.dst_off[p] >> 2 : a.dst_off[p];
    const float* from = x.region[p] + (size_t)par * x.nf;
    for (int i = t; i < units; i += stride) {
      if (VEC) {
        const float4 v = p == x.rank ? reinterpret_cast<const float4*>(src)[fo + i]
                                     : rx_xg_load4(from, (size_t)(fo + i));
        reinterpret_cast<float4*>(dst)[dof + i] = v;
      } else {
        dst[dof + i] = p == x.rank ? src[fo + i]
                                   : __hip_atomic_load(from + fo + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == gridDim.x - 1) {
      __hip_atomic_store(x.ctl + kXgDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(x.ctl + kXgDevSeq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Epoch-end vote of the fused step loop: publish this rank's error word into every peer's vote
// array, meet them (one flag round of sequence `seq`), and write the sum of all ranks' error
// words (+1 if this meeting itself timed out) into *out. Every rank that completes the meeting
// computes the same value.
__global__ __launch_bounds__(64) void xg_vote_kernel(XgDev x, unsigned seq, double* out) {
  if (threadIdx.x != 0) return;
  const unsigned mine = __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int p = 0; p < x.world; ++p)
    __hip_atomic_store(rx_xg_votes(x, p, seq) + x.rank, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  double sum = 0.0;
  if (rx_xg_rendezvous(x, seq)) {
    for (int p = 0; p < x.world; ++p)
      sum += (double)__hip_atomic_load(rx_xg_votes(x, x.rank, seq) + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    sum = 1.0 + (double)mine;
  }
  *out = sum;
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
  h->bytes = (2 * (size_t)nf + 3 * RX_XG_MAXR) * sizeof(float) +
             2 * (size_t)world * nf * sizeof(unsigned long long);   // tagged inbox (rx_xg_push)
  if (hipExtMallocWithFlags(&h->base, h->bytes, hipDeviceMallocUncached) != hipSuccess) {
    delete h;
    return nullptr;
  }
  unsigned* ctl = nullptr;
  if (hipMalloc(&ctl, kXgCtlWords * sizeof(unsigned)) != hipSuccess ||
      hipMemset(ctl, 0, kXgCtlWords * sizeof(unsigned)) != hipSuccess ||
      hipMemset(h->base, 0, h->bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipIpcGetMemHandle(&h->handle, h->base) != hipSuccess) {
    if (ctl) (void)hipFree(ctl);
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
  h->dev.layout = RX_XG_LAYOUT;
  h->dev.ctl = ctl;
  h->dev.err = ctl + kXgErr;
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
  if (h->ddev == nullptr && hipMalloc((void**)&h->ddev, sizeof(XgDev)) != hipSuccess) return -1;
  if (hipMemcpy(h->ddev, &h->dev, sizeof(XgDev), hipMemcpyHostToDevice) != hipSuccess) return -1;
  return 0;
}

// The descriptor in device memory (valid after rx_xg_open): what training kernels that exchange
// inside their launch read (XgStep::xd).
const XgDev* rx_xg_devptr(void* ctx) { return ((XgHost*)ctx)->ddev; }

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

// Switch a fresh communicator to host-side sequence numbers (before its first use): required by
// the fused step loop (rx_xg_take_seq) and rx_xg_vote; rx_xg_allreduce then takes its number on
// the host too (not graph-replayable).
int rx_xg_set_host_seq(void* ctx, int on) {
  ((XgHost*)ctx)->host_seq = on != 0;
  return 0;
}

// Largest n rx_xg_allreduce takes: the slot.
int rx_xg_max_floats(void* ctx) { return ((XgHost*)ctx)->dev.nf; }

// In-place all-reduce of n floats on `stream`, times `scale` (1/world: an average with no
// extra pass): one launch whose arguments depend only on (buf, n, scale), so a captured graph
// replays it correctly.
int rx_xg_allreduce_scaled(float* buf, int n, float scale, void* ctx, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (n < 0 || n > rx_xg_max_floats(ctx)) return -2;
  if (n == 0) return 0;
  if (h->dev.world == 1) {
    if (scale == 1.0f) return 0;
  }
  const bool vec = (reinterpret_cast<uintptr_t>(buf) & 15u) == 0;
  const long units = vec ? (long)(n >> 2) : (long)n;
  // ~4 units per thread before the grid grows, at most kMaxBlocks (then grid-stride)
  long blocks = (units + (long)kThreads * 4 - 1) / ((long)kThreads * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  const unsigned hseq = h->host_seq ? rx_xg_take_seq(ctx, 1) : 0u;
  if (vec)
    hipLaunchKernelGGL(xg_allreduce_kernel<true>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, buf, n,
                       hseq, scale);
  else
    hipLaunchKernelGGL(xg_allreduce_kernel<false>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, buf,
                       n, hseq, scale);
  return (int)hipGetLastError();
}

// Two-shot in-place all-reduce (device-sequenced communicators only; n % 4 == 0 and buf 16-B
// aligned, else -4 and the caller takes the one-shot path). -2: n outside the slot; -3:
// host-sequenced communicator.
int rx_xg_allreduce2_scaled(float* buf, int n, float scale, void* ctx, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (h->host_seq) return -3;
  if (n < 0 || n > h->dev.nf) return -2;
  if (n == 0) return 0;
  if ((n & 3) || (reinterpret_cast<uintptr_t>(buf) & 15u)) return -4;
  const int world = h->dev.world;
  const int n4 = n >> 2;
  const int chunk4 = (n4 + world - 1) / world;
  // the busiest phase moves (world - 1) chunks per rank: ~4 float4 per thread before the grid
  // grows, at most kMaxBlocks
  const long units = (long)chunk4 * (world > 1 ? world - 1 : 1);
  long blocks = (units + (long)kThreads * 4 - 1) / ((long)kThreads * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  hipLaunchKernelGGL(xg_allreduce2_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, buf, n, chunk4,
                     scale);
  return (int)hipGetLastError();
}

// All-gather of n 4-byte words per rank into dst (world * n words), device-sequenced.
int rx_xg_allgather(const float* src, float* dst, int n, void* ctx, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (h->host_seq) return -3;
  if (n < 0 || n > h->dev.nf) return -2;
  if (n == 0) return 0;
  const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0 && (n & 3) == 0;
  const long units = vec ? (long)(n >> 2) : (long)n;
  long blocks = (units + (long)kThreads * 4 - 1) / ((long)kThreads * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  if (vec)
    hipLaunchKernelGGL(xg_allgather_kernel<true>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, src, dst, n);
  else
    hipLaunchKernelGGL(xg_allgather_kernel<false>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, src, dst,
                       n);
  return (int)hipGetLastError();
}

int rx_xg_a2a_size() { return (int)sizeof(XgA2A); }

// Variable-split all-to-all (device-sequenced communicators only). -2: a count outside the slot
// or negative; -3: host-sequenced communicator.
int rx_xg_alltoallv(const float* src, float* dst, const XgA2A* a, void* ctx, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (h->host_seq) return -3;
  const int world = h->dev.world;
  if (a->src_words < 0 || a->src_words > h->dev.nf) return -2;
  long most = a->src_words;
  unsigned bits = (unsigned)a->src_words | (unsigned)(reinterpret_cast<uintptr_t>(src) & 15u) |
                  (unsigned)(reinterpret_cast<uintptr_t>(dst) & 15u);
  for (int p = 0; p < world; ++p) {
    if (a->len[p] < 0 || a->from_off[p] < 0 || a->dst_off[p] < 0 || (long)a->from_off[p] + a->len[p] > h->dev.nf)
      return -2;
    most = a->len[p] > most ? a->len[p] : most;
    bits |= (unsigned)a->len[p] | (unsigned)a->from_off[p] | (unsigned)a->dst_off[p];
  }
  const bool vec = (bits & 3u) == 0 && ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0;
  const long units = vec ? most >> 2 : most;
  long blocks = (units + (long)kThreads * 4 - 1) / ((long)kThreads * 4);
  if (blocks < 1) blocks = 1;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  if (vec)
    hipLaunchKernelGGL(xg_alltoallv_kernel<true>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, src, dst, *a);
  else
    hipLaunchKernelGGL(xg_alltoallv_kernel<false>, dim3((unsigned)blocks), dim3(kThreads), 0, stream, h->dev, src, dst,
                       *a);
  return (int)hipGetLastError();
}

// In-place all-reduce (sum) of n floats on `stream`.
int rx_xg_allreduce(float* buf, int n, void* ctx, hipStream_t stream) {
  return rx_xg_allreduce_scaled(buf, n, 1.0f, ctx, stream);
}

// Epoch-end agreement for host-sequenced users (the fused step loop): *out (device double) =
// sum over ranks of their error words, or > 0 when this meeting timed out.
int rx_xg_vote(void* ctx, double* out, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  if (!h->host_seq) return -3;
  if (h->dev.world == 1) return (int)hipMemsetAsync(out, 0, sizeof(double), stream);
  const unsigned seq = rx_xg_take_seq(ctx, 1);
  hipLaunchKernelGGL(xg_vote_kernel, dim3(1), dim3(64), 0, stream, h->dev, seq, out);
  return (int)hipGetLastError();
}

// Test hook: set this rank's error word (as a peer timeout would).
int rx_xg_set_error(void* ctx, int v) {
  XgHost* h = (XgHost*)ctx;
  const unsigned u = (unsigned)v;
  return (int)hipMemcpy(h->dev.err, &u, sizeof(u), hipMemcpyHostToDevice);
}

int rx_xg_error(void* ctx) {
  XgHost* h = (XgHost*)ctx;
  unsigned v = 0;
  if (hipMemcpy(&v, h->dev.err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return (int)v;
}

// Stream-ordered copy of the error word into (pinned) host memory: a step loop reads the value a
// few steps later instead of synchronising the device (and it is legal inside a graph capture).
int rx_xg_error_async(void* ctx, unsigned* host, hipStream_t stream) {
  XgHost* h = (XgHost*)ctx;
  return (int)hipMemcpyAsync(host, h->dev.err, sizeof(unsigned), hipMemcpyDeviceToHost, stream);
}

int rx_xg_destroy(void* ctx) {
  XgHost* h = (XgHost*)ctx;
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipDeviceSynchronize();
  for (int p = 0; p < h->dev.world; ++p)
    if (h->opened[p]) (void)hipIpcCloseMemHandle(h->dev.region[p]);
  (void)hipFree(h->dev.ctl);
  if (h->ddev) (void)hipFree(h->ddev);
  (void)hipFree(h->base);
  delete h;
  return 0;
}

}  // extern "C"
