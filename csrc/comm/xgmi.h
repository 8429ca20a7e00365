// One-shot all-reduce over xGMI peer memory: the device-side protocol shared by the stand-alone
// reduce kernel (csrc/comm/xgmi_allreduce.hip) and the fused "reduce + optimizer" kernel of the
// NYC step loop (csrc/hip/fused_mlp.hip).
//
// Why: the reference's gradient all-reduce is DDP/Horovod over NCCL rings
// (python/raydp/torch/estimator.py:243 prepare_model; examples/horovod_nyctaxi.py:133-138). The
// NYC model's whole gradient is 194 KB, so a ring is pure latency: 2*(N-1) link hops, each a
// kernel-to-kernel hand-off. MI355X GPUs of a node are fully connected by xGMI (7 links per
// GPU), so every rank can read every peer's gradient directly: one flag exchange, then each
// rank sums the N buffers itself (N-1 reads in parallel, one per link). No staging copy.
//
// Memory: each rank owns one exchange region allocated uncached (hipDeviceMallocUncached, so
// no L2 on either side holds a stale line) and exports it with hipIpcGetMemHandle:
//   [slot 0: nf floats][slot 1: nf floats][flags: RX_XG_MAXR u32][votes: 2 x RX_XG_MAXR u32]
//   [tile flags: RX_XG_MAXT x RX_XG_MAXR u32]
// Step s writes its gradient into slot (s & 1) of its own region, then publishes seq = s + base
// by storing it into flags[rank] of EVERY peer's region, waits until its own flags[p] >= seq for
// every peer p, and reads slot (s & 1) of every region.
// Double buffering makes one flag round per step enough: rank r overwrites slot (s & 1) at step
// s + 2 only after its kernel of step s + 1 saw every peer's seq s + 1 flag, which each peer
// publishes only after its step-s kernel (the reads of slot (s & 1)) ended.
//
// One rendezvous per LAUNCH, not per workgroup: every workgroup counts itself in on a local
// arrival word; the last one to arrive does the cross-rank flag exchange and then opens a local
// "go" word the others spin on (rx_xg_grid_rendezvous). A 1 MiB bucket is one flag round.
//
// Sequence numbers: the fused step loop takes them on the host (rx_xg_take_seq); the stand-alone
// all-reduce keeps them on the device (ctl[1], bumped by the launch's last workgroup), so its
// launch arguments never change and a HIP graph can replay it. A communicator is used in one
// of the two modes only (raydp_amd/ops/comm.py keys them apart).
//
// Every wait is bounded (spin_ticks of the 100 MHz wall clock): a missing peer sets ctl[0] and
// the kernel returns instead of hanging the GPU; the host reads it with the epoch's metrics.
#pragma once
#include <hip/hip_runtime.h>

#define RX_XG_MAXR 16
// per-tile flags of the in-kernel gradient exchange (rx_xg_tile_*): tile ids per region
#define RX_XG_MAXT 1024

// ctl words (this rank's local device memory, zeroed at create)
enum : int { kXgErr = 0, kXgDevSeq = 1, kXgArrive = 2, kXgGo = 3, kXgDone = 4, kXgCtlWords = 16 };

struct XgDev {
  float* region[RX_XG_MAXR];  // region base of rank p, mapped into this process
  unsigned* err;              // == ctl + kXgErr
  unsigned* ctl;              // local control words (kXg*)
  unsigned long long spin_ticks;
  int world, rank, nf;        // nf: floats per slot (multiple of 64)
  int pad_;
};

__device__ __forceinline__ unsigned* rx_xg_flags(const XgDev& x, int p) {
  return reinterpret_cast<unsigned*>(x.region[p] + 2 * (size_t)x.nf);
}

// vote words of rank p's region for a meeting of sequence seq (double-buffered by parity)
__device__ __forceinline__ unsigned* rx_xg_votes(const XgDev& x, int p, unsigned seq) {
  return rx_xg_flags(x, p) + RX_XG_MAXR * (1 + (int)(seq & 1u));
}

__device__ __forceinline__ void rx_xg_fail(const XgDev& x) {
  __hip_atomic_store(x.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Publish `seq` to every peer and wait for theirs. Call from ONE lane. Returns false on timeout
// (after setting *err).
__device__ __forceinline__ bool rx_xg_rendezvous(const XgDev& x, unsigned seq) {
  // my slot was written before this call (previous kernel, or this launch's workgroups before
  // they counted themselves in): make it visible to readers on other devices before they can
  // see the flag
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  for (int p = 0; p < x.world; ++p)
    if (p != x.rank)
      __hip_atomic_store(rx_xg_flags(x, p) + x.rank, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned* mine = rx_xg_flags(x, x.rank);
  const long long t0 = wall_clock64();
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank) continue;
    while ((int)(__hip_atomic_load(mine + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
      if ((unsigned long long)(wall_clock64() - t0) > x.spin_ticks) {
        rx_xg_fail(x);
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

// Launch-wide rendezvous: `nblocks` workgroups of this launch call it (all threads). The last
// workgroup to arrive meets the peers; the others wait on the local go word. Returns false on
// every workgroup when the exchange failed. All `nblocks` workgroups must be able to be
// resident together (callers launch at most a few hundred small workgroups).
__device__ __forceinline__ bool rx_xg_grid_rendezvous(const XgDev& x, unsigned seq, unsigned nblocks) {
  __shared__ int ok_s;
  __syncthreads();  // this workgroup's slot writes are done
  if (threadIdx.x == 0) {
    int ok = 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope) my part of the slot
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgArrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblocks - 1) {
      __hip_atomic_store(x.ctl + kXgArrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = rx_xg_rendezvous(x, seq) ? 1 : 0;
      // open the gate even on failure (the others read the error word next)
      __hip_atomic_store(x.ctl + kXgGo, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const long long t0 = wall_clock64();
      while ((int)(__hip_atomic_load(x.ctl + kXgGo, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0) {
        if ((unsigned long long)(wall_clock64() - t0) > x.spin_ticks) {
          rx_xg_fail(x);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope) the peers' slots
    }
    if (ok && __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) ok = 0;
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}

// 16-byte system-coherent load from a (possibly peer-mapped) region: sc0|sc1, never a stale
// line of this device's caches.
__device__ __forceinline__ float4 rx_xg_load4(const float* base, size_t idx4) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7ffffff0, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(idx4 * 16), 0, 17);
  return __builtin_bit_cast(float4, v);
}

// Sum of element idx of slot `par` over all ranks, always in rank order so every rank computes
// bit-identical sums (replicas stay identical, as under DDP).
__device__ __forceinline__ float rx_xg_sum(const XgDev& x, int par, int idx) {
  const size_t off = (size_t)par * x.nf + idx;
  float s = 0.f;
  for (int p = 0; p < x.world; ++p)
    s += p == x.rank ? x.region[p][off]
                     : __hip_atomic_load(x.region[p] + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return s;
}

// ---- per-tile exchange inside a training launch (persistent epoch / multi-workgroup step) ----
// The gradient all-reduce of the fused NYC engine at world > 1 without a launch, a pass or a
// rendezvous of its own: the workgroup that finishes a 32x32 weight tile's gradient (or a chunk
// of the bias / BatchNorm gradients) stores it into its rank's slot at the flat gradient offsets
// (system-scope write-through stores), drains them, publishes tile id t at the step's sequence
// number into every peer's tile-flag row, waits until every peer published t, and sums the world
// values of each of its elements in rank order (bit-identical on every rank) before it updates.
// 4 KB per tile crosses each link -- the 194 KB NYC gradient per step in all -- instead of the
// batch-sized X^T / G^T exports (7.8 MB at batch 4096). Slot reuse: a rank rewrites tile t of
// slot (seq & 1) two steps later, after it saw every peer's flag t of the step between, which each
// peer publishes after its reads of this step's tile t (same workgroup, program order).
struct XgStep {
  const XgDev* xd;  // the communicator's descriptor in DEVICE memory (rx_xg_devptr): read with scalar
                    // loads, so a kernel argument holding this stays small and register-resident
  unsigned seq;     // sequence number of this launch's (first) step
  int on;           // 0: one GPU (nothing exchanged)
  float gscale;     // 1 / world: the DDP average
  int pad_;
};

__device__ __forceinline__ float* rx_xg_region(const XgDev& x, int p) { return x.region[p]; }

// A specialised one-GPU code object (raydp_amd/ops/mlp_jit.py, world 1) is compiled with
// RX_XG_KERNELS 0: every exchange branch of the training kernels folds away and the kernels keep
// the one-GPU register allocation. The ahead-of-time build keeps them (1).
#ifndef RX_XG_KERNELS
#define RX_XG_KERNELS 1
#endif
__device__ __forceinline__ bool rx_xg_active(const XgStep& xs) { return RX_XG_KERNELS && xs.on; }

__device__ __forceinline__ unsigned* rx_xg_tflags_of(float* region, const XgDev& x) {
  return reinterpret_cast<unsigned*>(region + 2 * (size_t)x.nf) + 3 * RX_XG_MAXR;
}

__device__ __forceinline__ float* rx_xg_slotp(const XgDev& x, int p, unsigned seq) {
  return rx_xg_region(x, p) + (size_t)(seq & 1u) * x.nf;
}

// write-through (sc0 sc1) store into this rank's slot, and the matching peer load: global_
// instructions (address space 1), never flat_
typedef __attribute__((address_space(1))) float rx_xg_gf;
typedef __attribute__((address_space(1))) unsigned rx_xg_gu;
__device__ __forceinline__ void rx_xg_put(float* p, float v) {
  __hip_atomic_store((rx_xg_gf*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float rx_xg_get(const float* p) {
  return __hip_atomic_load((rx_xg_gf*)const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One lane, after every storing wave of its workgroup drained its rx_xg_put stores and joined a
// barrier: tile t of sequence seq is in this rank's slot.
__device__ __forceinline__ void rx_xg_tile_publish(const XgDev& x, int t, unsigned seq) {
  for (int p = 0; p < x.world; ++p)
    if (p != x.rank)
      __hip_atomic_store((rx_xg_gu*)(rx_xg_tflags_of(x.region[p], x) + t * RX_XG_MAXR + x.rank), seq,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One lane (or a whole wave: every lane polls the same words): wait until every peer published
// tile t of sequence seq. False on timeout (error word set) or when the error word was already set.
__device__ __forceinline__ bool rx_xg_tile_wait(const XgDev& x, int t, unsigned seq) {
  const unsigned* mine = rx_xg_tflags_of(rx_xg_region(x, x.rank), x) + t * RX_XG_MAXR;
  const unsigned long long t0 = wall_clock64();
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank) continue;
    int k = 0;
    while ((int)(__hip_atomic_load((rx_xg_gu*)const_cast<unsigned*>(mine + p), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
      if ((++k & 15) == 0) {
        if (__hip_atomic_load((rx_xg_gu*)x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return false;
        if ((unsigned long long)(wall_clock64() - t0) > x.spin_ticks) {
          rx_xg_fail(x);
          return false;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return true;
}

// Sum over ranks (rank order) of flat element idx of sequence seq's slots; this rank's own value is
// `mine` (the bits it stored).
__device__ __forceinline__ float rx_xg_tile_sum(const XgDev& x, unsigned seq, int idx, float mine) {
  float s = 0.f;
  const size_t off = (size_t)(seq & 1u) * x.nf + idx;
  for (int p = 0; p < x.world; ++p) s += p == x.rank ? mine : rx_xg_get(x.region[p] + off);
  return s;
}
