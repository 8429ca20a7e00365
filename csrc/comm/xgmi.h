// One-shot all-reduce over xGMI peer memory: the device-side protocol shared by the stand-alone
// reduce kernel (csrc/comm/xgmi_allreduce.hip) and the fused "reduce + optimizer" kernel of the
// NYC step loop (csrc/hip/fused_mlp.hip).
//
// Why: the reference's gradient all-reduce is DDP/Horovod over NCCL rings
// (python/raydp/torch/estimator.py:243 prepare_model; examples/horovod_nyctaxi.py:133-138). The
// NYC model's whole gradient is 194 KB, so a ring is pure latency: 2*(N-1) link hops, each a
// kernel-to-kernel hand-off. MI355X GPUs of a node are fully connected by xGMI (7 links per
// GPU), so every rank can read every peer's gradient directly: one flag exchange, then each
// rank sums the N buffers itself while it applies the optimizer (N-1 reads in parallel, one per
// link). No extra launch, no staging copy.
//
// Memory: each rank owns one exchange region allocated uncached (hipDeviceMallocUncached, so
// no L2 on either side holds a stale line) and exports it with hipIpcGetMemHandle:
//   [slot 0: nf floats][slot 1: nf floats][flags: RX_XG_MAXR u32]
// Step s writes its gradient into slot (s & 1) of its own region, then (in the consumer kernel)
// publishes seq = s + base by storing it into flags[rank] of EVERY peer's region, waits until
// its own flags[p] >= seq for every peer p, and reads slot (s & 1) of every region.
// Double buffering makes one flag round per step enough: rank r overwrites slot (s & 1) at step
// s + 2 only after its consumer kernel of step s + 1 saw every peer's seq s + 1 flag, which
// each peer publishes only after its step-s consumer kernel (the reads of slot (s & 1)) ended.
//
// Every wait is bounded (spin_ticks of the 100 MHz wall clock): a missing peer sets *err and
// the kernel returns instead of hanging the GPU; the host checks *err after the epoch.
#pragma once
#include <hip/hip_runtime.h>

#define RX_XG_MAXR 16

struct XgDev {
  float* region[RX_XG_MAXR];  // region base of rank p, mapped into this process
  unsigned* err;              // this rank's error word (device memory)
  unsigned long long spin_ticks;
  int world, rank, nf;        // nf: floats per slot (multiple of 64)
  int pad_;
};

__device__ __forceinline__ unsigned* rx_xg_flags(const XgDev& x, int p) {
  return reinterpret_cast<unsigned*>(x.region[p] + 2 * (size_t)x.nf);
}

// Publish `seq` to every peer and wait for theirs. Call from ONE lane; the caller then
// barriers its workgroup. Returns false on timeout (after setting *err).
__device__ __forceinline__ bool rx_xg_rendezvous(const XgDev& x, unsigned seq) {
  // my slot was written by the previous kernel (or by this rank's copy): make it visible to
  // readers on other devices before they can see the flag
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
        __hip_atomic_store(x.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

// Sum of element idx of slot `par` over all ranks, always in rank order so every rank computes
// bit-identical sums (replicas stay identical, as under DDP). Peer lines are read with
// system-scope loads: they must come from the peer's memory, never from a cache here.
__device__ __forceinline__ float rx_xg_sum(const XgDev& x, int par, int idx) {
  const size_t off = (size_t)par * x.nf + idx;
  float s = 0.f;
  for (int p = 0; p < x.world; ++p)
    s += p == x.rank ? x.region[p][off]
                     : __hip_atomic_load(x.region[p] + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return s;
}
