// Grid-wide hand-off primitives for persistent gfx950 kernels (one workgroup per CU, all
// co-resident): sc1 loads/stores and a counter barrier.
//
// Form (MI355X_MICROARCH.md "inter-workgroup visibility", first row of the sc1 table): every wave
// stores its hand-off bytes with sc1 (write-through) stores and drains them (s_waitcnt vmcnt(0)),
// the workgroup joins a barrier, then ONE lane adds to an agent-scope monotonic counter; the
// consumer's lane 0 polls the counter with sc1 loads, its workgroup joins a barrier and every
// wave reads the handed-off bytes with sc1 (L2-served) loads. Within one launch a hand-off buffer
// is written once and read only after that write (a consumer XCD's L2 must not hold a line of it
// from earlier in the same launch); across launches the kernel boundary makes writes visible.
#pragma once
#include "rx_common.h"

#define RX_MW_CTR 0
#define RX_MW_DONE 1
#define RX_MW_ERR 2

// Global-qualified on purpose: through a generic pointer (any pointer read out of a descriptor or
// a by-value struct) these become flat_* sc1 accesses, and a hand-off must be read by global_ /
// buffer_ sc1 loads, never flat_ (MI355X_MICROARCH.md, consumer condition (1)).
__device__ __forceinline__ float rx_ld_sc1f(const float* p) {
  return __hip_atomic_load(rx_g(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void rx_st_sc1f(float* p, float v) {
  __hip_atomic_store(rx_g(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned rx_ld_sc1u(const unsigned* p) {
  return __hip_atomic_load(rx_g(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 8-B sc1 load through a buffer descriptor (`base` wave-uniform).
__device__ __forceinline__ uint2 rx_load8_sc1(const void* base, int byte_off) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, byte_off, 0, 16);
  return uint2{v[0], v[1]};
}
__device__ __forceinline__ void rx_store8_sc1(void* base, int byte_off, uint2 v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7ffffff0, 0x00020000);
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{v.x, v.y}, rsrc, byte_off, 0, 16);
}

// Grid barrier number `k` (1-based, counted by the caller over the launch) of G workgroups on
// ctl[RX_MW_CTR]. Every thread of every workgroup calls it. Returns false once any workgroup timed
// out (ctl[RX_MW_ERR] set; every later barrier then returns at once).
__device__ __forceinline__ bool rx_grid_barrier(unsigned* ctl, int G, int k, unsigned long long ticks) {
  __shared__ int rx_gb_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have left
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __hip_atomic_fetch_add(rx_g(ctl) + RX_MW_CTR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (unsigned)(k * G);
    const unsigned long long t0 = wall_clock64();
    for (int it = 1;; ++it) {
      if (rx_ld_sc1u(ctl + RX_MW_CTR) >= target) break;
      if ((it & 15) == 0) {
        if (rx_ld_sc1u(ctl + RX_MW_ERR) != 0u || wall_clock64() - t0 > ticks) {
          __hip_atomic_store(rx_g(ctl) + RX_MW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
    rx_gb_ok = ok;
  }
  __syncthreads();
  return rx_gb_ok != 0;
}

// End of the launch: the last workgroup through resets the barrier counter for the next launch
// and, with `flip`, toggles ctl[flip_word] (a parity the next launch reads at its start).
__device__ __forceinline__ void rx_grid_finish(unsigned* ctl, int G, int flip_word = -1) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(rx_g(ctl) + RX_MW_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (counters only: a
    // relaxed device-scope RMW suffices, the next launch is ordered by the kernel boundary; acq_rel
    // cost every workgroup an L2 write-back + invalidate, ~3.5 us, at the end of every launch)
    if (old == (unsigned)G - 1u) {
      __hip_atomic_store(rx_g(ctl) + RX_MW_CTR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rx_g(ctl) + RX_MW_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (flip_word >= 0)
        __hip_atomic_fetch_xor(rx_g(ctl) + flip_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
