// Shared device helpers for the gfx950 kernels (wave64, bf16 MFMA, bf16 packing).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define RX_WAVE 64

// Pointers read out of a descriptor in memory are "generic" to the compiler, so every access
// through them becomes a flat_* instruction -- and a flat load is waited for with vmcnt(0) AND
// lgkmcnt(0), serialising everything around it. Casting them to the global address space
// restores global_load/global_store with counted waits.
#define RX_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ RX_GLOBAL T* rx_g(T* p) {
  return (RX_GLOBAL T*)p;
}

// Thread index behind an opaque (volatile) register move. The persistent epoch kernel runs the
// step body in a loop: with a plain threadIdx.x the compiler hoists every lane-dependent address
// of every layer out of that loop, keeps them all live across it and spills to scratch. The
// wave index goes back to an SGPR through readfirstlane (it is wave-uniform).
// Outside such loops (OPQ = false) it is the plain threadIdx.x.
template <bool OPQ = true>
__device__ __forceinline__ int rx_tid() {
  if constexpr (!OPQ) return (int)threadIdx.x;
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return (int)threadIdx.x + z;
}
template <bool OPQ = true>
__device__ __forceinline__ int rx_wave() {
  if constexpr (!OPQ) return (int)(threadIdx.x >> 6);
  return __builtin_amdgcn_readfirstlane(rx_tid<true>() >> 6);
}

// round-to-nearest-even fp32 -> bf16 bits: gfx950's v_cvt_pk_bf16_f32 (one VALU op per PAIR of
// values; the integer rounding sequence it replaces was 5 ops per value)
typedef __bf16 rx_bf16x2 __attribute__((ext_vector_type(2)));
typedef float rx_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t rx_f2bf2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((rx_f32x2){a, b}, rx_bf16x2));
}
__device__ __forceinline__ u16 rx_f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }

__device__ __forceinline__ float rx_bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }

// sum over the 4 lanes that share (lane & 15): lanes l, l^16, l^32, l^48. gfx950's
// v_permlane16_swap / v_permlane32_swap exchange rows / halves of the wave in the VALU (a
// __shfl_xor is an LDS-pipeline ds_bpermute round trip); swapping a value with itself leaves
// x[l] in one result and x[l^16] (x[l^32]) in the other, and a + b == b + a exactly, so every
// lane gets the bit-identical sum.
__device__ __forceinline__ float rx_colsum16(float v) {
  const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

__device__ __forceinline__ float rx_wavesum(float v) {
  v = rx_colsum16(v);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ f32x4 rx_mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// 16-B write-through (sc1) store through a buffer descriptor: tens of KB published by one
// workgroup drain far faster write-through than as plain write-back stores
// (MI355X_MICROARCH.md "publish-large"). `base` must be wave-uniform.
__device__ __forceinline__ void rx_store16_wt(float* base, int byte_off, const f32x4& v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7ffffff0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rsrc, byte_off, 0, 16);
}

// 16-B sc1 load / store through a buffer descriptor (`base` wave-uniform). sc1 loads bypass
// the CU's L1 and are served by L2, sc1 stores write through: the pair is how workgroups of one
// persistent launch hand data to each other without acquire/release fences
// (MI355X_MICROARCH.md "Workgroup dispatch ... inter-workgroup visibility", valid forms).
__device__ __forceinline__ u32x4 rx_load16_sc1(const void* base, int byte_off) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc, byte_off, 0, 16);
}
__device__ __forceinline__ void rx_store16_sc1(void* base, int byte_off, const u32x4& v) {
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7ffffff0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, byte_off, 0, 16);
}

#define RX_CHECK(x)                                                     \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) return (int)e_;                               \
  } while (0)
