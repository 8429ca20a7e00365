// Shared device helpers for the gfx950 kernels (wave64, bf16 MFMA, bf16 packing).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;
typedef unsigned int rx_u32x2 __attribute__((ext_vector_type(2)));

#define RX_WAVE 64

// compile-time bool carried through a generic lambda's argument
template <bool B>
struct rx_bool {
  static constexpr bool value = B;
};

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

// DPP lane moves inside a row of 16 lanes (one VALU op, no LDS round trip):
// quad_perm [1,0,3,2] (lane ^ 1), quad_perm [2,3,0,1] (lane ^ 2), row_half_mirror, row_mirror
#define RX_DPP_XOR1 0xB1
#define RX_DPP_XOR2 0x4E
#define RX_DPP_HALF_MIRROR 0x141
#define RX_DPP_MIRROR 0x140
template <int CTRL>
__device__ __forceinline__ float rx_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ uint32_t rx_dppu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}

// sum over the 16 lanes of a row (lane & ~15): four DPP steps; every lane of the row gets the
// bit-identical total (each step adds a value and its mirror image, and a + b == b + a)
__device__ __forceinline__ float rx_rowsum16(float v) {
  v += rx_dpp<RX_DPP_XOR1>(v);
  v += rx_dpp<RX_DPP_XOR2>(v);
  v += rx_dpp<RX_DPP_HALF_MIRROR>(v);
  v += rx_dpp<RX_DPP_MIRROR>(v);
  return v;
}

// whole-wave sum: rows by DPP, then the four row sums by the permlane swaps (no LDS pipeline)
__device__ __forceinline__ float rx_wavesum(float v) { return rx_colsum16(rx_rowsum16(v)); }

// Transpose of a bf16 4x4 block held by the 4 lanes of a quad: lane q holds column q of rows
// 0..3 as {p.x = (row 0, row 1), p.y = (row 2, row 3)} (an MFMA accumulator's 4 rows, packed);
// afterwards lane q holds row q of columns 0..3 as {(col 0, col 1), (col 2, col 3)}, i.e. 8
// contiguous bytes of a row-major image -- one ds_write_b64 instead of four ds_write_b16.
// Two exchange rounds (lane ^ 2, then lane ^ 1): 3 DPP moves, 3 selects, 2 byte permutes.
__device__ __forceinline__ uint2 rx_quad_transpose(uint2 p, int q) {
  const bool hi2 = (q & 2) != 0;
  const uint32_t y = rx_dppu<RX_DPP_XOR2>(hi2 ? p.x : p.y);
  const uint32_t a = hi2 ? y : p.x;   // rows (q & 2) .. +1 of column q & 1
  const uint32_t b = hi2 ? p.y : y;   //                  ... of column (q & 1) + 2
  const uint32_t pa = rx_dppu<RX_DPP_XOR1>(a), pb = rx_dppu<RX_DPP_XOR1>(b);
  // even lanes keep the low halves (their row is even): (own, partner); odd: (partner, own)
  const uint32_t sel = (q & 1) ? 0x03020706u : 0x05040100u;
  return make_uint2(__builtin_amdgcn_perm(pa, a, sel), __builtin_amdgcn_perm(pb, b, sel));
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
