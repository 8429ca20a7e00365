// Fused Linear(+bias)(+ReLU) GEMMs for MLP towers wider than the single-workgroup fused MLP
// (the DLRM bottom / top MLPs of the reference notebook: examples/pytorch_dlrm.ipynb cell 9,
// TorchMlp 13->512->128->32 and 384->1024->1024->512->256->1).
//
// One MFMA kernel, three epilogues (bf16 operands, fp32 accumulation on
// v_mfma_f32_16x16x32_bf16):
//   FWD   Y  = act(X W^T + b)          A = X [M][K] rows,      B = W [N][K] rows
//   DGRAD dX = (dY W) * (Xin > 0)       A = G [M][N] rows,      B = W [N][K] read transposed
//   WGRAD dW = G^T X (+ db = sum_m G)   A = G [M][N] transposed, B = X [M][K] transposed
// so the ReLU mask of a layer is applied ONCE, in the epilogue of the dgrad that produces its
// output gradient (the input activation of the layer above is that layer's ReLU output), the
// bias gradient is the row sum of the wgrad's A fragments (no separate reduction kernel), and
// fp32 operands (the dense features, the dot-interaction output) are converted to bf16 while
// they are staged into LDS (no cast kernels).
//
// Tiling: TM x TN output tile per 256-thread workgroup (4 waves as 2x2; each wave owns a
// (TM/2) x (TN/2) block = (TM/32) x (TN/32) MFMA tiles), 64-deep K stages double-buffered in LDS.
// Two tile shapes are built: 64x64 (narrow layers, ragged edges) and 128x128 (the wide tower
// GEMMs: 4x the MFMAs per staged byte and per barrier -- a 64x64 tile moves 32 FLOP per L2 byte
// and spends its K loop waiting on loads, profiles/r2_linear_gemm_kernel_times.txt), plus the
// two mixed 128x64 / 64x128 shapes; rx_lin_plan picks the shape and split-K factor per GEMM.
// Each operand tile is staged in its memory orientation with 16-B row chunks; operands whose
// reduction index is the slow one in memory are read with gfx950's transposing LDS read
// (ds_read_b64_tr_b16), so no layout needs a transposed copy in HBM. Edges (any M, N, K, any
// leading dimension) are zero-filled on load and masked on store; a stage whose whole tile is
// in bounds and 16-B aligned takes unchecked vector loads.
#include "rx_common.h"

#include <string.h>

#define LIN_BK 64   // K-stage depth
#define LIN_S 80    // ROW image row stride in elements (160 B = 10 16-B units: ds_read_b128 fragment reads
                    // conflict-free for gfx950's lane groups {0-3,12-15,20-27}, ... ; 144 B was 2-way)
#define LIN_TMAX 128

enum { LIN_ROW = 0, LIN_RED = 1 };
enum { LIN_FWD = 0, LIN_DGRAD = 1, LIN_WGRAD = 2 };
// tile shapes (LinArgs.tile): 0 = planned by rx_lin_plan
enum { LIN_TILE_AUTO = 0, LIN_TILE_64x64 = 1, LIN_TILE_128x128 = 2, LIN_TILE_128x64 = 3, LIN_TILE_64x128 = 4 };

struct LinOperand {
  const void* p;
  long long ld;  // elements between consecutive memory-major indices
  int f32;       // 1: fp32 in memory (converted while staging), 0: bf16
  int lay;       // LIN_ROW: stored [row][k]; LIN_RED: stored [k][row]
};

struct LinArgs {
  int M, N, K;  // C[M][N] = sum_k A(m, k) B(k, n)
  int epi;
  LinOperand a, b;
  const float* bias;  // FWD: [N]
  int relu;           // FWD
  int out_f32;        // FWD/DGRAD: 1 -> fp32 output
  void* out;          // FWD/DGRAD: [M][ldo] bf16 (or fp32); WGRAD: fp32 [M][ldo]
  long long ldo;
  float* out2;  // FWD: optional fp32 copy of the activation [M][ldo2]
  long long ldo2;
  const u16* mask;  // DGRAD: zero the output where mask[m][n] (bf16) <= 0
  long long ldm;
  float* dbias;  // WGRAD: [M] row sums of A (bias gradient)
  float beta;    // WGRAD: out = beta * out + acc (same for dbias)
  int splits;    // split-K factor (grid.z); > 1 needs ws + counters
  float* ws;     // [tiles][splits][TM*TN + TM] fp32 partial tiles (+ partial row sums)
  unsigned* counters;  // [tiles], zero between calls (the last block of a tile resets it)
  int tile;            // LIN_TILE_*
  int pad_;
};

typedef short rx_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) rx_v4s rx_lds_v4s;

// LDS image of one operand tile of T rows: ROW -> [T][LIN_S] (row-major, k fastest);
// RED -> [LIN_BK][T + 16] (k-major, rows fastest)
template <int LAY, int T>
struct LinImg {
  static constexpr int stride = LAY == LIN_ROW ? LIN_S : T + 16;
  static constexpr int elems = LAY == LIN_ROW ? T * LIN_S : LIN_BK * (T + 16);
};

// ---- operand staging: global -> registers -> LDS, branch-free ----
// Every stage issues the same loads in the same order whatever the tile position: the loads of
// stage k+2 stay in flight (counted vmcnt) while stage k is multiplied and stage k+1 is written
// to LDS. Edges need no branches: each load goes through a buffer resource whose num_records
// is the operand's extent, and a chunk outside [0, I) x [0, J) gets an offset past it, which the
// hardware answers with zeros. (A data-dependent branch around a load makes hipcc wait for
// vmcnt(0) -- the whole prefetch pipeline then drains every stage.)
// Staging modes (host-selected per operand, LinArgs operand f32 / alignment):
//   LIN_V16: bf16, 16-B aligned rows, J % 8 == 0   -> one 16-B load per 8-element chunk
//   LIN_V32: fp32, same conditions                  -> two 16-B loads, converted at the LDS write
//   LIN_G16 / LIN_G32: any leading dimension / edge -> eight 2- / 4-byte loads per chunk
enum { LIN_V16 = 0, LIN_V32 = 1, LIN_G16 = 2, LIN_G32 = 3 };
#define LIN_OOB 0x80000000u  // byte offset past every operand extent (extents are < 2^31 bytes)

template <int MODE, int CH>
struct LinStage;  // CH chunks of 8 elements per thread
template <int CH>
struct LinStage<LIN_V16, CH> { u32x4 v[CH]; };
template <int CH>
struct LinStage<LIN_V32, CH> { u32x4 v[2 * CH]; };
template <int CH>
struct LinStage<LIN_G16, CH> { u16 v[8 * CH]; };
template <int CH>
struct LinStage<LIN_G32, CH> { uint32_t v[8 * CH]; };

// buffer resource over one operand: [I][ld] elements in memory, J valid along the fast index
template <int MODE>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lin_rsrc(const LinOperand& o, long long I, long long J) {
  const long long esz = (MODE == LIN_V32 || MODE == LIN_G32) ? 4 : 2;
  const long long ext = I > 0 && J > 0 ? ((I - 1) * o.ld + J) * esz : 0;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(o.p), 0, (int)ext, 0x00020000);
}

// The T/32 chunks a thread stages for one operand tile of T rows: tile rows r0..r0+T-1,
// reduction k0..k0+63 (memory orientation: ROW -> (i, j) = (row, k); RED -> (i, j) = (k, row)).
// Index math is 32-bit unsigned: the host bounds every operand extent below 2^31 bytes (the
// buffer resource's num_records), so no element offset needs 64 bits -- 64-bit multiplies per
// chunk per stage were most of the kernel's VALU work (profiles/pmc/SUMMARY.md: VALU/MFMA 12.3).
template <int MODE, int LAY, int T>
__device__ __forceinline__ void lin_fetch(__amdgpu_buffer_rsrc_t rs, long long ld, long long r0, long long k0,
                                          long long R, long long Kd, int tid, LinStage<MODE, T / 32>& st) {
  constexpr int CPR = LAY == LIN_ROW ? LIN_BK / 8 : T / 8;  // chunks per memory row of the tile
  const unsigned I = (unsigned)(LAY == LIN_ROW ? R : Kd), J = (unsigned)(LAY == LIN_ROW ? Kd : R);
  const unsigned ldu = (unsigned)ld, r0u = (unsigned)r0, k0u = (unsigned)k0;
#pragma unroll
  for (int t = 0; t < T / 32; ++t) {
    const int c = tid + 256 * t;
    const unsigned ci = (unsigned)(c / CPR), cj = (unsigned)((c % CPR) * 8);
    const unsigned i = LAY == LIN_ROW ? r0u + ci : k0u + ci;
    const unsigned j = LAY == LIN_ROW ? k0u + cj : r0u + cj;
    const unsigned e0 = i * ldu + j;  // element offset of the chunk
    if constexpr (MODE == LIN_V16) {
      const unsigned off = (i < I && j < J) ? (unsigned)(e0 * 2) : LIN_OOB;
      st.v[t] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
    } else if constexpr (MODE == LIN_V32) {
      const unsigned off = (i < I && j < J) ? (unsigned)(e0 * 4) : LIN_OOB;
      st.v[2 * t] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
      st.v[2 * t + 1] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(off + 16u), 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool ok = i < I && j + e < J;
        if constexpr (MODE == LIN_G16)
          st.v[8 * t + e] = __builtin_amdgcn_raw_buffer_load_b16(rs, (int)(ok ? (unsigned)((e0 + e) * 2) : LIN_OOB), 0, 0);
        else
          st.v[8 * t + e] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(ok ? (unsigned)((e0 + e) * 4) : LIN_OOB), 0, 0);
      }
    }
  }
}

// Write a staged tile into its LDS image as bf16 (fp32 operands converted here, after their
// loads have landed -- converting at the load would make the stage wait for them).
template <int MODE, int LAY, int T>
__device__ __forceinline__ void lin_stash(u16* img, int tid, const LinStage<MODE, T / 32>& st) {
  constexpr int CPR = LAY == LIN_ROW ? LIN_BK / 8 : T / 8;
#pragma unroll
  for (int t = 0; t < T / 32; ++t) {
    const int c = tid + 256 * t;
    const int ci = c / CPR, cj = (c % CPR) * 8;
    uint4 r;
    if constexpr (MODE == LIN_V16) {
      r = make_uint4(st.v[t][0], st.v[t][1], st.v[t][2], st.v[t][3]);
    } else if constexpr (MODE == LIN_V32) {
      const u32x4 x = st.v[2 * t], y = st.v[2 * t + 1];
      r.x = rx_f2bf2(__uint_as_float(x[0]), __uint_as_float(x[1]));
      r.y = rx_f2bf2(__uint_as_float(x[2]), __uint_as_float(x[3]));
      r.z = rx_f2bf2(__uint_as_float(y[0]), __uint_as_float(y[1]));
      r.w = rx_f2bf2(__uint_as_float(y[2]), __uint_as_float(y[3]));
    } else if constexpr (MODE == LIN_G16) {
      const u16* v = st.v + 8 * t;
      r.x = v[0] | ((uint32_t)v[1] << 16);
      r.y = v[2] | ((uint32_t)v[3] << 16);
      r.z = v[4] | ((uint32_t)v[5] << 16);
      r.w = v[6] | ((uint32_t)v[7] << 16);
    } else {
      const uint32_t* v = st.v + 8 * t;
      r.x = rx_f2bf2(__uint_as_float(v[0]), __uint_as_float(v[1]));
      r.y = rx_f2bf2(__uint_as_float(v[2]), __uint_as_float(v[3]));
      r.z = rx_f2bf2(__uint_as_float(v[4]), __uint_as_float(v[5]));
      r.w = rx_f2bf2(__uint_as_float(v[6]), __uint_as_float(v[7]));
    }
    *reinterpret_cast<uint4*>(img + ci * LinImg<LAY, T>::stride + cj) = r;
  }
}

// MFMA operand fragment for tile rows rb..rb+15, reduction ks..ks+31 (lane l: row rb + (l & 15),
// k = ks + 8 (l >> 4) + e).
template <int LAY, int T>
__device__ __forceinline__ bf16x8 lin_frag(const u16* img, int rb, int ks, int lane) {
  constexpr int S = LinImg<LAY, T>::stride;
  if constexpr (LAY == LIN_ROW) {
    const uint4 x = *reinterpret_cast<const uint4*>(img + (rb + (lane & 15)) * S + ks + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8, x);
  } else {
    // [k][row] image: each 16-lane group h reads rows k = ks + 8h + {0..3} and {4..7}; lane 4q+p
    // addresses row q, columns rb + 4p .. +3; lane i receives column rb + i
    const int h = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const u16* a0 = img + (ks + 8 * h + q) * S + rb + 4 * p;
    const u16* a1 = a0 + 4 * S;
    const rx_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (rx_lds_v4s*)((__attribute__((address_space(3))) char*)(uintptr_t)(a0)));
    const rx_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (rx_lds_v4s*)((__attribute__((address_space(3))) char*)(uintptr_t)(a1)));
    typedef short rx_v8s __attribute__((ext_vector_type(8)));
    const rx_v8s all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, all);
  }
}

__device__ __forceinline__ float lin_bsum(const bf16x8& f) {
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) s += (float)f[e];
  return s;
}

// LA / LB: the operands' memory orientations as template constants (FWD: ROW x ROW, DGRAD:
// ROW x RED, WGRAD: RED x RED), so the fragment reads compile to straight-line ds_reads the
// scheduler can batch ahead of the MFMAs instead of layout branches between them.
// LDS of one GEMM block: [buffer][A image | B image] (u16 elements)
template <int LA, int LB, int TM, int TN>
struct LinLds {
  static constexpr int IA = LinImg<LA, TM>::elems, IB = LinImg<LB, TN>::elems;
  static constexpr int elems = 2 * (IA + IB);
};

// One output tile (bx, by) / K split bz of a GEMM whose tile grid has gy columns. Shared by the
// single-GEMM kernel and the paired kernel (two independent GEMMs in one launch).
template <int AM, int BM, int LA, int LB, int TM, int TN>
__device__ __forceinline__ void lin_gemm_body(const LinArgs& a, u16* lds, int bx, int by, int bz, int gy) {
  constexpr int FM = TM / 32, FN = TN / 32;  // MFMA tiles per wave along M / N
  constexpr int IA = LinLds<LA, LB, TM, TN>::IA, IB = LinLds<LA, LB, TM, TN>::IB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)bx * TM, n0 = (long long)by * TN;
  // split-K: this block reduces K stages [k_begin, k_end)
  const int nk_all = (a.K + LIN_BK - 1) / LIN_BK;
  const int per = (nk_all + a.splits - 1) / a.splits;
  const int k_begin = bz * per;
  const int k_end = min(nk_all, k_begin + per);
  const int nk = max(0, k_end - k_begin);
  const bool want_db = a.epi == LIN_WGRAD && a.dbias != nullptr && by == 0 && wn == 0;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int x = 0; x < FM; ++x)
#pragma unroll
    for (int y = 0; y < FN; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float asum[FM];
#pragma unroll
  for (int x = 0; x < FM; ++x) asum[x] = 0.f;

  const auto rsa = lin_rsrc<AM>(a.a, LA == LIN_ROW ? a.M : a.K, LA == LIN_ROW ? a.K : a.M);
  const auto rsb = lin_rsrc<BM>(a.b, LB == LIN_ROW ? a.N : a.K, LB == LIN_ROW ? a.K : a.N);
  // Global -> register -> LDS pipeline two stages deep: while stage kt is multiplied out of LDS,
  // stage kt+1 sits in one register set (loaded a stage ago, written to LDS after the MFMAs) and
  // stage kt+2's loads are in flight into the other set -- each load has two stages of MFMAs to
  // arrive in. The loop is unrolled by two so the sets swap roles without register copies.
  // The prefetch index is clamped (the last stages re-load stage nk-1 into a set nobody
  // reads) so every stage issues the same loads: no branch, counted waits.
  LinStage<AM, TM / 32> ra, qa;
  LinStage<BM, TN / 32> rb, qb;
  auto fetch = [&](int kt, LinStage<AM, TM / 32>& fa_, LinStage<BM, TN / 32>& fb_) {
    const long long k0 = (long long)(k_begin + kt) * LIN_BK;
    lin_fetch<AM, LA, TM>(rsa, a.a.ld, m0, k0, a.M, a.K, tid, fa_);
    lin_fetch<BM, LB, TN>(rsb, a.b.ld, n0, k0, a.N, a.K, tid, fb_);
  };
  auto img_a = [&](int buf) { return lds + buf * (IA + IB); };
  auto img_b = [&](int buf) { return lds + buf * (IA + IB) + IA; };
  auto stage = [&](int kt, const LinStage<AM, TM / 32>& sa, const LinStage<BM, TN / 32>& sb,
                   LinStage<AM, TM / 32>& la, LinStage<BM, TN / 32>& lb) {
    const int cur = kt & 1;
    fetch(min(kt + 2, nk - 1), la, lb);
    const u16* ia = img_a(cur);
    const u16* ib = img_b(cur);
#pragma unroll
    for (int ks = 0; ks < LIN_BK; ks += 32) {
      bf16x8 fa[FM], fb[FN];
#pragma unroll
      for (int x = 0; x < FM; ++x) fa[x] = lin_frag<LA, TM>(ia, wm * (TM / 2) + 16 * x, ks, lane);
#pragma unroll
      for (int y = 0; y < FN; ++y) fb[y] = lin_frag<LB, TN>(ib, wn * (TN / 2) + 16 * y, ks, lane);
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y) acc[x][y] = rx_mfma16(fa[x], fb[y], acc[x][y]);
      if (want_db) {
#pragma unroll
        for (int x = 0; x < FM; ++x) asum[x] += lin_bsum(fa[x]);
      }
    }
    // stage kt+1 into the other buffer (after the last stage: a re-loaded copy nobody reads)
    lin_stash<AM, LA, TM>(img_a(cur ^ 1), tid, sa);
    lin_stash<BM, LB, TN>(img_b(cur ^ 1), tid, sb);
    __syncthreads();
  };
  if (nk > 0) {
    fetch(0, ra, rb);
    lin_stash<AM, LA, TM>(img_a(0), tid, ra);
    lin_stash<BM, LB, TN>(img_b(0), tid, rb);
    fetch(min(1, nk - 1), ra, rb);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {
      stage(kt, ra, rb, qa, qb);      // write stage kt+1 from r*, load kt+2 into q*
      stage(kt + 1, qa, qb, ra, rb);  // write stage kt+2 from q*, load kt+3 into r*
    }
    if (kt < nk) stage(kt, ra, rb, qa, qb);
  }

  if (a.splits > 1) {
    // deterministic split-K fix-up: every split parks its fp32 tile (and its partial bias-row
    // sums) in the workspace; the block that arrives last sums ALL splits in split order -- the
    // result does not depend on which block came last -- and runs the epilogue. Hand-off
    // (MI355X: per-XCD L2s): write-through sc1 payload stores drained by every storing wave, a
    // barrier, ONE agent-scope counter add; the last block reads the payload with sc1 loads only
    // (they bypass its L1), so no release / acquire fence is needed.
    const int tile = bx * gy + by;
    const int TW = TM * TN + TM;
    float* mine = a.ws + ((long long)tile * a.splits + bz) * TW;
    const int slot = ((wave * 64 + lane) * (FM * FN * 4)) * 4;  // byte offset of this lane's floats
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
      for (int y = 0; y < FN; ++y)
        rx_store16_sc1(mine, slot + 16 * (FN * x + y), __builtin_bit_cast(u32x4, acc[x][y]));
    if (want_db) {
#pragma unroll
      for (int x = 0; x < FM; ++x) {
        const float sx = rx_colsum16(asum[x]);
        if (lane < 16)
          __hip_atomic_store(rx_g(mine) + TM * TN + wm * (TM / 2) + 16 * x + lane, sx, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    // the flag lives in the (now idle) operand images: a separate __shared__ word would add a
    // second LDS object (and push the 64x64 block past 40 KiB: one resident workgroup less per CU)
    unsigned* last_flag = reinterpret_cast<unsigned*>(&lds[0]);
    if (tid == 0) {
      const unsigned done = __hip_atomic_fetch_add(rx_g(a.counters) + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_flag = done + 1 == (unsigned)a.splits;
    }
    __syncthreads();
    if (!*last_flag) return;
    const float* base = a.ws + (long long)tile * a.splits * TW;
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
      for (int y = 0; y < FN; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float dsum[FM];
#pragma unroll
    for (int x = 0; x < FM; ++x) dsum[x] = 0.f;
    for (int sp = 0; sp < a.splits; ++sp) {
      const float* ps = base + (long long)sp * TW;
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
          acc[x][y] += __builtin_bit_cast(f32x4, rx_load16_sc1(ps, slot + 16 * (FN * x + y)));
      if (want_db && lane < 16) {
#pragma unroll
        for (int x = 0; x < FM; ++x)
          dsum[x] += __hip_atomic_load(rx_g(ps) + TM * TN + wm * (TM / 2) + 16 * x + lane, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (tid == 0) __hip_atomic_store(rx_g(a.counters) + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (want_db) {
#pragma unroll
      for (int x = 0; x < FM; ++x) {
        const long long m = m0 + wm * (TM / 2) + 16 * x + (lane & 15);
        if (lane < 16 && m < a.M) a.dbias[m] = a.beta != 0.f ? a.beta * a.dbias[m] + dsum[x] : dsum[x];
      }
    }
  }

  // Epilogue: lane holds rows rb + 4 (lane >> 4) + r (r = 0..3) of column cb + (lane & 15).
  // Branch-free like the staging: every access goes through a buffer resource sized to its
  // tensor (a null optional tensor gets num_records 0), out-of-range elements get an offset past
  // it (loads answer 0, stores are dropped), all loads of the tile are issued before the first
  // use, and index math is 32-bit (the host bounds every extent below 2^31 bytes).
  const unsigned M = (unsigned)a.M, N = (unsigned)a.N;
  const unsigned mb0 = (unsigned)m0 + wm * (TM / 2) + 4 * (lane >> 4), nb0 = (unsigned)n0 + wn * (TN / 2) + (lane & 15);
  // element index (row offset + column) of every accumulator element, or ~0u when out of range
  auto elem_idx = [&](unsigned ld, unsigned (&idx)[FM][FN][4]) {
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned m = mb0 + 16 * x + r;
        const unsigned ro = m * ld;
#pragma unroll
        for (int y = 0; y < FN; ++y) {
          const unsigned n = nb0 + 16 * y;
          idx[x][y][r] = ((m < M) & (n < N)) ? ro + n : ~0u;
        }
      }
  };
  auto boff = [](unsigned i, unsigned esz) -> int { return (int)(i != ~0u ? i * esz : LIN_OOB); };
  auto rsrc_of = [&](const void* p, long long ld, long long esz) {
    const long long ext = p != nullptr ? ((long long)(a.M - 1) * ld + a.N) * esz : 0;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)ext, 0x00020000);
  };
  unsigned idx[FM][FN][4];
  elem_idx((unsigned)a.ldo, idx);
  if (a.epi == LIN_FWD) {
    const auto rbias = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.bias), 0,
                                                         a.bias != nullptr ? a.N * 4 : 0, 0x00020000);
    float bv[FN];
#pragma unroll
    for (int y = 0; y < FN; ++y) {
      const unsigned n = nb0 + 16 * y;
      bv[y] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rbias, (int)(n < N ? n * 4 : LIN_OOB), 0, 0));
    }
    const float lo = a.relu ? 0.f : -INFINITY;
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
      for (int y = 0; y < FN; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[x][y][r] = fmaxf(acc[x][y][r] + bv[y], lo);
    const auto ro = rsrc_of(a.out, a.ldo, a.out_f32 ? 4 : 2);
    if (a.out_f32) {
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[x][y][r]), ro, boff(idx[x][y][r], 4), 0, 0);
    } else {
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b16(rx_f2bf(acc[x][y][r]), ro, boff(idx[x][y][r], 2), 0, 0);
    }
    if (a.out2 != nullptr) {
      const auto ro2 = rsrc_of(a.out2, a.ldo2, 4);
      elem_idx((unsigned)a.ldo2, idx);
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[x][y][r]), ro2, boff(idx[x][y][r], 4), 0, 0);
    }
  } else if (a.epi == LIN_DGRAD) {
    if (a.mask != nullptr) {
      const auto rm = rsrc_of(a.mask, a.ldm, 2);
      unsigned mi[FM][FN][4];
      elem_idx((unsigned)a.ldm, mi);
      u16 mk[FM][FN][4];
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) mk[x][y][r] = __builtin_amdgcn_raw_buffer_load_b16(rm, boff(mi[x][y][r], 2), 0, 0);
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[x][y][r] = rx_bf2f(mk[x][y][r]) > 0.f ? acc[x][y][r] : 0.f;
    }
    const auto ro = rsrc_of(a.out, a.ldo, a.out_f32 ? 4 : 2);
    if (a.out_f32) {
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[x][y][r]), ro, boff(idx[x][y][r], 4), 0, 0);
    } else {
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            __builtin_amdgcn_raw_buffer_store_b16(rx_f2bf(acc[x][y][r]), ro, boff(idx[x][y][r], 2), 0, 0);
    }
  } else {
    const auto ro = rsrc_of(a.out, a.ldo, 4);
    if (a.beta != 0.f) {
      float old[FM][FN][4];
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            old[x][y][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ro, boff(idx[x][y][r], 4), 0, 0));
#pragma unroll
      for (int x = 0; x < FM; ++x)
#pragma unroll
        for (int y = 0; y < FN; ++y)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[x][y][r] += a.beta * old[x][y][r];
    }
#pragma unroll
    for (int x = 0; x < FM; ++x)
#pragma unroll
      for (int y = 0; y < FN; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[x][y][r]), ro, boff(idx[x][y][r], 4), 0, 0);
  }
  if (want_db && a.splits <= 1) {
#pragma unroll
    for (int x = 0; x < FM; ++x) {
      const float s = rx_colsum16(asum[x]);  // the 4 lanes of row (lane & 15) hold k-quarters
      const long long m = m0 + wm * (TM / 2) + 16 * x + (lane & 15);
      if (lane < 16 && m < a.M) a.dbias[m] = a.beta != 0.f ? a.beta * a.dbias[m] + s : s;
    }
  }
}

template <int AM, int BM, int LA, int LB, int TM, int TN>
__global__ __launch_bounds__(256) void lin_gemm_kernel(LinArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[LinLds<LA, LB, TM, TN>::elems];
  lin_gemm_body<AM, BM, LA, LB, TM, TN>(a, lds, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.y);
}

// Two independent 64x64-tiled GEMMs in ONE launch: a layer's dgrad (ROW x RED, critical path of
// the backward) and its wgrad (RED x RED, needed only by the optimizer) both read only that
// layer's output gradient, so the tower backward issues one launch per layer instead of two
// (the DLRM step at the notebook's batch 128 is launch bound: ~5 us per dependent launch).
// Blocks [0, nb0) run problem 0, the rest problem 1; each problem's blocks are numbered
// (split, row tile, column tile) like the single kernel's grid. One LDS array of the larger size.
struct LinPair {
  LinArgs p[2];
  int gy[2];  // column tiles of each problem's grid
  int gxy[2]; // tiles per split of each problem
  int nb0;    // blocks of problem 0 (tiles x splits)
  int pad_;
};

template <int AM0, int BM0, int AM1, int BM1>
__global__ __launch_bounds__(256) void lin_pair_kernel(LinPair q) {
  constexpr int E0 = LinLds<LIN_ROW, LIN_RED, 64, 64>::elems, E1 = LinLds<LIN_RED, LIN_RED, 64, 64>::elems;
  __shared__ __attribute__((aligned(16))) u16 lds[E0 > E1 ? E0 : E1];
  int id = blockIdx.x;
  if (id < q.nb0) {
    const int bz = id / q.gxy[0], r = id - bz * q.gxy[0];
    lin_gemm_body<AM0, BM0, LIN_ROW, LIN_RED, 64, 64>(q.p[0], lds, r / q.gy[0], r % q.gy[0], bz, q.gy[0]);
  } else {
    id -= q.nb0;
    const int bz = id / q.gxy[1], r = id - bz * q.gxy[1];
    lin_gemm_body<AM1, BM1, LIN_RED, LIN_RED, 64, 64>(q.p[1], lds, r / q.gy[1], r % q.gy[1], bz, q.gy[1]);
  }
}

// G = gY * (Y > 0) (relu) or G = gY, fp32 -> bf16 (the tower's top-layer output gradient).
// gY rows are ldg floats apart (a column slice of a wider gradient, e.g. the DLRM interaction's
// bottom-MLP slot, is read in place); Y and G are dense [n / cols][cols].
__global__ __launch_bounds__(256) void lin_mask_cast_kernel(const float* __restrict__ g, const u16* __restrict__ y,
                                                            u16* __restrict__ out, long long n, int cols, long long ldg) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols;
    float v = g[r * ldg + (i - r * cols)];
    if (y != nullptr && !(rx_bf2f(y[i]) > 0.f)) v = 0.f;
    out[i] = rx_f2bf(v);
  }
}

// bf16 images of fp32 master weights, several tensors per launch.
struct LinRefresh {
  int n;
  int pad_;
  const float* src[16];
  u16* dst[16];
  long long len[16];
};

__global__ __launch_bounds__(256) void lin_refresh_kernel(LinRefresh r) {
  const int t = blockIdx.y;
  const float* s = r.src[t];
  u16* d = r.dst[t];
  const long long n = r.len[t];
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 2; i < n;
       i += (long long)gridDim.x * blockDim.x * 2) {
    if (i + 1 < n)
      *reinterpret_cast<uint32_t*>(d + i) = rx_f2bf2(s[i], s[i + 1]);
    else
      d[i] = rx_f2bf(s[i]);
  }
}

extern "C" {

int rx_lin_args_size() { return (int)sizeof(LinArgs); }
int rx_lin_refresh_size() { return (int)sizeof(LinRefresh); }

static void lin_tile_dims(int tile, int* tm, int* tn) {
  *tm = (tile == LIN_TILE_128x128 || tile == LIN_TILE_128x64) ? 128 : 64;
  *tn = (tile == LIN_TILE_128x128 || tile == LIN_TILE_64x128) ? 128 : 64;
}

static long long lin_tiles(int M, int N, int tile) {
  int tm, tn;
  lin_tile_dims(tile, &tm, &tn);
  return (long long)((M + tm - 1) / tm) * ((N + tn - 1) / tn);
}

// Tile shape and split-K factor for one GEMM, fitted to a measured sweep of every shape x
// split factor at the DLRM tower GEMMs (benchmarks/linear_gemm_bench.py --sweep,
// profiles/r3_linear_gemm_sweep.txt):
// * 64x64 tiles everywhere: at batch 2048 the 128-wide tiles leave half the CUs idle (128
//   workgroups for a 2048x1024 output) and their one wave per SIMD exposes every LDS and barrier
//   latency; splitting K to fill the chip costs more in the fix-up than it wins.
// * split-K only for problems with few output tiles AND a deep K (the weight gradients at
//   batch 2048, K = batch): about 192 workgroups, each split at least eight 64-deep stages
//   (s1 -> s4 is 17 -> 10.5 us at 2 tiles; at 512 tiles any split doubles the time). Below 24
//   stages the fix-up costs more than the shorter K loop saves: at the notebook's batch 128 the
//   1024-deep forward GEMMs run 8.06 / 7.95 us unsplit vs 8.83 / 8.64 us at s2
//   (profiles/r3_linear_gemm_sweep_batch128.txt).
// tile_force != 0 fixes the shape (sweeps / tests); the cus argument scales the target.
int rx_lin_plan(int M, int N, int K, int cus, int tile_force, int* tile_out) {
  const int tile = tile_force != LIN_TILE_AUTO ? tile_force : LIN_TILE_64x64;
  if (tile_out) *tile_out = tile;
  const long long tiles = lin_tiles(M, N, tile);
  const int nk = (K + LIN_BK - 1) / LIN_BK;
  const long long target = (3LL * (cus > 0 ? cus : 256)) / 4;  // 192 on MI355X
  long long want = (target + tiles - 1) / tiles;
  long long mx = nk >= 24 ? nk / 8 : 1;
  if (want > mx) want = mx;
  if (want > 64) want = 64;
  return want < 1 ? 1 : (int)want;
}

int rx_lin_splits(int M, int N, int K, int cus) { return rx_lin_plan(M, N, K, cus, LIN_TILE_AUTO, nullptr); }

int rx_lin_tile(int M, int N, int K, int cus) {
  int t = 0;
  rx_lin_plan(M, N, K, cus, LIN_TILE_AUTO, &t);
  return t;
}

// Split-K workspace for `splits` splits under ANY tile shape.
int rx_lin_ws_floats(int M, int N, int splits) {
  if (splits <= 1) return 0;
  long long need = 0;
  for (int t = LIN_TILE_64x64; t <= LIN_TILE_64x128; ++t) {
    int tm, tn;
    lin_tile_dims(t, &tm, &tn);
    const long long f = lin_tiles(M, N, t) * splits * (tm * tn + tm);
    need = f > need ? f : need;
  }
  return (int)need;
}

}  // extern "C"

template <int AM, int BM, int TM, int TN>
static void lin_launch_lay(const LinArgs* a, dim3 grid, hipStream_t stream) {
  if (a->a.lay == LIN_ROW && a->b.lay == LIN_ROW)
    hipLaunchKernelGGL((lin_gemm_kernel<AM, BM, LIN_ROW, LIN_ROW, TM, TN>), grid, dim3(256), 0, stream, *a);
  else if (a->a.lay == LIN_ROW)
    hipLaunchKernelGGL((lin_gemm_kernel<AM, BM, LIN_ROW, LIN_RED, TM, TN>), grid, dim3(256), 0, stream, *a);
  else if (a->b.lay == LIN_ROW)
    hipLaunchKernelGGL((lin_gemm_kernel<AM, BM, LIN_RED, LIN_ROW, TM, TN>), grid, dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL((lin_gemm_kernel<AM, BM, LIN_RED, LIN_RED, TM, TN>), grid, dim3(256), 0, stream, *a);
}

// Staging mode of one operand: vector loads when every row starts 16-B aligned and the fast
// index's extent is a multiple of 8 (so no 8-element chunk straddles the edge).
static int lin_mode(const LinOperand& o, long long J) {
  const int esz = o.f32 ? 4 : 2;
  const bool vec = ((uintptr_t)o.p & 15) == 0 && (o.ld * esz) % 16 == 0 && J % 8 == 0;
  return (vec ? 0 : 2) + (o.f32 ? 1 : 0);
}

// the wider tiles are built for the vector modes only (the generic modes serve the narrow,
// unaligned layers, e.g. the 13 dense features)
template <int TM, int TN>
static void lin_launch_vec(const LinArgs* a, int ma, int mb, hipStream_t stream) {
  const dim3 grid((unsigned)((a->M + TM - 1) / TM), (unsigned)((a->N + TN - 1) / TN), (unsigned)a->splits);
  if (ma == LIN_V16 && mb == LIN_V16)
    lin_launch_lay<LIN_V16, LIN_V16, TM, TN>(a, grid, stream);
  else if (ma == LIN_V16)
    lin_launch_lay<LIN_V16, LIN_V32, TM, TN>(a, grid, stream);
  else if (mb == LIN_V16)
    lin_launch_lay<LIN_V32, LIN_V16, TM, TN>(a, grid, stream);
  else
    lin_launch_lay<LIN_V32, LIN_V32, TM, TN>(a, grid, stream);
}

template <int AM>
static void lin_launch_64_b(const LinArgs* a, int mb, dim3 grid, hipStream_t stream) {
  switch (mb) {
    case LIN_V16: lin_launch_lay<AM, LIN_V16, 64, 64>(a, grid, stream); break;
    case LIN_V32: lin_launch_lay<AM, LIN_V32, 64, 64>(a, grid, stream); break;
    case LIN_G16: lin_launch_lay<AM, LIN_G16, 64, 64>(a, grid, stream); break;
    default: lin_launch_lay<AM, LIN_G32, 64, 64>(a, grid, stream); break;
  }
}

static void lin_launch_64(const LinArgs* a, int ma, int mb, hipStream_t stream) {
  const dim3 grid((unsigned)((a->M + 63) / 64), (unsigned)((a->N + 63) / 64), (unsigned)a->splits);
  switch (ma) {
    case LIN_V16: lin_launch_64_b<LIN_V16>(a, mb, grid, stream); break;
    case LIN_V32: lin_launch_64_b<LIN_V32>(a, mb, grid, stream); break;
    case LIN_G16: lin_launch_64_b<LIN_G16>(a, mb, grid, stream); break;
    default: lin_launch_64_b<LIN_G32>(a, mb, grid, stream); break;
  }
}

extern "C" {

// a->tile == LIN_TILE_AUTO: the shape rx_lin_plan picks (for the same M, N, K); a->splits is
// used as given. Operands that need the generic (element-wise) staging run on 64x64 tiles.
int rx_lin_gemm(const LinArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  if (a->K < 0 || a->epi < 0 || a->epi > 2 || a->splits < 1 || a->tile < 0 || a->tile > LIN_TILE_64x128) return -1;
  if (a->splits > 1 && (a->ws == nullptr || a->counters == nullptr)) return -1;
  // buffer-resource extents are 31-bit byte counts
  const long long ea = (long long)(a->a.lay == LIN_ROW ? a->M : a->K) * a->a.ld * (a->a.f32 ? 4 : 2);
  const long long eb = (long long)(a->b.lay == LIN_ROW ? a->N : a->K) * a->b.ld * (a->b.f32 ? 4 : 2);
  if (ea >= (1LL << 31) || eb >= (1LL << 31)) return -2;
  int tile = a->tile;
  if (tile == LIN_TILE_AUTO) rx_lin_plan(a->M, a->N, a->K, 256, LIN_TILE_AUTO, &tile);
  const int ma = lin_mode(a->a, a->a.lay == LIN_ROW ? a->K : a->M);
  const int mb = lin_mode(a->b, a->b.lay == LIN_ROW ? a->K : a->N);
  if (ma >= LIN_G16 || mb >= LIN_G16) tile = LIN_TILE_64x64;
  switch (tile) {
    case LIN_TILE_128x128: lin_launch_vec<128, 128>(a, ma, mb, stream); break;
    case LIN_TILE_128x64: lin_launch_vec<128, 64>(a, ma, mb, stream); break;
    case LIN_TILE_64x128: lin_launch_vec<64, 128>(a, ma, mb, stream); break;
    default: lin_launch_64(a, ma, mb, stream); break;
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- whole-tower drivers ----
// One host call per tower direction (the per-GEMM Python/ctypes cost was comparable to the
// kernels themselves at DLRM sizes).
struct LinLayer {
  const u16* W;       // bf16 image [N][K]
  const float* bias;  // [N] or null
  float* dW;          // [N][K] fp32 gradient out (backward; null: no weight gradient)
  float* db;          // [N] fp32 (null: none)
  int N, K;
  int relu;
  int pad_;
};

struct LinScratch {
  float* ws;
  unsigned* counters;
  long long ws_floats;
  int counters_len;
  int cus;
  int pair;  // 1: the backward pairs each layer's dgrad and wgrad in one launch (needs the
             //    workspace / counters sized for two problems: each gets one half)
  int pad_;
};

int rx_lin_mask_cast(const float* g, const u16* y, u16* out, long long n, hipStream_t stream);
static int lin_mask_cast2(const float* g, long long ldg, const u16* y, u16* out, int rows, int cols,
                          hipStream_t stream);

static int lin_run(LinArgs& a, const LinScratch& sc, hipStream_t stream) {
  int tile = LIN_TILE_AUTO;
  a.splits = rx_lin_plan(a.M, a.N, a.K, sc.cus, LIN_TILE_AUTO, &tile);
  a.tile = tile;
  if (a.splits > 1 && ((long long)rx_lin_ws_floats(a.M, a.N, a.splits) > sc.ws_floats ||
                       lin_tiles(a.M, a.N, tile) > sc.counters_len))
    a.splits = 1;  // scratch too small for this shape: run unsplit
  a.ws = a.splits > 1 ? sc.ws : nullptr;
  a.counters = a.splits > 1 ? sc.counters : nullptr;
  return rx_lin_gemm(&a, stream);
}

// Plan one problem of a pair into its half of the scratch.
static void lin_plan_half(LinArgs& a, const LinScratch& sc, int half) {
  int tile = LIN_TILE_AUTO;
  a.splits = rx_lin_plan(a.M, a.N, a.K, sc.cus, LIN_TILE_AUTO, &tile);
  a.tile = LIN_TILE_64x64;
  const long long wsh = sc.ws_floats / 2, ch = sc.counters_len / 2;
  if (a.splits > 1 && ((long long)rx_lin_ws_floats(a.M, a.N, a.splits) > wsh || lin_tiles(a.M, a.N, LIN_TILE_64x64) > ch))
    a.splits = 1;
  a.ws = a.splits > 1 ? sc.ws + half * wsh : nullptr;
  a.counters = a.splits > 1 ? sc.counters + half * ch : nullptr;
}

// dgrad d (ROW x RED) and wgrad w (RED x RED) of one layer in one launch when both take the
// 64x64 tile and the staging modes the paired kernel is built for (bf16 vector operands; the
// wgrad's activation operand bf16 or fp32 vector); otherwise two launches.
static int lin_run_pair(LinArgs& d, LinArgs& w, const LinScratch& sc, hipStream_t stream) {
  const int dma = lin_mode(d.a, d.K), dmb = lin_mode(d.b, d.N);
  const int wma = lin_mode(w.a, w.M), wmb = lin_mode(w.b, w.N);
  int td = 0, tw = 0;
  rx_lin_plan(d.M, d.N, d.K, sc.cus, LIN_TILE_AUTO, &td);
  rx_lin_plan(w.M, w.N, w.K, sc.cus, LIN_TILE_AUTO, &tw);
  // built pairs (A modes = the layer gradient G, staged the same way by both problems):
  //   G bf16:  <V16, V16 | V16, V16 or V32>   (any layer below the top; X bf16 or fp32 input)
  //   G fp32:  <V32, V16 | V32, V16>          (top layer of a tower whose gradient arrives fp32)
  //            <G32, V16 | G32, V16>          (the same with an unaligned width, e.g. the logit)
  const bool gv16 = dma == LIN_V16 && wma == LIN_V16 && (wmb == LIN_V16 || wmb == LIN_V32);
  const bool gf32 = ((dma == LIN_V32 && wma == LIN_V32) || (dma == LIN_G32 && wma == LIN_G32)) && wmb == LIN_V16;
  const bool ok = sc.pair && d.M > 0 && d.N > 0 && w.M > 0 && w.N > 0 && td == LIN_TILE_64x64 &&
                  tw == LIN_TILE_64x64 && dmb == LIN_V16 && (gv16 || gf32);
  if (!ok) {
    int rc = lin_run(w, sc, stream);
    return rc ? rc : lin_run(d, sc, stream);
  }
  const long long ed = (long long)d.M * d.a.ld * (d.a.f32 ? 4 : 2), eb = (long long)d.K * d.b.ld * 2;
  const long long ewa = (long long)w.K * w.a.ld * (w.a.f32 ? 4 : 2), ewb = (long long)w.K * w.b.ld * (w.b.f32 ? 4 : 2);
  if (ed >= (1LL << 31) || eb >= (1LL << 31) || ewa >= (1LL << 31) || ewb >= (1LL << 31)) return -2;
  LinPair q;
  memset(&q, 0, sizeof(q));
  lin_plan_half(d, sc, 0);
  lin_plan_half(w, sc, 1);
  q.p[0] = d;
  q.p[1] = w;
  const int gx0 = (d.M + 63) / 64, gy0 = (d.N + 63) / 64, gx1 = (w.M + 63) / 64, gy1 = (w.N + 63) / 64;
  q.gy[0] = gy0, q.gy[1] = gy1;
  q.gxy[0] = gx0 * gy0, q.gxy[1] = gx1 * gy1;
  q.nb0 = q.gxy[0] * d.splits;
  const unsigned blocks = (unsigned)(q.nb0 + q.gxy[1] * w.splits);
  if (dma == LIN_V32)
    hipLaunchKernelGGL((lin_pair_kernel<LIN_V32, LIN_V16, LIN_V32, LIN_V16>), dim3(blocks), dim3(256), 0, stream, q);
  else if (dma == LIN_G32)
    hipLaunchKernelGGL((lin_pair_kernel<LIN_G32, LIN_V16, LIN_G32, LIN_V16>), dim3(blocks), dim3(256), 0, stream, q);
  else if (wmb == LIN_V16)
    hipLaunchKernelGGL((lin_pair_kernel<LIN_V16, LIN_V16, LIN_V16, LIN_V16>), dim3(blocks), dim3(256), 0, stream, q);
  else
    hipLaunchKernelGGL((lin_pair_kernel<LIN_V16, LIN_V16, LIN_V16, LIN_V32>), dim3(blocks), dim3(256), 0, stream, q);
  return (int)hipGetLastError();
}

static LinArgs lin_args0() {
  LinArgs a;
  memset(&a, 0, sizeof(a));
  a.splits = 1;
  return a;
}

// acts[l] = act(acts[l-1] W_l^T + b_l) (acts[-1] = x), bf16; out32 (nullable): fp32 copy of the
// last layer's output.
int rx_lin_tower_fwd(const LinLayer* L, int nl, int M, const void* x, int x_f32, long long ldx, u16* const* acts,
                     float* out32, const LinScratch* sc, hipStream_t stream) {
  for (int l = 0; l < nl; ++l) {
    LinArgs a = lin_args0();
    a.M = M, a.N = L[l].N, a.K = L[l].K, a.epi = LIN_FWD;
    if (l == 0)
      a.a = LinOperand{x, ldx, x_f32, LIN_ROW};
    else
      a.a = LinOperand{acts[l - 1], L[l - 1].N, 0, LIN_ROW};
    a.b = LinOperand{L[l].W, L[l].K, 0, LIN_ROW};
    a.bias = L[l].bias;
    a.relu = L[l].relu;
    a.out = acts[l];
    a.ldo = L[l].N;
    if (l == nl - 1 && out32 != nullptr) {
      a.out2 = out32;
      a.ldo2 = L[l].N;
    }
    const int rc = lin_run(a, *sc, stream);
    if (rc) return rc;
  }
  return 0;
}

// Backward of rx_lin_tower_fwd from gout (fp32 [M][N_last]): weight / bias gradients of every
// layer with a dW, and dx (nullable; fp32 when x_f32 else bf16). g0 / g1: bf16 ping-pong buffers
// of M * max(N_l) elements.
int rx_lin_tower_bwd(const LinLayer* L, int nl, int M, const void* x, int x_f32, long long ldx, u16* const* acts,
                     const float* gout, long long ldg, int gout_masked, void* dx, u16* g0, u16* g1,
                     const LinScratch* sc, hipStream_t stream) {
  // the top layer's gradient: without a ReLU (or with the ReLU mask already applied by the
  // producer of gout: gout_masked) it is gout itself (fp32, converted to bf16 while the GEMMs
  // stage it); otherwise one mask+cast launch
  const void* G = gout;
  int g_f32 = 1;
  int rc = 0;
  if (L[nl - 1].relu && !gout_masked) {
    if ((rc = lin_mask_cast2(gout, ldg, acts[nl - 1], g0, M, L[nl - 1].N, stream))) return rc;
    G = g0;
    g_f32 = 0;
  }
  for (int l = nl - 1; l >= 0; --l) {
    const int N = L[l].N, K = L[l].K;
    const LinOperand Xl = l == 0 ? LinOperand{x, ldx, x_f32, LIN_RED} : LinOperand{acts[l - 1], K, 0, LIN_RED};
    LinArgs w = lin_args0();
    const bool has_w = L[l].dW != nullptr;
    if (has_w) {
      w.M = N, w.N = K, w.K = M, w.epi = LIN_WGRAD;
      w.a = LinOperand{G, g_f32 ? ldg : N, g_f32, LIN_RED};
      w.b = Xl;
      w.out = L[l].dW;
      w.ldo = K;
      w.dbias = L[l].db;
    }
    if (l > 0 || dx != nullptr) {
      LinArgs a = lin_args0();
      a.M = M, a.N = K, a.K = N, a.epi = LIN_DGRAD;
      a.a = LinOperand{G, g_f32 ? ldg : N, g_f32, LIN_ROW};
      a.b = LinOperand{L[l].W, K, 0, LIN_RED};
      u16* nextG = G == g0 ? g1 : g0;
      if (l > 0) {
        if (L[l - 1].relu) {
          a.mask = acts[l - 1];
          a.ldm = K;
        }
        a.out = nextG;
      } else {
        a.out = dx;
        a.out_f32 = x_f32;
      }
      a.ldo = K;
      rc = has_w ? lin_run_pair(a, w, *sc, stream) : lin_run(a, *sc, stream);
      if (rc) return rc;
      G = nextG;
      g_f32 = 0;
    } else if (has_w) {
      if ((rc = lin_run(w, *sc, stream))) return rc;
    }
  }
  return 0;
}

int rx_lin_layer_size() { return (int)sizeof(LinLayer); }
int rx_lin_scratch_size() { return (int)sizeof(LinScratch); }

int rx_lin_mask_cast(const float* g, const u16* y, u16* out, long long n, hipStream_t stream) {
  if (n <= 0) return 0;
  const long long blocks = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL(lin_mask_cast_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, y, out, n, 1, 1LL);
  return (int)hipGetLastError();
}

static int lin_mask_cast2(const float* g, long long ldg, const u16* y, u16* out, int rows, int cols,
                          hipStream_t stream) {
  const long long n = (long long)rows * cols;
  if (n <= 0) return 0;
  const long long blocks = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL(lin_mask_cast_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, y, out, n, cols, ldg);
  return (int)hipGetLastError();
}


int rx_lin_refresh(const LinRefresh* r, hipStream_t stream) {
  if (r->n <= 0) return 0;
  if (r->n > 16) return -1;
  long long mx = 0;
  for (int t = 0; t < r->n; ++t) mx = r->len[t] > mx ? r->len[t] : mx;
  long long bx = (mx / 2 + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
  hipLaunchKernelGGL(lin_refresh_kernel, dim3((unsigned)bx, (unsigned)r->n), dim3(256), 0, stream, *r);
  return (int)hipGetLastError();
}

}  // extern "C"
