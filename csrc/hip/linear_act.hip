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
// Tiling: 64x64 output tile per 256-thread workgroup (4 waves as 2x2, 32x32 per wave = 2x2
// MFMA tiles), 64-deep K stages double-buffered in LDS. Each operand tile is staged in its
// memory orientation with 16-B row chunks; operands whose reduction index is the slow one in
// memory are read with gfx950's transposing LDS read (ds_read_b64_tr_b16), so no layout needs a
// transposed copy in HBM. Edges (any M, N, K, any leading dimension) are zero-filled on load
// and masked on store.
#include "rx_common.h"

#include <string.h>

#define LIN_T 64    // output tile edge and K-stage depth
#define LIN_S 80    // LDS image row stride in elements (160 B = 10 16-B units: ds_read_b128 fragment reads
                    // conflict-free for gfx950's lane groups {0-3,12-15,20-27}, ... ; 144 B was 2-way)

enum { LIN_ROW = 0, LIN_RED = 1 };
enum { LIN_FWD = 0, LIN_DGRAD = 1, LIN_WGRAD = 2 };

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
  float* ws;     // [tiles][splits][64*64 + 64] fp32 partial tiles (+ partial row sums)
  unsigned* counters;  // [tiles], zero between calls (the last block of a tile resets it)
};

typedef short rx_v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) rx_v4s rx_lds_v4s;

// Load the 8 consecutive elements (i, j .. j+7) of an operand as bf16 (zero outside [0, I) x [0, J)).
template <int F32>
__device__ __forceinline__ uint4 lin_load8(const LinOperand& o, long long i, long long j, long long I, long long J) {
  uint4 r = make_uint4(0, 0, 0, 0);
  if (i >= I || j >= J) return r;
  if constexpr (F32) {
    const float* p = reinterpret_cast<const float*>(o.p) + i * o.ld + j;
    float v[8];
    if (j + 8 <= J && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      const float4 x = *reinterpret_cast<const float4*>(p);
      const float4 y = *reinterpret_cast<const float4*>(p + 4);
      v[0] = x.x, v[1] = x.y, v[2] = x.z, v[3] = x.w, v[4] = y.x, v[5] = y.y, v[6] = y.z, v[7] = y.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = j + e < J ? p[e] : 0.f;
    }
    r.x = rx_f2bf2(v[0], v[1]);
    r.y = rx_f2bf2(v[2], v[3]);
    r.z = rx_f2bf2(v[4], v[5]);
    r.w = rx_f2bf2(v[6], v[7]);
  } else {
    const u16* p = reinterpret_cast<const u16*>(o.p) + i * o.ld + j;
    if (j + 8 <= J && ((reinterpret_cast<uintptr_t>(p) & 15) == 0)) {
      r = *reinterpret_cast<const uint4*>(p);
    } else {
      u16 v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = j + e < J ? p[e] : (u16)0;
      r.x = v[0] | ((uint32_t)v[1] << 16);
      r.y = v[2] | ((uint32_t)v[3] << 16);
      r.z = v[4] | ((uint32_t)v[5] << 16);
      r.w = v[6] | ((uint32_t)v[7] << 16);
    }
  }
  return r;
}

// The two 16-B chunks a thread stages for one operand tile: tile rows r0.., reduction k0..
// (memory orientation: ROW -> (i, j) = (row, k); RED -> (i, j) = (k, row)).
template <int F32, int LAY>
__device__ __forceinline__ void lin_fetch(const LinOperand& o, long long r0, long long k0, long long R, long long Kd,
                                          int tid, uint4 (&v)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = tid + 256 * t;
    const int i = c >> 3, jc = (c & 7) * 8;
    if (LAY == LIN_ROW)
      v[t] = lin_load8<F32>(o, r0 + i, k0 + jc, R, Kd);
    else
      v[t] = lin_load8<F32>(o, k0 + i, r0 + jc, Kd, R);
  }
}

__device__ __forceinline__ void lin_stash(u16* img, int tid, const uint4 (&v)[2]) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int c = tid + 256 * t;
    const int i = c >> 3, jc = (c & 7) * 8;
    *reinterpret_cast<uint4*>(img + i * LIN_S + jc) = v[t];
  }
}

// MFMA operand fragment for tile rows rb..rb+15, reduction ks..ks+31 (lane l: row rb + (l & 15),
// k = ks + 8 (l >> 4) + e).
__device__ __forceinline__ bf16x8 lin_frag(const u16* img, int lay, int rb, int ks, int lane) {
  if (lay == LIN_ROW) {
    const uint4 x = *reinterpret_cast<const uint4*>(img + (rb + (lane & 15)) * LIN_S + ks + 8 * (lane >> 4));
    return __builtin_bit_cast(bf16x8, x);
  }
  // [k][row] image: each 16-lane group h reads rows k = ks + 8h + {0..3} and {4..7}; lane 4q+p
  // addresses row q, columns rb + 4p .. +3; lane i receives column rb + i
  const int h = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const u16* a0 = img + (ks + 8 * h + q) * LIN_S + rb + 4 * p;
  const u16* a1 = a0 + 4 * LIN_S;
  const rx_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (rx_lds_v4s*)((__attribute__((address_space(3))) char*)(uintptr_t)(a0)));
  const rx_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (rx_lds_v4s*)((__attribute__((address_space(3))) char*)(uintptr_t)(a1)));
  typedef short rx_v8s __attribute__((ext_vector_type(8)));
  const rx_v8s all = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, all);
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
template <int AF32, int BF32, int LA, int LB>
__global__ __launch_bounds__(256) void lin_gemm_kernel(LinArgs a) {
  __shared__ __attribute__((aligned(16))) u16 lds[2][2][LIN_T * LIN_S];  // [buffer][A|B]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const long long m0 = (long long)blockIdx.x * LIN_T, n0 = (long long)blockIdx.y * LIN_T;
  // split-K: this block reduces K stages [k_begin, k_end)
  const int nk_all = (a.K + LIN_T - 1) / LIN_T;
  const int per = (nk_all + a.splits - 1) / a.splits;
  const int k_begin = blockIdx.z * per;
  const int k_end = min(nk_all, k_begin + per);
  const int nk = max(0, k_end - k_begin);
  const bool want_db = a.epi == LIN_WGRAD && a.dbias != nullptr && blockIdx.y == 0 && wn == 0;

  f32x4 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float asum[2] = {0.f, 0.f};

  // Global -> register -> LDS pipeline two stages deep: while stage kt is multiplied out of LDS,
  // stage kt+1 sits in one register set (loaded an iteration ago, stashed after the MFMAs) and
  // stage kt+2's loads are in flight into the other set -- each load has two stages of MFMAs to
  // arrive in. The loop is unrolled by two so the sets swap roles without register copies
  // (a copy would wait for the loads it copies).
  uint4 ra[2], rb[2], qa[2], qb[2];
  auto fetch = [&](int kt, uint4 (&fa_)[2], uint4 (&fb_)[2]) {
    lin_fetch<AF32, LA>(a.a, m0, (long long)(k_begin + kt) * LIN_T, a.M, a.K, tid, fa_);
    lin_fetch<BF32, LB>(a.b, n0, (long long)(k_begin + kt) * LIN_T, a.N, a.K, tid, fb_);
  };
  auto stage = [&](int kt, uint4 (&sa)[2], uint4 (&sb)[2], uint4 (&la)[2], uint4 (&lb)[2]) {
    const int cur = kt & 1;
    if (kt + 2 < nk) fetch(kt + 2, la, lb);
    const u16* ia = lds[cur][0];
    const u16* ib = lds[cur][1];
#pragma unroll
    for (int ks = 0; ks < LIN_T; ks += 32) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) fa[x] = lin_frag(ia, LA, wm * 32 + 16 * x, ks, lane);
#pragma unroll
      for (int y = 0; y < 2; ++y) fb[y] = lin_frag(ib, LB, wn * 32 + 16 * y, ks, lane);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = rx_mfma16(fa[x], fb[y], acc[x][y]);
      if (want_db) {
#pragma unroll
        for (int x = 0; x < 2; ++x) asum[x] += lin_bsum(fa[x]);
      }
    }
    if (kt + 1 < nk) {
      lin_stash(lds[cur ^ 1][0], tid, sa);
      lin_stash(lds[cur ^ 1][1], tid, sb);
    }
    __syncthreads();
  };
  if (nk > 0) {
    fetch(0, ra, rb);
    lin_stash(lds[0][0], tid, ra);
    lin_stash(lds[0][1], tid, rb);
    if (nk > 1) fetch(1, ra, rb);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; kt += 2) {
    stage(kt, ra, rb, qa, qb);                  // stash stage kt+1 from r*, load kt+2 into q*
    if (kt + 1 < nk) stage(kt + 1, qa, qb, ra, rb);
  }

  if (a.splits > 1) {
    // deterministic split-K fix-up: every split parks its fp32 tile (and its partial bias-row
    // sums) in the workspace; the block that arrives last sums ALL splits in split order -- the
    // result does not depend on which block came last -- and runs the epilogue. Hand-off
    // (MI355X: per-XCD L2s): write-through sc1 payload stores drained by every storing wave, a
    // barrier, ONE agent-scope counter add; the last block reads the payload with sc1 loads only
    // (they bypass its L1), so no release / acquire fence is needed.
    const int tile = blockIdx.x * gridDim.y + blockIdx.y;
    const int TW = LIN_T * LIN_T + LIN_T;
    float* mine = a.ws + ((long long)tile * a.splits + blockIdx.z) * TW;
    const int slot = ((wave * 64 + lane) * 16) * 4;  // byte offset of this lane's 16 floats
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
        rx_store16_sc1(mine, slot + 16 * (2 * x + y), __builtin_bit_cast(u32x4, acc[x][y]));
    if (want_db) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const float sx = rx_colsum16(asum[x]);
        if (lane < 16)
          __hip_atomic_store(mine + LIN_T * LIN_T + wm * 32 + 16 * x + lane, sx, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    // the flag lives in the (now idle) operand images: a separate __shared__ word would push the
    // block past 40 KiB of LDS and cost a fourth resident workgroup per CU
    unsigned* last_flag = reinterpret_cast<unsigned*>(&lds[0][0][0]);
    if (tid == 0) {
      const unsigned done = __hip_atomic_fetch_add(a.counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last_flag = done + 1 == (unsigned)a.splits;
    }
    __syncthreads();
    if (!*last_flag) return;
    const float* base = a.ws + (long long)tile * a.splits * TW;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[x][y] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float dsum[2] = {0.f, 0.f};
    for (int sp = 0; sp < a.splits; ++sp) {
      const float* ps = base + (long long)sp * TW;
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
          acc[x][y] += __builtin_bit_cast(f32x4, rx_load16_sc1(ps, slot + 16 * (2 * x + y)));
      if (want_db && lane < 16) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
          dsum[x] += __hip_atomic_load(ps + LIN_T * LIN_T + wm * 32 + 16 * x + lane, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (tid == 0) __hip_atomic_store(a.counters + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (want_db) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const long long m = m0 + wm * 32 + 16 * x + (lane & 15);
        if (lane < 16 && m < a.M) a.dbias[m] = a.beta != 0.f ? a.beta * a.dbias[m] + dsum[x] : dsum[x];
      }
    }
  }

  // epilogue: lane holds rows rb + 4 (lane >> 4) + r (r = 0..3), column cb + (lane & 15)
#pragma unroll
  for (int x = 0; x < 2; ++x) {
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const long long n = n0 + wn * 32 + 16 * y + (lane & 15);
      if (n >= a.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long m = m0 + wm * 32 + 16 * x + 4 * (lane >> 4) + r;
        if (m >= a.M) continue;
        float v = acc[x][y][r];
        if (a.epi == LIN_FWD) {
          if (a.bias != nullptr) v += a.bias[n];
          if (a.relu) v = fmaxf(v, 0.f);
          if (a.out_f32)
            reinterpret_cast<float*>(a.out)[m * a.ldo + n] = v;
          else
            reinterpret_cast<u16*>(a.out)[m * a.ldo + n] = rx_f2bf(v);
          if (a.out2 != nullptr) a.out2[m * a.ldo2 + n] = v;
        } else if (a.epi == LIN_DGRAD) {
          if (a.mask != nullptr && !(rx_bf2f(a.mask[m * a.ldm + n]) > 0.f)) v = 0.f;
          if (a.out_f32)
            reinterpret_cast<float*>(a.out)[m * a.ldo + n] = v;
          else
            reinterpret_cast<u16*>(a.out)[m * a.ldo + n] = rx_f2bf(v);
        } else {
          float* o = reinterpret_cast<float*>(a.out) + m * a.ldo + n;
          *o = a.beta != 0.f ? a.beta * *o + v : v;
        }
      }
    }
  }
  if (want_db && a.splits <= 1) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const float s = rx_colsum16(asum[x]);  // the 4 lanes of row (lane & 15) hold k-quarters
      const long long m = m0 + wm * 32 + 16 * x + (lane & 15);
      if (lane < 16 && m < a.M) a.dbias[m] = a.beta != 0.f ? a.beta * a.dbias[m] + s : s;
    }
  }
}

// G = gY * (Y > 0) (relu) or G = gY, fp32 -> bf16 (the tower's top-layer output gradient).
__global__ __launch_bounds__(256) void lin_mask_cast_kernel(const float* __restrict__ g, const u16* __restrict__ y,
                                                            u16* __restrict__ out, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float v = g[i];
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

// Split-K factor for a problem: about two workgroups per CU, each split at least four 64-deep
// stages. Measured per DLRM tower GEMM (profiles/r2_linear_gemm_kernel_times.txt): the
// split-K fix-up costs more than it hides once a problem has ~one tile per CU (the wide
// forward / dgrad GEMMs run fastest unsplit), while the weight-gradient GEMMs (few output tiles,
// K = batch) gain 2-3x from 2-8 splits.
int rx_lin_splits(int M, int N, int K, int cus) {
  const long long tiles = (long long)((M + LIN_T - 1) / LIN_T) * ((N + LIN_T - 1) / LIN_T);
  const int nk = (K + LIN_T - 1) / LIN_T;
  long long want = (2LL * cus + tiles - 1) / tiles;
  long long mx = nk / 4;
  if (want > mx) want = mx;
  if (want > 64) want = 64;
  return want < 1 ? 1 : (int)want;
}

int rx_lin_ws_floats(int M, int N, int splits) {
  const long long tiles = (long long)((M + LIN_T - 1) / LIN_T) * ((N + LIN_T - 1) / LIN_T);
  return splits > 1 ? (int)(tiles * splits * (LIN_T * LIN_T + LIN_T)) : 0;
}

int rx_lin_gemm(const LinArgs* a, hipStream_t stream) {
  if (a->M <= 0 || a->N <= 0) return 0;
  if (a->K < 0 || a->epi < 0 || a->epi > 2 || a->splits < 1) return -1;
  if (a->splits > 1 && (a->ws == nullptr || a->counters == nullptr)) return -1;
  const dim3 grid((unsigned)((a->M + LIN_T - 1) / LIN_T), (unsigned)((a->N + LIN_T - 1) / LIN_T),
                  (unsigned)a->splits);
#define RX_LIN_LAY(AF, BF)                                                                          \
  if (a->a.lay == LIN_ROW && a->b.lay == LIN_ROW)                                                  \
    hipLaunchKernelGGL((lin_gemm_kernel<AF, BF, LIN_ROW, LIN_ROW>), grid, dim3(256), 0, stream, *a); \
  else if (a->a.lay == LIN_ROW)                                                                    \
    hipLaunchKernelGGL((lin_gemm_kernel<AF, BF, LIN_ROW, LIN_RED>), grid, dim3(256), 0, stream, *a); \
  else if (a->b.lay == LIN_ROW)                                                                    \
    hipLaunchKernelGGL((lin_gemm_kernel<AF, BF, LIN_RED, LIN_ROW>), grid, dim3(256), 0, stream, *a); \
  else                                                                                             \
    hipLaunchKernelGGL((lin_gemm_kernel<AF, BF, LIN_RED, LIN_RED>), grid, dim3(256), 0, stream, *a);
  if (a->a.f32 && a->b.f32) {
    RX_LIN_LAY(1, 1)
  } else if (a->a.f32) {
    RX_LIN_LAY(1, 0)
  } else if (a->b.f32) {
    RX_LIN_LAY(0, 1)
  } else {
    RX_LIN_LAY(0, 0)
  }
#undef RX_LIN_LAY
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
};

int rx_lin_mask_cast(const float* g, const u16* y, u16* out, long long n, hipStream_t stream);

static int lin_run(LinArgs& a, const LinScratch& sc, hipStream_t stream) {
  a.splits = rx_lin_splits(a.M, a.N, a.K, sc.cus);
  const long long tiles = (long long)((a.M + LIN_T - 1) / LIN_T) * ((a.N + LIN_T - 1) / LIN_T);
  if (a.splits > 1 && ((long long)rx_lin_ws_floats(a.M, a.N, a.splits) > sc.ws_floats || tiles > sc.counters_len))
    a.splits = 1;  // scratch too small for this shape: run unsplit
  a.ws = a.splits > 1 ? sc.ws : nullptr;
  a.counters = a.splits > 1 ? sc.counters : nullptr;
  return rx_lin_gemm(&a, stream);
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
                     const float* gout, void* dx, u16* g0, u16* g1, const LinScratch* sc, hipStream_t stream) {
  u16* G = g0;
  int rc = rx_lin_mask_cast(gout, L[nl - 1].relu ? acts[nl - 1] : nullptr, G, (long long)M * L[nl - 1].N, stream);
  if (rc) return rc;
  for (int l = nl - 1; l >= 0; --l) {
    const int N = L[l].N, K = L[l].K;
    const LinOperand Xl = l == 0 ? LinOperand{x, ldx, x_f32, LIN_RED} : LinOperand{acts[l - 1], K, 0, LIN_RED};
    if (L[l].dW != nullptr) {
      LinArgs a = lin_args0();
      a.M = N, a.N = K, a.K = M, a.epi = LIN_WGRAD;
      a.a = LinOperand{G, N, 0, LIN_RED};
      a.b = Xl;
      a.out = L[l].dW;
      a.ldo = K;
      a.dbias = L[l].db;
      if ((rc = lin_run(a, *sc, stream))) return rc;
    }
    if (l > 0 || dx != nullptr) {
      LinArgs a = lin_args0();
      a.M = M, a.N = K, a.K = N, a.epi = LIN_DGRAD;
      a.a = LinOperand{G, N, 0, LIN_ROW};
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
      if ((rc = lin_run(a, *sc, stream))) return rc;
      G = nextG;
    }
  }
  return 0;
}

int rx_lin_layer_size() { return (int)sizeof(LinLayer); }
int rx_lin_scratch_size() { return (int)sizeof(LinScratch); }

int rx_lin_mask_cast(const float* g, const u16* y, u16* out, long long n, hipStream_t stream) {
  if (n <= 0) return 0;
  const long long blocks = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL(lin_mask_cast_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, y, out, n);
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
