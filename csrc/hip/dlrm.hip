// DLRM hot ops for CDNA4 (gfx950): multi-table embedding gather, fused sparse-SGD embedding
// update, and the dot-product feature interaction (forward + backward) on MFMA.
//
// Reference model: examples/pytorch_dlrm.ipynb (cells 9, 14) -- MultiTableEmbeddings of 26
// nn.Embedding(sparse=True) tables, DotInteraction = bmm(X, X^T) + strict-lower-triangle
// gather + concat(bottom_mlp_out, tril, zero pad). Here all tables live in ONE row-major fp32
// buffer [sum(rows), D] addressed through per-table row offsets, and the interaction input
// X[b] = [bottom_mlp_out; emb_0; ...; emb_{T-1}] (F = T + 1 rows of D) is produced directly by
// the gather kernel, so the concat never materialises separately.
//
// Interaction: per sample, Z = X X^T (F x F, F <= 32 padded to 32) on
// v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulate) -- only the three 16x16 blocks
// that touch the strict lower triangle are computed. Output row:
//   [ X[0, 0:D] | Z[i][j] for i > j in row-major (i, j) order | 0 ]   (D + F(F-1)/2 + 1)
// Backward: dX = S X with S symmetric (S[i][j] = S[j][i] = dZ_ij, zero diagonal), plus the
// pass-through gradient of the first D outputs into dX[0].
#include "rx_common.h"

namespace {

constexpr int kMaxF = 32;  // interaction rows (1 + tables), padded

// ---------------------------------------------------------------- embeddings --------------
// X[b][1 + t][:] = W[offsets[t] + idx[b][t]][:]   (one 16-B chunk of D per thread)
// and, with `head`, X[b][0][:] = head[b][:] (the bottom-MLP output: the interaction input is
// written whole by this one launch, no separate concat copy)
__global__ __launch_bounds__(256) void emb_gather_kernel(const float* __restrict__ W, const long long* __restrict__ offs,
                                                         const long long* __restrict__ idx, float* __restrict__ X,
                                                         const float* __restrict__ head, int B, int T, int D, int F,
                                                         long long total_rows, int col0) {
  const int chunks = D >> 2;
  const long long n = (long long)B * T * chunks;
  const long long nh = head != nullptr ? (long long)B * chunks : 0;
  for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n + nh; g += (long long)gridDim.x * blockDim.x) {
    if (g >= n) {
      const long long h = g - n;
      const int c = (int)(h % chunks);
      const long long b = h / chunks;
      *reinterpret_cast<f32x4*>(X + (b * F) * D + 4 * c) = *reinterpret_cast<const f32x4*>(head + b * D + 4 * c);
      continue;
    }
    const int c = (int)(g % chunks);
    const long long bt = g / chunks;
    const int t = (int)(bt % T);
    const long long b = bt / T;
    long long row = offs[t] + idx[b * T + t];
    row = row < 0 ? 0 : (row >= total_rows ? total_rows - 1 : row);  // never read out of bounds
    const f32x4 v = *reinterpret_cast<const f32x4*>(W + row * D + 4 * c);
    *reinterpret_cast<f32x4*>(X + (b * F + col0 + t) * D + 4 * c) = v;
  }
}

// W[row] -= lr * dX[b][1 + t]   (duplicates accumulate through fp32 atomics)
__global__ __launch_bounds__(256) void emb_sgd_kernel(float* __restrict__ W, const long long* __restrict__ offs,
                                                      const long long* __restrict__ idx, const float* __restrict__ dX,
                                                      int B, int T, int D, int F, float lr, long long total_rows,
                                                      int col0) {
  const long long n = (long long)B * T * D;
  for (long long g = blockIdx.x * (long long)blockDim.x + threadIdx.x; g < n; g += (long long)gridDim.x * blockDim.x) {
    const int d = (int)(g % D);
    const long long bt = g / D;
    const int t = (int)(bt % T);
    const long long b = bt / T;
    long long row = offs[t] + idx[b * T + t];
    if (row < 0 || row >= total_rows) continue;
    atomicAdd(W + row * D + d, -lr * dX[(b * F + col0 + t) * D + d]);
  }
}

// ---------------------------------------------------------------- interaction -------------
// LDS image of one sample: Xs[row][k] bf16, row stride D + 8 (16-B pad: conflict-free b128).
template <int D>
__device__ __forceinline__ void load_sample(const float* __restrict__ x, u16* Xs, int F, int lane) {
  constexpr int RS = D + 8;
  for (int e = lane; e < kMaxF * D; e += 64) {
    const int r = e / D, k = e % D;
    Xs[r * RS + k] = r < F ? rx_f2bf(x[r * D + k]) : (u16)0;
  }
}

// one wave per sample, 4 samples per workgroup
template <int D>
__global__ __launch_bounds__(256) void dot_fwd_kernel(const float* __restrict__ X, float* __restrict__ out, int B, int F) {
  constexpr int RS = D + 8;
  __shared__ __attribute__((aligned(16))) u16 lds[4][kMaxF * RS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wave;
  const bool valid = b < B;  // no early exit: every wave reaches the barrier
  const float* x = X + (long long)(valid ? b : 0) * F * D;
  u16* Xs = lds[wave];
  if (valid) load_sample<D>(x, Xs, F, lane);
  __syncthreads();
  if (!valid) return;
  const int lr = lane & 15, lg = lane >> 4;
  // blocks (I, J) in {(0,0), (1,0), (1,1)} of Z = Xs Xs^T
  f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int k0 = 0; k0 < D; k0 += 32) {
    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Xs + lr * RS + k0 + 8 * lg);
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Xs + (16 + lr) * RS + k0 + 8 * lg);
    // B operand = Xs^T: lane (col n, k-group) holds Xs[n][k0 + 8lg ..] -- the same fragments
    acc[0] = rx_mfma16(a0, a0, acc[0]);
    acc[1] = rx_mfma16(a1, a0, acc[1]);
    acc[2] = rx_mfma16(a1, a1, acc[2]);
  }
  float* o = out + (long long)b * (D + F * (F - 1) / 2 + 1);
  // pass-through of the bottom-MLP row (fp32, exact)
  for (int k = lane; k < D; k += 64) o[k] = x[k];
  // C layout: col = lane & 15, row = 4 * (lane >> 4) + r
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const int I = blk == 0 ? 0 : 1, J = blk == 2 ? 1 : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = I * 16 + 4 * lg + r, j = J * 16 + lr;
      if (i < F && j < i) o[D + i * (i - 1) / 2 + j] = acc[blk][r];
    }
  }
  if (lane == 0) o[D + F * (F - 1) / 2] = 0.f;
}

// dX = S X (+ pass-through into row 0); S[i][j] = S[j][i] = dO[D + tri(i, j)], diag 0
template <int D>
__global__ __launch_bounds__(256) void dot_bwd_kernel(const float* __restrict__ X, const float* __restrict__ dO,
                                                      float* __restrict__ dX, int B, int F) {
  constexpr int XS = kMaxF + 8;  // XT[d][k] row stride (k = interaction row)
  __shared__ __attribute__((aligned(16))) u16 xt[4][D * XS];
  __shared__ __attribute__((aligned(16))) u16 ss[4][kMaxF * XS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wave;
  const bool valid = b < B;
  const float* x = X + (long long)(valid ? b : 0) * F * D;
  const float* g = dO + (long long)(valid ? b : 0) * (D + F * (F - 1) / 2 + 1);
  u16* XT = xt[wave];
  u16* S = ss[wave];
  for (int e = lane; valid && e < kMaxF * D; e += 64) {
    const int r = e / D, k = e % D;
    XT[k * XS + r] = r < F ? rx_f2bf(x[r * D + k]) : (u16)0;
  }
  for (int e = lane; valid && e < kMaxF * kMaxF; e += 64) {
    const int i = e / kMaxF, j = e % kMaxF;
    float v = 0.f;
    if (i < F && j < F && i != j) {
      const int hi = i > j ? i : j, lo = i > j ? j : i;
      v = g[D + hi * (hi - 1) / 2 + lo];
    }
    S[i * XS + j] = rx_f2bf(v);
  }
  __syncthreads();
  if (!valid) return;
  const int lr = lane & 15, lg = lane >> 4;
  // C[i][d] = sum_k S[i][k] XT[d][k]: A = S rows (K = 32 = padded F), B[k][n=d] = XT[d][k]
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(S + (mi * 16 + lr) * XS + 8 * lg);
#pragma unroll
    for (int nd = 0; nd < D / 16; ++nd) {
      const bf16x8 bb = *reinterpret_cast<const bf16x8*>(XT + (nd * 16 + lr) * XS + 8 * lg);
      f32x4 c = rx_mfma16(a, bb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = mi * 16 + 4 * lg + r, d = nd * 16 + lr;
        if (i < F) dX[((long long)b * F + i) * D + d] = c[r] + (i == 0 ? g[d] : 0.f);
      }
    }
  }
}

// ---------------------------------------------------------------- gather + interaction -----
// The replicated-table forward in ONE launch: each wave gathers its sample's interaction input
// straight from the tables (row 0 = the bottom-MLP output `head`, row 1 + t = W[offs[t] +
// idx[b][t]]), 16-B chunks), writes it to X (fp32: the backward's operand) and keeps its bf16
// image in LDS for the MFMA interaction -- the emb_gather launch and the interaction kernel's
// re-read of X are gone.
template <int D>
__global__ __launch_bounds__(256) void emb_dot_fwd_kernel(const float* __restrict__ W, const long long* __restrict__ offs,
                                                          const long long* __restrict__ idx,
                                                          const float* __restrict__ head, float* __restrict__ X,
                                                          float* __restrict__ out, int B, int F,
                                                          long long total_rows) {
  constexpr int RS = D + 8, CH = D / 4;
  __shared__ __attribute__((aligned(16))) u16 lds[4][kMaxF * RS];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = blockIdx.x * 4 + wave;
  const bool valid = b < B;
  const int T = F - 1;
  u16* Xs = lds[wave];
  if (valid) {
    float* x = X + (long long)b * F * D;
    for (int e = lane; e < kMaxF * CH; e += 64) {
      const int r = e / CH, c = e % CH;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      if (r == 0) {
        v = *reinterpret_cast<const f32x4*>(head + (long long)b * D + 4 * c);
      } else if (r < F) {
        long long row = offs[r - 1] + idx[(long long)b * T + r - 1];
        row = row < 0 ? 0 : (row >= total_rows ? total_rows - 1 : row);  // never read out of bounds
        v = *reinterpret_cast<const f32x4*>(W + row * D + 4 * c);
      }
      if (r < F) *reinterpret_cast<f32x4*>(x + r * D + 4 * c) = v;
      uint2 pk;
      pk.x = rx_f2bf2(v[0], v[1]);
      pk.y = rx_f2bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(Xs + r * RS + 4 * c) = pk;
    }
  }
  __syncthreads();
  if (!valid) return;
  const int lr = lane & 15, lg = lane >> 4;
  f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int k0 = 0; k0 < D; k0 += 32) {
    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(Xs + lr * RS + k0 + 8 * lg);
    const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(Xs + (16 + lr) * RS + k0 + 8 * lg);
    acc[0] = rx_mfma16(a0, a0, acc[0]);
    acc[1] = rx_mfma16(a1, a0, acc[1]);
    acc[2] = rx_mfma16(a1, a1, acc[2]);
  }
  float* o = out + (long long)b * (D + F * (F - 1) / 2 + 1);
  for (int k = lane; k < D; k += 64) o[k] = head[(long long)b * D + k];
#pragma unroll
  for (int blk = 0; blk < 3; ++blk) {
    const int I = blk == 0 ? 0 : 1, J = blk == 2 ? 1 : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = I * 16 + 4 * lg + r, j = J * 16 + lr;
      if (i < F && j < i) o[D + i * (i - 1) / 2 + j] = acc[blk][r];
    }
  }
  if (lane == 0) o[D + F * (F - 1) / 2] = 0.f;
}

// Interaction backward with the embedding SGD applied in its epilogue: dX = S X as in
// dot_bwd_kernel, but only row 0 (the bottom-MLP gradient) is stored, to dmlp [B][D]; the
// embedding rows' gradients go straight into the tables, W[row] -= lr * dX[b][1 + t] (fp32
// atomics, as emb_sgd_kernel) -- no dX buffer, no second launch. relu_mask: row 0 of X is the
// output of a ReLU (the bottom MLP's last layer), so dmlp is stored already multiplied by
// relu'(.) = (X[b][0] > 0): the bottom tower's backward then skips its mask kernel.
// One workgroup per sample (4 waves): the operand staging is spread over 256 threads (16-B
// loads of X) and each wave owns MFMA tiles of dX, so the per-sample dependent chain (load ->
// LDS -> MFMA -> atomics) is a quarter as long as with one wave per sample; at the notebook's
// batch 128 that one-wave chain, not bandwidth, was the kernel's time.
template <int D>
__global__ __launch_bounds__(256) void dot_bwd_sgd_kernel(const float* __restrict__ X, const float* __restrict__ dO,
                                                          float* __restrict__ dmlp, float* __restrict__ W,
                                                          const long long* __restrict__ offs,
                                                          const long long* __restrict__ idx, int B, int F, float lr,
                                                          long long total_rows, int relu_mask) {
  constexpr int XS = kMaxF + 8, CH = D / 4;
  __shared__ __attribute__((aligned(16))) u16 XT[D * XS];
  __shared__ __attribute__((aligned(16))) u16 S[kMaxF * XS];
  __shared__ long long rows_s[kMaxF];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int T = F - 1;
  const float* x = X + (long long)b * F * D;
  const float* g = dO + (long long)b * (D + F * (F - 1) / 2 + 1);
  for (int e = tid; e < kMaxF * CH; e += 256) {
    const int r = e / CH, c = (e % CH) * 4;
    const f32x4 v = r < F ? *reinterpret_cast<const f32x4*>(x + r * D + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) XT[(c + q) * XS + r] = rx_f2bf(v[q]);
  }
  for (int e = tid; e < kMaxF * kMaxF; e += 256) {
    const int i = e / kMaxF, j = e % kMaxF;
    float v = 0.f;
    if (i < F && j < F && i != j) {
      const int hi = i > j ? i : j, lo = i > j ? j : i;
      v = g[D + hi * (hi - 1) / 2 + lo];
    }
    S[i * XS + j] = rx_f2bf(v);
  }
  if (tid < kMaxF) {
    long long row = -1;
    if (tid >= 1 && tid < F) {
      row = offs[tid - 1] + idx[(long long)b * T + tid - 1];
      if (row < 0 || row >= total_rows) row = -1;
    }
    rows_s[tid] = row;
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63, lr_ = lane & 15, lg = lane >> 4;
  constexpr int NT = 2 * (D / 16);  // (row tile mi) x (column tile nd) of dX [32 x D]
  for (int t = wave; t < NT; t += 4) {
    const int mi = t / (D / 16), nd = t % (D / 16);
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(S + (mi * 16 + lr_) * XS + 8 * lg);
    const bf16x8 bb = *reinterpret_cast<const bf16x8*>(XT + (nd * 16 + lr_) * XS + 8 * lg);
    const f32x4 c = rx_mfma16(a, bb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = mi * 16 + 4 * lg + r, d = nd * 16 + lr_;
      if (i == 0) {
        dmlp[(long long)b * D + d] = (relu_mask && !(x[d] > 0.f)) ? 0.f : c[r] + g[d];
      } else if (i < F) {
        const long long row = rows_s[i];
        if (row >= 0) atomicAdd(W + row * D + d, -lr * c[r]);
      }
    }
  }
}

template <int D>
int launch_fwd(const float* X, float* out, int B, int F, hipStream_t s) {
  hipLaunchKernelGGL(dot_fwd_kernel<D>, dim3((B + 3) / 4), dim3(256), 0, s, X, out, B, F);
  return (int)hipGetLastError();
}

template <int D>
int launch_bwd(const float* X, const float* dO, float* dX, int B, int F, hipStream_t s) {
  hipLaunchKernelGGL(dot_bwd_kernel<D>, dim3((B + 3) / 4), dim3(256), 0, s, X, dO, dX, B, F);
  return (int)hipGetLastError();
}

int grid_for(long long n) {
  long long g = (n + 255) / 256;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

// head (nullable, [B, D] fp32, 16-B aligned rows): copied into X[b][0] by the same launch.
int rx_emb_gather(const float* W, const long long* offs, const long long* idx, float* X, const float* head, int B,
                  int T, int D, int F, long long total_rows, hipStream_t s) {
  if (D % 4 != 0 || F < T + 1) return -1;
  const long long units = (long long)B * (T + (head != nullptr ? 1 : 0)) * (D / 4);
  hipLaunchKernelGGL(emb_gather_kernel, dim3(grid_for(units)), dim3(256), 0, s, W, offs, idx, X, head, B, T, D, F,
                     total_rows, 1);
  return (int)hipGetLastError();
}

// Packed variant for the owner side of table-wise sharding: Y[b][t] = W[offs[t] + idx[b][t]]
// ([B, T, D], no interaction slot) -- the rows an owner returns over all-to-all.
int rx_emb_gather_rows(const float* W, const long long* offs, const long long* idx, float* Y, int B, int T, int D,
                       long long total_rows, hipStream_t s) {
  if (D % 4 != 0) return -1;
  hipLaunchKernelGGL(emb_gather_kernel, dim3(grid_for((long long)B * T * (D / 4))), dim3(256), 0, s, W, offs, idx, Y,
                     (const float*)nullptr, B, T, D, T, total_rows, 0);
  return (int)hipGetLastError();
}

// W[offs[t] + idx[b][t]] -= lr * G[b][t]: the sparse SGD of the owner's local tables, applied
// straight from the gradient rows that came back over all-to-all.
int rx_emb_sgd_rows(float* W, const long long* offs, const long long* idx, const float* G, int B, int T, int D,
                    float lr, long long total_rows, hipStream_t s) {
  hipLaunchKernelGGL(emb_sgd_kernel, dim3(grid_for((long long)B * T * D)), dim3(256), 0, s, W, offs, idx, G, B, T, D, T,
                     lr, total_rows, 0);
  return (int)hipGetLastError();
}

int rx_emb_sgd(float* W, const long long* offs, const long long* idx, const float* dX, int B, int T, int D, int F,
               float lr, long long total_rows, hipStream_t s) {
  hipLaunchKernelGGL(emb_sgd_kernel, dim3(grid_for((long long)B * T * D)), dim3(256), 0, s, W, offs, idx, dX, B, T, D, F,
                     lr, total_rows, 1);
  return (int)hipGetLastError();
}

int rx_dot_interaction_fwd(const float* X, float* out, int B, int F, int D, hipStream_t s) {
  if (F > kMaxF || F < 2) return -1;
  switch (D) {
    case 32: return launch_fwd<32>(X, out, B, F, s);
    case 64: return launch_fwd<64>(X, out, B, F, s);
    case 128: return launch_fwd<128>(X, out, B, F, s);
    default: return -1;
  }
}

// Gather + interaction in one launch (replicated tables): X [B][F][D] written for the backward,
// out = the interaction output. head: [B][D] fp32, 16-B aligned rows.
int rx_emb_dot_fwd(const float* W, const long long* offs, const long long* idx, const float* head, float* X,
                   float* out, int B, int F, int D, long long total_rows, hipStream_t s) {
  if (F > kMaxF || F < 2) return -1;
  const dim3 grid((B + 3) / 4);
  switch (D) {
    case 32: hipLaunchKernelGGL(emb_dot_fwd_kernel<32>, grid, dim3(256), 0, s, W, offs, idx, head, X, out, B, F, total_rows); break;
    case 64: hipLaunchKernelGGL(emb_dot_fwd_kernel<64>, grid, dim3(256), 0, s, W, offs, idx, head, X, out, B, F, total_rows); break;
    case 128: hipLaunchKernelGGL(emb_dot_fwd_kernel<128>, grid, dim3(256), 0, s, W, offs, idx, head, X, out, B, F, total_rows); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

// Interaction backward + fused embedding SGD: dmlp [B][D] = the bottom-MLP gradient; the table
// rows are updated in place.
int rx_dot_bwd_sgd(const float* X, const float* dO, float* dmlp, float* W, const long long* offs, const long long* idx,
                   int B, int F, int D, float lr, long long total_rows, int relu_mask, hipStream_t s) {
  if (F > kMaxF || F < 2) return -1;
  if (B <= 0) return 0;
  const dim3 grid(B);
  switch (D) {
    case 32: hipLaunchKernelGGL(dot_bwd_sgd_kernel<32>, grid, dim3(256), 0, s, X, dO, dmlp, W, offs, idx, B, F, lr, total_rows, relu_mask); break;
    case 64: hipLaunchKernelGGL(dot_bwd_sgd_kernel<64>, grid, dim3(256), 0, s, X, dO, dmlp, W, offs, idx, B, F, lr, total_rows, relu_mask); break;
    case 128: hipLaunchKernelGGL(dot_bwd_sgd_kernel<128>, grid, dim3(256), 0, s, X, dO, dmlp, W, offs, idx, B, F, lr, total_rows, relu_mask); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

int rx_dot_interaction_bwd(const float* X, const float* dO, float* dX, int B, int F, int D, hipStream_t s) {
  if (F > kMaxF || F < 2) return -1;
  switch (D) {
    case 32: return launch_bwd<32>(X, dO, dX, B, F, s);
    case 64: return launch_bwd<64>(X, dO, dX, B, F, s);
    case 128: return launch_bwd<128>(X, dO, dX, B, F, s);
    default: return -1;
  }
}

}  // extern "C"
