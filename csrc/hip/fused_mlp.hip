// Fused MLP training step for CDNA4 (gfx950): forward + loss + backward of a
// [Linear -> act -> BatchNorm1d]* -> Linear network in ONE workgroup, bf16 MFMA
// (v_mfma_f32_16x16x32_bf16) with fp32 accumulation, followed by a wide fused
// Adam/AdamW/SGD kernel that also refreshes the bf16 weight images.
//
// Why one workgroup: the reference workloads (NYC_Model in examples/pytorch_nyctaxi.py:69-92,
// batch 64; the stroke tutorial MLPs; DLRM's MLP towers) are ~6 MFLOP per step, so the step is
// latency bound. A chain of ~60 PyTorch launches costs far more than the math; here the whole
// dependency chain (10 GEMMs, 4 BatchNorm reductions, loss) runs in one CU with every
// activation resident in LDS, and column reductions stay inside a wave (each wave owns whole
// 16-column output tiles, so BN statistics are wave-local shuffles).
//
// Layouts (all bf16 LDS matrices have a +16 B row pad: ds_read_b128 of 16 rows at the same
// column then hits 16 distinct 16-B slots of the 256-B bank row -> conflict free):
//   R  [Bpad][max_k]    row-major activations (fwd A operand) / gradients (dgrad A operand)
//   GT [max_n][Bpad]    transposed gradient (wgrad A operand)
//   XT_l [in_n][Bpad]   transposed layer inputs saved for wgrad (wgrad B operand)
// Weights come from global memory as two bf16 images written by the optimizer kernel:
//   W  [out_n][in_k]  (fwd B operand, K = in contiguous)
//   Wt [in_n][out_k]  (dgrad B operand, K = out contiguous)
#include "rx_common.h"

#define RX_MAXL 8
#define RX_NW 8          // waves per workgroup
#define RX_THREADS (RX_NW * RX_WAVE)

struct MlpLayer {
  int in, out;
  int in_k, out_k;   // K padding (multiple of 32)
  int in_n, out_n;   // N padding (multiple of 16)
  const u16* W;
  const u16* Wt;
  int w_off, b_off;  // offsets into the flat fp32 parameter / gradient vectors
  int act;           // 0 identity, 1 relu
  int bn;            // 0 none, 1 act->bn, 2 bn->act
  int g_off, be_off; // BN affine params (-1: not affine)
  float* run_mean;
  float* run_var;
  float eps, momentum;
  int xt_off;        // LDS byte offset of XT_l
  int stat_off;      // float offset of (mean, invstd) pairs for this layer's outputs in LDS
  int r_off;         // float offset of the saved pre-BN values in the scratch buffer
  int pr_off;        // float offset of [bias|gamma|beta|run_mean|run_var] (x out_n) in LDS
};

struct MlpDesc {
  int L;
  int r_lds_off, gt_lds_off, stats_lds_off, lds_bytes;
  int max_k, max_n;
  int loss;          // 0 mse, 1 smooth_l1, 2 l1
  float beta;        // smooth_l1 beta
  int out_dim;
  int feat_k;        // row stride of the bf16 feature matrix
  MlpLayer layer[RX_MAXL];
  unsigned long long* stamps;  // optional: per-phase s_memtime stamps (profiling builds/tests)
  int pr_lds_off;    // LDS byte offset of the per-column parameter block
  int pr_total;      // floats in that block
};

namespace {

template <int MT>
struct Tile {
  static constexpr int BP = MT * 16;         // padded batch rows
  static constexpr int NTW = 16 / MT;        // max output n-tiles per wave (64 acc regs)
  static constexpr int XS = BP + 8;          // stride (elements) of transposed matrices
};

__device__ __forceinline__ float act_fwd(int act, float z) { return act == 1 ? fmaxf(z, 0.f) : z; }

// C[Bpad x 16-col tile n] += A (LDS, row-major, K contiguous) x Bt (global bf16, [n][K]).
// The weight fragments of up to KC k-steps are fetched in ONE burst of unconditional
// (address-clamped) 16-B loads before any MFMA consumes them, so a layer costs one global
// round trip per 16-column tile instead of one per 32-deep k-step: the step is latency bound
// and the weights arrive from the Infinity Cache / another XCD's L2 after each optimizer step.
template <int MT>
__device__ __forceinline__ void gemm_tile(f32x4 (&acc)[MT], const u16* __restrict__ Arow, int RS,
                                          const u16* __restrict__ Brow, int K, int lg) {
  constexpr int KC = 8;
  const int nks = K >> 5;
  for (int kc = 0; kc < nks; kc += KC) {
    bf16x8 bfr[KC];
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const int ks = min(kc + s, nks - 1);
      bfr[s] = *reinterpret_cast<const bf16x8*>(Brow + ks * 32 + 8 * lg);
    }
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      if (kc + s < nks) {
        const int k0 = (kc + s) * 32 + 8 * lg;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(Arow + mt * 16 * RS + k0);
          acc[mt] = rx_mfma16(a, bfr[s], acc[mt]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// forward of layer l for the rows of this workgroup. Leaves y (the layer output after
// act/BN) in R (row-major) and in XT_{l+1}; for the last layer computes loss, metrics and
// writes dL/dy into R/GT as G_{L-1}.
// ------------------------------------------------------------------------------------------
template <int MT, bool TRAIN>
__device__ void layer_forward(const MlpDesc& d, int l, char* smem, const float* __restrict__ P,
                              float* __restrict__ Gr, const float* __restrict__ labels,
                              const int* __restrict__ rowidx, int nvalid, float* __restrict__ scratch,
                              double* __restrict__ metrics) {
  using T = Tile<MT>;
  const MlpLayer& ly = d.layer[l];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int RS = d.max_k + 8;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* GT = reinterpret_cast<u16*>(smem + d.gt_lds_off);
  float* stats = reinterpret_cast<float*>(smem + d.stats_lds_off);
  const bool last = (l == d.L - 1);
  const int ntiles = ly.out_n >> 4;

  f32x4 acc[T::NTW * MT];
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    f32x4 part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) part[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = wave + j * RX_NW;
    if (n < ntiles) gemm_tile<MT>(part, R + lr * RS, RS, ly.W + (n * 16 + lr) * ly.in_k, ly.in_k, lg);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[j * MT + mt] = part[mt];
  }

  // ---- epilogue in registers, in place on acc: bias, act, BN, loss ----
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    const int n = wave + j * RX_NW;
    if (n < ntiles) {
      const int c = n * 16 + lr;
      const bool colok = c < ly.out;
      const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off) + ly.pr_off;
      const float bias = pr[c];
      const bool act_first = ly.bn != 2;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = acc[j * MT + mt][r] + bias;
          acc[j * MT + mt][r] = act_first ? act_fwd(ly.act, z) : z;
        }
      if (ly.bn != 0) {
        float mean, invstd;
        if (TRAIN) {
          float s = 0.f;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              s += (mt * 16 + lg * 4 + r < nvalid) ? acc[j * MT + mt][r] : 0.f;
          s = rx_colsum16(s);
          mean = s / (float)nvalid;
          float v = 0.f;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float dv = acc[j * MT + mt][r] - mean;
              v += (mt * 16 + lg * 4 + r < nvalid) ? dv * dv : 0.f;
            }
          v = rx_colsum16(v);
          const float var = v / (float)nvalid;
          invstd = rsqrtf(var + ly.eps);
          if (colok && lg == 0) {
            stats[ly.stat_off + 2 * c] = mean;
            stats[ly.stat_off + 2 * c + 1] = invstd;
            const float unb = nvalid > 1 ? var * (float)nvalid / (float)(nvalid - 1) : var;
            float* prw = reinterpret_cast<float*>(smem + d.pr_lds_off) + ly.pr_off;
            prw[3 * ly.out_n + c] = (1.f - ly.momentum) * prw[3 * ly.out_n + c] + ly.momentum * mean;
            prw[4 * ly.out_n + c] = (1.f - ly.momentum) * prw[4 * ly.out_n + c] + ly.momentum * unb;
          }
          // save the BN input for the backward pass (thread-private slots)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              scratch[ly.r_off + (mt * 16 + lg * 4 + r) * ly.out_n + c] = acc[j * MT + mt][r];
        } else {
          mean = colok ? pr[3 * ly.out_n + c] : 0.f;
          invstd = colok ? rsqrtf(pr[4 * ly.out_n + c] + ly.eps) : 0.f;
        }
        const float gam = pr[ly.out_n + c];
        const float bet = pr[2 * ly.out_n + c];
        const bool act_after = ly.bn == 2;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t = (acc[j * MT + mt][r] - mean) * invstd * gam + bet;
            acc[j * MT + mt][r] = act_after ? act_fwd(ly.act, t) : t;
          }
      } else if (TRAIN && !last) {
        // ReLU mask source for the backward pass
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            scratch[ly.r_off + (mt * 16 + lg * 4 + r) * ly.out_n + c] = colok ? acc[j * MT + mt][r] : 0.f;
      }
      // padded rows / columns carry exact zeros through every GEMM
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!colok || mt * 16 + lg * 4 + r >= nvalid) acc[j * MT + mt][r] = 0.f;
      if (last) {
        // loss, metrics and dL/dy (mean reduction over nvalid * out_dim elements)
        float lsum = 0.f, asum = 0.f, ssum = 0.f, gsum = 0.f;
        const float inv_n = 1.f / (float)(nvalid * ly.out);
        const int lcode = d.loss;
        const float beta = d.beta;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = mt * 16 + lg * 4 + r;
            float g = 0.f;
            if (colok && row < nvalid) {
              const float t = labels[rowidx[row] * d.out_dim + c];
              const float e = acc[j * MT + mt][r] - t;
              const float ae = fabsf(e);
              asum += ae;
              ssum += e * e;
              const float sgn = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
              const bool quad = ae < beta;
              lsum += quad ? 0.5f * e * e / beta : ae - 0.5f * beta;  // smooth-L1 term
              g = lcode == 0 ? 2.f * e : (lcode == 1 && quad ? e / beta : sgn);
              g *= inv_n;
            }
            acc[j * MT + mt][r] = g;  // acc now holds G_{L-1}
            gsum += g;
          }
        lsum = rx_wavesum(lsum);
        asum = rx_wavesum(asum);
        ssum = rx_wavesum(ssum);
        if (lcode == 0) lsum = ssum;
        else if (lcode == 2) lsum = asum;
        if (lane == 0) {
          atomicAdd(&metrics[0], (double)(lsum * inv_n));
          atomicAdd(&metrics[1], (double)asum);
          atomicAdd(&metrics[2], (double)ssum);
          if (n == 0) {
            atomicAdd(&metrics[3], (double)(nvalid * ly.out));
            atomicAdd(&metrics[4], 1.0);
          }
        }
        if (TRAIN) {
          gsum = rx_colsum16(gsum);
          if (colok && lg == 0 && ly.b_off >= 0) Gr[ly.b_off + c] = gsum;
        }
      }
    }
  }
  __syncthreads();  // every wave finished reading R for this layer
  if (last && !TRAIN) return;

  // ---- publish y (or G_{L-1}) as bf16: row-major into R, transposed into XT_{l+1} / GT ----
  const int XS = T::XS;
  u16* dstT = last ? GT : reinterpret_cast<u16*>(smem + d.layer[l + 1].xt_off);
  const int tstride = last ? (T::BP + 8) : XS;
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    const int n = wave + j * RX_NW;
    if (n < ntiles) {
      const int c = n * 16 + lr;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        u16 h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[r] = rx_f2bf(acc[j * MT + mt][r]);
          R[(mt * 16 + lg * 4 + r) * RS + c] = h[r];
        }
        if (TRAIN || !last) {
          uint2 pk;
          pk.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
          pk.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
          *reinterpret_cast<uint2*>(dstT + c * tstride + mt * 16 + lg * 4) = pk;
        }
      }
    }
  }
  // zero the K padding columns [out_n, out_k) of R so the next GEMM's K tail is exact
  const int kpad = (last ? ly.out_k : d.layer[l + 1].in_k) - ly.out_n;
  if (kpad > 0) {
    for (int idx = threadIdx.x; idx < T::BP * kpad; idx += RX_THREADS) {
      const int row = idx / kpad, cc = ly.out_n + idx % kpad;
      R[row * RS + cc] = 0;
    }
  }
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// backward of layer l: G_l is in R (row-major) and GT (transposed).
// ------------------------------------------------------------------------------------------
template <int MT>
__device__ void layer_backward(const MlpDesc& d, int l, char* smem, const float* __restrict__ P,
                               float* __restrict__ Gr, int nvalid, const float* __restrict__ scratch) {
  using T = Tile<MT>;
  const MlpLayer& ly = d.layer[l];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int RS = d.max_k + 8;
  const int XS = T::XS;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* GT = reinterpret_cast<u16*>(smem + d.gt_lds_off);
  const u16* XT = reinterpret_cast<const u16*>(smem + ly.xt_off);
  float* stats = reinterpret_cast<float*>(smem + d.stats_lds_off);

  // ---- wgrad, computed transposed: dW^T[i][o] = sum_b X[b][i] G[b][o]  (A = XT, B = GT) ----
  // each lane then holds 4 consecutive i of one o = 16 contiguous bytes of dW[o][:] ->
  // one dwordx4 store instead of four dword stores (the step is store-queue bound here)
  {
    const int mo_tiles = ly.out_n >> 4, ni_tiles = ly.in_n >> 4;
    const int ntile = mo_tiles * ni_tiles;
    const bool vec = ((ly.w_off | ly.in) & 3) == 0;
    for (int t = wave; t < ntile; t += RX_NW) {
      const int mo = t / ni_tiles, ni = t % ni_tiles;
      f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < T::BP; k0 += 32) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(XT + (ni * 16 + lr) * XS + k0 + 8 * lg);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(GT + (mo * 16 + lr) * XS + k0 + 8 * lg);
        a4 = rx_mfma16(a, b, a4);
      }
      const int o = mo * 16 + lr, i0 = ni * 16 + lg * 4;
      if (o < ly.out) {
        float* dst = Gr + ly.w_off + o * ly.in + i0;
        if (vec && i0 + 3 < ly.in) {
          *reinterpret_cast<f32x4*>(dst) = a4;
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (i0 + r < ly.in) dst[r] = a4[r];
        }
      }
    }
  }
  if (d.stamps != nullptr && threadIdx.x == 0) d.stamps[20 + 4 * l] = __builtin_amdgcn_s_memtime();
  if (l == 0) return;

  // ---- dgrad: dX[b][i] = sum_o G[b][o] W[o][i]  (A = R, B = Wt, K = out_k) ----
  const MlpLayer& pv = d.layer[l - 1];  // owns the post-ops between layer l-1 and l
  const int ntiles = ly.in_n >> 4;
  f32x4 acc[T::NTW * MT];
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    f32x4 part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) part[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = wave + j * RX_NW;
    if (n < ntiles) gemm_tile<MT>(part, R + lr * RS, RS, ly.Wt + (n * 16 + lr) * ly.out_k, ly.out_k, lg);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[j * MT + mt] = part[mt];
  }
  if (d.stamps != nullptr && threadIdx.x == 0) d.stamps[21 + 4 * l] = __builtin_amdgcn_s_memtime();
  __syncthreads();  // all reads of G_l (R, GT) are done; they are overwritten with G_{l-1}
  if (d.stamps != nullptr && threadIdx.x == 0) d.stamps[22 + 4 * l] = __builtin_amdgcn_s_memtime();

  // ---- post-op backward of layer l-1 (BN / act), producing G_{l-1} ----
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) continue;
    const int c = n * 16 + lr;
    const bool colok = c < pv.out;
    float g[MT * 4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + lg * 4 + r;
        g[mt * 4 + r] = (row < nvalid && colok) ? acc[j * MT + mt][r] : 0.f;
      }
    if (pv.bn == 0) {
      if (pv.act == 1) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = mt * 16 + lg * 4 + r;
            const float a = scratch[pv.r_off + row * pv.out_n + c];
            if (!(a > 0.f)) g[mt * 4 + r] = 0.f;
          }
      }
    } else {
      const float mean = colok ? stats[pv.stat_off + 2 * c] : 0.f;
      const float invstd = colok ? stats[pv.stat_off + 2 * c + 1] : 0.f;
      const float* ppr = reinterpret_cast<const float*>(smem + d.pr_lds_off) + pv.pr_off;
      const float gam = ppr[pv.out_n + c];
      const float bet = ppr[2 * pv.out_n + c];
      float xh[MT * 4], s[MT * 4];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mt * 16 + lg * 4 + r;
          s[mt * 4 + r] = scratch[pv.r_off + row * pv.out_n + c];
          xh[mt * 4 + r] = (s[mt * 4 + r] - mean) * invstd;
          if (pv.bn == 2 && pv.act == 1 && !(xh[mt * 4 + r] * gam + bet > 0.f)) g[mt * 4 + r] = 0.f;
        }
      float sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int q = 0; q < MT * 4; ++q) {
        sg += g[q];
        sgx += g[q] * xh[q];
      }
      sg = rx_colsum16(sg);
      sgx = rx_colsum16(sgx);
      if (colok && lg == 0) {
        if (pv.g_off >= 0) Gr[pv.g_off + c] = sgx;
        if (pv.be_off >= 0) Gr[pv.be_off + c] = sg;
      }
      const float inv_n = 1.f / (float)nvalid;
      const float k1 = gam * invstd;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = mt * 16 + lg * 4 + r;
          const int q = mt * 4 + r;
          float dz = k1 * (g[q] - sg * inv_n - xh[q] * sgx * inv_n);
          if (pv.bn == 1 && pv.act == 1 && !(s[q] > 0.f)) dz = 0.f;
          g[q] = (row < nvalid && colok) ? dz : 0.f;
        }
    }
    // bias grad of layer l-1
    float bs = 0.f;
#pragma unroll
    for (int q = 0; q < MT * 4; ++q) bs += g[q];
    bs = rx_colsum16(bs);
    if (colok && lg == 0 && pv.b_off >= 0) Gr[pv.b_off + c] = bs;
    // publish G_{l-1}
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      u16 h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        h[r] = rx_f2bf(g[mt * 4 + r]);
        R[(mt * 16 + lg * 4 + r) * RS + c] = h[r];
      }
      uint2 pk;
      pk.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      pk.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
      *reinterpret_cast<uint2*>(GT + c * XS + mt * 16 + lg * 4) = pk;
    }
  }
  if (d.stamps != nullptr && threadIdx.x == 0) d.stamps[23 + 4 * l] = __builtin_amdgcn_s_memtime();
  // zero the K tail [out_n, out_k) of G_{l-1} in R for the next dgrad
  const int kpad = pv.out_k - pv.out_n;
  if (kpad > 0) {
    for (int idx = threadIdx.x; idx < T::BP * kpad; idx += RX_THREADS) {
      const int row = idx / kpad, cc = pv.out_n + idx % kpad;
      R[row * RS + cc] = 0;
    }
  }
  __syncthreads();
}

// Stage every layer's per-column parameters (bias, BN gamma/beta, running mean/var) into LDS
// with ONE burst of independent loads per thread (column c = threadIdx.x of every layer,
// address-clamped so no load sits behind a per-element branch). Saves two dependent
// cross-XCD round trips per layer in the epilogues.
__device__ void load_params(const MlpDesc& d, char* smem, const float* __restrict__ P) {
  float* pr = reinterpret_cast<float*>(smem + d.pr_lds_off);
  const int c = threadIdx.x;
  float v[RX_MAXL][5];
#pragma unroll
  for (int l = 0; l < RX_MAXL; ++l) {
    if (l < d.L) {
      const MlpLayer& ly = d.layer[l];
      const bool ok = c < ly.out;
      const int cc = ok ? c : 0;
      const float b = P[ly.b_off >= 0 ? ly.b_off + cc : 0];
      const float g = P[ly.g_off >= 0 ? ly.g_off + cc : 0];
      const float be = P[ly.be_off >= 0 ? ly.be_off + cc : 0];
      const float* rmp = ly.run_mean ? ly.run_mean : P;
      const float* rvp = ly.run_var ? ly.run_var : P;
      const float rm = rmp[ly.run_mean ? cc : 0];
      const float rv = rvp[ly.run_var ? cc : 0];
      v[l][0] = (ok && ly.b_off >= 0) ? b : 0.f;
      v[l][1] = (ok && ly.g_off >= 0) ? g : 1.f;
      v[l][2] = (ok && ly.be_off >= 0) ? be : 0.f;
      v[l][3] = (ok && ly.run_mean) ? rm : 0.f;
      v[l][4] = (ok && ly.run_var) ? rv : 1.f;
    }
  }
#pragma unroll
  for (int l = 0; l < RX_MAXL; ++l) {
    if (l < d.L) {
      const MlpLayer& ly = d.layer[l];
      if (c < ly.out_n) {
#pragma unroll
        for (int k = 0; k < 5; ++k) pr[ly.pr_off + k * ly.out_n + c] = v[l][k];
      }
    }
  }
}

// write the updated BatchNorm running statistics back (once per step, after the forward)
__device__ void store_running_stats(const MlpDesc& d, char* smem) {
  const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off);
  const int c = threadIdx.x;
  for (int l = 0; l < d.L; ++l) {
    const MlpLayer& ly = d.layer[l];
    if (ly.run_mean != nullptr && c < ly.out) {
      ly.run_mean[c] = pr[ly.pr_off + 3 * ly.out_n + c];
      ly.run_var[c] = pr[ly.pr_off + 4 * ly.out_n + c];
    }
  }
}

// load the batch's feature rows (gathered through the epoch permutation) into R and XT_0
template <int MT>
__device__ void load_inputs(const MlpDesc& d, char* smem, const u16* __restrict__ feats,
                            const int* __restrict__ rowidx, int nvalid, bool need_t) {
  using T = Tile<MT>;
  const int RS = d.max_k + 8;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* XT = reinterpret_cast<u16*>(smem + d.layer[0].xt_off);
  const int in_n = d.layer[0].in_n;
  const int chunks = d.feat_k >> 3;  // 8 bf16 per 16-B chunk
  for (int idx = threadIdx.x; idx < T::BP * chunks; idx += RX_THREADS) {
    const int row = idx / chunks, ch = idx % chunks;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < nvalid) v = *reinterpret_cast<const uint4*>(feats + (size_t)rowidx[row] * d.feat_k + ch * 8);
    *reinterpret_cast<uint4*>(R + row * RS + ch * 8) = v;
    if (need_t) {
      const u16* h = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = ch * 8 + e;
        if (k < in_n) XT[k * T::XS + row] = h[e];
      }
    }
  }
  __syncthreads();
}

template <int MT>
__global__ __launch_bounds__(RX_THREADS) void mlp_train_step_kernel(
    const MlpDesc* __restrict__ dp, const float* __restrict__ P, float* __restrict__ Gr, const u16* __restrict__ feats,
    const float* __restrict__ labels, const int* __restrict__ perm, int row0, int nvalid,
    float* __restrict__ scratch, double* __restrict__ metrics) {
  const MlpDesc& d = *dp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int rowidx[Tile<MT>::BP];
  unsigned long long* st = d.stamps;
  int si = 0;
#define RX_STAMP()                                                        \
  do {                                                                    \
    if (st != nullptr && threadIdx.x == 0) st[si] = __builtin_amdgcn_s_memtime(); \
    ++si;                                                                 \
  } while (0)
  RX_STAMP();
  for (int i = threadIdx.x; i < Tile<MT>::BP; i += RX_THREADS)
    rowidx[i] = i < nvalid ? (perm ? perm[row0 + i] : row0 + i) : 0;
  load_params(d, smem, P);
  __syncthreads();
  load_inputs<MT>(d, smem, feats, rowidx, nvalid, true);
  RX_STAMP();
  for (int l = 0; l < d.L; ++l) {
    layer_forward<MT, true>(d, l, smem, P, Gr, labels, rowidx, nvalid, scratch, metrics);
    RX_STAMP();
  }
  store_running_stats(d, smem);
  for (int l = d.L - 1; l >= 0; --l) {
    layer_backward<MT>(d, l, smem, P, Gr, nvalid, scratch);
    RX_STAMP();
  }
#undef RX_STAMP
}

template <int MT>
__global__ __launch_bounds__(RX_THREADS) void mlp_eval_kernel(
    const MlpDesc* __restrict__ dp, const float* __restrict__ P, const u16* __restrict__ feats,
    const float* __restrict__ labels, int n_rows, int batch, double* __restrict__ metrics,
    float* __restrict__ out) {
  const MlpDesc& d = *dp;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int rowidx[Tile<MT>::BP];
  const int row0 = blockIdx.x * batch;
  const int nvalid = min(batch, n_rows - row0);
  for (int i = threadIdx.x; i < Tile<MT>::BP; i += RX_THREADS) rowidx[i] = i < nvalid ? row0 + i : 0;
  load_params(d, smem, P);
  __syncthreads();
  load_inputs<MT>(d, smem, feats, rowidx, nvalid, false);
  for (int l = 0; l < d.L; ++l) {
    if (l == d.L - 1 && out != nullptr) {
      // prediction mode is handled by the host (not needed by the estimator path)
    }
    layer_forward<MT, false>(d, l, smem, P, nullptr, labels, rowidx, nvalid, nullptr, metrics);
  }
}

// ------------------------------------------------------------------------------------------
// optimizer: fused Adam / AdamW / SGD(momentum, nesterov) over the flat parameter vector,
// refreshing the bf16 W / Wt images of every Linear weight in the same pass.
// ------------------------------------------------------------------------------------------
#define RX_MAXSEG (4 * RX_MAXL)
struct OptSeg {
  int start, len, kind;  // kind 1: linear weight (needs bf16 images)
  int out, in, in_k, out_k;
  u16* W;
  u16* Wt;
};
struct OptDesc {
  int nseg, total;
  int algo;  // 0 adam, 1 adamw, 2 sgd
  float b1, b2, eps, wd, momentum, dampening;
  int nesterov, maximize;
  OptSeg seg[RX_MAXSEG];
};

__device__ __forceinline__ float opt_update(const OptDesc& o, int idx, float* __restrict__ p,
                                            const float* __restrict__ g, float* __restrict__ m,
                                            float* __restrict__ v, float lr, float bc1, float bc2,
                                            float gscale, int first) {
  float gr = g[idx] * gscale;
  if (o.maximize) gr = -gr;
  float pv = p[idx];
  if (o.algo == 2) {
    if (o.wd != 0.f) gr += o.wd * pv;
    if (o.momentum != 0.f) {
      const float b = first ? gr : o.momentum * m[idx] + (1.f - o.dampening) * gr;
      m[idx] = b;
      gr = o.nesterov ? gr + o.momentum * b : b;
    }
    pv -= lr * gr;
  } else {
    if (o.algo == 1) pv *= (1.f - lr * o.wd);
    else if (o.wd != 0.f) gr += o.wd * pv;
    const float mm = o.b1 * m[idx] + (1.f - o.b1) * gr;
    const float vv = o.b2 * v[idx] + (1.f - o.b2) * gr * gr;
    m[idx] = mm;
    v[idx] = vv;
    pv -= (lr / bc1) * mm / (sqrtf(vv) / sqrtf(bc2) + o.eps);
  }
  p[idx] = pv;
  return pv;
}

// Tiled optimizer: block b -> (segment, 32x32 weight tile | 1024-element vector chunk).
// Weight tiles update p/m/v coalesced along `in`, then transpose through LDS so the W
// ([out][in_k]) and Wt ([in][out_k]) bf16 images are both written with coalesced rows.
__global__ __launch_bounds__(256) void opt_tiled_kernel(const OptDesc* __restrict__ op, float* __restrict__ p,
                                                        const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float lr, float bc1, float bc2, float gscale,
                                                        int first) {
  const OptDesc& o = *op;
  __shared__ u16 tile[32][33];
  int b = blockIdx.x;
  int s = 0;
  for (; s < o.nseg; ++s) {
    const OptSeg& sg = o.seg[s];
    const int nb = sg.kind == 1 ? ((sg.out + 31) / 32) * ((sg.in + 31) / 32) : (sg.len + 1023) / 1024;
    if (b < nb) break;
    b -= nb;
  }
  if (s >= o.nseg) return;
  const OptSeg& sg = o.seg[s];
  if (sg.kind != 1) {
    for (int q = b * 1024 + threadIdx.x; q < min(sg.len, (b + 1) * 1024); q += 256)
      opt_update(o, sg.start + q, p, g, m, v, lr, bc1, bc2, gscale, first);
    return;
  }
  const int tiles_i = (sg.in + 31) / 32;
  const int o0 = (b / tiles_i) * 32, i0 = (b % tiles_i) * 32;
  const int ti = threadIdx.x & 31, to = threadIdx.x >> 5;  // 8 rows per pass
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oo = o0 + to + r * 8, ii = i0 + ti;
    u16 h = 0;
    if (oo < sg.out && ii < sg.in) {
      const float pv = opt_update(o, sg.start + oo * sg.in + ii, p, g, m, v, lr, bc1, bc2, gscale, first);
      h = rx_f2bf(pv);
      sg.W[oo * sg.in_k + ii] = h;
    }
    tile[to + r * 8][ti] = h;
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ii = i0 + to + r * 8, oo = o0 + ti;
    if (oo < sg.out && ii < sg.in) sg.Wt[ii * sg.out_k + oo] = tile[ti][to + r * 8];
  }
}

int opt_tiled_blocks(const OptDesc& o) {
  int nb = 0;
  for (int s = 0; s < o.nseg; ++s) {
    const OptSeg& sg = o.seg[s];
    nb += sg.kind == 1 ? ((sg.out + 31) / 32) * ((sg.in + 31) / 32) : (sg.len + 1023) / 1024;
  }
  return nb < 1 ? 1 : nb;
}

template <int MT>
int set_lds(int bytes) {
  RX_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_train_step_kernel<MT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  RX_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&mlp_eval_kernel<MT>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  return 0;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C API
// ------------------------------------------------------------------------------------------
typedef int (*rx_allreduce_fn)(float* buf, int n, void* ctx, hipStream_t s);

extern "C" {

int rx_mlp_desc_size() { return (int)sizeof(MlpDesc); }
int rx_opt_desc_size() { return (int)sizeof(OptDesc); }

// One or more training steps over rows [first_row, first_row + nsteps * batch) of the epoch
// permutation. Per step: fused fwd/bwd kernel -> (optional) gradient all-reduce -> optimizer.
int rx_mlp_train_steps(const MlpDesc* d, const MlpDesc* d_dev, const OptDesc* o, const OptDesc* o_dev, int mt, float* params, float* grads,
                       float* m, float* v, const u16* feats, const float* labels, const int* perm,
                       int n_rows, int batch, int first_step, int nsteps, const float* lrs,
                       const float* bc1s, const float* bc2s, float gscale, int opt_first_step,
                       float* scratch, double* metrics, hipStream_t stream,
                       rx_allreduce_fn allreduce, void* ar_ctx) {
  static int lds_set[9] = {0};
  if (mt != 2 && mt != 4 && mt != 8) return -1;
  if (lds_set[mt] < d->lds_bytes) {
    int rc = mt == 2 ? set_lds<2>(d->lds_bytes) : mt == 4 ? set_lds<4>(d->lds_bytes) : set_lds<8>(d->lds_bytes);
    if (rc) return rc;
    lds_set[mt] = d->lds_bytes;
  }
  const int opt_blocks = opt_tiled_blocks(*o);
  for (int s = 0; s < nsteps; ++s) {
    const int step = first_step + s;
    const int row0 = step * batch;
    const int nvalid = n_rows - row0 < batch ? n_rows - row0 : batch;
    if (nvalid <= 0) break;
    if (mt == 2)
      hipLaunchKernelGGL(mlp_train_step_kernel<2>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                         params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
    else if (mt == 4)
      hipLaunchKernelGGL(mlp_train_step_kernel<4>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                         params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
    else
      hipLaunchKernelGGL(mlp_train_step_kernel<8>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                         params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
    if (allreduce) {
      int rc = allreduce(grads, o->total, ar_ctx, stream);
      if (rc) return rc;
    }
    hipLaunchKernelGGL(opt_tiled_kernel, dim3(opt_blocks), dim3(256), 0, stream, o_dev, params, grads, m, v,
                       lrs[s], bc1s[s], bc2s[s], gscale, (opt_first_step && s == 0) ? 1 : 0);
  }
  return (int)hipGetLastError();
}

// Single pieces of a step for callers that interleave their own collective between the
// backward and the optimizer (torch.distributed fallback path).
int rx_mlp_fwdbwd(const MlpDesc* d, const MlpDesc* d_dev, int mt, const float* params, float* grads, const u16* feats,
                  const float* labels, const int* perm, int n_rows, int batch, int step,
                  float* scratch, double* metrics, hipStream_t stream) {
  static int lds_set[9] = {0};
  if (mt != 2 && mt != 4 && mt != 8) return -1;
  if (lds_set[mt] < d->lds_bytes) {
    int rc = mt == 2 ? set_lds<2>(d->lds_bytes) : mt == 4 ? set_lds<4>(d->lds_bytes) : set_lds<8>(d->lds_bytes);
    if (rc) return rc;
    lds_set[mt] = d->lds_bytes;
  }
  const int row0 = step * batch;
  const int nvalid = n_rows - row0 < batch ? n_rows - row0 : batch;
  if (nvalid <= 0) return 0;
  if (mt == 2)
    hipLaunchKernelGGL(mlp_train_step_kernel<2>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                       params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
  else if (mt == 4)
    hipLaunchKernelGGL(mlp_train_step_kernel<4>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                       params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
  else
    hipLaunchKernelGGL(mlp_train_step_kernel<8>, dim3(1), dim3(RX_THREADS), d->lds_bytes, stream, d_dev,
                       params, grads, feats, labels, perm, row0, nvalid, scratch, metrics);
  return (int)hipGetLastError();
}

int rx_opt_step(const OptDesc* o, const OptDesc* o_dev, float* params, const float* grads, float* m, float* v, float lr,
                float bc1, float bc2, float gscale, int first, hipStream_t stream) {
  const int opt_blocks = opt_tiled_blocks(*o);
  hipLaunchKernelGGL(opt_tiled_kernel, dim3(opt_blocks), dim3(256), 0, stream, o_dev, params, grads, m, v,
                     lr, bc1, bc2, gscale, first);
  return (int)hipGetLastError();
}

int rx_mlp_eval(const MlpDesc* d, const MlpDesc* d_dev, int mt, const float* params, const u16* feats, const float* labels,
                int n_rows, int batch, double* metrics, hipStream_t stream) {
  static int lds_set[9] = {0};
  if (mt != 2 && mt != 4 && mt != 8) return -1;
  if (lds_set[mt] < d->lds_bytes) {
    int rc = mt == 2 ? set_lds<2>(d->lds_bytes) : mt == 4 ? set_lds<4>(d->lds_bytes) : set_lds<8>(d->lds_bytes);
    if (rc) return rc;
    lds_set[mt] = d->lds_bytes;
  }
  const int nb = (n_rows + batch - 1) / batch;
  if (nb <= 0) return 0;
  if (mt == 2)
    hipLaunchKernelGGL(mlp_eval_kernel<2>, dim3(nb), dim3(RX_THREADS), d->lds_bytes, stream, d_dev, params,
                       feats, labels, n_rows, batch, metrics, nullptr);
  else if (mt == 4)
    hipLaunchKernelGGL(mlp_eval_kernel<4>, dim3(nb), dim3(RX_THREADS), d->lds_bytes, stream, d_dev, params,
                       feats, labels, n_rows, batch, metrics, nullptr);
  else
    hipLaunchKernelGGL(mlp_eval_kernel<8>, dim3(nb), dim3(RX_THREADS), d->lds_bytes, stream, d_dev, params,
                       feats, labels, n_rows, batch, metrics, nullptr);
  return (int)hipGetLastError();
}

// Refresh the bf16 images from the fp32 master weights (initialisation / after load).
int rx_mlp_refresh_images(const OptDesc* o, const OptDesc* o_dev, const float* params, hipStream_t stream);

}  // extern "C"

namespace {
__global__ void refresh_kernel(const OptDesc* __restrict__ op, const float* __restrict__ p) {
  const OptDesc& o = *op;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < o.total; idx += gridDim.x * blockDim.x) {
    for (int s = 0; s < o.nseg; ++s) {
      const OptSeg& sg = o.seg[s];
      if (idx >= sg.start && idx < sg.start + sg.len) {
        if (sg.kind == 1) {
          const int q = idx - sg.start;
          const int oo = q / sg.in, ii = q - oo * sg.in;
          const u16 h = rx_f2bf(p[idx]);
          sg.W[oo * sg.in_k + ii] = h;
          sg.Wt[ii * sg.out_k + oo] = h;
        }
        break;
      }
    }
  }
}
}  // namespace

extern "C" int rx_mlp_refresh_images(const OptDesc* o, const OptDesc* o_dev, const float* params, hipStream_t stream) {
  const int blocks = (o->total + 255) / 256 < 1024 ? (o->total + 255) / 256 : 1024;
  hipLaunchKernelGGL(refresh_kernel, dim3(blocks), dim3(256), 0, stream, o_dev, params);
  return (int)hipGetLastError();
}
