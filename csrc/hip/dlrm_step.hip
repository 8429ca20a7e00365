// The whole DLRM training step as ONE persistent launch on gfx950 (replicated tables, one GPU,
// plain SGD, BCE-with-logits): bottom MLP, embedding gather, dot interaction, top MLP, loss, the
// backward of every layer, the dense SGD and the sparse embedding SGD -- 14 grid-wide phases
// separated by counter barriers (rx_grid.h), instead of the 21 dependent launches of the
// launch-per-op step (csrc/hip/linear_act.hip + dlrm.hip), each of which is >= 4.6 us at the
// notebook's batch of 128 (profiles/r3_linear_gemm_sweep_batch128.txt).
//
// Reference model: examples/pytorch_dlrm.ipynb cells 9, 14 (Dlrm: bottom 13-512-128-32, 26
// tables x 32, dot interaction, top 1024-1024-512-256-1, BCEWithLogitsLoss, SGD) trained by
// TorchEstimator (python/raydp/torch/estimator.py:280-320 runs it as an eager torch loop).
//
// Phases (B = batch rows, a multiple of 32, <= 256):
//   BOTTOM  per 16-row block: dense rows (gathered through the epoch permutation) -> bottom MLP
//           in LDS (MFMA 16x16x32 bf16) -> interaction input X = [bottom out; 26 table rows] ->
//           Z = [x0 | strict lower triangle of X X^T | 0]; stores H_l, H_l^T, X, Z, Z^T
//   GEMM    top forward layers: tiles of Y = relu(A W^T + b), stored row-major and transposed
//   HEAD    per 16-row block: last layer (N = 1) + BCE + its backward -> dA of layer L-1 and the
//           block's partial of the last layer's gradient (its SGD: one workgroup, next phase)
//   GEMM    per top layer, backward: dgrad tiles (dX = dY W, ReLU mask of X) AND wgrad tiles
//           (dW = dY^T X with the SGD update of the fp32 master in the epilogue) in ONE phase
//   IBWD    per 16 samples: dX = S X (S = symmetric dZ), bottom-MLP gradient (ReLU-masked),
//           the table rows updated in place (fp32 atomics, as rx_dot_bwd_sgd)
//   GEMM    bottom backward (the first layer wgrad only)
// A layer's dgrad reads its bf16 weight image of parity p while its wgrad epilogue writes the
// updated weights into the images of parity 1 - p: the two never race inside the launch, and the
// next launch (the parity word flips at the end) reads the new ones. fp32 masters (the torch
// parameters' storage) are read and written only by the workgroup owning the tile.
// Hand-offs between workgroups: 16-/8-B sc1 stores, rx_grid_barrier, sc1 loads; every hand-off
// buffer is written once per launch.
#include "rx_common.h"
#include "rx_grid.h"

namespace {

constexpr int NT = 256;
constexpr int MAXF = 32;     // interaction rows (1 + tables), padded
constexpr int MAXPH = 24;
constexpr int MAXBOT = 4;
constexpr int CTL_PAR = 3;   // parity word of ctl

enum { PH_GEMM = 0, PH_BOTTOM = 1, PH_HEAD = 2, PH_IBWD = 3 };
enum { EPI_FWD = 0, EPI_DGRAD = 1, EPI_WGRAD = 2 };

// One GEMM of a phase: C[M x N] = A[M][K] * Bm[N][K]^T (both bf16, K contiguous), tiled tm x tn.
struct GSpec {
  const u16* A;
  const u16* Bm[2];        // by parity (the same pointer twice when not a weight image)
  long long lda, ldb;
  int M, N, K;             // K: multiple of 32
  int tm, tn;              // 16, 32 or 64
  int epi, relu;
  int pad0;
  const float* bias;       // FWD: [N]
  const u16* mask;         // DGRAD: C *= (mask[m][n] > 0)
  long long ldmask;
  u16* Y;                  // bf16 row-major [M][ldy] (nullable)
  long long ldy;
  u16* YT;                 // bf16 transposed [N][ldyt] (nullable)
  long long ldyt;
  float* Yf;               // fp32 row-major [M][ldyf] (nullable)
  long long ldyf;
  // WGRAD: rows m = output features, cols n = input features
  float* W;                // fp32 master [M][kvalid]
  int kvalid, pad1;
  u16* img[2];             // images written for parity (1 - p): [M][ldimg] and [N][ldimgT]
  u16* imgT[2];
  long long ldimg, ldimgT;
  float* b;                // bias master [M] (nullable): b[m] -= lr * sum_r dyT[m][r]
  const u16* dyT;
  long long lddyT;
  int brows, pad2;
};

struct Phase {
  int kind, nspec;
  GSpec s[2];
};

struct BotLayer {
  const u16* img[2];       // [N][Kp] bf16 by parity
  const float* bias;       // [N]
  int N, K, Kp, pad;
  u16* H;                  // output row-major [B][N] (nullable: the last layer's lives in X)
  u16* HT;                 // output transposed [N][B] (nullable)
};

struct DlrmDesc {
  int B, nph, nbot, F, D, ZP, G, pad0;
  Phase ph[MAXPH];
  BotLayer bot[MAXBOT];
  const float* dense;      // [rows][ld_dense] fp32
  long long ld_dense;
  int ndense, pad1;
  const long long* cats;   // [rows][ld_cats] int64 (table-local ids)
  long long ld_cats;
  const float* labels;     // [rows] (stride ld_lab)
  long long ld_lab;
  u16* XdT;                // dense transposed [Kp0][B] bf16
  float* emb;              // [emb_rows][D] fp32
  const long long* offs;   // [F - 1]
  long long emb_rows;
  u16* ximg;               // [B][32][D] bf16 interaction inputs
  u16* Z;                  // [B][ZP]
  u16* ZT;                 // [ZP][B]
  // HEAD
  const u16* A_last;       // [B][K_last] (the top tower's last hidden activation)
  int K_last, pad2;
  float* w_last;           // [K_last] fp32 master
  float* b_last;           // [1]
  u16* dA;                 // [B][K_last]
  u16* dAT;                // [K_last][B]
  float* logits;           // [B] (nullable)
  double* loss_acc;        // += mean loss of every step
  float* step_loss;        // the last step's mean loss
  // IBWD
  const float* dZ;         // [B][ZP] fp32
  u16* dmlp;               // [B][D]
  u16* dmlpT;              // [D][B]
  float lr;
  int pad3;
  unsigned* ctl;           // [0] barrier counter, [1] done, [2] error, [3] parity
  unsigned long long ticks;
  unsigned long long* stamps;  // nullable: [MAXPH + 1] wall-clock stamps of workgroup 0 (phase profile)
  float* head_part;        // [B / 16][head_ld]: per 16-row block sum dz A (K_last), sum dz, sum loss
  int head_ld, pad4;
};

__device__ __forceinline__ long long src_row(const long long* perm, long long row0, int i, int nvalid) {
  return perm[row0 + (i < nvalid ? i : nvalid - 1)];
}

__device__ __forceinline__ bf16x8 ld16(const u16* base, long long elem) {
  return __builtin_bit_cast(bf16x8, rx_load16_sc1(base, (int)(elem * 2)));
}

__device__ __forceinline__ void unpack8(const u32x4& v, float (&f)[8]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(v[j] << 16);
    f[2 * j + 1] = __uint_as_float(v[j] & 0xffff0000u);
  }
}

__device__ __forceinline__ u32x4 pack8(const float (&f)[8]) {
  return u32x4{rx_f2bf2(f[0], f[1]), rx_f2bf2(f[2], f[3]), rx_f2bf2(f[4], f[5]), rx_f2bf2(f[6], f[7])};
}

// Transposed store of a bf16 tile staged in LDS (st[r * ss + c], r < TM, c < TN) into
// out[(c0 + c) * ld + r0 + r]: 16-B chunks of 8 consecutive rows.
__device__ __forceinline__ void store_transposed(const u16* st, int ss, int TM, int TN, u16* out, long long ld,
                                                 int r0, int c0) {
  const int rch = TM >> 3;
  for (int idx = threadIdx.x; idx < TN * rch; idx += NT) {
    const int c = idx / rch, r8 = (idx % rch) * 8;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = rx_bf2f(st[(r8 + j) * ss + c]);
    rx_store16_sc1(out, (int)(((long long)(c0 + c) * ld + r0 + r8) * 2), pack8(f));
  }
}

// ------------------------------------------------------------------------------------- GEMM --
// Every global operand of a job is requested before the job waits for any: the K loop's A / B
// fragments in bursts, and ahead of them the epilogue's own operands that do not depend on the
// product (fp32 master weights of a WGRAD tile, the FWD bias, the DGRAD ReLU mask), so their
// latency hides under the K loop instead of following it.
template <int MS, int NS>
__device__ void gemm_job(const GSpec& s, int p, int mt, int nt, float lr, char* lds) {
  constexpr int TM = MS * 16, TN = NS * 16;
  constexpr int KC = (32 / (MS + NS)) > 8 ? 8 : (32 / (MS + NS));
  constexpr int PS = TN + 4;             // fp32 partial row stride
  constexpr int SS = TN + 8;             // bf16 staging row stride
  constexpr int CC = TN / 8;             // 8-column chunks per row
  constexpr int IT = (TM * CC + NT - 1) / NT;   // epilogue chunks per thread
  float* part = reinterpret_cast<float*>(lds);                       // [4][TM][PS]
  u16* st = reinterpret_cast<u16*>(lds + 4 * TM * PS * 4);          // [TM][SS]
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr_ = lane & 15, lg = lane >> 4;
  const int m0 = mt * TM, n0 = nt * TN;
  const u16* A = s.A;
  const u16* Bm = s.Bm[p];
  const int nks = s.K >> 5;
  const int per = (nks + 3) >> 2;
  const int k0s = wave * per, k1s = min(nks, k0s + per);
  float pre[IT][8];
  u32x4 mk[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = tid + it * NT;
    const int r = idx / CC, c = (idx % CC) * 8, m = m0 + r, n = n0 + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) pre[it][j] = 0.f;
    mk[it] = u32x4{0u, 0u, 0u, 0u};
    if (idx < TM * CC) {
      if (s.epi == EPI_WGRAD) {
        const RX_GLOBAL float* w = rx_g(s.W) + (long long)m * s.kvalid;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (n + j < s.kvalid) pre[it][j] = w[n + j];
      } else if (s.epi == EPI_FWD) {
        const RX_GLOBAL float* bias = rx_g(s.bias);
#pragma unroll
        for (int j = 0; j < 8; ++j) pre[it][j] = bias[n + j];
      } else if (s.mask != nullptr) {
        mk[it] = rx_load16_sc1(s.mask, (int)(((long long)m * s.ldmask + n) * 2));
      }
    }
  }
  f32x4 acc[MS][NS];
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = k0s; kc < k1s; kc += KC) {
    bf16x8 af[KC][MS], bfr[KC][NS];
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      const int ks = min(kc + q, k1s - 1);
#pragma unroll
      for (int i = 0; i < MS; ++i) af[q][i] = ld16(A, (long long)(m0 + 16 * i + lr_) * s.lda + ks * 32 + 8 * lg);
#pragma unroll
      for (int j = 0; j < NS; ++j) bfr[q][j] = ld16(Bm, (long long)(n0 + 16 * j + lr_) * s.ldb + ks * 32 + 8 * lg);
    }
#pragma unroll
    for (int q = 0; q < KC; ++q)
      if (kc + q < k1s)
#pragma unroll
        for (int i = 0; i < MS; ++i)
#pragma unroll
          for (int j = 0; j < NS; ++j) acc[i][j] = rx_mfma16(af[q][i], bfr[q][j], acc[i][j]);
  }
  // C layout: row = 16 i + 4 lg + r, col = 16 j + lr_
#pragma unroll
  for (int i = 0; i < MS; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[(wave * TM + 16 * i + 4 * lg + r) * PS + 16 * j + lr_] = acc[i][j][r];
  __syncthreads();
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = tid + it * NT;
    if (idx >= TM * CC) break;
    const int r = idx / CC, c = (idx % CC) * 8;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int o = r * PS + c + j;
      v[j] = part[o] + part[TM * PS + o] + part[2 * TM * PS + o] + part[3 * TM * PS + o];
    }
    const int m = m0 + r, n = n0 + c;
    if (s.epi == EPI_WGRAD) {
      // SGD on the fp32 master (columns past kvalid are the image's zero padding)
      RX_GLOBAL float* w = rx_g(s.W) + (long long)m * s.kvalid;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (n + j < s.kvalid) {
          const float nw = pre[it][j] - lr * v[j];
          w[n + j] = nw;
          v[j] = nw;
        } else {
          v[j] = 0.f;
        }
      }
      rx_store16_sc1(s.img[1 - p], (int)(((long long)m * s.ldimg + n) * 2), pack8(v));
    } else {
      if (s.epi == EPI_FWD) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[j] += pre[it][j];
          if (s.relu) v[j] = fmaxf(v[j], 0.f);
        }
      } else if (s.mask != nullptr) {
        float mf[8];
        unpack8(mk[it], mf);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = mf[j] > 0.f ? v[j] : 0.f;
      }
      if (s.Yf != nullptr) {
        const int bo = (int)(((long long)m * s.ldyf + n) * 4);
        rx_store16_sc1(s.Yf, bo, __builtin_bit_cast(u32x4, f32x4{v[0], v[1], v[2], v[3]}));
        rx_store16_sc1(s.Yf, bo + 16, __builtin_bit_cast(u32x4, f32x4{v[4], v[5], v[6], v[7]}));
      }
      if (s.Y != nullptr) rx_store16_sc1(s.Y, (int)(((long long)m * s.ldy + n) * 2), pack8(v));
    }
    *reinterpret_cast<u32x4*>(st + r * SS + c) = pack8(v);
  }
  __syncthreads();
  if (s.epi == EPI_WGRAD) {
    if (s.imgT[1 - p] != nullptr) store_transposed(st, SS, TM, TN, s.imgT[1 - p], s.ldimgT, m0, n0);
    if (s.b != nullptr && nt == 0) {
      // bias gradient = row sums of dY^T over the batch (brows <= 256: at most 32 chunks of 8
      // per row, dealt over the TPR adjacent lanes of the row); SGD on the fp32 bias
      constexpr int TPR = NT / TM;
      const int r = tid / TPR, q = tid % TPR;
      float a1 = 0.f;
#pragma unroll
      for (int i = 0; i < 32 / TPR + (32 % TPR != 0); ++i) {
        const int c = (q + i * TPR) * 8;
        if (c < s.brows) {
          float f[8];
          unpack8(rx_load16_sc1(s.dyT, (int)(((long long)(m0 + r) * s.lddyT + c) * 2)), f);
          a1 += ((f[0] + f[1]) + (f[2] + f[3])) + ((f[4] + f[5]) + (f[6] + f[7]));
        }
      }
#pragma unroll
      for (int o = TPR / 2; o > 0; o >>= 1) a1 += __shfl_xor(a1, o);
      if (q == 0) rx_g(s.b)[m0 + r] -= lr * a1;
    }
  } else if (s.YT != nullptr) {
    store_transposed(st, SS, TM, TN, s.YT, s.ldyt, m0, n0);
  }
  __syncthreads();  // LDS reused by the next job
}

__device__ void run_job(const GSpec& s, int p, int t, float lr, char* lds) {
  const int tn_tiles = s.N / s.tn;
  const int mt = t / tn_tiles, nt = t % tn_tiles;
  const int code = (s.tm >> 4) * 8 + (s.tn >> 4);
  switch (code) {
    case 1 * 8 + 1: gemm_job<1, 1>(s, p, mt, nt, lr, lds); break;
    case 1 * 8 + 2: gemm_job<1, 2>(s, p, mt, nt, lr, lds); break;
    case 2 * 8 + 1: gemm_job<2, 1>(s, p, mt, nt, lr, lds); break;
    case 2 * 8 + 2: gemm_job<2, 2>(s, p, mt, nt, lr, lds); break;
    case 1 * 8 + 4: gemm_job<1, 4>(s, p, mt, nt, lr, lds); break;
    case 4 * 8 + 1: gemm_job<4, 1>(s, p, mt, nt, lr, lds); break;
    case 2 * 8 + 4: gemm_job<2, 4>(s, p, mt, nt, lr, lds); break;
    case 4 * 8 + 2: gemm_job<4, 2>(s, p, mt, nt, lr, lds); break;
    case 4 * 8 + 4: gemm_job<4, 4>(s, p, mt, nt, lr, lds); break;
    default: break;  // the host only plans the shapes above
  }
}

__device__ void gemm_phase(const Phase& P, int p, float lr, int G, char* lds) {
  const int j0 = (P.s[0].M / P.s[0].tm) * (P.s[0].N / P.s[0].tn);
  const int j1 = P.nspec > 1 ? (P.s[1].M / P.s[1].tm) * (P.s[1].N / P.s[1].tn) : 0;
  // second spec's jobs dealt from the top of the grid down, so a short phase spreads both over
  // disjoint workgroups
  for (int t = blockIdx.x; t < j0 + j1; t += G) {
    if (t < j0)
      run_job(P.s[0], p, t, lr, lds);
    else
      run_job(P.s[1], p, j1 - 1 - (t - j0), lr, lds);
  }
}

// ----------------------------------------------------------------------------------- BOTTOM --
// One 16-row block: bottom MLP in LDS, then gather + interaction for its 16 samples. The
// dependent index chain (permutation -> source row -> table-local id) runs once for the whole
// block; the embedding rows are requested before the MLP and land while it computes.
template <int D>
__device__ void bottom_block(const DlrmDesc* __restrict__ d, int p, int rb, const long long* __restrict__ perm,
                             long long row0, int nvalid, char* lds) {
  constexpr int XR = D + 8;            // interaction image row stride (bf16)
  constexpr int CH = D / 8;            // 16-B bf16 chunks per interaction row
  constexpr int GI = 16 * MAXF * CH / NT;   // gathered chunks per thread
  static_assert(16 * MAXF * CH % NT == 0, "gather split");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr_ = lane & 15, lg = lane >> 4;
  const int r0 = rb * 16;
  const int B = d->B, F = d->F, ZP = d->ZP, nbot = d->nbot;
  // LDS: embedding row ids [16][MAXF], two activation buffers [16][HS], the interaction images
  // [16][MAXF][XR], Z staging [16][ZS]
  int maxw = 32;
  for (int l = 0; l < nbot; ++l) maxw = max(maxw, max(d->bot[l].Kp, d->bot[l].N));
  const int HS = maxw + 8;
  long long* erow = reinterpret_cast<long long*>(lds);
  u16* h0 = reinterpret_cast<u16*>(erow + 16 * MAXF);
  u16* h1 = h0 + 16 * HS;
  u16* xs = h1 + 16 * HS;              // [16][MAXF][XR]
  const int ZS = ZP + 8;
  u16* zs = xs + 16 * MAXF * XR;       // [16][ZS]
  const int Kp0 = d->bot[0].Kp;        // <= 32 (host-checked)
  const RX_GLOBAL float* dense = rx_g(d->dense);
  const RX_GLOBAL long long* cats = rx_g(d->cats);
  const RX_GLOBAL long long* offs = rx_g(d->offs);
  // (sample, column) pairs: dense features -> h0, table ids -> erow (-1: no table row)
#pragma unroll
  for (int i = 0; i < 16 * MAXF / NT; ++i) {
    const int t = tid + i * NT, sm = t / MAXF, c = t % MAXF;
    const long long src = src_row(perm, row0, r0 + sm, nvalid);
    float v = 0.f;
    if (c < d->ndense) v = dense[src * d->ld_dense + c];
    long long row = -1;
    if (c >= 1 && c < F) {
      row = offs[c - 1] + cats[src * d->ld_cats + c - 1];
      row = row < 0 ? 0 : (row >= d->emb_rows ? d->emb_rows - 1 : row);
    }
    erow[sm * MAXF + c] = row;
    if (c < Kp0) h0[sm * HS + c] = rx_f2bf(v);
  }
  __syncthreads();
  f32x4 ga[GI], gb[GI];
  {
    const RX_GLOBAL float* emb = rx_g(d->emb);
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int e = tid + i * NT, sm = e / (MAXF * CH), rem = e % (MAXF * CH), r = rem / CH, c = (rem % CH) * 8;
      const long long row = erow[sm * MAXF + r];
      ga[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      gb[i] = ga[i];
      if (row >= 0) {
        ga[i] = *reinterpret_cast<const RX_GLOBAL f32x4*>(emb + row * D + c);
        gb[i] = *reinterpret_cast<const RX_GLOBAL f32x4*>(emb + row * D + c + 4);
      }
    }
  }
  store_transposed(h0, HS, 16, Kp0, d->XdT, B, r0, 0);
  u16* hin = h0;
  u16* hout = h1;
  for (int l = 0; l < nbot; ++l) {
    const BotLayer& L = d->bot[l];
    const u16* img = L.img[p];
    const RX_GLOBAL float* bias = rx_g(L.bias);
    const int ntile = L.N >> 4, nks = L.Kp >> 5;
    if (nks == 1) {
      // K <= 32: up to 8 of this wave's tiles per burst of weight loads
      for (int t0 = wave; t0 < ntile; t0 += 32) {
        bf16x8 bfr[8];
        float bv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int t = min(t0 + 4 * j, ntile - 1);
          bfr[j] = ld16(img, (long long)(t * 16 + lr_) * L.Kp + 8 * lg);
          bv[j] = bias[t * 16 + lr_];
        }
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(hin + lr_ * HS + 8 * lg);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int t = t0 + 4 * j;
          if (t < ntile) {
            const f32x4 acc = rx_mfma16(a, bfr[j], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) hout[(4 * lg + r) * HS + t * 16 + lr_] = rx_f2bf(fmaxf(acc[r] + bv[j], 0.f));
          }
        }
      }
    } else {
      for (int t = wave; t < ntile; t += 4) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        const float bv = bias[t * 16 + lr_];
        for (int kc = 0; kc < nks; kc += 16) {
          bf16x8 bfr[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int ks = min(kc + q, nks - 1);
            bfr[q] = ld16(img, (long long)(t * 16 + lr_) * L.Kp + ks * 32 + 8 * lg);
          }
#pragma unroll
          for (int q = 0; q < 16; ++q)
            if (kc + q < nks) {
              const bf16x8 a = *reinterpret_cast<const bf16x8*>(hin + lr_ * HS + (kc + q) * 32 + 8 * lg);
              acc = rx_mfma16(a, bfr[q], acc);
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) hout[(4 * lg + r) * HS + t * 16 + lr_] = rx_f2bf(fmaxf(acc[r] + bv, 0.f));
      }
    }
    __syncthreads();
    if (L.H != nullptr) {
      const int cc = L.N >> 3;
      for (int idx = tid; idx < 16 * cc; idx += NT) {
        const int r = idx / cc, c = (idx % cc) * 8;
        rx_store16_sc1(L.H, (int)(((long long)(r0 + r) * L.N + c) * 2),
                       *reinterpret_cast<const u32x4*>(hout + r * HS + c));
      }
    }
    if (L.HT != nullptr) store_transposed(hout, HS, 16, L.N, L.HT, B, r0, 0);
    u16* t_ = hin;
    hin = hout;
    hout = t_;
    __syncthreads();
  }
  // hin: the bottom output [16][D] (ReLU'd), row 0 of every sample's interaction input; rows
  // 1..T the gathered table rows
#pragma unroll
  for (int i = 0; i < GI; ++i) {
    const int e = tid + i * NT, sm = e / (MAXF * CH), rem = e % (MAXF * CH), r = rem / CH, c = (rem % CH) * 8;
    u32x4 v;
    if (r == 0)
      v = *reinterpret_cast<const u32x4*>(hin + sm * HS + c);
    else
      v = u32x4{rx_f2bf2(ga[i][0], ga[i][1]), rx_f2bf2(ga[i][2], ga[i][3]), rx_f2bf2(gb[i][0], gb[i][1]),
                rx_f2bf2(gb[i][2], gb[i][3])};
    *reinterpret_cast<u32x4*>(xs + (sm * MAXF + r) * XR + c) = v;
    rx_store16_sc1(d->ximg, (int)((((long long)(r0 + sm) * MAXF + r) * D + c) * 2), v);
  }
  // Z staging: x0 in front, zeros everywhere else (the triangle is scattered in below)
  for (int e = tid; e < 16 * ZP; e += NT) {
    const int sm = e / ZP, c = e % ZP;
    zs[sm * ZS + c] = c < D ? hin[sm * HS + c] : (u16)0;
  }
  __syncthreads();
  for (int sm = wave; sm < 16; sm += 4) {
    const u16* X = xs + sm * MAXF * XR;
    f32x4 acc[3] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int k0 = 0; k0 < D; k0 += 32) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(X + lr_ * XR + k0 + 8 * lg);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(X + (16 + lr_) * XR + k0 + 8 * lg);
      acc[0] = rx_mfma16(a0, a0, acc[0]);
      acc[1] = rx_mfma16(a1, a0, acc[1]);
      acc[2] = rx_mfma16(a1, a1, acc[2]);
    }
#pragma unroll
    for (int blk = 0; blk < 3; ++blk) {
      const int I = blk == 0 ? 0 : 1, J = blk == 2 ? 1 : 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = I * 16 + 4 * lg + r, j = J * 16 + lr_;
        if (i < F && j < i) zs[sm * ZS + D + i * (i - 1) / 2 + j] = rx_f2bf(acc[blk][r]);
      }
    }
  }
  __syncthreads();
  const int zc = ZP >> 3;
  for (int idx = tid; idx < 16 * zc; idx += NT) {
    const int r = idx / zc, c = (idx % zc) * 8;
    rx_store16_sc1(d->Z, (int)(((long long)(r0 + r) * ZP + c) * 2), *reinterpret_cast<const u32x4*>(zs + r * ZS + c));
  }
  store_transposed(zs, ZS, 16, ZP, d->ZT, B, r0, 0);
  __syncthreads();
}

// ------------------------------------------------------------------------------------- HEAD --
// Last layer (N = 1) and BCE with logits over one 16-row block: logits, the mean-loss gradient
// dz, dA = dz w (x) relu'(A) (row-major and transposed, for the next layer's dgrad / wgrad), and
// this block's partial of the last layer's own gradient (sum dz A, sum dz, sum loss), which ONE
// workgroup reduces and applies in the next phase (head_finish). K_last <= 512, multiple of 32.
__device__ void head_block(const DlrmDesc* __restrict__ d, int rb, const long long* __restrict__ perm, long long row0,
                           int nvalid, char* lds) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int B = d->B, K = d->K_last, r0 = rb * 16;
  const int AS = K + 8, ch = K >> 3;
  u16* a = reinterpret_cast<u16*>(lds);                  // [16][AS]: A rows, then dA rows
  float* red = reinterpret_cast<float*>(a + 16 * AS);    // [4][K] per-wave partial dw
  float* rowv = red + 4 * K;                             // [16] dz, [16] loss, [16] labels
  u32x4 av[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * NT;
    av[i] = u32x4{0u, 0u, 0u, 0u};
    if (idx < 16 * ch) av[i] = rx_load16_sc1(d->A_last, (int)(((long long)(r0 + idx / ch) * K + (idx % ch) * 8) * 2));
  }
  if (tid < 16) {
    const int b = r0 + tid;
    rowv[32 + tid] = b < nvalid ? rx_g(d->labels)[src_row(perm, row0, b, nvalid) * d->ld_lab] : 0.f;
  }
  float w[8];
  {
    const RX_GLOBAL float* wl = rx_g(d->w_last);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = h * 256 + lane * 4 + j;
        w[h * 4 + j] = k < K ? wl[k] : 0.f;
      }
  }
  const float bl = rx_g(d->b_last)[0];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = tid + i * NT;
    if (idx < 16 * ch) *reinterpret_cast<u32x4*>(a + (idx / ch) * AS + (idx % ch) * 8) = av[i];
  }
  __syncthreads();
  float dw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wave * 4 + rr, b = r0 + r;
    float x[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = h * 256 + lane * 4;
      uint2 q = uint2{0u, 0u};
      if (k < K) q = *reinterpret_cast<const uint2*>(a + r * AS + k);
      x[h * 4 + 0] = __uint_as_float(q.x << 16);
      x[h * 4 + 1] = __uint_as_float(q.x & 0xffff0000u);
      x[h * 4 + 2] = __uint_as_float(q.y << 16);
      x[h * 4 + 3] = __uint_as_float(q.y & 0xffff0000u);
    }
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j] * w[j];
    acc = rx_wavesum(acc);
    const float z = acc + bl;
    const bool valid = b < nvalid;
    const float y = rowv[32 + r];
    const float g = valid ? (1.f / (1.f + expf(-z)) - y) / (float)nvalid : 0.f;
    if (lane == 0) {
      rowv[r] = g;
      rowv[16 + r] = valid ? fmaxf(z, 0.f) - z * y + log1pf(expf(-fabsf(z))) : 0.f;
      if (d->logits != nullptr) rx_g(d->logits)[b] = z;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = h * 256 + lane * 4;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dw[h * 4 + j] += g * x[h * 4 + j];
        o[j] = x[h * 4 + j] > 0.f ? g * w[h * 4 + j] : 0.f;
      }
      if (k < K) *reinterpret_cast<uint2*>(a + r * AS + k) = uint2{rx_f2bf2(o[0], o[1]), rx_f2bf2(o[2], o[3])};
    }
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = h * 256 + lane * 4 + j;
      if (k < K) red[wave * K + k] = dw[h * 4 + j];
    }
  __syncthreads();
  for (int idx = tid; idx < 16 * ch; idx += NT) {
    const int r = idx / ch, c = (idx % ch) * 8;
    rx_store16_sc1(d->dA, (int)(((long long)(r0 + r) * K + c) * 2), *reinterpret_cast<const u32x4*>(a + r * AS + c));
  }
  store_transposed(a, AS, 16, K, d->dAT, B, r0, 0);
  float* hp = d->head_part + (long long)rb * d->head_ld;
  for (int k = tid * 4; k < K + 4; k += NT * 4) {
    f32x4 v;
    if (k < K) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = red[k + j] + red[K + k + j] + red[2 * K + k + j] + red[3 * K + k + j];
    } else {
      float sd = 0.f, sl = 0.f;
      for (int r = 0; r < 16; ++r) {
        sd += rowv[r];
        sl += rowv[16 + r];
      }
      v = f32x4{sd, sl, 0.f, 0.f};
    }
    rx_store16_sc1(hp, k * 4, __builtin_bit_cast(u32x4, v));
  }
  __syncthreads();
}

// The last layer's SGD from the blocks' partials (one workgroup, the phase after HEAD).
__device__ void head_finish(const DlrmDesc* __restrict__ d, int nvalid) {
  const int K = d->K_last, nblk = d->B >> 4;
  const float lr = d->lr;
  for (int k = (int)threadIdx.x * 4; k < K + 4; k += NT * 4) {
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 v[16];
#pragma unroll
    for (int rb = 0; rb < 16; ++rb)
      v[rb] = rb < nblk ? rx_load16_sc1(d->head_part, (int)(((long long)rb * d->head_ld + k) * 4)) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int rb = 0; rb < 16; ++rb) s += __builtin_bit_cast(f32x4, v[rb]);
    if (k < K) {
      RX_GLOBAL float* w = rx_g(d->w_last);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[k + j] -= lr * s[j];
    } else {
      rx_g(d->b_last)[0] -= lr * s[0];
      const float L = s[1] / (float)nvalid;
      rx_g(d->step_loss)[0] = L;
      rx_g(d->loss_acc)[0] += (double)L;
    }
  }
}

// ------------------------------------------------------------------------------------- IBWD --
// 16 samples: dX = S X per sample; row 0 -> the bottom-MLP gradient (masked by x0 > 0), rows
// 1..T -> W_emb[row] -= lr * dX[t] (fp32 atomics: duplicate ids accumulate). Every load of the
// block (table ids, dZ rows, interaction inputs) is in flight before any is waited for.
template <int D>
__device__ void ibwd_block(const DlrmDesc* __restrict__ d, int rb, const long long* __restrict__ perm, long long row0,
                           int nvalid, char* lds) {
  constexpr int XS = MAXF + 8;
  constexpr int DS = D + 8;
  constexpr int CH = D / 8;
  constexpr int XI = 16 * MAXF * CH / NT;   // interaction-input chunks per thread
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr_ = lane & 15, lg = lane >> 4;
  const int r0 = rb * 16, F = d->F, ZP = d->ZP, B = d->B;
  const float lr = d->lr;
  float* dzr = reinterpret_cast<float*>(lds);                  // [16][ZP]
  u16* XT = reinterpret_cast<u16*>(dzr + 16 * ZP);             // [16][D][XS]
  u16* S = XT + 16 * D * XS;                                   // [4][MAXF][XS] (one per wave)
  long long* rows = reinterpret_cast<long long*>(S + 4 * MAXF * XS);   // [16][MAXF]
  u16* dm = reinterpret_cast<u16*>(rows + 16 * MAXF);          // [16][DS]
  u32x4 xv[XI];
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int e = tid + i * NT, sm = e / (MAXF * CH), rem = e % (MAXF * CH);
    xv[i] = rx_load16_sc1(d->ximg, (int)((((long long)(r0 + sm) * MAXF + rem / CH) * D + (rem % CH) * 8) * 2));
  }
  {
    const RX_GLOBAL long long* cats = rx_g(d->cats);
    const RX_GLOBAL long long* offs = rx_g(d->offs);
#pragma unroll
    for (int i = 0; i < 16 * MAXF / NT; ++i) {
      const int t = tid + i * NT, sm = t / MAXF, c = t % MAXF, b = r0 + sm;
      long long row = -1;
      if (c >= 1 && c < F && b < nvalid) {
        row = offs[c - 1] + cats[src_row(perm, row0, b, nvalid) * d->ld_cats + c - 1];
        if (row < 0 || row >= d->emb_rows) row = -1;
      }
      rows[sm * MAXF + c] = row;
    }
  }
  const int zq = ZP >> 2;
#pragma unroll 4
  for (int e = tid; e < 16 * zq; e += NT) {
    const int sm = e / zq, c = (e % zq) * 4;
    *reinterpret_cast<u32x4*>(dzr + sm * ZP + c) = rx_load16_sc1(d->dZ, (int)(((long long)(r0 + sm) * ZP + c) * 4));
  }
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int e = tid + i * NT, sm = e / (MAXF * CH), rem = e % (MAXF * CH), r = rem / CH, c = (rem % CH) * 8;
    u16* Xw = XT + sm * D * XS;
    float f[8];
    unpack8(xv[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) Xw[(c + j) * XS + r] = rx_f2bf(f[j]);
  }
  __syncthreads();
  u16* Sw = S + wave * MAXF * XS;
  for (int k = 0; k < 4; ++k) {
    const int sl = wave * 4 + k;
    const float* zr = dzr + sl * ZP;
    const u16* Xw = XT + sl * D * XS;
    for (int e = lane; e < MAXF * MAXF; e += 64) {
      const int i = e / MAXF, j = e % MAXF;
      float v = 0.f;
      if (i < F && j < F && i != j) {
        const int hi = i > j ? i : j, lo = i > j ? j : i;
        v = zr[D + hi * (hi - 1) / 2 + lo];
      }
      Sw[i * XS + j] = rx_f2bf(v);
    }
    __syncthreads();
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(Sw + (mi * 16 + lr_) * XS + 8 * lg);
#pragma unroll
      for (int nd = 0; nd < D / 16; ++nd) {
        const bf16x8 bb = *reinterpret_cast<const bf16x8*>(Xw + (nd * 16 + lr_) * XS + 8 * lg);
        const f32x4 c = rx_mfma16(a, bb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = mi * 16 + 4 * lg + r, dd = nd * 16 + lr_;
          if (i == 0) {
            const float x0 = rx_bf2f(Xw[dd * XS]);
            dm[sl * DS + dd] = rx_f2bf(x0 > 0.f ? c[r] + zr[dd] : 0.f);
          } else if (i < F) {
            const long long row = rows[sl * MAXF + i];
            if (row >= 0)
              __hip_atomic_fetch_add(rx_g(d->emb) + row * D + dd, -lr * c[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
      }
    }
    __syncthreads();
  }
  const int cc = D / 8;
  for (int idx = tid; idx < 16 * cc; idx += NT) {
    const int r = idx / cc, c = (idx % cc) * 8;
    rx_store16_sc1(d->dmlp, (int)(((long long)(r0 + r) * D + c) * 2), *reinterpret_cast<const u32x4*>(dm + r * DS + c));
  }
  store_transposed(dm, DS, 16, D, d->dmlpT, B, r0, 0);
  __syncthreads();
}

template <int D>
__global__ __launch_bounds__(NT) void dlrm_step_kernel(const DlrmDesc* __restrict__ d, const long long* __restrict__ perm,
                                                       long long row0, int nvalid) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int G = d->G;
  unsigned* ctl = d->ctl;
  const int p = (int)(rx_ld_sc1u(ctl + CTL_PAR) & 1u);
  const float lr = d->lr;
  int k = 0;
  const int nph = d->nph, nblk = d->B >> 4;
  unsigned long long* stamps = blockIdx.x == 0 && threadIdx.x == 0 ? d->stamps : nullptr;
  if (stamps != nullptr) stamps[0] = wall_clock64();
  bool head_done = false;
  for (int ph = 0; ph < nph; ++ph) {
    const Phase& P = d->ph[ph];
    if (head_done) {
      // the phase after HEAD: the last workgroup applies the last layer's SGD
      if (blockIdx.x == G - 1) head_finish(d, nvalid);
      head_done = false;
    }
    if (P.kind == PH_GEMM) {
      gemm_phase(P, p, lr, G, lds);
    } else if (P.kind == PH_BOTTOM) {
      for (int rb = blockIdx.x; rb < nblk; rb += G) bottom_block<D>(d, p, rb, perm, row0, nvalid, lds);
    } else if (P.kind == PH_HEAD) {
      for (int rb = blockIdx.x; rb < nblk; rb += G) head_block(d, rb, perm, row0, nvalid, lds);
      head_done = true;
    } else {
      // IBWD: blocks dealt from the top of the grid down
      for (int rb = (int)(G - 1 - blockIdx.x); rb < nblk; rb += G) ibwd_block<D>(d, rb, perm, row0, nvalid, lds);
    }
    if (ph + 1 < nph && !rx_grid_barrier(ctl, G, ++k, d->ticks)) break;
    if (stamps != nullptr) stamps[ph + 1] = wall_clock64();
  }
  rx_grid_finish(ctl, G, CTL_PAR);
}

template <int D>
int occupancy(int lds, int* per_cu) {
  return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, reinterpret_cast<const void*>(&dlrm_step_kernel<D>),
                                                           NT, lds);
}

}  // namespace

extern "C" {

int rx_dlrm_desc_size() { return (int)sizeof(DlrmDesc); }
int rx_dlrm_phase_size() { return (int)sizeof(Phase); }
int rx_dlrm_ctl_words() { return 8; }
int rx_dlrm_err_index() { return RX_MW_ERR; }
int rx_dlrm_parity_index() { return CTL_PAR; }
unsigned long long rx_dlrm_ticks(double seconds) {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0ull;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0ull;
  return (unsigned long long)(seconds * khz * 1000.0);
}
int rx_dlrm_gspec_size() { return (int)sizeof(GSpec); }
int rx_dlrm_max_phases() { return MAXPH; }

// 0 when G workgroups with `lds` bytes of dynamic LDS are co-resident, -4 if not, else a HIP error.
int rx_dlrm_resident(int D, int lds, int G) {
  int dev = 0, cus = 0, per_cu = 0;
  RX_CHECK(hipGetDevice(&dev));
  RX_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (D != 32) return -1;
  if (lds > 65536)
    RX_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&dlrm_step_kernel<32>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  RX_CHECK((hipError_t)occupancy<32>(lds, &per_cu));
  return (long long)per_cu * cus >= G ? 0 : -4;
}

// nsteps consecutive steps over rows perm[row0 + j * B ...]; the last step has nvalid_last valid
// rows (<= B), every other step B. d_dev: the descriptor in device memory; G / lds as checked by
// rx_dlrm_resident.
int rx_dlrm_train_steps(const void* d_dev, int D, int B, int G, int lds, const long long* perm, long long row0,
                        int nsteps, int nvalid_last, hipStream_t s) {
  if (D != 32 || B <= 0 || (B & 31) || nvalid_last <= 0 || nvalid_last > B) return -1;
  const DlrmDesc* d = reinterpret_cast<const DlrmDesc*>(d_dev);
  for (int j = 0; j < nsteps; ++j) {
    const int nv = j + 1 == nsteps ? nvalid_last : B;
    hipLaunchKernelGGL(dlrm_step_kernel<32>, dim3(G), dim3(NT), lds, s, d, perm, row0 + (long long)j * B, nv);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
