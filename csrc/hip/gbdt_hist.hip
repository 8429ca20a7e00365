// Gradient-histogram build for the histogram GBDT behind XGBoostEstimator (gfx950).
//
// The reference boosts through xgboost-ray (python/raydp/xgboost/estimator.py:54-81), whose
// `hist` tree method spends its time building per-node (gradient, hessian) histograms over the
// quantised feature matrix, then all-reduces them (Rabit). Here that build is one kernel per
// tree level; the all-reduce stays on torch.distributed (RCCL over xGMI on MI355X).
//
// Layout
//   binsT [F][n] int16  column-major bin ids (0 = missing), transposed once per training run so
//                       a wavefront reads 64 consecutive rows of one feature (128 B, coalesced);
//   pos   [n]    int64  row -> node index within the level (-1: row sits in a finished leaf);
//   gq,hq [n]    int32  gradient / hessian in fixed point (power-of-two scale per tree, chosen by
//                       the host from the global max |g|, |h| so |q| <= 2^30);
//   hist  [K][F][B][2] int64, zeroed by the caller, accumulated here.
//
// Fixed-point (integer) accumulation is what makes the histogram exact: integer adds are
// associative, so the result does not depend on the order in which LDS and global atomics land
// (run-to-run reproducible), equals the CPU path's index_add_ bit for bit, survives the
// cross-rank all-reduce and the sibling subtraction without rounding. XGBoost's GPU hist uses the
// same idea (quantised gradient pairs).
//
// Grid: x = row chunks, y = feature, z = node group (KG nodes). Each workgroup privatises the
// KG x B (g, h) slice of its feature in LDS (64-bit LDS atomics, ds_add_u64), then flushes the
// non-zero entries with global 64-bit atomics. Chunks are sized so the whole launch is ~2048
// workgroups (>> 256 CUs) while keeping the global flush traffic at a few entries per row chunk.
// When one node's slice does not fit in LDS (B > 4096 bins) the kernel runs in global mode: the
// same loop with its atomics aimed straight at the output.
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

#define GH_THREADS 256
#define GH_LDS_BYTES 65536

#define GH_UNROLL 4

typedef unsigned long long gh_u64;

__global__ __launch_bounds__(GH_THREADS) void gbdt_hist_kernel(const int16_t* __restrict__ binsT,
                                                              const long long* __restrict__ pos,
                                                              const int* __restrict__ gq,
                                                              const int* __restrict__ hq, long long* __restrict__ hist,
                                                              long long n, int F, int B, int K, int KG,
                                                              long long rows_per_chunk) {
  // Two planes (sum g | sum h) rather than interleaved pairs: an 8-byte word at index 2b maps
  // onto only 16 distinct bank pairs of the 64-bank LDS, index b onto 32.
  extern __shared__ gh_u64 sh[];
  const int tid = threadIdx.x;
  const int f = blockIdx.y;
  const bool global_mode = KG == 0;
  const int k0 = global_mode ? 0 : blockIdx.z * KG;
  const int kg = global_mode ? K : min(KG, K - k0);
  const int plane = kg * B;
  gh_u64* shg = sh;
  gh_u64* shh = sh + plane;
  if (!global_mode) {
    for (int i = tid; i < 2 * plane; i += GH_THREADS) sh[i] = 0ull;
    __syncthreads();
  }
  gh_u64* const gout = reinterpret_cast<gh_u64*>(hist);

  const long long r0 = (long long)blockIdx.x * rows_per_chunk;
  const long long r1 = min(n, r0 + rows_per_chunk);
  const int16_t* col = binsT + (long long)f * n;
  // GH_UNROLL rows per thread per trip: all loads of a trip are issued before the first LDS
  // atomic, so each wave keeps several HBM requests in flight instead of one.
  for (long long base = r0; base < r1; base += (long long)GH_THREADS * GH_UNROLL) {
    long long p[GH_UNROLL];
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      const long long r = base + tid + u * GH_THREADS;
      p[u] = r < r1 ? pos[r] : -1;
    }
    unsigned slot[GH_UNROLL];
    long long gv[GH_UNROLL], hv[GH_UNROLL];
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      const long long r = base + tid + u * GH_THREADS;
      const unsigned kk = (unsigned)(p[u] - k0);
      slot[u] = 0xffffffffu;
      gv[u] = 0;
      hv[u] = 0;
      if (p[u] >= 0 && kk < (unsigned)kg) {
        const unsigned b = (unsigned)(unsigned short)col[r];
        if (b < (unsigned)B) slot[u] = kk * B + b;
        gv[u] = gq[r];
        hv[u] = hq[r];
      }
    }
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      if (slot[u] == 0xffffffffu) continue;
      if (global_mode) {
        const unsigned kk = slot[u] / (unsigned)B, b = slot[u] - kk * (unsigned)B;
        gh_u64* dst = gout + ((long long)kk * F + f) * (2 * B) + 2 * b;
        atomicAdd(dst, (gh_u64)gv[u]);
        atomicAdd(dst + 1, (gh_u64)hv[u]);
      } else {
        atomicAdd(shg + slot[u], (gh_u64)gv[u]);
        atomicAdd(shh + slot[u], (gh_u64)hv[u]);
      }
    }
  }
  if (global_mode) return;
  __syncthreads();

  // node kk of this feature: hist[((k0 + kk) * F + f) * B * 2 + 2 * b + c]
  const bool owner = gridDim.x == 1;  // single row chunk: this workgroup owns the slice outright
  for (int i = tid; i < 2 * plane; i += GH_THREADS) {
    const int c = i >= plane;
    const int e = i - c * plane;
    const int kk = e / B, b = e - kk * B;
    gh_u64* dst = gout + ((long long)(k0 + kk) * F + f) * (2 * B) + 2 * b + c;
    const gh_u64 v = sh[i];
    if (owner)
      *dst = v;
    else if (v != 0ull)
      atomicAdd(dst, v);
  }
}

// ---------------------------------------------------------------------------- split search ----
// One wavefront per (node, feature): the B-1 candidate thresholds (bins 1..t go left) are split
// into contiguous runs per lane; a wave-wide exclusive scan of the run sums gives every lane its
// starting prefix, then each lane walks its run evaluating XGBoost's gain for both default
// directions of missing values (dl = 1: bin 0 goes left). Replaces the cumsum + ~40 elementwise
// kernels + 2 reductions of the tensor formulation with one launch per level.
//
// Prefix sums are int64 (exact), so every (L, R) pair is the same integer the CPU path's cumsum
// produces; converted with the per-tree scale and pushed through the gain formula in the same
// operation order with FP contraction off, the gains are bit-identical to the CPU path's, and
// ties resolve the same way (lowest t, then lowest feature on the host). A candidate is invalid
// (never chosen) unless both children have hessian >= min_child_weight and H + lambda > 0, so a
// zero-hessian child with lambda = 0 cannot produce a NaN gain.
// out[(k * F + f) * 4 + {0,1,2,3}] = {gain dl=1, t dl=1, gain dl=0, t dl=0}; ties keep the lowest t.
__device__ __forceinline__ double gh_soft(double g, double alpha) {
  if (alpha <= 0.0) return g;
  const double a = fabs(g) - alpha;
  return a > 0.0 ? copysign(a, g) : 0.0;
}

__device__ __forceinline__ void gh_best_reduce(double& gain, int& t) {
  for (int off = 32; off > 0; off >>= 1) {
    const double og = __shfl_xor(gain, off, 64);
    const int ot = __shfl_xor(t, off, 64);
    if (og > gain || (og == gain && ot < t)) {
      gain = og;
      t = ot;
    }
  }
}

__global__ __launch_bounds__(64) void gbdt_split_kernel(const long long* __restrict__ hist,
                                                       const long long* __restrict__ tot,
                                                       const int* __restrict__ ncuts,
                                                       const unsigned char* __restrict__ fmask, double* __restrict__ out,
                                                       int F, int B, double inv_g, double inv_h, double lam,
                                                       double alpha, double mcw) {
  const int kf = blockIdx.x;
  const int k = kf / F, f = kf - k * F;
  const int lane = threadIdx.x;
  double* o = out + (long long)kf * 4;
  if (fmask != nullptr && !fmask[f]) {
    if (lane == 0) {
      o[0] = -1.0; o[1] = 0.0; o[2] = -1.0; o[3] = 0.0;
    }
    return;
  }
  const long long* hf = hist + (long long)kf * B * 2;
  const int nt = B - 1;                 // thresholds t = 0 .. B-2 (bins 1..t+1 go left)
  const int valid_t = ncuts[f];         // t must index a real cut
  const int run = (nt + 63) / 64;
  const int t0 = min(lane * run, nt), t1 = min(t0 + run, nt);
  long long sg = 0, sh = 0;
  for (int t = t0; t < t1; ++t) {
    sg += hf[2 * (t + 1)];
    sh += hf[2 * (t + 1) + 1];
  }
  // inclusive scan over lanes, then exclusive = inclusive - own (exact in integers)
  long long ig = sg, ih = sh;
  for (int off = 1; off < 64; off <<= 1) {
    const long long ug = __shfl_up(ig, off, 64), uh = __shfl_up(ih, off, 64);
    if (lane >= off) {
      ig += ug;
      ih += uh;
    }
  }
  long long cg = ig - sg, ch = ih - sh;
  const long long Gq = tot[2 * k], Hq = tot[2 * k + 1];
  const long long mg = hf[0], mh = hf[1];
  const double G = (double)Gq * inv_g, H = (double)Hq * inv_h;
  const double sG = gh_soft(G, alpha);
  const double parent = sG * sG / (H + lam);
  double best1 = -1.0, best0 = -1.0;
  int bt1 = 0x7fffffff, bt0 = 0x7fffffff;
  for (int t = t0; t < t1; ++t) {
    cg += hf[2 * (t + 1)];
    ch += hf[2 * (t + 1) + 1];
    if (t >= valid_t) continue;
#pragma unroll
    for (int dl = 1; dl >= 0; --dl) {
      const long long Lgq = cg + (dl ? mg : 0), Lhq = ch + (dl ? mh : 0);
      const double Lg = (double)Lgq * inv_g, Lh = (double)Lhq * inv_h;
      const double Rg = (double)(Gq - Lgq) * inv_g, Rh = (double)(Hq - Lhq) * inv_h;
      if (!(Lh >= mcw && Rh >= mcw && Lh + lam > 0.0 && Rh + lam > 0.0)) continue;
      const double sl = gh_soft(Lg, alpha), sr = gh_soft(Rg, alpha);
      const double gain = sl * sl / (Lh + lam) + sr * sr / (Rh + lam) - parent;
      if (dl) {
        if (gain > best1) { best1 = gain; bt1 = t; }
      } else {
        if (gain > best0) { best0 = gain; bt0 = t; }
      }
    }
  }
  gh_best_reduce(best1, bt1);
  gh_best_reduce(best0, bt0);
  if (lane == 0) {
    o[0] = best1; o[1] = bt1 == 0x7fffffff ? 0.0 : (double)bt1;
    o[2] = best0; o[3] = bt0 == 0x7fffffff ? 0.0 : (double)bt0;
  }
}

// ------------------------------------------------------------------------- row partition ----
// Moves every active row one level down in place: node table tab[k] = {remap, feature, split
// bin, default_left, tree node id} (remap < 0: node k became a leaf, its rows record the leaf id
// and leave the active set). Replaces ~10 gather/where kernels per level of the tensor version.
__global__ __launch_bounds__(256) void gbdt_partition_kernel(const int16_t* __restrict__ binsT,
                                                            const long long* __restrict__ tab, long long* __restrict__ pos,
                                                            long long* __restrict__ leaf, long long n, int K) {
  const long long r = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const long long p = pos[r];
  if (p < 0 || p >= K) return;
  const long long* t = tab + p * 5;
  const long long rm = t[0];
  if (rm < 0) {
    leaf[r] = t[4];
    pos[r] = -1;
    return;
  }
  const int b = (int)(unsigned short)binsT[t[1] * n + r];
  const bool left = b == 0 ? t[3] != 0 : b <= t[2];
  pos[r] = rm + (left ? 0 : 1);
}

static inline long long gh_cdiv(long long a, long long b) { return (a + b - 1) / b; }

extern "C" {

// Node-group size that keeps the LDS slice within GH_LDS_BYTES (0: B too large for one node;
// the histogram then runs in global-atomic mode).
int rx_gbdt_hist_group(int K, int B) {
  const long long per_node = (long long)B * 2 * sizeof(gh_u64);
  if (per_node > GH_LDS_BYTES) return 0;
  const int kg = (int)(GH_LDS_BYTES / per_node);
  return kg < K ? kg : K;
}

int rx_gbdt_hist(const int16_t* binsT, const long long* pos, const int* gq, const int* hq, long long* hist,
                 long long n, int F, int B, int K, hipStream_t s) {
  if (n <= 0 || F <= 0 || K <= 0) return 0;
  if (B <= 0 || B > 32768) return -1;
  const int KG = rx_gbdt_hist_group(K, B);
  const int groups = KG > 0 ? (K + KG - 1) / KG : 1;
  const long long want = 2048 / ((long long)F * groups);
  long long chunks = want < 1 ? 1 : want;
  const long long max_chunks = gh_cdiv(n, 2048);  // at least 2048 rows per workgroup
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks > 65535) chunks = 65535;
  const long long rpc = gh_cdiv(n, chunks);
  chunks = gh_cdiv(n, rpc);
  const size_t lds = KG > 0 ? (size_t)KG * B * 2 * sizeof(gh_u64) : 0;
  hipLaunchKernelGGL(gbdt_hist_kernel, dim3((unsigned)chunks, (unsigned)F, (unsigned)groups), dim3(GH_THREADS), lds, s,
                     binsT, pos, gq, hq, hist, n, F, B, K, KG, rpc);
  return (int)hipGetLastError();
}

// Best split per (node, feature) for both default directions (see gbdt_split_kernel).
int rx_gbdt_split(const long long* hist, const long long* tot, const int* ncuts, const unsigned char* fmask,
                  double* out, int K, int F, int B, double inv_g, double inv_h, double lam, double alpha, double mcw,
                  hipStream_t s) {
  if (K <= 0 || F <= 0 || B < 2) return K <= 0 || F <= 0 ? 0 : -1;
  hipLaunchKernelGGL(gbdt_split_kernel, dim3((unsigned)(K * F)), dim3(64), 0, s, hist, tot, ncuts, fmask, out, F, B,
                     inv_g, inv_h, lam, alpha, mcw);
  return (int)hipGetLastError();
}

// One level of row partitioning (see gbdt_partition_kernel); pos/leaf are updated in place.
int rx_gbdt_partition(const int16_t* binsT, const long long* tab, long long* pos, long long* leaf, long long n, int K,
                      hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gbdt_partition_kernel, dim3((unsigned)gh_cdiv(n, 256)), dim3(256), 0, s, binsT, tab, pos, leaf, n,
                     K);
  return (int)hipGetLastError();
}

}  // extern "C"
