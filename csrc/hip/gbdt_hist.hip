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
//   g, h  [n]    fp32   gradient / hessian;
//   hist  [K][F][B][2] fp64, zeroed by the caller, accumulated here.
//
// Grid: x = row chunks, y = feature, z = node group (KG nodes). Each workgroup privatises the
// KG x B (g, h) slice of its feature in LDS (fp64 LDS atomics, ds_add_f64), then flushes the
// non-zero entries with global fp64 atomics. Chunks are sized so the whole launch is ~2048
// workgroups (>> 256 CUs) while keeping the global flush traffic at a few entries per row chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GH_THREADS 256
#define GH_LDS_BYTES 65536

#define GH_UNROLL 4

__global__ __launch_bounds__(GH_THREADS) void gbdt_hist_kernel(const int16_t* __restrict__ binsT,
                                                              const long long* __restrict__ pos,
                                                              const float* __restrict__ g,
                                                              const float* __restrict__ h, double* __restrict__ hist,
                                                              long long n, int F, int B, int K, int KG,
                                                              long long rows_per_chunk) {
  // Two planes (sum g | sum h) rather than interleaved pairs: a double at index 2b maps onto
  // only 16 distinct bank pairs of the 64-bank LDS, index b onto 32.
  extern __shared__ double sh[];
  const int tid = threadIdx.x;
  const int f = blockIdx.y;
  const int k0 = blockIdx.z * KG;
  const int kg = min(KG, K - k0);
  const int plane = kg * B;
  double* shg = sh;
  double* shh = sh + plane;
  for (int i = tid; i < 2 * plane; i += GH_THREADS) sh[i] = 0.0;
  __syncthreads();

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
    float gv[GH_UNROLL], hv[GH_UNROLL];
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      const long long r = base + tid + u * GH_THREADS;
      const unsigned kk = (unsigned)(p[u] - k0);
      slot[u] = 0xffffffffu;
      gv[u] = 0.f;
      hv[u] = 0.f;
      if (p[u] >= 0 && kk < (unsigned)kg) {
        const unsigned b = (unsigned)(unsigned short)col[r];
        if (b < (unsigned)B) slot[u] = kk * B + b;
        gv[u] = g[r];
        hv[u] = h[r];
      }
    }
#pragma unroll
    for (int u = 0; u < GH_UNROLL; ++u) {
      if (slot[u] != 0xffffffffu) {
        atomicAdd(shg + slot[u], (double)gv[u]);
        atomicAdd(shh + slot[u], (double)hv[u]);
      }
    }
  }
  __syncthreads();

  // node kk of this feature: hist[((k0 + kk) * F + f) * B * 2 + 2 * b + c]
  const bool owner = gridDim.x == 1;  // single row chunk: this workgroup owns the slice outright
  for (int i = tid; i < 2 * plane; i += GH_THREADS) {
    const int c = i >= plane;
    const int e = i - c * plane;
    const int kk = e / B, b = e - kk * B;
    double* dst = hist + ((long long)(k0 + kk) * F + f) * (2 * B) + 2 * b + c;
    const double v = sh[i];
    if (owner)
      *dst = v;
    else if (v != 0.0)
      unsafeAtomicAdd(dst, v);
  }
}

static inline long long gh_cdiv(long long a, long long b) { return (a + b - 1) / b; }

extern "C" {

// Node-group size that keeps the LDS slice within GH_LDS_BYTES (0: B too large for one node).
int rx_gbdt_hist_group(int K, int B) {
  const long long per_node = (long long)B * 2 * sizeof(double);
  if (per_node > GH_LDS_BYTES) return 0;
  const int kg = (int)(GH_LDS_BYTES / per_node);
  return kg < K ? kg : K;
}

int rx_gbdt_hist(const int16_t* binsT, const long long* pos, const float* g, const float* h, double* hist,
                 long long n, int F, int B, int K, hipStream_t s) {
  if (n <= 0 || F <= 0 || K <= 0) return 0;
  const int KG = rx_gbdt_hist_group(K, B);
  if (KG <= 0) return -1;
  const int groups = (K + KG - 1) / KG;
  const long long want = 2048 / ((long long)F * groups);
  long long chunks = want < 1 ? 1 : want;
  const long long max_chunks = gh_cdiv(n, 2048);  // at least 2048 rows per workgroup
  if (chunks > max_chunks) chunks = max_chunks;
  if (chunks > 65535) chunks = 65535;
  const long long rpc = gh_cdiv(n, chunks);
  chunks = gh_cdiv(n, rpc);
  const size_t lds = (size_t)KG * B * 2 * sizeof(double);
  hipLaunchKernelGGL(gbdt_hist_kernel, dim3((unsigned)chunks, (unsigned)F, (unsigned)groups), dim3(GH_THREADS), lds, s,
                     binsT, pos, g, h, hist, n, F, B, K, KG, rpc);
  return (int)hipGetLastError();
}

}  // extern "C"
