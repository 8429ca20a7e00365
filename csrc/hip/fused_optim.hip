// Multi-tensor optimizer and loss kernels for the torch-loop engine (models the fused MLP
// kernel does not cover: DLRM, the stroke tutorial's NET_Model, user MLPs under DDP).
//
// Reference: the DLRM notebook trains with torch.optim.SGD + BCEWithLogitsLoss
// (examples/pytorch_dlrm.ipynb cells 9, 14); eager PyTorch runs that as one add kernel per
// parameter tensor, a separate pass that rebuilds the bf16 operand images of the fused MFMA
// towers (csrc/hip/linear_act.hip) after every update, and ~6 elementwise / reduction kernels
// for the loss and its gradient.
//
//   mt_sgd_kernel   one launch for up to kMtMax parameter tensors: weight decay, momentum
//                   (+ nesterov, dampening), maximize, the update -- and, for weights a fused
//                   tower reads, the bf16 image written from the fresh fp32 value in the same
//                   pass (no re-read of the weight)
//   mt_adam_kernel  the same for Adam / AdamW (user loops: Horovod's DistributedOptimizer)
//   bce_fwd_kernel  mean binary cross-entropy with logits (one workgroup, LDS reduction)
//   bce_bwd_kernel  its gradient (sigmoid(x) - y) * go / n straight from the saved operands
#include "rx_common.h"

namespace {

constexpr int kMtMax = 24;

struct MtSgd {
  int n;          // tensors in this launch
  int first;      // 1: momentum buffers are fresh (buf = g), as torch's first step
  float lr, wd, momentum, dampening;
  int nesterov, maximize;
  float* p[kMtMax];
  const float* g[kMtMax];
  float* buf[kMtMax];   // momentum buffers (null without momentum)
  u16* img[kMtMax];     // bf16 image of p (null: none)
  long long len[kMtMax];
};

__global__ __launch_bounds__(256) void mt_sgd_kernel(MtSgd a) {
  const int t = blockIdx.y;
  float* __restrict__ p = a.p[t];
  const float* __restrict__ g = a.g[t];
  float* __restrict__ mb = a.buf[t];
  u16* __restrict__ img = a.img[t];
  const long long n = a.len[t];
  // two elements per thread per pass (one packed bf16x2 image store)
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 2; i < n;
       i += (long long)gridDim.x * blockDim.x * 2) {
    const int m = i + 1 < n ? 2 : 1;
    float out[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k >= m) break;
      const long long j = i + k;
      const float pv = p[j];
      float d = a.maximize ? -g[j] : g[j];
      if (a.wd != 0.f) d += a.wd * pv;
      if (mb != nullptr) {
        const float b = a.first ? d : a.momentum * mb[j] + (1.f - a.dampening) * d;
        mb[j] = b;
        d = a.nesterov ? d + a.momentum * b : b;
      }
      out[k] = pv - a.lr * d;
      p[j] = out[k];
    }
    if (img != nullptr) {
      if (m == 2)
        *reinterpret_cast<uint32_t*>(img + i) = rx_f2bf2(out[0], out[1]);
      else
        img[i] = rx_f2bf(out[0]);
    }
  }
}

// Adam / AdamW over up to kMtMax fp32 tensors in one launch (torch.optim.Adam / AdamW semantics,
// amsgrad off): torch's default (foreach) implementation runs ~10 multi-tensor kernels per step
// for this, its single-tensor one ~6 per parameter. Per tensor the host passes the step's
// element-independent factors from that tensor's own step count: nlr_bc1 = -lr / (1 - b1^t),
// rs_bc2 = 1 / sqrt(1 - b2^t). Four elements per thread per pass (16-B accesses when the tensor
// allows them).
struct MtAdam {
  int n;           // tensors in this launch
  int adamw;       // 1: decoupled weight decay (p *= 1 - lr wd), 0: L2 (g += wd p)
  int maximize;
  float lr, b1, b2, eps, wd;
  float nlr_bc1[kMtMax];
  float rs_bc2[kMtMax];
  float* p[kMtMax];
  const float* g[kMtMax];
  float* m[kMtMax];
  float* v[kMtMax];
  long long len[kMtMax];
};

__device__ __forceinline__ void adam_elem(const MtAdam& a, float nlr_bc1, float rs_bc2, float& p, float g, float& m,
                                          float& v) {
  if (a.maximize) g = -g;
  if (a.adamw) p *= 1.f - a.lr * a.wd;
  else if (a.wd != 0.f) g = fmaf(a.wd, p, g);
  m = fmaf(1.f - a.b1, g - m, m);                 // torch: exp_avg.lerp_(grad, 1 - beta1)
  v = fmaf(a.b2, v, (1.f - a.b2) * g * g);        // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float den = sqrtf(v) * rs_bc2 + a.eps;    // exp_avg_sq.sqrt() / sqrt(bc2) + eps
  p = fmaf(nlr_bc1, m / den, p);                  // p.addcdiv_(exp_avg, denom, -lr / bc1)
}

__global__ __launch_bounds__(256) void mt_adam_kernel(MtAdam a) {
  const int t = blockIdx.y;
  float* __restrict__ p = a.p[t];
  const float* __restrict__ g = a.g[t];
  float* __restrict__ m = a.m[t];
  float* __restrict__ v = a.v[t];
  const long long n = a.len[t];
  const float f1 = a.nlr_bc1[t], f2 = a.rs_bc2[t];
  const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0;
  for (long long i = (blockIdx.x * (long long)blockDim.x + threadIdx.x) * 4; i < n;
       i += (long long)gridDim.x * blockDim.x * 4) {
    if (vec && i + 4 <= n) {
      f32x4 pv = *reinterpret_cast<const f32x4*>(p + i), gv = *reinterpret_cast<const f32x4*>(g + i);
      f32x4 mv = *reinterpret_cast<const f32x4*>(m + i), vv = *reinterpret_cast<const f32x4*>(v + i);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float pk = pv[k], mk = mv[k], vk = vv[k];
        adam_elem(a, f1, f2, pk, gv[k], mk, vk);
        pv[k] = pk;
        mv[k] = mk;
        vv[k] = vk;
      }
      *reinterpret_cast<f32x4*>(p + i) = pv;
      *reinterpret_cast<f32x4*>(m + i) = mv;
      *reinterpret_cast<f32x4*>(v + i) = vv;
    } else {
      for (long long j = i; j < i + 4 && j < n; ++j) {
        float pj = p[j], mj = m[j], vj = v[j];
        adam_elem(a, f1, f2, pj, g[j], mj, vj);
        p[j] = pj;
        m[j] = mj;
        v[j] = vj;
      }
    }
  }
}

// softplus-form BCE with logits, stable for either sign of x:
//   l(x, y) = max(x, 0) - x * y + log1p(exp(-|x|))
__device__ __forceinline__ float bce_term(float x, float y) {
  return fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
}

// one workgroup: loss[0] = mean over n of l(x, y)
__global__ __launch_bounds__(1024) void bce_fwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                       long long n, float* __restrict__ loss) {
  float s = 0.f;
  for (long long i = threadIdx.x; i < n; i += blockDim.x) s += bce_term(x[i], y[i]);
  s = rx_wavesum(s);
  __shared__ float part[16];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) part[w] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k];
    loss[0] = t / (float)n;
  }
}

// dx = (sigmoid(x) - y) * go[0] / n
__global__ __launch_bounds__(256) void bce_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                      const float* __restrict__ go, long long n,
                                                      float* __restrict__ dx) {
  const float sc = go[0] / (float)n;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = x[i];
    const float sig = 1.f / (1.f + __expf(-v));
    dx[i] = (sig - y[i]) * sc;
  }
}

}  // namespace

extern "C" {

int rx_mt_sgd_size() { return (int)sizeof(MtSgd); }
int rx_mt_sgd_max() { return kMtMax; }

int rx_mt_sgd(const MtSgd* a, hipStream_t stream) {
  if (a->n <= 0) return 0;
  if (a->n > kMtMax) return -1;
  long long mx = 0;
  for (int t = 0; t < a->n; ++t) mx = a->len[t] > mx ? a->len[t] : mx;
  long long bx = (mx / 2 + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
  hipLaunchKernelGGL(mt_sgd_kernel, dim3((unsigned)bx, (unsigned)a->n), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

int rx_mt_adam_size() { return (int)sizeof(MtAdam); }

int rx_mt_adam(const MtAdam* a, hipStream_t stream) {
  if (a->n <= 0) return 0;
  if (a->n > kMtMax) return -1;
  long long mx = 0;
  for (int t = 0; t < a->n; ++t) mx = a->len[t] > mx ? a->len[t] : mx;
  long long bx = (mx / 4 + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
  hipLaunchKernelGGL(mt_adam_kernel, dim3((unsigned)bx, (unsigned)a->n), dim3(256), 0, stream, *a);
  return (int)hipGetLastError();
}

int rx_bce_logits_fwd(const float* x, const float* y, long long n, float* loss, hipStream_t stream) {
  if (n <= 0) return -1;
  hipLaunchKernelGGL(bce_fwd_kernel, dim3(1), dim3(1024), 0, stream, x, y, n, loss);
  return (int)hipGetLastError();
}

int rx_bce_logits_bwd(const float* x, const float* y, const float* go, long long n, float* dx, hipStream_t stream) {
  if (n <= 0) return -1;
  long long bx = (n + 255) / 256;
  bx = bx > 1024 ? 1024 : bx;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3((unsigned)bx), dim3(256), 0, stream, x, y, go, n, dx);
  return (int)hipGetLastError();
}

}  // extern "C"
