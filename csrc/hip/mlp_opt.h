// Optimizer descriptor and element update of the fused MLP trainer, shared by the
// ahead-of-time build (fused_mlp.hip) and the per-model specialised build (mlp_jit.py), whose
// persistent epoch kernel (mlp_persist.h) updates parameters inside the training launch.
//
// Reference role: the torch.optim.Adam / AdamW / SGD step of the NYC / stroke models
// (python/raydp/torch/estimator.py:286-288, examples/pytorch_nyctaxi.py:96), same update
// formulas as torch (bias-corrected Adam, decoupled AdamW decay, SGD momentum/dampening/nesterov).
#pragma once
#include "rx_common.h"

#pragma clang fp contract(off)  // see mlp_core.h

#ifndef RX_MAXL
#define RX_MAXL 8
#endif
#define RX_MAXSEG (4 * RX_MAXL)

struct OptSeg {
  int start, len, kind;  // kind 1: linear weight (needs bf16 images)
  int out, in, in_k, out_k;
  int in_n, out_n;       // rows of the exported X^T / G^T of this layer (wgrad_mode 1)
  int xg_off, gg_off;    // their bf16 offsets in the activation area
  u16* W;
  u16* Wt;
};
struct OptDesc {
  int nseg, total;
  int algo;  // 0 adam, 1 adamw, 2 sgd
  float b1, b2, eps, wd, momentum, dampening;
  int nesterov, maximize;
  OptSeg seg[RX_MAXSEG];
  int act_off;     // float offset of the activation area in the gradient buffer / xGMI slot
  int act_floats;  // its size
  int bp;          // padded batch rows (K of the optimizer-side wgrad)
  int wgrad_mode;  // mirrors MlpDesc::wgrad_mode
  int ps_l0_inline; // persistent epoch: layer 0's weight is updated by the step workgroup itself
                    // (MlpDesc::w0s_lds_off), no optimizer workgroups for its segment
};

// One element: p, m, v in registers (the persistent kernel keeps them there for a whole epoch).
// Every multiply-add is an explicit fmaf: left to the compiler, contraction depends on the
// inlining context, and the same update would round differently in the launch-per-step
// optimizer kernel and in the persistent kernel (the two must agree bit for bit).
// `o`: the runtime descriptor, or (specialised kernels) an empty struct whose hyperparameters are
// static constexpr members -- the branches on the algorithm fold away. nlr_bc1 = -(lr / bc1) and
// rs_bc2 = 1 / sqrt(bc2) are the step's element-independent factors (opt_update_reg computes
// them from lr, bc1, bc2; a caller updating elements one at a time passes them precomputed --
// the same values, so the same bits).
template <class O>
__device__ __forceinline__ void opt_update_pre(const O& o, float& pv, float& mv, float& vv, float gsum, float lr,
                                               float nlr_bc1, float rs_bc2, float gscale, int first) {
  float gr = gsum * gscale;
  if (o.maximize) gr = -gr;
  if (o.algo == 2) {
    if (o.wd != 0.f) gr = fmaf(o.wd, pv, gr);
    if (o.momentum != 0.f) {
      const float b = first ? gr : fmaf(o.momentum, mv, (1.f - o.dampening) * gr);
      mv = b;
      gr = o.nesterov ? fmaf(o.momentum, b, gr) : b;
    }
    pv = fmaf(-lr, gr, pv);
  } else {
    if (o.algo == 1) pv *= fmaf(-lr, o.wd, 1.f);
    else if (o.wd != 0.f) gr = fmaf(o.wd, pv, gr);
    mv = fmaf(o.b1, mv, (1.f - o.b1) * gr);
    vv = fmaf(o.b2, vv, ((1.f - o.b2) * gr) * gr);
    // the per-element sqrt / reciprocal are the 1-ulp hardware ones (v_sqrt_f32 / v_rcp_f32)
    // instead of the ~10-instruction correctly rounded sequences: the update is VALU-bound where
    // one workgroup updates many elements
    const float den = fmaf(__builtin_amdgcn_sqrtf(vv), rs_bc2, o.eps);
    pv = fmaf(nlr_bc1, mv * __builtin_amdgcn_rcpf(den), pv);
  }
}

// Four elements at once: Adam / AdamW in packed-fp32 operations (v_pk_fma_f32 / v_pk_mul_f32 on
// pairs), the same operations per element as opt_update_pre -- so the same bits; other algorithms
// and options element by element.
template <class O>
__device__ __forceinline__ void opt_update_pre4(const O& o, f32x4& pv, f32x4& mv, f32x4& vv, f32x4 g, float lr,
                                                float nlr_bc1, float rs_bc2, int first) {
  if (o.algo == 2 || o.maximize || (o.algo == 0 && o.wd != 0.f)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p_ = pv[r], m_ = mv[r], v_ = vv[r];
      opt_update_pre(o, p_, m_, v_, g[r], lr, nlr_bc1, rs_bc2, 1.f, first);
      pv[r] = p_;
      mv[r] = m_;
      vv[r] = v_;
    }
    return;
  }
  auto splat = [](float x) { return f32x4{x, x, x, x}; };
  g = g * splat(1.f);                                        // (gsum * gscale, gscale = 1)
  if (o.algo == 1) pv *= splat(fmaf(-lr, o.wd, 1.f));
  mv = __builtin_elementwise_fma(splat(o.b1), mv, splat(1.f - o.b1) * g);
  vv = __builtin_elementwise_fma(splat(o.b2), vv, (splat(1.f - o.b2) * g) * g);
  f32x4 q;
#pragma unroll
  for (int r = 0; r < 4; ++r) q[r] = __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_sqrtf(vv[r]), rs_bc2, o.eps));
  pv = __builtin_elementwise_fma(splat(nlr_bc1), mv * q, pv);
}

template <class O>
__device__ __forceinline__ void opt_update_reg(const O& o, float& pv, float& mv, float& vv, float gsum, float lr,
                                               float bc1, float bc2, float gscale, int first) {
  opt_update_pre(o, pv, mv, vv, gsum, lr, -(lr / bc1), 1.f / sqrtf(bc2), gscale, first);
}

// gsum: this element's gradient (summed over ranks when the reduction is fused in)
__device__ __forceinline__ float opt_update(const OptDesc& o, int idx, float* __restrict__ p, float gsum,
                                            float* __restrict__ m, float* __restrict__ v, float lr, float bc1,
                                            float bc2, float gscale, int first) {
  float pv = p[idx], mv = m[idx], vv = v[idx];
  opt_update_reg(o, pv, mv, vv, gsum, lr, bc1, bc2, gscale, first);
  m[idx] = mv;
  if (o.algo != 2) v[idx] = vv;
  p[idx] = pv;
  return pv;
}

// blocks of the tiled optimizer per segment: 32x32 weight tiles, 1024-element vector chunks
__host__ __device__ __forceinline__ int opt_seg_blocks(const OptSeg& sg) {
  return sg.kind == 1 ? ((sg.out + 31) / 32) * ((sg.in + 31) / 32) : (sg.len + 1023) / 1024;
}
