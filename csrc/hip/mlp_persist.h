// Persistent epoch kernel of the fused MLP trainer (one GPU): a whole epoch of training steps in
// ONE launch, with the optimizer running beside the backward pass instead of after it.
//
// The launch-per-step loop (fused_mlp.hip rx_mlp_train_steps) pays, per step, two dependent
// kernel boundaries (~1.5 us each, MI355X_MICROARCH.md "boundary") and runs the whole optimizer
// (weight gradients dW = X^T G for every layer, Adam, bf16 image rewrite) after the last
// backward layer. Here:
//   * block 0 (the step workgroup) runs forward + loss + backward exactly as the step kernel does
//     (mlp_core.h, PS = true), keeps the bias / BatchNorm parameters and running statistics in
//     LDS for the whole epoch and updates those vector parameters itself, inside the epilogue
//     that produces each gradient (mlp_core.h PsVec);
//   * blocks 1.. (optimizer workgroups) each own two 32x32 tiles of one Linear weight, with the
//     fp32 master weight and both Adam moments of those tiles in REGISTERS for the whole epoch.
//     As soon as the backward has finished with layer l (its G^T exported and its dgrad done),
//     the step workgroup raises flag l; layer l's optimizer workgroups compute their dW tiles
//     from the exported X^T / G^T, update, and rewrite their slice of the W_l / Wt_l images
//     while the backward continues with layers l-1 .. 0. Only layer 0's update (the smallest
//     weight) is left between one step's backward and the next step's forward, and the next
//     batch's input gather overlaps it.
//
// Hand-offs (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement & inter-workgroup
// visibility", valid form: sc1 payload stores, s_waitcnt vmcnt(0) in every storing wave, a
// workgroup barrier, one lane's sc1 flag store or agent-scope atomic add; the consumer polls with
// sc1 loads, joins a barrier and reads every handed-off byte with sc1 loads):
//   step -> optimizer: X^T_l / G^T_l in the activation area of Gr,   flag sync[32 l] = step + 1
//   optimizer -> step: W_l / Wt_l image tiles,                        counter sync[32 (RX_MAXL + l)]
// Every wait is bounded (wall clock); a timeout sets the error word and every workgroup leaves
// its loop, so the grid always drains.
//
// World > 1 (XgStep::on, one persistent launch per rank and epoch): the data-parallel gradient
// all-reduce happens inside the same launch. Each optimizer workgroup, once its dW tiles of a step
// are computed, exchanges them with the peers' workgroups of the same tiles (csrc/comm/xgmi.h
// rx_xg_push / rx_xg_pull_sum_n: each element goes once, as a tagged 8-B granule, into every peer's
// inbox; each lane polls its own inbox and sums in rank order) and updates with the rank sum x
// 1 / world; the step workgroup pushes the step's bias / BatchNorm gradients after its backward,
// and the next step's vector update (waves 1..7, beside wave 0's counter poll) sums them over the
// ranks. Layer 0 then goes to optimizer workgroups (the host keeps
// ps_l0_inline off) and the vector updates leave the epilogues (they need every rank's gradient).
//
// Reference role: the per-batch train loop of TorchEstimator (python/raydp/torch/estimator.py:
// 272-293: zero_grad / forward / loss.backward / optimizer.step; DDP's all-reduce at :243), same
// arithmetic as mlp_train_step_body + opt_tiled_body.
#pragma once
#include "mlp_core.h"
#include "mlp_opt.h"
#include "../comm/xgmi.h"

#define RX_PS_FLAG(l) (32 * (l))
#define RX_PS_CNT(l) (32 * (RX_MAXL + (l)))
#define RX_PS_ERR (64 * RX_MAXL)
#define RX_PS_XCC (64 * RX_MAXL + 32)  // [worker] = 1 + XCD id of that workgroup
#define RX_PS_MAXW 256
#define RX_PS_WORDS (RX_PS_XCC + RX_PS_MAXW)
#define RX_PS_OPT_LDS (2 * 32 * 33 * 4 + 2 * 32 * 40 * 2)  // dynamic LDS an optimizer workgroup uses

__device__ __forceinline__ unsigned rx_ps_load(const unsigned* p) {
  return __hip_atomic_load(rx_g(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load sc1
}

// One lane: wait until *p >= target. False (error word set) on timeout, or at once when another
// workgroup has already failed.
__device__ __forceinline__ bool rx_ps_wait(unsigned* sync, const unsigned* p, unsigned target,
                                           unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  int k = 0;
  while (rx_ps_load(p) < target) {
    if ((++k & 15) == 0) {
      if (rx_ps_load(sync + RX_PS_ERR) != 0u) return false;
      if (wall_clock64() - t0 > ticks) {
        __hip_atomic_store(rx_g(sync) + RX_PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

__device__ __forceinline__ unsigned rx_xcc_id() {
  return __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // hwreg(HW_REG_XCC_ID, 0, 4)
}

// optimizer workgroups of a weight segment (two 32x32 tiles each)
__host__ __device__ __forceinline__ int ps_seg_blocks(const OptSeg& sg) { return (opt_seg_blocks(sg) + 1) / 2; }

// optimizer workgroups of the l-th weight segment (q: its index in o.seg); none for layer 0 when
// the step workgroup updates it itself (OptDesc::ps_l0_inline)
__host__ __device__ __forceinline__ int ps_seg_workers(const OptDesc& o, int q, int l) {
  return (l == 0 && o.ps_l0_inline) ? 0 : ps_seg_blocks(o.seg[q]);
}

__host__ __device__ __forceinline__ int ps_grid_blocks(const OptDesc& o) {
  int nb = 1, l = 0;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind == 1) nb += ps_seg_workers(o, s, l++);
  return nb;
}

// Bias / BatchNorm gamma, beta of every layer: one optimizer update per element from a step's
// gradients in Gr (written by this workgroup), parameters in the LDS parameter block.
// The elements of all layers are dealt round-robin over the worker threads [64, 512) -- waves
// 1..7; wave 0 meanwhile polls the optimizer workgroups' layer counters, so the update of step
// s - 1 runs in the shadow of the wait for layer 0's new weights of step s (column-per-thread
// would leave the first 16 threads with 15 updates each: the update is VALU bound) -- and every
// gradient / moment load of a thread's elements is issued before its first update.
#define RX_PS_VEC_T0 64
// World > 1 (xs.on): the gradients are the rank sums of step `seq` (each element polled from this
// rank's inbox, rx_xg_pull_sum_n), times 1 / world.
template <class C, class D>
__device__ __forceinline__ void ps_vector_update(const D& d, const OptDesc& o, char* smem, const float* __restrict__ Gr,
                                                 float* __restrict__ m, float* __restrict__ v, float lr, float bc1,
                                                 float bc2, int first, const XgStep& xs, unsigned seq,
                                                 unsigned* __restrict__ sync) {
  constexpr int J = 4;  // elements per thread per pass
  constexpr int NW = RX_THREADS - RX_PS_VEC_T0;
  float* pr = reinterpret_cast<float*>(smem + d.pr_lds_off);
  int total = 0;
  C::each_layer(d, [&](const auto& ly, int) {
    total += ((ly.b_off >= 0) + (ly.g_off >= 0) + (ly.be_off >= 0)) * ly.out;
  });
  const int tid = rx_tid() - RX_PS_VEC_T0;
  if (tid < 0) return;
  const float gsc = rx_xg_active(xs) ? xs.gscale : 1.f;
  bool xok = true;
  for (int e0 = 0; e0 < total; e0 += J * NW) {
    int idx[J], slot[J];
    float g[J], mv[J], vv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = e0 + j * NW + tid;
      int base = 0, id = -1, sl = 0;
      C::each_layer(d, [&](const auto& ly, int) {
        const int offs[3] = {ly.b_off, ly.g_off, ly.be_off};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (offs[k] >= 0) {
            const int c = e - base;
            if (c >= 0 && c < ly.out) {
              id = offs[k] + c;
              sl = ly.pr_off + k * ly.out_n + c;
            }
            base += ly.out;
          }
        }
      });
      idx[j] = id;
      slot[j] = sl;
      const int q = id >= 0 ? id : 0;
      g[j] = rx_g(Gr)[q];
      mv[j] = rx_g(m)[q];
      vv[j] = rx_g(v)[q];
    }
    if (rx_xg_active(xs)) {
      bool val[J];
#pragma unroll
      for (int j = 0; j < J; ++j) val[j] = idx[j] >= 0;
      rx_xg_pull_sum_v<J, 1, true>(XgView{*xs.xd}, *xs.xd, seq, idx, val, g, xok);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if (idx[j] >= 0) {
        float pv = pr[slot[j]];
        opt_update_reg(o, pv, mv[j], vv[j], g[j], lr, bc1, bc2, gsc, first);
        pr[slot[j]] = pv;
        rx_g(m)[idx[j]] = mv[j];
        rx_g(v)[idx[j]] = vv[j];
      }
    }
  }
  if (!xok) __hip_atomic_store(rx_g(sync) + RX_PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class C, class D>
__device__ __forceinline__ void ps_store_vectors(const D& d, const char* smem, float* __restrict__ P) {
  const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off);
  C::each_layer(d, [&](const auto& ly, int) {
    for (int c = rx_tid(); c < ly.out; c += RX_THREADS) {
      if (ly.b_off >= 0) rx_g(P)[ly.b_off + c] = pr[ly.pr_off + c];
      if (ly.g_off >= 0) rx_g(P)[ly.g_off + c] = pr[ly.pr_off + ly.out_n + c];
      if (ly.be_off >= 0) rx_g(P)[ly.be_off + c] = pr[ly.pr_off + 2 * ly.out_n + c];
    }
  });
}

// Layer l's weights are first read where layer l-1's forward prefetches them: each wave reads
// layer l's optimizer counter at the start of layer l-1 (issue) and compares it with this step's
// target there (wait), polling on only if the optimizer workgroups are not done yet -- no wait for
// every layer at the start of the step, no workgroup barrier (every wave that reads the weights
// has matched the counter itself: MI355X_MICROARCH.md valid forms, first row). After a timeout
// or another workgroup's failure the waits stop: the epoch runs to its end and the host rolls it
// back.
struct PsNxWait {
  unsigned* sync;
  const int* workers;       // LDS: optimizer workgroups per layer
  int s;
  unsigned long long ticks;
  unsigned v = 0;
  __device__ void issue(int l) { v = rx_ps_load(sync + RX_PS_CNT(l)); }
  __device__ void wait(int l) {
    const unsigned target = (unsigned)(workers[l] * s);
    if (__builtin_amdgcn_readfirstlane(v) >= target) return;
    const unsigned long long t0 = wall_clock64();
    for (int k = 1;; ++k) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_readfirstlane(rx_ps_load(sync + RX_PS_CNT(l))) >= target) return;
      if ((k & 15) == 0) {
        if (__builtin_amdgcn_readfirstlane(rx_ps_load(sync + RX_PS_ERR)) != 0u) return;
        if (wall_clock64() - t0 > ticks) {
          if ((rx_tid() & 63) == 0)
            __hip_atomic_store(rx_g(sync) + RX_PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return;
        }
      }
    }
  }
};

// ---- layer 0 updated by the step workgroup (OptDesc::ps_l0_inline) ----
// Layer 0's update sat between one step's backward and the next step's forward: G^T_0 export ->
// flag -> optimizer workgroups (sc1 reads of X^T_0 / G^T_0, wgrad, update, image stores) ->
// counter -> the step workgroup's weight reads, ~4 us of hand-off latency per step (profiles/
// r5_persist_*). Its weight is small (NYC: 256 x 20): the step workgroup keeps the fp32 master
// and both moments in LDS (w0s_lds_off), computes dW_0^T = X_0^T G_0 from its own LDS images (the
// X^T_0 copy load_inputs kept, G^T_0 the backward left), updates, and keeps the new bf16 weight
// in REGISTERS as the next forward's B fragments: wave w owns output tiles n = w + 8 j (j < 2,
// as in the forward) and both 16-column halves mi of the K = 32 input padding, so lane (lr, lg)
// holds W_0[16 n + lr][16 mi + 4 lg + r] -- a forward B fragment in the k order pi (mlp_core.h
// ld_afrag_pi). Eligible: one workgroup, in <= 20, in_k == 32, out == out_n <= 256.
// State slots (fp32 each of master | m | v, real elements only): half mi = 0 at
// ((2 w + j) 64 + lane) 4 + r, half mi = 1 (lanes lg == 0: columns 16..19) at
// 16 * 64 * 4 + ((2 w + j) 16 + lr) 4 + r.
#define RX_W0S_N (16 * 64 * 4 + 16 * 16 * 4)   // elements per array (5120)

__device__ __forceinline__ int ps_w0_slot(int w, int j, int mi, int lane) {
  return mi == 0 ? ((2 * w + j) * 64 + lane) * 4 : 16 * 64 * 4 + ((2 * w + j) * 16 + (lane & 15)) * 4;
}

// epoch start: state from P / m / v (row-major [out][in] at w_off), B fragments from the master
template <class LY>
__device__ __forceinline__ void ps_l0_load(const LY& ly, char* smem, int w0s_off, const float* __restrict__ P,
                                           const float* __restrict__ m, const float* __restrict__ v,
                                           bf16x8 (&w0b)[RX_W0J]) {
  const int lane = rx_tid() & 63, wave = rx_wave(), lr = lane & 15, lg = lane >> 4;
  float* S = reinterpret_cast<float*>(smem + w0s_off);
  const int ntiles = ly.out_n >> 4;
#pragma unroll
  for (int j = 0; j < RX_W0J; ++j) {
    const int n = wave + j * RX_NW;
    float h[8];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int i0 = 16 * mi + 4 * lg;
      const int slot = ps_w0_slot(wave, j, mi, lane);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool real = n < ntiles && i0 + r < ly.in;
        const int idx = ly.w_off + (n * 16 + lr) * ly.in + i0 + r;
        const float pv = real ? rx_g(P)[idx] : 0.f;
        if (real) {
          S[slot + r] = pv;
          S[RX_W0S_N + slot + r] = rx_g(m)[idx];
          S[2 * RX_W0S_N + slot + r] = rx_g(v)[idx];
        }
        h[4 * mi + r] = pv;
      }
    }
    w0b[j] = __builtin_bit_cast(bf16x8, u32x4{rx_f2bf2(h[0], h[1]), rx_f2bf2(h[2], h[3]), rx_f2bf2(h[4], h[5]),
                                              rx_f2bf2(h[6], h[7])});
  }
}

// end of a step's backward (G^T_0 in the transposed image): dW_0, the update, the new B fragments
template <int MT, class D, class LY, class O>
__device__ __forceinline__ void ps_l0_update(const D& d, const LY& ly, char* smem, const O& hp, const float* vsc,
                                             bf16x8 (&w0b)[RX_W0J]) {
  using T = Tile<MT>;
  constexpr int KS = T::BP / 32;
  const int lane = rx_tid() & 63, wave = rx_wave(), lr = lane & 15, lg = lane >> 4;
  const u16* GT = reinterpret_cast<const u16*>(smem + d.gt_lds_off);
  const u16* XC = reinterpret_cast<const u16*>(smem + d.x0c_lds_off);
  float* S = reinterpret_cast<float*>(smem + d.w0s_lds_off);
  const f32x4 sc = *reinterpret_cast<const f32x4*>(vsc);   // lr, -(lr / bc1), 1 / sqrt(bc2), first
  const int first = sc[3] != 0.f ? 1 : 0;
  const int ntiles = ly.out_n >> 4;
#pragma unroll
  for (int j = 0; j < RX_W0J; ++j) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) continue;
    bf16x8 gb[KS], xa[2][KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      gb[ks] = *reinterpret_cast<const bf16x8*>(GT + T::tix(n * 16 + lr, ks * 32 + 8 * lg));
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
        xa[mi][ks] = *reinterpret_cast<const bf16x8*>(XC + T::tix(16 * mi + lr, ks * 32 + 8 * lg));
    }
    float h[8];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) a4 = rx_mfma16(xa[mi][ks], gb[ks], a4);
      const bool real = 16 * mi + 4 * lg < ly.in;   // (the slot exists; its columns past `in` stay 0)
      const int slot = ps_w0_slot(wave, j, mi, lane);
      f32x4 pv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (real) {
        pv = *reinterpret_cast<const f32x4*>(S + slot);
        f32x4 mv = *reinterpret_cast<const f32x4*>(S + RX_W0S_N + slot);
        f32x4 vv = *reinterpret_cast<const f32x4*>(S + 2 * RX_W0S_N + slot);
        if (16 * mi + 4 * lg + 3 < ly.in) {
          opt_update_pre4(hp, pv, mv, vv, a4, sc[0], sc[1], sc[2], first);   // four real columns
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (16 * mi + 4 * lg + r < ly.in) {
              float p_ = pv[r], m_ = mv[r], v_ = vv[r];
              opt_update_pre(hp, p_, m_, v_, a4[r], sc[0], sc[1], sc[2], 1.f, first);
              pv[r] = p_;
              mv[r] = m_;
              vv[r] = v_;
            }
          }
        }
        *reinterpret_cast<f32x4*>(S + slot) = pv;
        *reinterpret_cast<f32x4*>(S + RX_W0S_N + slot) = mv;
        *reinterpret_cast<f32x4*>(S + 2 * RX_W0S_N + slot) = vv;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) h[4 * mi + r] = 16 * mi + 4 * lg + r < ly.in ? pv[r] : 0.f;   // padding: 0
    }
    w0b[j] = __builtin_bit_cast(bf16x8, u32x4{rx_f2bf2(h[0], h[1]), rx_f2bf2(h[2], h[3]), rx_f2bf2(h[4], h[5]),
                                              rx_f2bf2(h[6], h[7])});
  }
}

// epoch end: master / moments back to P / m / v, the bf16 W_0 image (zeros in its padding)
template <class LY>
__device__ __forceinline__ void ps_l0_store(const LY& ly, const char* smem, int w0s_off, float* __restrict__ P,
                                            float* __restrict__ m, float* __restrict__ v, u16* __restrict__ W) {
  const int lane = rx_tid() & 63, wave = rx_wave(), lr = lane & 15, lg = lane >> 4;
  const float* S = reinterpret_cast<const float*>(smem + w0s_off);
  const int ntiles = ly.out_n >> 4;
#pragma unroll
  for (int j = 0; j < RX_W0J; ++j) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) continue;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int i0 = 16 * mi + 4 * lg;
      const int slot = ps_w0_slot(wave, j, mi, lane);
      float h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool real = i0 + r < ly.in;
        h[r] = real ? S[slot + r] : 0.f;
        if (real) {
          const int idx = ly.w_off + (n * 16 + lr) * ly.in + i0 + r;
          rx_g(P)[idx] = h[r];
          rx_g(m)[idx] = S[RX_W0S_N + slot + r];
          rx_g(v)[idx] = S[2 * RX_W0S_N + slot + r];
        }
      }
      *reinterpret_cast<RX_GLOBAL rx_u32x2*>(rx_g(W) + ly.w_img + (n * 16 + lr) * ly.in_k + i0) =
          rx_u32x2{rx_f2bf2(h[0], h[1]), rx_f2bf2(h[2], h[3])};
    }
  }
}

// stamps[0..31]: phase stamps of the middle step (diagnostics); stamps[32 + s]: start of step s,
// stamps[32 + nsteps]: end of the last step; stamps[33 + nsteps + k], k < RX_PS_LAYER_STAMPS:
// the middle step's intra-layer shader-clock stamps (s_memtime; layer_forward [40 + 5 l + k],
// layer_backward [20 + 4 l + k]) -- a stamps buffer holds 33 + nsteps + RX_PS_LAYER_STAMPS words
#define RX_PS_STEP_STAMPS 32
#define RX_PS_LAYER_STAMPS 96

template <class C, int MT>
__device__ __forceinline__ void ps_step_wg(const MlpDesc* __restrict__ dp, const OptDesc& o, const u16* __restrict__ img,
                                           float* __restrict__ rstats, float* __restrict__ P, float* __restrict__ Gr,
                                           const u16* __restrict__ feats, const float* __restrict__ labels,
                                           const int* __restrict__ perm, int n_rows, int batch, int nsteps,
                                           float* __restrict__ scratch, double* __restrict__ metrics,
                                           float* __restrict__ m, float* __restrict__ v, const float* __restrict__ sched,
                                           int opt_first, unsigned* __restrict__ sync, unsigned long long ticks,
                                           char* smem, int* rowidx, int* flag_lds,
                                           unsigned long long* __restrict__ stamps, const XgStep& xs) {
  auto&& d = C::desc(dp);
  // optional timeline of the middle step (wall clock, 100 MHz; scripts/dev/persist_time.py)
  const int sstep = nsteps / 2;
  auto stamp = [&](int s, int k) {
    if (stamps != nullptr && s == sstep && rx_tid() == 0) rx_g(stamps)[k] = wall_clock64();
  };
  // XCD census: plain (L2-resident) X^T / G^T exports when every optimizer workgroup shares this
  // XCD's L2, write-through (sc1) ones otherwise
  if (rx_tid() == 0) {
    const unsigned me = rx_xcc_id() + 1u;
    __hip_atomic_store(rx_g(sync) + RX_PS_XCC, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nw = ps_grid_blocks(o);
    bool ok = true, same = true;
    for (int w = 1; w < nw && ok; ++w) {
      ok = rx_ps_wait(sync, sync + RX_PS_XCC + w, 1u, ticks);
      same = same && rx_ps_load(sync + RX_PS_XCC + w) == me;
    }
    flag_lds[0] = ok ? 0 : 1;
    flag_lds[1] = same ? 0 : 1;
  }
  load_params<C>(d, smem, P, rstats);
  // optimizer workgroups per layer (PsNxWait targets), in LDS
  int* workers = flag_lds + 8;
  if (rx_tid() == 0) {
    int l = 0;
    for (int q = 0; q < o.nseg && l < RX_MAXL; ++q)
      if (o.seg[q].kind == 1) {
        workers[l] = ps_seg_workers(o, q, l);
        ++l;
      }
  }
  // layer 0 updated here (see ps_l0_update): its state into LDS, its first B fragments
  const bool l0_in = o.ps_l0_inline != 0 && d.w0s_lds_off >= 0;
  bf16x8 w0b[RX_W0J];
  if (l0_in) {
    ps_l0_load(C::first(d), smem, d.w0s_lds_off, P, m, v, w0b);
    // the X^T_0 copy's K-tail rows [in_n, in_k): zeros for the whole epoch (nothing writes them)
    zero_t_rows<MT, true>(reinterpret_cast<u16*>(smem + d.x0c_lds_off), C::first(d).in_n, C::first(d).in_k);
  }
  __syncthreads();
  if (flag_lds[0]) return;
  const bool ps_wt = flag_lds[1] != 0;
  // bias / BatchNorm affine updates inside the epilogues (mlp_core.h PsVec) unless the last
  // layer carries a BatchNorm (its affine gradients are not produced by a post-op)
  bool last_affine = false;
  C::each_layer(d, [&](const auto& ly, int) { last_affine = ly.g_off >= 0 || ly.be_off >= 0; });
  const bool vec_inline = !last_affine && !rx_xg_active(xs);   // (world > 1: the rank sums come after the step)
  using O = typename rx_opt_type<C>::type;
  const rx_opt_holder<O> oh;
  const O& oc = oh.get(o);
  float* vsc = reinterpret_cast<float*>(flag_lds + 4);   // the step's optimizer scalars (PsVec::sc)
  // next-batch prefetch during the backward (one input chunk per thread, no embedding front)
  const bool pf = Tile<MT>::BP * (d.feat_k >> 3) <= RX_THREADS && d.front_n == 0;
  int pr_i = 0;                 // next step: this thread's row index (threads < BP)
  float sch[3] = {0.f, 1.f, 1.f};   // thread 0: the step's lr, bc1, bc2
  u32x4 xin = u32x4{0u, 0u, 0u, 0u};
  float labn[MT * 4], labp[MT * 4];
#pragma unroll
  for (int q = 0; q < MT * 4; ++q) labn[q] = 0.f;
  for (int s = 0; s < nsteps; ++s) {
    stamp(s, 0);
    // per-step start times (stamps[32 + s], one lane, one vector store): the step-time
    // histogram of raydp_amd/utils/devmon.py
    if (stamps != nullptr && rx_tid() == 0) rx_g(stamps)[RX_PS_STEP_STAMPS + s] = wall_clock64();
    const int row0 = s * batch;
    const int nvalid = min(batch, n_rows - row0);
    if (rx_tid() == 0) {
      // this step's lr and bias corrections: read during the previous step's backward (a global
      // read here would hold every wave at the next barrier for its round trip)
      if (s == 0) {
        sch[0] = rx_g(sched)[0];
        sch[1] = rx_g(sched)[nsteps];
        sch[2] = rx_g(sched)[2 * nsteps];
      }
      const float lr = sch[0], bc1 = sch[1], bc2 = sch[2];
      *reinterpret_cast<f32x4*>(vsc) = f32x4{lr, -(lr / bc1), 1.f / sqrtf(bc2), (opt_first && s == 0) ? 1.f : 0.f};
    }
    if (s > 0 && pf) {
      // this batch was fetched during the previous step's backward: rows, features and labels
      // are already in registers
      if (rx_tid() < Tile<MT>::BP) rowidx[rx_tid()] = pr_i;
      if (d.r_lds_off < 0)
        scatter_input_quads<MT>(d, C::first(d), smem, rx_tid(), xin);
      else
        scatter_input_chunk<MT>(d, C::first(d), smem, rx_tid(), xin);
      if (d.r_lds_off < 0 && C::first(d).in_k > C::first(d).in_n)   // T mode: XT_0's K tail rows
        zero_t_rows<MT, true>(reinterpret_cast<u16*>(smem + C::first(d).xt_off), C::first(d).in_n,
                              C::first(d).in_k);
#pragma unroll
      for (int q = 0; q < MT * 4; ++q) labp[q] = labn[q];
      __syncthreads();
    } else {
      for (int i = rx_tid(); i < Tile<MT>::BP; i += RX_THREADS)
        rowidx[i] = i < nvalid ? (perm ? rx_g(perm)[row0 + i] : row0 + i) : (perm ? rx_g(perm)[row0] : row0);
      __syncthreads();
      // the batch gather does not depend on the weights: it overlaps the last optimizer tiles
      load_inputs<MT, true>(d, C::first(d), smem, feats, rowidx, nvalid, true, dp, P, metrics);
      prefetch_labels<MT, true>(d, labels, rowidx, labp);
    }
    stamp(s, 1);
    // waves 1..7: the vector update of step s - 1 when it is not inside the epilogues (its flag
    // is out, its gradients are in Gr), beside wave 0's counter poll
    if (s > 0 && !vec_inline)
      ps_vector_update<C>(d, o, smem, Gr, m, v, rx_g(sched)[s - 1], rx_g(sched)[nsteps + s - 1],
                          rx_g(sched)[2 * nsteps + s - 1], (opt_first && s == 1) ? 1 : 0, xs,
                          xs.seq + (unsigned)(s - 1), sync);
    // layers >= 1 are waited for where their weights are first read (PsNxWait); layer 0 here,
    // unless the step workgroup updates it itself
    if (s > 0 && !l0_in) {
      if (rx_tid() < RX_PS_VEC_T0) {
        // lane l polls layer l's counter: all layers in flight at once (a sequential poll pays
        // one L2 round trip per layer even when the counters are long complete)
        const int lane = rx_tid();
        unsigned target = 0u;
        int l = 0;
        for (int q = 0; q < o.nseg; ++q) {
          if (o.seg[q].kind != 1) continue;
          if (l == lane && l == 0) target = (unsigned)(ps_seg_workers(o, q, l) * s);
          ++l;
        }
        const unsigned* cnt = sync + RX_PS_CNT(lane < RX_MAXL ? lane : 0);
        const unsigned long long t0 = wall_clock64();
        bool ok = true;
        for (int k = 1;; ++k) {
          const bool done = lane >= l || rx_ps_load(cnt) >= target;
          if (__builtin_amdgcn_ballot_w64(!done) == 0) break;  // wave-uniform exit
          if ((k & 15) == 0) {
            const bool bad = rx_ps_load(sync + RX_PS_ERR) != 0u || wall_clock64() - t0 > ticks;
            if (__builtin_amdgcn_readfirstlane(bad ? 1 : 0)) {
              if (lane == 0) __hip_atomic_store(rx_g(sync) + RX_PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok = false;
              break;
            }
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (lane == 0) flag_lds[0] = ok ? 0 : 1;
      }
      __syncthreads();
      if (flag_lds[0]) return;
    } else if (s > 0 && !vec_inline) {
      __syncthreads();   // the vector update's parameter writes before the forward reads them
    }
    stamp(s, 2);
#ifdef RX_LAYER_STAMPS
    unsigned long long* lst =
        (stamps != nullptr && s == sstep) ? stamps + RX_PS_STEP_STAMPS + nsteps + 1 : nullptr;
#else
    unsigned long long* lst = nullptr;
#endif
    PsNxWait nxw{sync, workers, s, ticks};
    PsVec<O> vo;
    if (vec_inline) {
      vo.o = &oc;
      vo.m = m;
      vo.v = v;
      vo.sc = vsc;
    }
    bf16x8 wpre[RX_PJ][RX_PK];
    if (!l0_in) fwd_prefetch<true>(C::first(d), img, wpre, d.w0s_lds_off >= 0);
    // every step but a ragged last one fills the tile: the full-batch body has no row masks
    auto body = [&](auto full) {
      constexpr bool F = decltype(full)::value;
      C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
        layer_forward<MT, true, true, F>(d, ly, nx, last, smem, img, P, Gr, labels, rowidx, nvalid, scratch, metrics,
                                         wpre, ps_wt, l, lst, labp, static_cast<NoMw*>(nullptr), vo,
                                         (l == 0 && l0_in) ? w0b : nullptr, &nxw);
      });
      stamp(s, 3);
      // next batch, part 1: the data rows this thread needs (its own row index, its feature
      // chunk's row, its label slots' rows) -- global reads the first backward layer hides; every
      // thread reads its own, so no barrier joins the two parts
      if (rx_tid() == 0 && s + 1 < nsteps) {
        sch[0] = rx_g(sched)[s + 1];
        sch[1] = rx_g(sched)[nsteps + s + 1];
        sch[2] = rx_g(sched)[2 * nsteps + s + 1];
      }
      const bool pf_next = pf && s + 1 < nsteps;
      const int row0n = row0 + batch, nvalid_n = min(batch, n_rows - row0n);
      int pr_f = 0, pr_l[MT * 4];
      if (pf_next) {
        auto prow = [&](int i) {
          return i < nvalid_n ? (perm ? rx_g(perm)[row0n + i] : row0n + i) : (perm ? rx_g(perm)[row0n] : row0n);
        };
        pr_i = prow(rx_tid() < Tile<MT>::BP ? rx_tid() : 0);
        int frow, fch;
        if (d.r_lds_off < 0)
          input_chunk_pos<true>(rx_tid(), d.feat_k >> 3, frow, fch);
        else
          input_chunk_pos<false>(rx_tid(), d.feat_k >> 3, frow, fch);
        pr_f = prow(min(frow, Tile<MT>::BP - 1));
#pragma unroll
        for (int q = 0; q < MT * 4; ++q) {
          const int r = label_row<MT>(d, rx_tid() & 63, q);
          pr_l[q] = r >= 0 ? prow(r) : 0;
        }
      }
      bool first_bwd = true;
      C::bwd_layers(d, [&](const auto& ly, const auto& pv, int l) {
        if (l == 0 && l0_in)
          ps_l0_update<MT>(d, ly, smem, oc, vsc, w0b);
        else
          layer_backward<MT, true, F>(d, ly, pv, l, smem, img, P, Gr, nvalid, scratch, lst, sync, s, ps_wt,
                                      static_cast<NoMw*>(nullptr), vo, l0_in ? w0b : nullptr);
        if (first_bwd && pf_next) {
          // part 2, after the first backward layer: the feature chunk and the labels into
          // registers (held until the next step scatters them)
          xin = d.r_lds_off < 0 ? gather_input_chunk<MT, true>(d, feats, pr_f, nvalid_n, rx_tid())
                                : gather_input_chunk<MT, false>(d, feats, pr_f, nvalid_n, rx_tid());
          prefetch_labels_rows<MT, true>(d, labels, pr_l, labn);
        }
        first_bwd = false;
        stamp(s, 8 + l);
      });
    };
    if (nvalid == Tile<MT>::BP)
      body(rx_bool<true>{});
    else
      body(rx_bool<false>{});
    if (!l0_in) {
      // layer 0's backward ends with its G^T export (no dgrad): drained, then its flag
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (rx_tid() == 0)
        __hip_atomic_store(rx_g(sync) + RX_PS_FLAG(0), (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rx_xg_active(xs)) {
        // world > 1: the step's bias / BatchNorm gradients (this workgroup's own Gr stores, drained
        // above) pushed into every peer's inbox; the peers' are summed by the next step's vector
        // update. (Pushing each where the epilogues produce it would start them earlier, but the
        // push code inside the epilogues spilled ~700 B per lane of the step body.)
        // (up to 4 elements per thread: their loads in flight together, then the pushes)
        int nvec = 0;
        for (int q = 0; q < o.nseg; ++q)
          if (o.seg[q].kind != 1) nvec += o.seg[q].len;
        for (int e0 = 0; e0 < nvec; e0 += 4 * RX_THREADS) {
          int gi[4];
          float gv[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            int e = e0 + j * RX_THREADS + rx_tid();
            gi[j] = -1;
            for (int q = 0; q < o.nseg && gi[j] < 0 && e < nvec; ++q) {
              const OptSeg& sg = o.seg[q];
              if (sg.kind == 1) continue;
              if (e < sg.len)
                gi[j] = sg.start + e;
              else
                e -= sg.len;
            }
            gv[j] = gi[j] >= 0 ? rx_g(Gr)[gi[j]] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (gi[j] >= 0) rx_xg_push(*xs.xd, xs.seq + (unsigned)s, gi[j], gv[j]);
        }
      }
    } else {
      __syncthreads();   // every read of this step's LDS images is done before the next batch lands
    }
    stamp(s, 4);
    stamp(s, 5);
  }
  // the last step's vector update (the others ran under the next step's counter wait)
  if (nsteps > 0 && !vec_inline) {
    const int s = nsteps - 1;
    ps_vector_update<C>(d, o, smem, Gr, m, v, rx_g(sched)[s], rx_g(sched)[nsteps + s], rx_g(sched)[2 * nsteps + s],
                        (opt_first && s == 0) ? 1 : 0, xs, xs.seq + (unsigned)s, sync);
    __syncthreads();
  }
  if (stamps != nullptr && rx_tid() == 0) rx_g(stamps)[RX_PS_STEP_STAMPS + nsteps] = wall_clock64();
  if (l0_in) ps_l0_store(C::first(d), smem, d.w0s_lds_off, P, m, v, const_cast<u16*>(img));
  ps_store_vectors<C>(d, smem, P);
  store_running_stats<C>(d, smem, rstats);
}

// One wave's 16x16 block of the dW tile [o0, o0+32) x [i0, i0+32) of its half-workgroup (4
// waves: wh = 2 ms + ns) from the exported X^T / G^T, every byte read with an sc1 load (written
// by the step workgroup of this launch). xo / go: this lane's byte offsets of its X^T and G^T
// rows (computed once per epoch); nk: 32-row k-steps of the batch. All loads are issued back to
// back, address-clamped and unconditional (one L2 round trip, not one per k-step; a load under a
// branch is waited for before the next one issues). Lane (lr, lg) gets
// dW[o0 + 16 ms + lr][i0 + 16 ns + 4 lg + r], r = 0..3 -- the elements it owns.
__device__ __forceinline__ f32x4 ps_wgrad_block(const float* __restrict__ Gr, int xo, int go, int nk) {
  constexpr int KMAX = 4;   // bp <= 128: the persistent kernel runs one-workgroup batches
  u32x4 xa[KMAX], gb[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int kk = k < nk ? k : 0;
    xa[k] = rx_load16_sc1(Gr, xo + kk * 64);
    gb[k] = rx_load16_sc1(Gr, go + kk * 64);
  }
  f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
    if (k < nk) a4 = rx_mfma16(__builtin_bit_cast(bf16x8, xa[k]), __builtin_bit_cast(bf16x8, gb[k]), a4);
  return a4;
}

// An optimizer workgroup: two 32x32 tiles of one Linear weight (one per half-workgroup), master
// weight and moments in registers for the epoch. Per step: wait for the layer's flag, wgrad (the
// MFMA accumulator IS the update's input: each lane updates the 4 elements it holds), bf16
// image stores straight from registers -- W_l rows as 8-B stores, Wt_l rows through a quad
// transpose (rx_quad_transpose) as 8-B stores; layer 0 has no dgrad and no Wt image to keep --
// drain, count. No LDS round trip and one barrier between flag and counter.
template <class O>
__device__ __forceinline__ void ps_opt_wg(const OptDesc& o, const O& hp, int b, float* __restrict__ P,
                                          const float* __restrict__ Gr,
                                          float* __restrict__ m, float* __restrict__ v, const float* __restrict__ sched,
                                          int nsteps, int opt_first, unsigned* __restrict__ sync,
                                          unsigned long long ticks, char* smem, int* flag_lds,
                                          unsigned long long* __restrict__ stamps, const XgStep& xs) {
  const int bw = b;
  int seg = -1, l = 0;
  for (int q = 0; q < o.nseg; ++q) {
    if (o.seg[q].kind != 1) continue;
    const int nbk = ps_seg_workers(o, q, l);
    if (b < nbk) {
      seg = q;
      break;
    }
    b -= nbk;
    ++l;
  }
  if (seg < 0) return;
  const OptSeg& sg = o.seg[seg];
  const int half = rx_tid() >> 8;
  const int t = 2 * b + half;
  const bool valid = t < opt_seg_blocks(sg);
  const int tiles_i = (sg.in + 31) / 32;
  const int o0 = valid ? (t / tiles_i) * 32 : 0, i0 = valid ? (t % tiles_i) * 32 : 0;
  const int lane = rx_tid() & 63, wh = rx_wave() & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int oo = o0 + (wh >> 1) * 16 + lr;             // this lane's weight row
  const int ib = i0 + (wh & 1) * 16 + 4 * lg;          // and its 4 columns ib .. ib + 3
  // everything the step loop needs from the descriptors, read once (inside the loop every field
  // would be a scalar load behind an lgkmcnt wait, on the layer-0 critical path)
  const int nk = (o.bp + 31) / 32;
  const int xo = o.act_off * 4 + (sg.xg_off + min(i0 + (wh & 1) * 16 + lr, sg.in_n - 1) * o.bp + 8 * lg) * 2;
  const int go = o.act_off * 4 + (sg.gg_off + min(o0 + (wh >> 1) * 16 + lr, sg.out_n - 1) * o.bp + 8 * lg) * 2;
  u16* const Wimg = sg.W;
  u16* const Wtimg = sg.Wt;
  const int in_k = sg.in_k, out_k = sg.out_k;

  float pr_[4], mr[4], vr[4];
  int idx[4];
  bool ok[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    ok[r] = valid && oo < sg.out && ib + r < sg.in;
    idx[r] = ok[r] ? sg.start + oo * sg.in + ib + r : sg.start;
    pr_[r] = rx_g(P)[idx[r]];
    mr[r] = rx_g(m)[idx[r]];
    vr[r] = rx_g(v)[idx[r]];
  }
  // image rows this lane writes: W_l row oo (cols ib..+3) and, after the quad transpose, Wt_l row
  // i0 + 16 ns + 4 lg + (lr & 3) (cols o0 + 16 ms + (lr & ~3) .. +3); padding rows stay unwritten
  const bool w_row = valid && oo < sg.out_n;
  const int it = i0 + (wh & 1) * 16 + 4 * lg + (lr & 3);
  const int ot = o0 + (wh >> 1) * 16 + (lr & ~3);
  const bool wt_row = valid && l > 0 && it < sg.in_n && ot < sg.out_n;
  // plain (L2-resident) image stores when this workgroup shares the step workgroup's XCD,
  // write-through (sc1) ones otherwise; the step workgroup reads them with sc1 loads either way
  if (rx_tid() == 0) {
    const unsigned me = rx_xcc_id() + 1u;
    __hip_atomic_store(rx_g(sync) + RX_PS_XCC + 1 + bw, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool okw = rx_ps_wait(sync, sync + RX_PS_XCC, 1u, ticks);
    flag_lds[0] = okw ? 0 : 1;
    flag_lds[1] = (okw && rx_ps_load(sync + RX_PS_XCC) == me) ? 0 : 1;
    // world > 1: the inbox row pointers into LDS (this workgroup leaves its dynamic LDS unused)
    if (rx_xg_active(xs)) rx_xg_rows_init(*xs.xd, reinterpret_cast<XgRows*>(smem));
  }
  __syncthreads();
  const bool wt_ = flag_lds[1] != 0;
  for (int s = 0; s < nsteps; ++s) {
    const float lr_ = rx_g(sched)[s], bc1 = rx_g(sched)[nsteps + s], bc2 = rx_g(sched)[2 * nsteps + s];
    if (rx_tid() == 0 && flag_lds[0] == 0)
      flag_lds[0] = rx_ps_wait(sync, sync + RX_PS_FLAG(l), (unsigned)(s + 1), ticks) ? 0 : 1;
    __syncthreads();
    if (flag_lds[0]) break;
    const bool st = stamps != nullptr && s == nsteps / 2 && b == 0 && rx_tid() == 0;
    if (st) rx_g(stamps)[16 + 2 * l] = wall_clock64();
    f32x4 gw = ps_wgrad_block(Gr, xo, go, nk);
    if (st && l == 0) {   // layer 0: its X^T / G^T fragments arrived
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      rx_g(stamps)[28] = wall_clock64();
    }
    float gsc = 1.f;
    if (rx_xg_active(xs)) {
      // world > 1: each lane pushes its 4 gradient elements into every peer's inbox and sums the
      // peers' (rank order, polled from its own inbox) in place of the local gradient
      const unsigned seq = xs.seq + (unsigned)s;
      const XgRowsView xv{reinterpret_cast<const XgRows*>(smem), *xs.xd};
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (ok[r]) rx_xg_push_v(xv, seq, idx[r], gw[r]);
      if (st && l == 0) rx_g(stamps)[29] = wall_clock64();   // layer 0: pushes issued
      bool okx = true;
      float gv[4] = {gw[0], gw[1], gw[2], gw[3]};
      rx_xg_pull_sum_v<4, 4, true>(xv, *xs.xd, seq, idx, ok, gv, okx);
#pragma unroll
      for (int r = 0; r < 4; ++r) gw[r] = gv[r];
      if (st && l == 0) rx_g(stamps)[31] = wall_clock64();   // lane 0's peer values summed
      if (__syncthreads_or(okx ? 0 : 1)) {
        if (rx_tid() == 0) __hip_atomic_store(rx_g(sync) + RX_PS_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      if (st && l == 0) rx_g(stamps)[30] = wall_clock64();   // the workgroup's sums done
      gsc = xs.gscale;
    }
    const int first = (opt_first && s == 0) ? 1 : 0;
    float h[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (ok[r]) opt_update_reg(hp, pr_[r], mr[r], vr[r], gw[r], lr_, bc1, bc2, gsc, first);
      h[r] = ok[r] ? pr_[r] : 0.f;   // zeros in the padding, which the images must keep
    }
    if (st && l == 0) rx_g(stamps)[26] = wall_clock64();   // layer 0: wgrad + update done
    const uint2 wv = make_uint2(rx_f2bf2(h[0], h[1]), rx_f2bf2(h[2], h[3]));
    const uint2 tv = rx_quad_transpose(wv, lr & 3);   // (every lane of the quad takes part)
    if (w_row) {
      const int off = oo * in_k + ib;
      if (wt_)
        rx_store8_sc1(Wimg, off * 2, wv);
      else
        *reinterpret_cast<RX_GLOBAL rx_u32x2*>(rx_g(Wimg) + off) = rx_u32x2{wv.x, wv.y};
    }
    if (wt_row) {
      const int off = it * out_k + ot;
      if (wt_)
        rx_store8_sc1(Wtimg, off * 2, tv);
      else
        *reinterpret_cast<RX_GLOBAL rx_u32x2*>(rx_g(Wtimg) + off) = rx_u32x2{tv.x, tv.y};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (st && l == 0) rx_g(stamps)[27] = wall_clock64();   // its image stores drained
    __syncthreads();
    if (rx_tid() == 0) __hip_atomic_fetch_add(rx_g(sync) + RX_PS_CNT(l), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (st) rx_g(stamps)[17 + 2 * l] = wall_clock64();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (ok[r]) {
      rx_g(P)[idx[r]] = pr_[r];
      rx_g(m)[idx[r]] = mr[r];
      rx_g(v)[idx[r]] = vr[r];
    }
}

template <class C, int MT>
__device__ __forceinline__ void mlp_persist_body(const MlpDesc* __restrict__ dp, const OptDesc* __restrict__ od,
                                                 const u16* __restrict__ img, float* __restrict__ rstats,
                                                 float* __restrict__ P, float* __restrict__ Gr,
                                                 const u16* __restrict__ feats, const float* __restrict__ labels,
                                                 const int* __restrict__ perm, int n_rows, int batch, int nsteps,
                                                 float* __restrict__ scratch, double* __restrict__ metrics,
                                                 float* __restrict__ m, float* __restrict__ v,
                                                 const float* __restrict__ sched, int opt_first,
                                                 unsigned* __restrict__ sync, unsigned long long ticks, char* smem,
                                                 int* rowidx, int* flag_lds,
                                                 unsigned long long* __restrict__ stamps, const XgStep& xs) {
  const OptDesc& o = *od;
  // workers are blocks 0, stride, 2 stride, ... (stride 8: one XCD under round-robin dispatch;
  // placement only changes which hand-off form a worker picks, never correctness)
  const int nw = ps_grid_blocks(o);
  const int stride = nw > 1 ? ((int)gridDim.x - 1) / (nw - 1) : 1;
  if ((int)blockIdx.x % stride != 0) return;
  const int w = (int)blockIdx.x / stride;
  if (w >= nw) return;
  if (w == 0) {
    ps_step_wg<C, MT>(dp, o, img, rstats, P, Gr, feats, labels, perm, n_rows, batch, nsteps, scratch, metrics, m, v,
                      sched, opt_first, sync, ticks, smem, rowidx, flag_lds, stamps, xs);
  } else {
    // hyperparameters: compile-time constants in a specialised kernel (C::Opt), else the descriptor
    using O = typename rx_opt_type<C>::type;
    const rx_opt_holder<O> oh;
    ps_opt_wg(o, oh.get(o), w - 1, P, Gr, m, v, sched, nsteps, opt_first, sync, ticks, smem, flag_lds, stamps, xs);
  }
}
