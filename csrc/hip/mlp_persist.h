// Persistent epoch kernel of the fused MLP trainer (one GPU): a whole epoch of training steps in
// ONE launch, with the optimizer running beside the backward pass instead of after it.
//
// The launch-per-step loop (fused_mlp.hip rx_mlp_train_steps) pays, per step, two dependent
// kernel boundaries (~1.5 us each, MI355X_MICROARCH.md "boundary") and runs the whole optimizer
// (weight gradients dW = X^T G for every layer, Adam, bf16 image rewrite) after the last
// backward layer. Here:
//   * block 0 (the step workgroup) runs forward + loss + backward exactly as the step kernel does
//     (mlp_core.h, PS = true), keeps the bias / BatchNorm parameters and running statistics in
//     LDS for the whole epoch and updates those vector parameters itself at the end of each step;
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
// Reference role: the per-batch train loop of TorchEstimator (python/raydp/torch/estimator.py:
// 272-293: zero_grad / forward / loss.backward / optimizer.step), same arithmetic as
// mlp_train_step_body + opt_tiled_body.
#pragma once
#include "mlp_core.h"
#include "mlp_opt.h"

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

__host__ __device__ __forceinline__ int ps_grid_blocks(const OptDesc& o) {
  int nb = 1;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind == 1) nb += ps_seg_blocks(o.seg[s]);
  return nb;
}

// Bias / BatchNorm gamma, beta of every layer: one optimizer update per element from this
// step's gradients in Gr (written by this workgroup), parameters in the LDS parameter block.
// The elements of all layers are dealt round-robin over the 512 threads (column-per-thread would
// leave the first 16 threads with 15 updates each while 256 threads idle: the update is VALU
// bound), and every gradient / moment load of a thread's elements is issued before its first
// update.
template <class C, class D>
__device__ __forceinline__ void ps_vector_update(const D& d, const OptDesc& o, char* smem, const float* __restrict__ Gr,
                                                 float* __restrict__ m, float* __restrict__ v, float lr, float bc1,
                                                 float bc2, int first) {
  constexpr int J = 4;  // elements per thread per pass
  float* pr = reinterpret_cast<float*>(smem + d.pr_lds_off);
  int total = 0;
  C::each_layer(d, [&](const auto& ly, int) {
    total += ((ly.b_off >= 0) + (ly.g_off >= 0) + (ly.be_off >= 0)) * ly.out;
  });
  const int tid = rx_tid();
  for (int e0 = 0; e0 < total; e0 += J * RX_THREADS) {
    int idx[J], slot[J];
    float g[J], mv[J], vv[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int e = e0 + j * RX_THREADS + tid;
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
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if (idx[j] >= 0) {
        float pv = pr[slot[j]];
        opt_update_reg(o, pv, mv[j], vv[j], g[j], lr, bc1, bc2, 1.f, first);
        pr[slot[j]] = pv;
        rx_g(m)[idx[j]] = mv[j];
        rx_g(v)[idx[j]] = vv[j];
      }
    }
  }
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
                                           unsigned long long* __restrict__ stamps) {
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
  __syncthreads();
  if (flag_lds[0]) return;
  const bool ps_wt = flag_lds[1] != 0;
  for (int s = 0; s < nsteps; ++s) {
    stamp(s, 0);
    // per-step start times (stamps[32 + s], one lane, one vector store): the step-time
    // histogram of raydp_amd/utils/devmon.py
    if (stamps != nullptr && rx_tid() == 0) rx_g(stamps)[RX_PS_STEP_STAMPS + s] = wall_clock64();
    const int row0 = s * batch;
    const int nvalid = min(batch, n_rows - row0);
    for (int i = rx_tid(); i < Tile<MT>::BP; i += RX_THREADS)
      rowidx[i] = i < nvalid ? (perm ? rx_g(perm)[row0 + i] : row0 + i) : (perm ? rx_g(perm)[row0] : row0);
    __syncthreads();
    // the batch gather does not depend on the weights: it overlaps the last optimizer tiles
    load_inputs<MT, true>(d, C::first(d), smem, feats, rowidx, nvalid, true, dp, P, metrics);
    float labp[MT * 4];
    prefetch_labels<MT, true>(d, labels, rowidx, labp);
    stamp(s, 1);
    if (s > 0) {
      if (rx_tid() < 64) {
        // lane l polls layer l's counter: all layers in flight at once (a sequential poll pays
        // one L2 round trip per layer even when the counters are long complete)
        const int lane = rx_tid();
        unsigned target = 0u;
        int l = 0;
        for (int q = 0; q < o.nseg; ++q) {
          if (o.seg[q].kind != 1) continue;
          if (l == lane) target = (unsigned)(ps_seg_blocks(o.seg[q]) * s);
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
    }
    stamp(s, 2);
#ifdef RX_LAYER_STAMPS
    unsigned long long* lst =
        (stamps != nullptr && s == sstep) ? stamps + RX_PS_STEP_STAMPS + nsteps + 1 : nullptr;
#else
    unsigned long long* lst = nullptr;
#endif
    bf16x8 wpre[RX_PJ][RX_PK];
    fwd_prefetch<true>(C::first(d), img, wpre);
    // every step but a ragged last one fills the tile: the full-batch body has no row masks
    auto body = [&](auto full) {
      constexpr bool F = decltype(full)::value;
      C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
        layer_forward<MT, true, true, F>(d, ly, nx, last, smem, img, P, Gr, labels, rowidx, nvalid, scratch, metrics,
                                         wpre, ps_wt, l, lst, labp);
      });
      stamp(s, 3);
      C::bwd_layers(d, [&](const auto& ly, const auto& pv, int l) {
        layer_backward<MT, true, F>(d, ly, pv, l, smem, img, P, Gr, nvalid, scratch, lst, sync, s, ps_wt);
        stamp(s, 8 + l);
      });
    };
    if (nvalid == Tile<MT>::BP)
      body(rx_bool<true>{});
    else
      body(rx_bool<false>{});
    // layer 0's backward ends with its G^T export (no dgrad)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (rx_tid() == 0)
      __hip_atomic_store(rx_g(sync) + RX_PS_FLAG(0), (unsigned)(s + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    stamp(s, 4);
    ps_vector_update<C>(d, o, smem, Gr, m, v, rx_g(sched)[s], rx_g(sched)[nsteps + s], rx_g(sched)[2 * nsteps + s],
                        (opt_first && s == 0) ? 1 : 0);
    stamp(s, 6);
    __syncthreads();
    stamp(s, 5);
  }
  if (stamps != nullptr && rx_tid() == 0) rx_g(stamps)[RX_PS_STEP_STAMPS + nsteps] = wall_clock64();
  ps_store_vectors<C>(d, smem, P);
  store_running_stats<C>(d, smem, rstats);
}

// dW tile [o0, o0+32) x [i0, i0+32) of one half-workgroup (4 waves) from the exported X^T / G^T,
// every byte read with an sc1 load (written by the step workgroup of this launch).
__device__ __forceinline__ void ps_wgrad_tile(const OptSeg& sg, const OptDesc& o, int o0, int i0,
                                              const float* __restrict__ Gr, float (*gtile)[33]) {
  const int lane = rx_tid() & 63, wh = rx_wave() & 3;
  const int lr = lane & 15, lg = lane >> 4;
  const int ms = wh >> 1, ns = wh & 1;
  const int orow = min(o0 + ms * 16 + lr, sg.out_n - 1);
  const int irow = min(i0 + ns * 16 + lr, sg.in_n - 1);
  const int base = o.act_off * 4;
  const int xo = base + (sg.xg_off + irow * o.bp + 8 * lg) * 2;
  const int go = base + (sg.gg_off + orow * o.bp + 8 * lg) * 2;
  f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < o.bp; k0 += 32) {
    const bf16x8 a = __builtin_bit_cast(bf16x8, rx_load16_sc1(Gr, xo + k0 * 2));
    const bf16x8 b = __builtin_bit_cast(bf16x8, rx_load16_sc1(Gr, go + k0 * 2));
    a4 = rx_mfma16(a, b, a4);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) gtile[ms * 16 + lr][ns * 16 + lg * 4 + r] = a4[r];
}

__device__ __forceinline__ void ps_opt_wg(const OptDesc& o, int b, float* __restrict__ P, const float* __restrict__ Gr,
                                          float* __restrict__ m, float* __restrict__ v, const float* __restrict__ sched,
                                          int nsteps, int opt_first, unsigned* __restrict__ sync,
                                          unsigned long long ticks, char* smem, int* flag_lds,
                                          unsigned long long* __restrict__ stamps) {
  const int bw = b;
  int seg = -1, l = 0;
  for (int q = 0; q < o.nseg; ++q) {
    if (o.seg[q].kind != 1) continue;
    const int nbk = ps_seg_blocks(o.seg[q]);
    if (b < nbk) {
      seg = q;
      break;
    }
    b -= nbk;
    ++l;
  }
  if (seg < 0) return;
  const OptSeg& sg = o.seg[seg];
  const int half = rx_tid() >> 8, ht = rx_tid() & 255;
  const int t = 2 * b + half;
  const bool valid = t < opt_seg_blocks(sg);
  const int tiles_i = (sg.in + 31) / 32;
  const int o0 = valid ? (t / tiles_i) * 32 : 0, i0 = valid ? (t % tiles_i) * 32 : 0;
  const int ti = ht & 31, to = ht >> 5;
  float pr_[4], mr[4], vr[4];
  int idx[4];
  bool ok[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oo = o0 + to + 8 * r, ii = i0 + ti;
    ok[r] = valid && oo < sg.out && ii < sg.in;
    idx[r] = ok[r] ? sg.start + oo * sg.in + ii : sg.start;
    pr_[r] = rx_g(P)[idx[r]];
    mr[r] = rx_g(m)[idx[r]];
    vr[r] = rx_g(v)[idx[r]];
  }
  // plain (L2-resident) image stores when this workgroup shares the step workgroup's XCD,
  // write-through (sc1) ones otherwise; the step workgroup reads them with sc1 loads either way
  if (rx_tid() == 0) {
    const unsigned me = rx_xcc_id() + 1u;
    __hip_atomic_store(rx_g(sync) + RX_PS_XCC + 1 + bw, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool ok = rx_ps_wait(sync, sync + RX_PS_XCC, 1u, ticks);
    flag_lds[0] = ok ? 0 : 1;
    flag_lds[1] = (ok && rx_ps_load(sync + RX_PS_XCC) == me) ? 0 : 1;
  }
  __syncthreads();
  const bool wt_ = flag_lds[1] != 0;
  float (*gtile)[33] = reinterpret_cast<float (*)[33]>(smem) + half * 32;
  u16 (*wt)[40] = reinterpret_cast<u16 (*)[40]>(smem + 2 * 32 * 33 * 4) + half * 32;
  for (int s = 0; s < nsteps; ++s) {
    const float lr = rx_g(sched)[s], bc1 = rx_g(sched)[nsteps + s], bc2 = rx_g(sched)[2 * nsteps + s];
    if (rx_tid() == 0 && flag_lds[0] == 0)
      flag_lds[0] = rx_ps_wait(sync, sync + RX_PS_FLAG(l), (unsigned)(s + 1), ticks) ? 0 : 1;
    __syncthreads();
    if (flag_lds[0]) break;
    const bool st = stamps != nullptr && s == nsteps / 2 && b == 0 && rx_tid() == 0;
    if (st) rx_g(stamps)[16 + 2 * l] = wall_clock64();
    if (valid) ps_wgrad_tile(sg, o, o0, i0, Gr, gtile);
    __syncthreads();
    const int first = (opt_first && s == 0) ? 1 : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      u16 h = 0;
      if (ok[r]) {
        opt_update_reg(o, pr_[r], mr[r], vr[r], gtile[to + 8 * r][ti], lr, bc1, bc2, 1.f, first);
        h = rx_f2bf(pr_[r]);
      }
      wt[to + 8 * r][ti] = h;
    }
    __syncthreads();
    // W_l rows [o0, o0+32) x cols [i0, i0+32) and Wt_l rows [i0, i0+32) x cols [o0, o0+32):
    // 16-B write-through stores (zeros in the padding, which the images must keep)
    if (valid) {
      if (ht < 128) {
        const int row = ht >> 2, ch = ht & 3;
        if (o0 + row < sg.out_n) {
          const u32x4 val = *reinterpret_cast<const u32x4*>(&wt[row][ch * 8]);
          const int off = (o0 + row) * sg.in_k + i0 + ch * 8;
          if (wt_)
            rx_store16_sc1(sg.W, off * 2, val);
          else
            *reinterpret_cast<RX_GLOBAL u32x4*>(rx_g(sg.W) + off) = val;
        }
      } else {
        const int q = ht - 128, row = q >> 2, ch = q & 3;
        if (i0 + row < sg.in_n) {
          u32x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            pk[e] = (uint32_t)wt[ch * 8 + 2 * e][row] | ((uint32_t)wt[ch * 8 + 2 * e + 1][row] << 16);
          const int off = (i0 + row) * sg.out_k + o0 + ch * 8;
          if (wt_)
            rx_store16_sc1(sg.Wt, off * 2, pk);
          else
            *reinterpret_cast<RX_GLOBAL u32x4*>(rx_g(sg.Wt) + off) = pk;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
                                                 unsigned long long* __restrict__ stamps) {
  const OptDesc& o = *od;
  // workers are blocks 0, stride, 2 stride, ... (stride 8: one XCD under round-robin dispatch;
  // placement only changes which hand-off form a worker picks, never correctness)
  const int nw = ps_grid_blocks(o);
  const int stride = nw > 1 ? ((int)gridDim.x - 1) / (nw - 1) : 1;
  if ((int)blockIdx.x % stride != 0) return;
  const int w = (int)blockIdx.x / stride;
  if (w >= nw) return;
  if (w == 0)
    ps_step_wg<C, MT>(dp, o, img, rstats, P, Gr, feats, labels, perm, n_rows, batch, nsteps, scratch, metrics, m, v,
                      sched, opt_first, sync, ticks, smem, rowidx, flag_lds, stamps);
  else
    ps_opt_wg(o, w - 1, P, Gr, m, v, sched, nsteps, opt_first, sync, ticks, smem, flag_lds, stamps);
}
