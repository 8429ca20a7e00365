// Multi-workgroup step: split-K weight gradient + optimizer update of one 32x32 weight tile, and
// the optimizer workgroups that run it INSIDE the step's own launch.
//
// A (tile, split) task: 4 waves (256 threads), each a 16x16 subtile, accumulate dW^T over
// RX_WSPLIT_K batch rows of the exported X^T_l / G^T_l (bf16, sc1 loads), store the fp32 partial
// with sc1 stores and count in on the tile's arrival counter; the LAST arriving task sums the S
// partials in split order (the same bits every run, independent of arrival order), updates p / m /
// v and rewrites the W / Wt bf16 images. Hand-off (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row of the sc1 table): sc1 stores, every wave's vmcnt(0), a barrier, one
// lane's agent-scope add; the last arriver reads every partial with sc1 loads.
//
// Fused (MwCtx::od set): workgroups G .. G+K-1 of the step's grid run the tasks while the G step
// workgroups are still in their backward -- the optimizer no longer follows the step as a
// launch of its own (~18 us at batch 4096, NYC). Layer l's tasks start once every step workgroup
// counted in on lcnt[l] (its X^T_l / G^T_l exports drained and its dgrad of layer l done: nothing
// of this launch reads W_l / Wt_l any more); tasks are dealt latest layer first, the order the
// backward produces them. Vector parameters (biases, BatchNorm) follow lcnt[RX_LCNT_VEC] (every
// step workgroup's bias gradient stores drained). The counters are never reset: after the n-th
// fused launch each holds G * n. Every counter is kept in RX_LCNT_REP replicas.
//
// World > 1 (MwOptArgs::xs.on): the gradient all-reduce rides in the same tasks -- a tile's last
// arriver, once it summed the split-K partials, exchanges the 32x32 tile with its peers (csrc/comm/
// xgmi.h XgStep: write-through store into this rank's slot, tile flag, wait for every peer's flag,
// rank-order sum) and updates with the rank sum times 1 / world; vector chunks likewise. Only the
// 194 KB gradient crosses the links, never the batch-sized X^T / G^T exports.
#pragma once
#include "rx_grid.h"
#include "mlp_opt.h"
#include "../comm/xgmi.h"

#ifndef RX_WSPLIT_K
#define RX_WSPLIT_K 256   // batch rows per split-K task (dev A/B of the fused role: RAYDP_MLP_DEFINES)
#endif
// the partial buffer is sized for 256-row splits (raydp_amd/ops/fused_mlp.py mw_wpart)
static_assert(RX_WSPLIT_K >= 256 && RX_WSPLIT_K % 32 == 0, "split-K partials sized for 256-row splits");
#define RX_LCNT_VEC 31
#define RX_LCNT_REP 8   // replicas of the done counters, one 128-B line each (lcnt[rep * 32 + idx])
#ifndef RX_MWOPT_SLEEP
#define RX_MWOPT_SLEEP 10
#endif

struct MwOptArgs {
  const OptDesc* od;  // device descriptor
  float* p;
  const float* g;
  float* m;
  float* v;
  float lr, bc1, bc2;
  int first;
  const u16* act;     // exported X^T / G^T (g + od->act_off)
  float* wpart;       // [tile][split][4 waves][64 lanes] f32x4 partials
  unsigned* wctr;     // per-tile arrival counters (the last arriver resets its own)
  unsigned need;      // fused launches: every done counter's value once this launch's step
                      // workgroups counted in (G x fused launches so far)
  XgStep xs;          // world > 1: the in-task gradient exchange (xs.on == 0: one GPU)
};

// tile ids of the exchange: weight tiles in segment order, then the vector chunks
__host__ __device__ __forceinline__ int mw_weight_tiles(const OptDesc& o) {
  int n = 0;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind == 1) n += opt_seg_blocks(o.seg[s]);
  return n;
}

// Task `b` (weight tiles in segment order, S splits per tile) -> segment, tile ordinal, tile
// within the segment, split. Returns the segment index (nseg: past the weight tasks).
__device__ __forceinline__ int mw_task_decode(const OptDesc& o, int S, int b, int& tile, int& tb, int& q) {
  int s = 0;
  tile = 0;
  for (; s < o.nseg; ++s) {
    const OptSeg& sg = o.seg[s];
    if (sg.kind != 1) continue;
    const int nb = opt_seg_blocks(sg) * S;
    if (b < nb) break;
    b -= nb;
    tile += opt_seg_blocks(sg);
  }
  tb = b / S;
  q = b % S;
  tile += tb;
  return s;
}

// One (tile, split) task on 256 threads (t = thread index within them). Every thread of the
// calling workgroup executes the same barriers: `valid` false runs them without work (the
// fused role pairs two tasks on 512 threads). The task's X^T and G^T slices (32 rows x
// RX_WSPLIT_K each, 32 KB) are loaded ONCE into LDS (`xs`, RX_MWT_XS) -- each 16-row fragment
// feeds two of the four waves, which loaded it from memory twice before (64 KB a task, 53 MB a
// step at batch 4096) -- then every wave's MFMA chain reads its fragments from there.
// gtile / wimg: 32 x 33 each.
#define RX_MWT_RS (RX_WSPLIT_K + 8)                 // LDS row stride (bf16): 16-B reads conflict-free
#define RX_MWT_XS (2 * 32 * RX_MWT_RS * 2)          // bytes of a task's X^T + G^T slices
__device__ __forceinline__ void mw_tile_task(const MwOptArgs& a, int s, int tile, int tb, int q, bool valid, int t,
                                             float* gtile, u16* wimg, int* last_lds, u16* xs) {
  const OptDesc& o = *a.od;
  const int S = (o.bp + RX_WSPLIT_K - 1) / RX_WSPLIT_K;
  const OptSeg& sg = o.seg[valid ? s : 0];
  const int tiles_i = (sg.in + 31) / 32;
  const int o0 = (tb / tiles_i) * 32, i0 = (tb % tiles_i) * 32;
  const int lane = t & 63, wave = t >> 6;
  const int lc = lane & 15, lg = lane >> 4;
  const int ms = wave >> 1, ns = wave & 1;
  constexpr int KSTEPS = RX_WSPLIT_K / 32, CPR = RX_WSPLIT_K / 8;   // 16-B chunks per row
  const int k0 = q * RX_WSPLIT_K;
  const int nks = (min(o.bp, k0 + RX_WSPLIT_K) - k0) >> 5;
  if (valid) {
    // rows 0..31: X^T_l rows i0.., 32..63: G^T_l rows o0.. (clamped rows, clamped k chunks)
    u32x4 v[64 * CPR / 256];
#pragma unroll
    for (int j = 0; j < 64 * CPR / 256; ++j) {
      const int e = t + 256 * j, r = e / CPR, c = min(e % CPR, nks * 4 - 1);
      const int row = r < 32 ? sg.xg_off + min(i0 + r, sg.in_n - 1) * o.bp
                             : sg.gg_off + min(o0 + r - 32, sg.out_n - 1) * o.bp;
      v[j] = rx_load16_sc1(a.act, (int)(((size_t)row + k0 + 8 * c) * 2));
    }
#pragma unroll
    for (int j = 0; j < 64 * CPR / 256; ++j) {
      const int e = t + 256 * j, r = e / CPR, c = e % CPR;
      *reinterpret_cast<u32x4*>(xs + r * RX_MWT_RS + 8 * c) = v[j];
    }
  }
  __syncthreads();
  if (valid) {
    const u16* xa = xs + (ns * 16 + lc) * RX_MWT_RS + 8 * lg;
    const u16* ga = xs + (32 + ms * 16 + lc) * RX_MWT_RS + 8 * lg;
    f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KSTEPS; ++ks)
      if (ks < nks)
        a4 = rx_mfma16(*reinterpret_cast<const bf16x8*>(xa + 32 * ks), *reinterpret_cast<const bf16x8*>(ga + 32 * ks),
                       a4);
    const int poff = (int)(((((size_t)tile * S + q) * 4 + wave) * 64 + lane) * 16);
    rx_store16_sc1(a.wpart, poff, __builtin_bit_cast(u32x4, a4));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t == 0) {
    int last = 0;
    if (valid) {
      const unsigned old = __hip_atomic_fetch_add(rx_g(a.wctr) + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = old == (unsigned)(S - 1) ? 1 : 0;
      if (last) __hip_atomic_store(rx_g(a.wctr) + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *last_lds = last;
  }
  __syncthreads();
  const bool last = *last_lds != 0;
  const int ti = t & 31, to = t >> 5;  // 8 rows per pass
  float pp[4], pm[4], pvv[4];
  if (last) {
    // this thread's four parameters and moments travel with the partials (one round trip fewer
    // on the tile's critical path)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = o0 + to + r * 8, ii = i0 + ti;
      const int idx = sg.start + min(oo, sg.out - 1) * sg.in + min(ii, sg.in - 1);
      pp[r] = a.p[idx];
      pm[r] = a.m[idx];
      pvv[r] = a.v[idx];
    }
    // the S partials of this wave's subtile summed in split order
    f32x4 t4 = f32x4{0.f, 0.f, 0.f, 0.f};
    const int pbase = (int)((((size_t)tile * S) * 4 + wave) * 64 + lane) * 16;
    for (int q0 = 0; q0 < S; q0 += 8) {
      f32x4 part[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        part[i] = __builtin_bit_cast(f32x4, rx_load16_sc1(a.wpart, pbase + min(q0 + i, S - 1) * 256 * 16));
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (q0 + i < S) t4 += part[i];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) gtile[(ms * 16 + lc) * 33 + ns * 16 + lg * 4 + r] = t4[r];
  }
  __syncthreads();
  const bool xlast = last;
  if (last && rx_xg_active(a.xs)) {
    // world > 1: this rank's tile pushed into every peer's inbox (tagged granules), before any
    // of this lane's polls for theirs
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = o0 + to + r * 8, ii = i0 + ti;
      if (oo < sg.out && ii < sg.in)
        rx_xg_push(*a.xs.xd, a.xs.seq, sg.start + oo * sg.in + ii, gtile[(to + r * 8) * 33 + ti]);
    }
  }
  if (xlast) {
    const float gsc = rx_xg_active(a.xs) ? a.xs.gscale : 1.f;
    bool okx = true;   // (a peer that never came: the error word is set, this element keeps its weight)
    float gs[4];
    int gi[4];
    bool gv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = o0 + to + r * 8, ii = i0 + ti;
      gv[r] = oo < sg.out && ii < sg.in;
      gi[r] = gv[r] ? sg.start + oo * sg.in + ii : sg.start;
      gs[r] = gtile[(to + r * 8) * 33 + ti];
    }
    if (rx_xg_active(a.xs)) rx_xg_pull_sum_n<4>(*a.xs.xd, a.xs.seq, gi, gv, gs, okx);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oo = o0 + to + r * 8, ii = i0 + ti;
      u16 h = 0;
      if (oo < sg.out && ii < sg.in) {
        const int idx = gi[r];
        float pv = pp[r], mv = pm[r], vv = pvv[r];   // opt_update with the loads hoisted
        const float gw = gs[r];
        if (okx) {
          opt_update_reg(o, pv, mv, vv, gw, a.lr, a.bc1, a.bc2, gsc, a.first);
          a.m[idx] = mv;
          if (o.algo != 2) a.v[idx] = vv;
          a.p[idx] = pv;
        }
        h = rx_f2bf(pv);
        rx_g(sg.W)[oo * sg.in_k + ii] = h;
      }
      wimg[(to + r * 8) * 33 + ti] = h;
    }
  }
  __syncthreads();
  if (xlast) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = i0 + to + r * 8, oo = o0 + ti;
      if (oo < sg.out && ii < sg.in) rx_g(sg.Wt)[ii * sg.out_k + oo] = wimg[ti * 33 + to + r * 8];
    }
  }
}

// Vector parameters: chunk `c` (CH elements) of the element-wise segments on NT threads (`t`).
// sc1: the gradients were stored in this launch (fused role). World > 1 (a.xs.on): the chunk is
// pushed to the peers and summed over the ranks element by element (rx_xg_push / rx_xg_pull_sum_n).
template <int CH, int NT>
__device__ __forceinline__ void mw_vector_chunk(const MwOptArgs& a, int c, int t, bool sc1) {
  const OptDesc& o = *a.od;
  for (int s = 0; s < o.nseg; ++s) {
    const OptSeg& sg = o.seg[s];
    if (sg.kind == 1) continue;
    const int nb = (sg.len + CH - 1) / CH;
    if (c < nb) {
      if (!rx_xg_active(a.xs)) {
        for (int q = c * CH + t; q < min(sg.len, (c + 1) * CH); q += NT) {
          const int idx = sg.start + q;
          opt_update(o, idx, a.p, sc1 ? rx_ld_sc1f(a.g + idx) : a.g[idx], a.m, a.v, a.lr, a.bc1, a.bc2, 1.f, a.first);
        }
        return;
      }
      // world > 1: the chunk's gradients pushed into every peer's inbox, then each summed over
      // the ranks from this lane's own inbox
      constexpr int J = CH / NT;
      const XgDev& x = *a.xs.xd;
      float gl[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int q = c * CH + t + j * NT;
        gl[j] = 0.f;
        if (q < sg.len) {
          const int idx = sg.start + q;
          gl[j] = sc1 ? rx_ld_sc1f(a.g + idx) : a.g[idx];
          rx_xg_push(x, a.xs.seq, idx, gl[j]);
        }
      }
      bool okx = true;
      int gi[J];
      bool gv[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int q = c * CH + t + j * NT;
        gv[j] = q < sg.len;
        gi[j] = gv[j] ? sg.start + q : sg.start;
      }
      rx_xg_pull_sum_n<J>(x, a.xs.seq, gi, gv, gl, okx);
      if (okx) {
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (gv[j]) opt_update(o, gi[j], a.p, gl[j], a.m, a.v, a.lr, a.bc1, a.bc2, a.xs.gscale, a.first);
      }
      return;
    }
    c -= nb;
  }
}

template <int CH>
__host__ __device__ __forceinline__ int mw_vector_chunks(const OptDesc& o) {
  int n = 0;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind != 1) n += (o.seg[s].len + CH - 1) / CH;
  return n;
}

// Weight tasks of the descriptor (tiles x splits).
__host__ __device__ __forceinline__ int mw_weight_tasks(const OptDesc& o) {
  const int S = (o.bp + RX_WSPLIT_K - 1) / RX_WSPLIT_K;
  int n = 0;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind == 1) n += opt_seg_blocks(o.seg[s]) * S;
  return n;
}

// Weight task `r` in latest-layer-first order -> segment (returned), tile ordinal (segment
// order, the wpart / wctr index), tile within the segment, split, layer.
__device__ __forceinline__ int mw_task_decode_rev(const OptDesc& o, int S, int r, int& tile, int& tb, int& q,
                                                  int& l) {
  int nl = 0, tiles = 0;
  for (int s = 0; s < o.nseg; ++s)
    if (o.seg[s].kind == 1) {
      ++nl;
      tiles += opt_seg_blocks(o.seg[s]);
    }
  for (int s = o.nseg - 1; s >= 0; --s) {
    const OptSeg& sg = o.seg[s];
    if (sg.kind != 1) continue;
    const int nbt = opt_seg_blocks(sg);
    tiles -= nbt;
    --nl;
    if (r < nbt * S) {
      tb = r / S;
      q = r % S;
      tile = tiles + tb;
      l = nl;
      return s;
    }
    r -= nbt * S;
  }
  tile = tb = q = l = 0;
  return o.nseg;
}

// One lane: wait (bounded) until counter lcnt[idx] reached `need`; a timeout sets the error word.
// The error word is not polled here: step workgroups count in even after a timed-out wait of
// their own, and the control line every step workgroup checks while it waits on BatchNorm
// granules stays off the path of up to 224 pollers.
template <class MWC>
__device__ __forceinline__ void mw_wait_count(const MWC& mw, int idx, unsigned need) {
  const unsigned long long t0 = wall_clock64();
  // the replica of this workgroup's XCD (dispatch deals workgroups round-robin over the 8 XCDs):
  // 28 pollers a line instead of 224 (MI355X_MICROARCH.md valid forms: a counter in R replicas,
  // each producer adding to every replica with one wave instruction of R active lanes)
  const unsigned* c = mw.lcnt + (blockIdx.x % RX_LCNT_REP) * 32 + idx;
  while ((int)(rx_ld_sc1u(c) - need) < 0) {
    if (wall_clock64() - t0 > mw.ticks) {
      __hip_atomic_store(rx_g(mw.ctl) + RX_MW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(RX_MWOPT_SLEEP);   // (~64 clocks a unit: 224 pollers of one line)
  }
}

// LDS of the fused role: two tasks' gtile (fp32) + wimg (bf16), 4 flag words, two tasks' slices.
#define RX_MWOPT_LDS (2 * 32 * 33 * 4 + 2 * 32 * 33 * 2 + 16 + 2 * RX_MWT_XS)

// The optimizer workgroups of a fused multi-workgroup step (blockIdx.x >= mw.G; 512 threads):
// two weight tasks at a time, one per 256-thread half, dealt latest layer first; then the vector
// chunks once the step workgroups' bias gradients are stored. A step that timed out (error word
// set) updates nothing more.
template <class MWC>
__device__ __forceinline__ void mw_opt_role(const MWC& mw, const MwOptArgs& a, char* smem) {
  const OptDesc& o = *a.od;
  const int S = (o.bp + RX_WSPLIT_K - 1) / RX_WSPLIT_K;
  const int K = (int)gridDim.x - mw.G, ko = (int)blockIdx.x - mw.G;
  const int half = (int)threadIdx.x >> 8, t = (int)threadIdx.x & 255;
  float* gtile = reinterpret_cast<float*>(smem) + half * 32 * 33;
  u16* wimg = reinterpret_cast<u16*>(smem + 2 * 32 * 33 * 4) + half * 32 * 33;
  int* flag = reinterpret_cast<int*>(smem + 2 * 32 * 33 * 4 + 2 * 32 * 33 * 2);
  u16* xs = reinterpret_cast<u16*>(smem + 2 * 32 * 33 * 4 + 2 * 32 * 33 * 2 + 16) + half * (RX_MWT_XS / 2);
  const unsigned need = a.need;
  const int nw = mw_weight_tasks(o);
  for (int t0 = 2 * ko; t0 < nw; t0 += 2 * K) {
    const int r = t0 + half;
    const bool valid = r < nw;
    int s = 0, tile = 0, tb = 0, q = 0, l = 0;
    if (valid) s = mw_task_decode_rev(o, S, r, tile, tb, q, l);
    if (t == 0 && valid) mw_wait_count(mw, l, need);
    __syncthreads();
    if (threadIdx.x == 0) flag[2] = rx_ld_sc1u(mw.ctl + RX_MW_ERR) == 0u ? 1 : 0;
    __syncthreads();
    if (!flag[2]) return;
    mw_tile_task(a, s, tile, tb, q, valid, t, gtile, wimg, flag + half, xs);
  }
  const int nv = mw_vector_chunks<512>(o);
  if (ko >= nv) return;
  if (threadIdx.x == 0) {
    mw_wait_count(mw, RX_LCNT_VEC, need);
    flag[2] = rx_ld_sc1u(mw.ctl + RX_MW_ERR) == 0u ? 1 : 0;
  }
  __syncthreads();
  if (!flag[2]) return;
  for (int c = ko; c < nv; c += K) mw_vector_chunk<512, 512>(a, c, (int)threadIdx.x, true);
}
