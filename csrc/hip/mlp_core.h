// Fused MLP training step for CDNA4 (gfx950) -- device code shared by the ahead-of-time
// build (fused_mlp.hip, runtime descriptor) and the per-model specialised build that
// raydp_amd/ops/mlp_jit.py generates (every dimension and offset a compile-time constant).
//
// Forward + loss + backward of a [Linear -> act -> BatchNorm1d]* -> Linear network runs in ONE
// workgroup, bf16 MFMA (v_mfma_f32_16x16x32_bf16) with fp32 accumulation. The reference
// workloads (NYC_Model in examples/pytorch_nyctaxi.py:69-92, batch 64; the stroke tutorial MLPs;
// DLRM's MLP towers) are ~6 MFLOP per step: the step is latency bound, so the whole dependency
// chain (10 GEMMs, 4 BatchNorm reductions, loss) stays in one CU with every activation resident
// in LDS, and column reductions stay inside a wave (each wave owns whole 16-column tiles).
//
// Layouts (bf16 LDS matrices carry a row pad; R's is RX_RPAD, chosen for gfx950's b128 lane
// groups -- see below):
//   R  [Bpad][max_k]    row-major activations (fwd A operand) / gradients (dgrad A operand)
//   GT [max_n][Bpad]    transposed gradient (wgrad A operand)
//   XT_l [in_n][Bpad]   transposed layer inputs saved for wgrad (wgrad B operand)
// Weights come from one global bf16 image buffer written by the optimizer kernel:
//   W_l  [out_n][in_k] at w_img   (fwd B operand, K = in contiguous)
//   Wt_l [in_n][out_k] at wt_img  (dgrad B operand, K = out contiguous)
//
// Descriptor access is generic over a "descriptor" type D and "layer" types: at run time they
// are the MlpDesc / MlpLayer structs below read from device memory; in a specialised build
// they are empty structs whose fields are static constexpr members, so `ly.out` etc. are
// compile-time constants and the compiler schedules each layer with full knowledge.
#pragma once
#include "rx_common.h"
#include "rx_grid.h"
#include "mlp_opt.h"
#include "mlp_mwopt.h"

#include <type_traits>

// No implicit multiply-add contraction in the training kernels: whether the compiler fuses an
// a * b + c depends on the inlining context (and on what the SLP vectorizer pairs into v_pk_*
// ops), so the same expression could round differently in the launch-per-step kernel and in
// the persistent epoch kernel. Fused multiply-adds are written out (fmaf) where they pay.
#pragma clang fp contract(off)

// Saved forward values (BN inputs / ReLU mask sources) stay fp32: a bf16 copy halves their
// bytes but the BN gamma/beta gradients cancel to near zero for some channels, and Adam turns
// their rounding error into sign flips of the update (measured: 12 % parameter error).
// They are stored FRAGMENT-major -- [16-column tile][row tile mt][lane][4 rows] -- i.e. exactly
// the MFMA accumulator layout, and the backward reads them back with the same lane mapping: one
// coalesced 16-B store / load per accumulator instead of four scattered 4-B ones (the CU's
// vector-memory pipe is the bottleneck of the epilogues).
template <int MT>
__device__ __forceinline__ int frag_off(int base, int n, int mt, int lane) {
  return base + ((n * MT + mt) * 64 + lane) * 4;
}


// Row pad (elements) of the row-major LDS activations R: a row stride of max_k + 16 elements is
// 2 (mod 4) 16-B units, which keeps the ds_read_b128 A-fragment reads (16 rows x 4 k-chunks per
// wave) conflict-free for gfx950's b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...;
// the former +8 (odd unit count) was 2-way (SQ_LDS_BANK_CONFLICT, profiles/pmc/SUMMARY.md).
// raydp_amd/ops/fused_mlp.py sizes the R region with the same pad.
#define RX_RPAD 16
#define RX_MAXL 8
#define RX_NW 8          // waves per workgroup
#define RX_THREADS (RX_NW * RX_WAVE)

struct MlpLayer {
  int in, out;
  int in_k, out_k;   // K padding (multiple of 32)
  int in_n, out_n;   // N padding (multiple of 16)
  int w_img, wt_img; // element offsets of W_l / Wt_l in the bf16 image buffer
  int w_off, b_off;  // offsets into the flat fp32 parameter / gradient vectors
  int act;           // 0 identity, 1 relu
  int bn;            // 0 none, 1 act->bn, 2 bn->act
  int g_off, be_off; // BN affine params (-1: not affine)
  int rs_off;        // float offset of [running_mean | running_var] in the stats buffer (-1: none)
  int mw_off;        // multi-workgroup step: float offset of this layer's partial block (MwCtx)
  float eps, momentum;
  int xt_off;        // LDS byte offset of XT_l
  int stat_off;      // float offset of (mean, invstd) pairs for this layer's outputs in LDS
  int r_off;         // float offset of the saved pre-BN values in the scratch buffer
  int pr_off;        // float offset of [bias|gamma|beta|run_mean|run_var] (x out_n) in LDS
  int xg_off;        // wgrad_mode 1: bf16 offset of X^T_l [in_n][BP] in the exported activation area
  int gg_off;        //               bf16 offset of G^T_l [out_n][BP]
  int sv_lds;        // LDS byte offset of the saved BN inputs / ReLU sources (fragment-major like
                     // r_off), or -1: they live in the global scratch buffer at r_off
};

// Embedding front (MlpDesc::front_n > 0): column k of the first Linear's input is either a copy
// of raw input column `src` (poff < 0) or element j of the embedding row selected by raw column
// `src` (poff = flat offset of the table's element [0][j], stride = embedding_dim, rows =
// num_embeddings). This is the stroke tutorial's NET_Model shape (per-column nn.Embedding
// lookups concatenated with dense columns in front of an MLP).
struct FrontCol {
  int src, poff, stride, rows;
};
#define RX_MAXF 64

struct MlpDesc {
  int L;
  int r_lds_off, gt_lds_off, stats_lds_off, lds_bytes;
  int max_k, max_n;
  int loss;          // 0 mse, 1 smooth_l1, 2 l1
  float beta;        // smooth_l1 beta
  int out_dim;
  int feat_k;        // row stride of the bf16 feature matrix
  MlpLayer layer[RX_MAXL];
  int pr_lds_off;    // LDS byte offset of the per-column parameter block
  int pr_total;      // floats in that block
  int act_off;       // float offset (in the gradient buffer) of the exported activation area
  int wgrad_mode;    // 0: weight gradients computed and stored here; 1: X^T / G^T exported and
                     //    the optimizer kernel computes dW = X^T G on its own workgroups
  int front_n;       // embedding front: columns it produces (0 = none; feats is layer 0's input)
  int front_q;       // (column, table row) pairs of the front's embedding columns
  int acc_mode;      // 1: binary accuracy, (pred > acc_thr) == (long)label counted in metrics[5]
  float acc_thr;
  FrontCol front[RX_MAXF];
  int front_qbase[RX_MAXF];  // prefix of `rows` over the front's embedding columns
  int loss_lds_off;  // >= 0: one output column, regression / BCE loss run a row per lane through
                     //       this LDS area (BP floats); -1: the tile-layout loss
  int w0s_lds_off;   // >= 0 (persistent epoch): layer 0's fp32 master weight and Adam / SGD moments
                     //       live here, updated by the step workgroup (mlp_persist.h ps_l0_update)
  int x0c_lds_off;   //       with its copy of X^T_0 ([in_k rows][BP], Tile::tix layout) here
};

// run-time descriptor: loops over layers are ordinary loops
struct DynCfg {
  __device__ static const MlpDesc& desc(const MlpDesc* dp) { return *dp; }
  template <class F>
  __device__ static void fwd_layers(const MlpDesc& d, F&& f) {
    for (int l = 0; l < d.L; ++l) f(d.layer[l], d.layer[l + 1 < d.L ? l + 1 : l], l, l == d.L - 1);
  }
  template <class F>
  __device__ static void bwd_layers(const MlpDesc& d, F&& f) {
    for (int l = d.L - 1; l >= 0; --l) f(d.layer[l], d.layer[l > 0 ? l - 1 : 0], l);
  }
  // unrolled visit (register arrays indexed by l stay in registers)
  template <class F>
  __device__ static void each_layer(const MlpDesc& d, F&& f) {
#pragma unroll
    for (int l = 0; l < RX_MAXL; ++l)
      if (l < d.L) f(d.layer[l], l);
  }
  __device__ static const MlpLayer& first(const MlpDesc& d) { return d.layer[0]; }
};


template <int MT>
struct Tile {
  static constexpr int BP = MT * 16;         // padded batch rows
  static constexpr int NTW = 16 / MT;        // max output n-tiles per wave (64 acc regs)
  // transposed matrices (XT_l, GT): rows of BP bf16, no padding; the 16-B chunks of row r are
  // XOR-permuted by swz(r). Every access keeps to whole chunks -- the publish step's 8-B stores
  // (16 rows per lane group), the wgrad fragments' and the export's 16-B reads -- so a chunk
  // permutation is free, and swz spreads each lane group over the banks: LDS cycles per
  // wave-instruction (ds_read_b128 ideal 4) export 8 -> 4, wgrad fragments 8 -> 4 at MT 4 / 8
  // (12 -> 4 export at MT 2); the 8-B stores stay at 8 (2 dwords per lane over 32 banks: 2-way is
  // the floor for a 16-B permutation). The padded stride BP + 8 this replaces gave 8 / 8 / 8.
  static constexpr int XS = BP;
  // chosen with a bank model (MI355X_MICROARCH.md §LDS) over the image's three access kinds:
  // ds_read_b64_tr_b16 A-operand reads (rows 8 apart in a 32-lane half: ideal 1 cycle per half),
  // the publish step's 8-B stores (unchanged) and the export's 16-B row reads (ideal)
  __host__ __device__ static constexpr int swz(int r) {
    return MT == 1   ? (r >> 2) & 1
           : MT == 2 ? ((r >> 1) & 1) | (((r >> 3) & 1) << 1)
           : MT == 4 ? (r & 3) | (((r >> 3) & 1) << 2)
                     : (r & 3) | (((r ^ (r >> 3)) & 1) << 2) | ((r & 1) << 3);
  }
  // element index of (row r, batch column e) in a transposed matrix
  __host__ __device__ static constexpr int tix(int r, int e) { return r * XS + (((e >> 3) ^ swz(r)) << 3) + (e & 7); }
};

// R, the row-major activation / gradient image (stride RS = max_k + RX_RPAD, b128-friendly):
// the 16-B chunks of row r are XOR-permuted by rx_rsw(r) in {0, 2}. The publish step writes R
// with 2-byte stores, rows 4 apart in the two 16-lane halves of a lane group, and at this
// stride those rows share banks (2-way); flipping chunk bit 1 between them separates them, and
// the GEMM A-fragment reads (rows lr of a 16-row tile, k-chunks s*4 + lg) stay conflict-free
// (bank model: publish 4 -> 2 LDS cycles per wave-instruction, A reads 4 -> 4, for max_k 64 ..
// 512). The permutation only touches chunk bit 1, so offsets of whole 4-chunk (64-B) steps --
// the GEMM's k-steps -- commute with it.
__host__ __device__ constexpr int rx_rsw(int r) { return (((r >> 2) ^ (r >> 3)) & 1) << 1; }
__host__ __device__ constexpr int rx_rix(int r, int k, int RS) {
  return r * RS + (((k >> 3) ^ rx_rsw(r)) << 3) + (k & 7);
}

// ------------------------------------------------------------------------------------------
// Multi-workgroup step (batch > one workgroup's 16 * MT rows; TorchEstimator batch_size 129 ..
// 16384, e.g. the reference's own test at batch 1000, python/raydp/tests/test_torch.py:70-80):
// G workgroups of the same launch each run the single-workgroup step on rows [wg * BP, wg * BP +
// BP) of the batch, activations in their own LDS. What couples the rows of a batch goes through
// global memory:
//   * BatchNorm batch statistics (forward) and the batch sums of its backward: each workgroup
//     publishes per-column partials (count-weighted sums and centred second moments, combined in
//     workgroup order: every workgroup computes bit-identical statistics), then a grid barrier;
//   * bias gradients: per-workgroup partial column sums, reduced in workgroup order after the
//     last barrier of the step into the gradient buffer (deterministic, no float atomics);
//   * weight gradients: every workgroup exports its rows of X^T / G^T into the batch-wide
//     activation area (row stride = the padded batch), and the optimizer kernel's dW = X^T G runs
//     over the whole batch (K = G * BP) as before;
//   * the loss mean and the BatchNorm averages divide by the batch's row count, not the tile's.
// Hand-off form (MI355X_MICROARCH.md "inter-workgroup visibility", first table row): partials are
// written with sc1 stores by every wave, each wave drains them (s_waitcnt vmcnt(0)), a workgroup
// barrier, then ONE lane's agent-scope add to a monotonic counter; the consumer lane polls the
// counter with sc1 loads, its workgroup joins a barrier and every wave reads the partials with
// sc1 loads. All G workgroups must be co-resident (the host checks occupancy); every wait is
// bounded and a timeout sets the error word, after which every barrier returns at once.
struct NoMw {  // one workgroup per step (the fields only make MWT::on ? a : b well-formed)
  static constexpr bool on = false;
  int k, ok, G, wg, n_total, stride;
  float* part;
};

struct MwCtx {
  static constexpr bool on = true;
  int k;                       // grid barriers passed so far in this step (uniform)
  int ok;                      // 0 once a barrier of this step timed out (uniform): no gradient,
                               // running statistic or bias partial is stored from then on
  float* part;                 // [G][stride] partials; layer l's block at mw_off_l: [fwd | bwd | bias]
  int stride;                  // floats per workgroup (a multiple of 32: 128-B lines)
  unsigned* ctl;               // [0] barrier counter, [1] done counter, [2] error word
  int G, wg;                   // workgroups of the step, this one's index
  int n_total;                 // valid rows of the whole batch
  unsigned long long ticks;    // wall-clock bound of one barrier wait
  unsigned long long* tstamp;  // optional: workgroup 0 stores the step's start (wall clock) here
  unsigned seq;                // launch sequence number (host, from 1): tags this launch's granules
  unsigned long long* lstamp;  // diagnostic build (RX_LAYER_STAMPS): workgroup 0's intra-layer
                               // shader-clock stamps of this step ([20 + 4 l ..] backward, [40 + 5 l ..]
                               // forward, [0 .. 2] the closing barrier / bias reduction)
  unsigned* lcnt;              // per-layer done counters (mlp_mwopt.h; [l] X^T_l / G^T_l exported and
                               // W_l read for the last time, [RX_LCNT_VEC] bias gradients stored), one
                               // add per step workgroup in a launch with optimizer workgroups
  MwOptArgs opt;               // opt.od set: workgroups G.. of the grid are optimizer workgroups
};

// A step workgroup's count-in on lcnt[idx] (multi-workgroup step with counters): every wave's
// stores drained, a barrier, one lane's agent-scope add (the producer side of mlp_mwopt.h).
template <class MWT>
__device__ __forceinline__ void mw_count_in(MWT* mw, int idx, int idx2 = -1) {
  if constexpr (MWT::on) {
    if (mw->opt.od == nullptr) return;   // (a launch without optimizer workgroups)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < RX_LCNT_REP) {   // one add per replica, one wave instruction
      unsigned* c = mw->lcnt + threadIdx.x * 32;
      __hip_atomic_fetch_add(rx_g(c) + idx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (idx2 >= 0) __hip_atomic_fetch_add(rx_g(c) + idx2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The persistent step's per-layer weight wait (mlp_persist.h PsNxWait): layer_forward(l) issues
// the read of layer l+1's optimizer counter at its start and waits on it only where it prefetches
// layer l+1's weights. NoNxWait: nothing (every other kernel).
struct NoNxWait {
  __device__ void issue(int) {}
  __device__ void wait(int) {}
};

// Persistent epoch kernel: the bias / BatchNorm affine parameters are updated where their
// gradients are produced. The four lanes holding a column's batch sums (every lane of a column
// gets them from the cross-lane reductions) each own one parameter -- lane group 0 the bias, 1
// gamma, 2 beta -- and apply the optimizer to it in place in the LDS parameter block, with its
// two moments prefetched at the start of the layer. No vector-update phase of its own, no
// gradient round trip through memory. `o == nullptr`: off (the optimizer kernel / the
// end-of-step update owns these parameters). O: OptDesc, or a specialised kernel's constexpr
// hyperparameter struct (C::Opt). The step's scalars live in LDS (sc: lr, -(lr / bc1),
// 1 / sqrt(bc2), first) and are read where they are used: nothing of this stays in SGPRs across
// the layers (the step body is at the SGPR limit; every extra live value is a spill).
template <class O = OptDesc>
struct PsVec {
  const O* o = nullptr;
  float* m = nullptr;
  float* v = nullptr;
  const float* sc = nullptr;
};

// the optimizer-hyperparameter type of a layer configuration: C::Opt where it has one
template <class C, class = void>
struct rx_opt_type {
  using type = OptDesc;
};
template <class C>
struct rx_opt_type<C, std::void_t<typename C::Opt>> {
  using type = typename C::Opt;
};
// the hyperparameters as a reference: the runtime descriptor itself, or an (empty) constexpr struct
template <class O>
struct rx_opt_holder {
  O v;
  __device__ const O& get(const OptDesc&) const { return v; }
};
template <>
struct rx_opt_holder<OptDesc> {
  __device__ const OptDesc& get(const OptDesc& o) const { return o; }
};

// flat parameter index of column c of layer ly that lane group lg updates (-1: none)
template <class LY>
__device__ __forceinline__ int ps_vec_index(const LY& ly, int lg, int c) {
  const int off = lg == 0 ? ly.b_off : (lg == 1 ? ly.g_off : (lg == 2 ? ly.be_off : -1));
  return off >= 0 ? off + c : -1;
}

// both moments of this lane's parameter of column c (address-clamped: issued unconditionally)
template <class VO, class LY>
__device__ __forceinline__ void ps_vec_prefetch(const VO& vo, const LY& ly, int lg, int c, float& mm,
                                                float& vv) {
  const int idx = c < ly.out ? ps_vec_index(ly, lg, c) : -1;
  const int q = idx >= 0 ? idx : 0;
  mm = rx_g(vo.m)[q];
  vv = rx_g(vo.v)[q];
}

// the update itself (same arithmetic as every other optimizer path: opt_update_reg)
template <class VO, class LY>
__device__ __forceinline__ void ps_vec_update(const VO& vo, const LY& ly, float* pr, int lg, int c, bool colok,
                                              float grad, float mm, float vv) {
  const int idx = ps_vec_index(ly, lg, c);
  if (colok && idx >= 0) {
    float* slot = pr + ly.pr_off + lg * ly.out_n + c;   // [bias | gamma | beta | ...] of the layer
    float p = *slot;
    const f32x4 sc = *reinterpret_cast<const f32x4*>(vo.sc);
    opt_update_pre(*vo.o, p, mm, vv, grad, sc[0], sc[1], sc[2], 1.f, sc[3] != 0.f ? 1 : 0);
    *slot = p;
    rx_g(vo.m)[idx] = mm;
    if (vo.o->algo != 2) rx_g(vo.v)[idx] = vv;
  }
}

// Partial blocks: every (layer, phase) region of every workgroup starts on its own 128-B line. A
// consumer's XCD must not hold a line of a region before that region's last write of the step
// (its L2 would then serve the stale copy to the sc1 loads): with regions sharing lines, reading
// layer l's forward statistics pulled in bytes of a region written only later in the backward.
__host__ __device__ __forceinline__ int rx_ru32(int x) { return (x + 31) & ~31; }
template <class LY>
__device__ __forceinline__ float* mw_fwd(float* part, int stride, const LY& ly, int w) {
  return part + (size_t)w * stride + ly.mw_off;
}
template <class LY>
__device__ __forceinline__ float* mw_bwd(float* part, int stride, const LY& ly, int w) {
  return part + (size_t)w * stride + ly.mw_off + rx_ru32(4 * ly.out_n);
}
template <class LY>
__device__ __forceinline__ float* mw_bias(float* part, int stride, const LY& ly, int w) {
  return part + (size_t)w * stride + ly.mw_off + 2 * rx_ru32(4 * ly.out_n);
}

// Grid barrier number `k` (1-based, counted by the caller) of the step. Every thread of every
// workgroup calls it. Returns false when any workgroup timed out (error word set).
__device__ __forceinline__ bool mw_barrier(const MwCtx& mw, int k) {
  __shared__ int mw_ok;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 partial stores have left
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __hip_atomic_fetch_add(rx_g(mw.ctl) + RX_MW_CTR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (unsigned)(k * mw.G);
    const unsigned long long t0 = wall_clock64();
    for (int it = 1;; ++it) {
      if (__hip_atomic_load(rx_g(mw.ctl) + RX_MW_CTR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if ((it & 15) == 0) {
        if (__hip_atomic_load(rx_g(mw.ctl) + RX_MW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
            wall_clock64() - t0 > mw.ticks) {
          __hip_atomic_store(rx_g(mw.ctl) + RX_MW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
    }
    mw_ok = ok;
  }
  __syncthreads();
  return mw_ok != 0;
}

// End of the step: the last workgroup through resets the barrier counter for the next launch
// (every workgroup has passed every wait by then).
__device__ __forceinline__ void mw_finish(const MwCtx& mw) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(rx_g(mw.ctl) + RX_MW_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (counters only: a
    // relaxed device-scope RMW suffices, the next launch is ordered by the kernel boundary; acq_rel
    // cost every workgroup an L2 write-back + invalidate, ~3.5 us, at the end of every launch)
    if (old == (unsigned)mw.G - 1u) {
      __hip_atomic_store(rx_g(mw.ctl) + RX_MW_CTR, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rx_g(mw.ctl) + RX_MW_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Rows of workgroup w when the batch's n valid rows are dealt BP per workgroup.
__device__ __forceinline__ int mw_rows(int n, int w, int bp) { return max(0, min(bp, n - w * bp)); }

// Granule hand-off of the per-workgroup partials (MI355X_MICROARCH.md's R2 form: an 8-B
// {data, tag} written by ONE sc1 store -- here two of them in one 16-B store -- read with sc1
// loads until the tag is this launch's): the reader waits for the data itself, so the step needs
// no grid barrier per BatchNorm reduction (one barrier was ~1.2 us plus the loads' round trip after
// it). Tag = launch sequence * 32 + phase; the partial buffer starts zeroed (tag 0 never valid).
// A pair (a, b) of column c of workgroup w: {a, tag, b, tag} at 16 c bytes into w's region.
__device__ __forceinline__ unsigned mw_tag(const MwCtx& mw, int k) { return mw.seq * 32u + (unsigned)k; }
__device__ __forceinline__ void mw_put_pair(const MwCtx& mw, const float* at, float a, float b, unsigned tag) {
  rx_store16_sc1(mw.part, (int)((at - mw.part) * 4), u32x4{__float_as_uint(a), tag, __float_as_uint(b), tag});
}
__device__ __forceinline__ void mw_put_one(const MwCtx& mw, const float* at, float a, unsigned tag) {
  rx_store8_sc1(mw.part, (int)((at - mw.part) * 4), make_uint2(__float_as_uint(a), tag));
}
// wait until every granule of v[] (16-B pairs, or 8-B singles when ONE) carries `tag`, reloading
// the stale ones; wave-uniform exit, bounded by the barrier timeout (then the error word is set,
// mw.ok cleared and the values are whatever arrived: the host rolls the step back)
template <int N, bool ONE>
__device__ __forceinline__ void mw_await(MwCtx& mw, u32x4 (&v)[N], const int (&off)[N], unsigned tag) {
  auto fresh = [&](const u32x4& x) { return x[1] == tag && (ONE || x[3] == tag); };
  const unsigned long long t0 = wall_clock64();
  for (int it = 1;; ++it) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < N; ++i) ok = ok && fresh(v[i]);
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) return;
    if ((it & 15) == 0) {
      const bool bad = __hip_atomic_load(rx_g(mw.ctl) + RX_MW_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u ||
                       wall_clock64() - t0 > mw.ticks;
      if (__builtin_amdgcn_readfirstlane(bad ? 1 : 0)) {
        __hip_atomic_store(rx_g(mw.ctl) + RX_MW_ERR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mw.ok = 0;
        return;
      }
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (!fresh(v[i])) {
        if constexpr (ONE) {
          const uint2 y = rx_load8_sc1(mw.part, off[i]);
          v[i] = u32x4{y.x, y.y, 0u, 0u};
        } else {
          v[i] = rx_load16_sc1(mw.part, off[i]);
        }
      }
  }
}

// Sums of the G workgroups' pairs of one column (lane group q takes w = q, q + 4, ...; the four
// lane sums added by rx_colsum16: bit-identical on every lane, in a fixed order), and -- for the
// forward BatchNorm -- the count-weighted centred second moment (Chan et al.) from the same pairs.
// `at0`: workgroup 0's pair of the column.
template <bool M2>
__device__ __forceinline__ void mw_reduce_pairs(MwCtx& mw, const float* at0, int q, unsigned tag, int n_batch, int bp,
                                                float& a, float& b) {
  const int G = mw.G, base = (int)((at0 - mw.part) * 4), wst = mw.stride * 4;
  float sa = 0.f, sb = 0.f;
  float keep_a[8], keep_b[8];
  for (int w0 = q; w0 < G; w0 += 32) {
    u32x4 v[8];
    int off[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int w = w0 + 4 * i;
      off[i] = base + (w < G ? w : q) * wst;
      v[i] = rx_load16_sc1(mw.part, off[i]);
    }
    mw_await<8, false>(mw, v, off, tag);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      keep_a[i] = __uint_as_float(v[i][0]);
      keep_b[i] = __uint_as_float(v[i][2]);
      if (w0 + 4 * i < G) {
        sa += keep_a[i];
        sb += keep_b[i];
      }
    }
  }
  a = rx_colsum16(sa);
  b = rx_colsum16(sb);
  if constexpr (M2) {
    const float mean = a / (float)n_batch;
    float m2 = 0.f;
    for (int w0 = q; w0 < G; w0 += 32) {
      if (G > 32) {   // (G <= 32: the one chunk's pairs are still in registers)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const u32x4 x = rx_load16_sc1(mw.part, base + (w0 + 4 * i < G ? w0 + 4 * i : q) * wst);
          keep_a[i] = __uint_as_float(x[0]);
          keep_b[i] = __uint_as_float(x[2]);
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int w = w0 + 4 * i;
        const int nwi = w < G ? mw_rows(n_batch, w, bp) : 0;
        if (nwi == 0) continue;      // an empty workgroup published nothing meaningful
        const float nw = (float)nwi;
        const float dm = keep_a[i] / nw - mean;
        m2 += keep_b[i];
        m2 = fmaf(nw * dm, dm, m2);
      }
    }
    a = mean;
    b = rx_colsum16(m2);
  }
}

// Sums over the G workgroups' partial pairs at p0 + w * stride + {0, 1}. The four lanes that
// share (lane & 15) split the workgroups (lane group q takes w = q, q + 4, ...), each issuing its
// loads 8 workgroups at a time, and rx_colsum16 adds the four lane sums -- every lane gets the
// bit-identical total, in a fixed order (deterministic). A loop of G dependent sc1 loads per
// column, the form this replaces, was most of the multi-workgroup step's time.
__device__ __forceinline__ void mw_pair_sum(const float* p0, int stride, int G, int q, float& a, float& b) {
  float sa = 0.f, sb = 0.f;
  for (int w0 = q; w0 < G; w0 += 32) {
    float va[8], vb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int w = w0 + 4 * i;
      const float* pp = p0 + (size_t)(w < G ? w : q) * (size_t)stride;
      va[i] = rx_ld_sc1f(pp);
      vb[i] = rx_ld_sc1f(pp + 1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (w0 + 4 * i < G) {
        sa += va[i];
        sb += vb[i];
      }
  }
  a = rx_colsum16(sa);
  b = rx_colsum16(sb);
}

// Count-weighted centred second moment of the batch from every workgroup's (sum, M2) pair of
// p0 + w * stride (Chan et al.'s parallel combination), split over lanes as mw_pair_sum.
__device__ __forceinline__ float mw_m2_sum(const float* p0, int stride, int G, int q, float mean, int n_batch,
                                           int bp) {
  float m2 = 0.f;
  for (int w0 = q; w0 < G; w0 += 32) {
    float vs[8], vm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int w = w0 + 4 * i;
      const float* pp = p0 + (size_t)(w < G ? w : q) * (size_t)stride;
      vs[i] = rx_ld_sc1f(pp);
      vm[i] = rx_ld_sc1f(pp + 1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int w = w0 + 4 * i;
      const int nwi = w < G ? mw_rows(n_batch, w, bp) : 0;
      if (nwi == 0) continue;      // an empty workgroup published nothing meaningful
      const float nw = (float)nwi;
      const float dm = vs[i] / nw - mean;
      m2 += vm[i];
      m2 = fmaf(nw * dm, dm, m2);
    }
  }
  return rx_colsum16(m2);
}

// mw_pair_sum's first component and mw_m2_sum with ONE round of partial loads when the grid is
// at most 32 workgroups (each lane's 8 pairs stay in registers for the second pass): the same
// additions in the same order, one cross-XCD round trip instead of two per BatchNorm layer
__device__ __forceinline__ void mw_mean_m2(const float* p0, int stride, int G, int q, int n_batch, int bp,
                                           float& mean, float& m2out) {
  if (G > 32) {
    float S, unused;
    mw_pair_sum(p0, stride, G, q, S, unused);
    mean = S / (float)n_batch;
    m2out = mw_m2_sum(p0, stride, G, q, mean, n_batch, bp);
    return;
  }
  float vs[8], vm[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int w = q + 4 * i;
    const float* pp = p0 + (size_t)(w < G ? w : q) * (size_t)stride;
    vs[i] = rx_ld_sc1f(pp);
    vm[i] = rx_ld_sc1f(pp + 1);
  }
  float sa = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (q + 4 * i < G) sa += vs[i];
  mean = rx_colsum16(sa) / (float)n_batch;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int w = q + 4 * i;
    const int nwi = w < G ? mw_rows(n_batch, w, bp) : 0;
    if (nwi == 0) continue;
    const float nw = (float)nwi;
    const float dm = vs[i] / nw - mean;
    m2 += vm[i];
    m2 = fmaf(nw * dm, dm, m2);
  }
  m2out = rx_colsum16(m2);
}

__device__ __forceinline__ float act_fwd(int act, float z) { return act == 1 ? fmaxf(z, 0.f) : z; }

// Element (mt, r) of an accumulator tile is batch row mt * 16 + 4 lg + r. FULL (the batch fills
// the workgroup's BP rows -- every step of an epoch but a ragged last one) makes every row valid
// at compile time: no per-element compare / select in the epilogues.
template <bool FULL>
__device__ __forceinline__ f32x4 rx_rowmask(f32x4 v, int mt, int lg, int nvalid) {
  if constexpr (!FULL) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (mt * 16 + lg * 4 + r >= nvalid) v[r] = 0.f;
  }
  return v;
}

// Sum of the MT x 4 (row-masked) values of one lane: a tree over packed-fp32 adds (depth
// log2(MT) + 2) instead of a serial chain of MT * 4 dependent adds.
template <int MT, bool FULL>
__device__ __forceinline__ float rx_lane_sum(const f32x4* a, int lg, int nvalid) {
  f32x4 s4 = rx_rowmask<FULL>(a[0], 0, lg, nvalid);
  if constexpr (MT >= 2) {
    f32x4 t4 = rx_rowmask<FULL>(a[1], 1, lg, nvalid);
#pragma unroll
    for (int mt = 2; mt < MT; mt += 2) {
      s4 += rx_rowmask<FULL>(a[mt], mt, lg, nvalid);
      t4 += rx_rowmask<FULL>(a[mt + 1], mt + 1, lg, nvalid);
    }
    s4 += t4;
  }
  return (s4[0] + s4[1]) + (s4[2] + s4[3]);
}

// Sum of the (row-masked) squared deviations from `mean`, same tree.
template <int MT, bool FULL>
__device__ __forceinline__ float rx_lane_sqdev(const f32x4* a, float mean, int lg, int nvalid) {
  const f32x4 m4 = f32x4{mean, mean, mean, mean};
  f32x4 s4 = f32x4{0.f, 0.f, 0.f, 0.f}, t4 = s4;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const f32x4 dv = rx_rowmask<FULL>(a[mt] - m4, mt, lg, nvalid);
    if (mt & 1)
      t4 = __builtin_elementwise_fma(dv, dv, t4);
    else
      s4 = __builtin_elementwise_fma(dv, dv, s4);
  }
  s4 += t4;
  return (s4[0] + s4[1]) + (s4[2] + s4[3]);
}

// Publish one accumulator tile's bf16 image into R (row-major [row][k]): the 4 lanes of a quad
// transpose their 4 x 4 block (rx_quad_transpose), so each lane stores 8 contiguous bytes of one
// row -- 4 ds_write_b64 per tile instead of 16 ds_write_b16. `pk[mt]` are the tile's packed rows.
template <int MT>
__device__ __forceinline__ void rx_publish_rows(u16* R, int RS, int c, int lane, const uint2 (&pk)[MT]) {
  const int lg = lane >> 4, q = lane & 3;
  const int c0 = c & ~3;                         // this quad's first column
  const int rin = lg * 4 + q;                    // the row (inside a 16-row tile) this lane writes
  u16* Rq = R + rin * RS + ((((c0 >> 3) ^ rx_rsw(rin)) << 3) | (c0 & 7));
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    *reinterpret_cast<uint2*>(Rq + mt * 16 * RS) = rx_quad_transpose(pk[mt], q);
}

// C[Bpad x 16-col tile n] += A (LDS, row-major, K contiguous) x Bt (global bf16, [n][K]).
// The weight fragments of up to KC k-steps are fetched in ONE burst of unconditional
// (address-clamped) 16-B loads before any MFMA consumes them, so a layer costs one global
// round trip per 16-column tile instead of one per 32-deep k-step: the step is latency bound
// and the weights arrive from the Infinity Cache / another XCD's L2 after each optimizer step.
// Weight-image load: plain in the launch-per-step loop; sc1 (L2-served) in the persistent epoch
// kernel, where other workgroups of the same launch rewrite the images every step.
template <bool PS>
__device__ __forceinline__ bf16x8 ld_w(const u16* __restrict__ img, int off) {
  if constexpr (PS)
    return __builtin_bit_cast(bf16x8, rx_load16_sc1(img, off * 2));
  else
    return *reinterpret_cast<const RX_GLOBAL bf16x8*>(rx_g(img) + off);
}

#define RX_LDS __attribute__((address_space(3)))
typedef short rx_v4s __attribute__((ext_vector_type(4)));

// A operand of the GEMMs: the layer input (forward) / G_l (dgrad), 16 batch rows x 8 k per lane.
//  * R mode (d.r_lds_off >= 0): the row-major image R, one ds_read_b128 per fragment;
//  * T mode (no R image): straight from the TRANSPOSED image [k][batch] the previous step
//    published for the export anyway, two ds_read_b64_tr_b16 per fragment (gfx950's hardware
//    transpose read: lane 4q + p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4 x 16
//    block; lane i receives column i of the 4 rows). No row-major copy is written at all.
struct AOp {
  const u16* base;  // R or the transposed image
  int RS;           // R's row stride (R mode)
  bool tr;          // T mode
};

template <int MT>
__device__ __forceinline__ bf16x8 ld_afrag(const AOp& A, int ks, int mt, int lane) {
  if (A.tr) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int r0 = ks * 32 + 8 * g + q, e = mt * 16 + 4 * p;
    const rx_v4s x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RX_LDS rx_v4s*)(A.base + Tile<MT>::tix(r0, e)));
    const rx_v4s y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RX_LDS rx_v4s*)(A.base + Tile<MT>::tix(r0 + 4, e)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
  }
  const int lr = lane & 15, lg = lane >> 4;
  const int k0 = ks * 32 + 8 * (lg ^ rx_rsw(lr));   // R's chunk swizzle
  return *reinterpret_cast<const bf16x8*>(A.base + (mt * 16 + lr) * A.RS + k0);
}

// A fragment of a K = 32 GEMM in the k order pi(g, j) = 16 (j >> 2) + 4 g + (j & 3) (transposed
// reads only): the order in which ps_l0_update's accumulators hold a layer-0 weight row, so the
// forward consumes those registers as B fragments directly (mlp_persist.h)
template <int MT>
__device__ __forceinline__ bf16x8 ld_afrag_pi(const AOp& A, int mt, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = 4 * g + q, e = mt * 16 + 4 * p;
  const rx_v4s x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RX_LDS rx_v4s*)(A.base + Tile<MT>::tix(r0, e)));
  const rx_v4s y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((RX_LDS rx_v4s*)(A.base + Tile<MT>::tix(r0 + 16, e)));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(x, y, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int MT, bool PS>
__device__ __forceinline__ void gemm_tile(f32x4 (&acc)[MT], const AOp& A, int lane, const u16* __restrict__ img,
                                          int boff, int ks0, int nks, int lg) {
  constexpr int KC = 8;
  for (int kc = ks0; kc < nks; kc += KC) {
    bf16x8 bfr[KC];
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      const int ks = min(kc + s, nks - 1);
      bfr[s] = ld_w<PS>(img, boff + ks * 32 + 8 * lg);
    }
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      if (kc + s < nks) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = rx_mfma16(ld_afrag<MT>(A, kc + s, mt, lane), bfr[s], acc[mt]);
      }
    }
  }
}

// Weight fragments fetched ahead of time (before the work that precedes the GEMM) so their global
// round trip overlaps that work. The buffer holds RX_PF fragments, dealt flat over this wave's
// (tile j, k-step s) pairs: fragment f = j * nks + s. At the NYC shapes that is every fragment of
// every GEMM (layer 1 forward: 1 tile x 8 k-steps; layer 1 dgrad: 2 tiles x 4), so no GEMM issues
// a load of its own: a load issued after the layer's stores would be waited for behind them
// (vmcnt retires in issue order).
constexpr int RX_W0J = 2;   // layer-0 weight tiles per wave the step workgroup can update (out <= 256)
constexpr int RX_PJ = 2;
constexpr int RX_PK = 4;
constexpr int RX_PF = RX_PJ * RX_PK;
template <bool PS>
__device__ __forceinline__ void gemm_prefetch_flat(bf16x8 (&pre)[RX_PJ][RX_PK], const u16* __restrict__ img,
                                                   int img_off, int ntiles, int K, int wave, int lr, int lg) {
  const int nks = K >> 5;
#pragma unroll
  for (int f = 0; f < RX_PF; ++f) {
    const int j = f / nks, s = f - (f / nks) * nks;
    if (j * RX_NW < ntiles) {   // some wave has a j-th tile (address-clamped for the others)
      const int n = min(wave + j * RX_NW, ntiles - 1);
      pre[f >> 2][f & 3] = ld_w<PS>(img, img_off + (n * 16 + lr) * K + s * 32 + 8 * lg);
    }
  }
}

// This wave's forward weight fragments of layer `ly` (W_l rows, K = in_k).
// pi: layer 0 of a model laid out for the persistent kernel's own layer-0 update
// (MlpDesc::w0s_lds_off >= 0, K = 32): every kernel of that model runs layer 0's GEMM in the k
// order pi of ld_afrag_pi, so the persistent epoch and the launch-per-step loop round alike --
// the fragment is two 8-B reads, columns 4 lg .. +3 and 16 + 4 lg .. +3.
template <bool PS, class LY>
__device__ __forceinline__ void fwd_prefetch(const LY& ly, const u16* __restrict__ img, bf16x8 (&wpre)[RX_PJ][RX_PK],
                                             bool pi = false) {
  const int lane = rx_tid<PS>() & 63, wave = rx_wave<PS>();
  if (pi) {
    const int ntiles = ly.out_n >> 4, lr = lane & 15, lg = lane >> 4;
#pragma unroll
    for (int j = 0; j < RX_PJ; ++j) {
      const int n = min(wave + j * RX_NW, ntiles - 1);
      const int off = ly.w_img + (n * 16 + lr) * ly.in_k + 4 * lg;
      uint2 a, b;
      if constexpr (PS) {
        a = rx_load8_sc1(img, off * 2);
        b = rx_load8_sc1(img, (off + 16) * 2);
      } else {
        const rx_u32x2 x = *reinterpret_cast<const RX_GLOBAL rx_u32x2*>(rx_g(img) + off);
        const rx_u32x2 y = *reinterpret_cast<const RX_GLOBAL rx_u32x2*>(rx_g(img) + off + 16);
        a = make_uint2(x[0], x[1]);
        b = make_uint2(y[0], y[1]);
      }
      wpre[j][0] = __builtin_bit_cast(bf16x8, u32x4{a.x, a.y, b.x, b.y});
    }
    return;
  }
  gemm_prefetch_flat<PS>(wpre, img, ly.w_img, ly.out_n >> 4, ly.in_k, wave, lane & 15, lane >> 4);
}

// Copy `rows` rows of a transposed bf16 LDS matrix (row stride XS) to global memory packed
// [rows][BP]: whole 128-B (BP = 64) rows, 16 B per lane. The optimizer kernel computes the
// weight gradients from these (wgrad_mode 1), so the step kernel's critical chain neither runs
// the wgrad GEMMs nor stores 4 B of fp32 gradient per weight.
// `byte_base`: byte offset of the destination inside the gradient buffer Gr. Persistent (PS) with
// `wt`: write-through sc1 stores (some optimizer workgroup of the launch sits on another XCD);
// plain stores otherwise (every reader shares this XCD's L2 and reads it with sc1 loads).
// Multi-workgroup step: `bp_total` (the exported rows' stride, the padded batch) and `col0` (this
// workgroup's first batch row) place the workgroup's BP columns inside the batch-wide area.
template <int MT, bool PS>
__device__ __forceinline__ void export_rows(const u16* lds, int rows, float* __restrict__ Gr, int byte_base,
                                            bool wt = true, int bp_total = Tile<MT>::BP, int col0 = 0) {
  constexpr int BP = Tile<MT>::BP, XS = Tile<MT>::XS, CH = BP / 8;
  if constexpr (PS) {
    // persistent epoch: straight-line, every thread the same number of 16-B write-through
    // stores (threads past the end repeat an earlier chunk's identical bytes), so the compiler
    // can count them when it waits for the loads issued before them
    const int total = rows * CH;
    const int iters = (total + RX_THREADS - 1) / RX_THREADS;
    for (int it = 0; it < iters; ++it) {
      int idx = rx_tid<PS>() + it * RX_THREADS;
      idx = idx < total ? idx : idx % total;
      const int r = idx / CH, c = idx % CH;
      const int boff = byte_base + (r * bp_total + col0 + c * 8) * 2;
      rx_store16_sc1(Gr, boff, *reinterpret_cast<const u32x4*>(lds + r * XS + ((c ^ Tile<MT>::swz(r)) << 3)));
    }
    (void)wt;
    return;
  }
  for (int idx = rx_tid<PS>(); idx < rows * CH; idx += RX_THREADS) {
    const int r = idx / CH, c = idx % CH;
    const int boff = byte_base + (r * bp_total + col0 + c * 8) * 2;
    const u32x4 val = *reinterpret_cast<const u32x4*>(lds + r * XS + ((c ^ Tile<MT>::swz(r)) << 3));
    *reinterpret_cast<RX_GLOBAL u32x4*>(rx_g(reinterpret_cast<char*>(Gr)) + boff) = val;
  }
}

// Tile j of this wave: the k-steps held in the flat prefetch buffer first (fragment f = j * nks +
// s, statically indexed), the rest loaded here in one burst.
template <int MT, bool PS>
__device__ __forceinline__ void gemm_tile_pre(f32x4 (&acc)[MT], const AOp& A, int lane, const u16* __restrict__ img,
                                              int boff, int K, int lg, const bf16x8 (&pre)[RX_PJ][RX_PK], int j) {
  const int nks = K >> 5;
#pragma unroll
  for (int f = 0; f < RX_PF; ++f) {
    const int s = f - j * nks;
    if (s >= 0 && s < nks) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = rx_mfma16(ld_afrag<MT>(A, s, mt, lane), pre[f >> 2][f & 3], acc[mt]);
    }
  }
  const int done = max(0, min(nks, RX_PF - j * nks));
  if (nks > done) gemm_tile<MT, PS>(acc, A, lane, img, boff, done, nks, lg);
}

// Saved forward values (BN inputs / ReLU sources) of layer `ly`: fragment-major, in LDS when the
// host found room (sv_lds >= 0: no global round trip on the step's critical chain), else in the
// global scratch buffer.
template <int MT, class LY>
__device__ __forceinline__ void sv_store(const LY& ly, char* smem, float* __restrict__ scratch, int n, int mt, int lane,
                                         const f32x4& v) {
  if (ly.sv_lds >= 0)
    *reinterpret_cast<f32x4*>(smem + ly.sv_lds + frag_off<MT>(0, n, mt, lane) * 4) = v;
  else
    *reinterpret_cast<RX_GLOBAL f32x4*>(rx_g(scratch) + frag_off<MT>(ly.r_off, n, mt, lane)) = v;
}
template <int MT, class LY>
__device__ __forceinline__ f32x4 sv_load(const LY& ly, const char* smem, const float* __restrict__ scratch, int n, int mt,
                                         int lane) {
  if (ly.sv_lds >= 0) return *reinterpret_cast<const f32x4*>(smem + ly.sv_lds + frag_off<MT>(0, n, mt, lane) * 4);
  return *reinterpret_cast<const RX_GLOBAL f32x4*>(rx_g(scratch) + frag_off<MT>(ly.r_off, n, mt, lane));
}

// Zero rows [r0, r1) of a transposed image (the K tail the next GEMM reads: T mode's analogue of
// zeroing R's padding columns), 16 B per thread and pass.
template <int MT, bool PS>
__device__ __forceinline__ void zero_t_rows(u16* Tm, int r0, int r1) {
  constexpr int CH = Tile<MT>::BP / 8;
  for (int idx = rx_tid<PS>(); idx < (r1 - r0) * CH; idx += RX_THREADS) {
    const int r = r0 + idx / CH, c = idx % CH;
    *reinterpret_cast<u32x4*>(Tm + r * Tile<MT>::XS + (c << 3)) = u32x4{0u, 0u, 0u, 0u};
  }
}

// ------------------------------------------------------------------------------------------
// forward of layer l for the rows of this workgroup. Leaves y (the layer output after
// act/BN) in R (row-major) and in XT_{l+1}; for the last layer computes loss, metrics and
// writes dL/dy into R/GT as G_{L-1}.
// ------------------------------------------------------------------------------------------
template <int MT, bool TRAIN, bool PS, bool FULL = false, class D, class LY, class NX, class MWT = NoMw,
          class VO = PsVec<>, class NXW = NoNxWait>
__device__ __forceinline__ void layer_forward(const D& d, const LY& ly, const NX& nx, bool last, char* smem,
                                              const u16* __restrict__ img, const float* __restrict__ P,
                              float* __restrict__ Gr, const float* __restrict__ labels,
                              const int* __restrict__ rowidx, int nvalid, float* __restrict__ scratch,
                              double* __restrict__ metrics, bf16x8 (&wpre)[RX_PJ][RX_PK], bool ps_wt = true,
                              int l = 0, unsigned long long* __restrict__ stamps = nullptr,
                              const float* lab_pre = nullptr, MWT* mw = nullptr, VO vo = VO{},
                              const bf16x8* w0b = nullptr, NXW* nxw = nullptr) {
  // optional intra-layer timeline (wave 0, s_memtime): [40 + 5 l ..] export, GEMM, epilogue,
  // first barrier, publish + second barrier
  auto fst = [&](int k) {
#ifdef RX_LAYER_STAMPS
    if (stamps != nullptr && rx_tid<PS>() == 0) rx_g(stamps)[40 + 5 * l + k] = __builtin_amdgcn_s_memtime();
#endif
  };
  using T = Tile<MT>;
  const int lane = rx_tid<PS>() & 63, wave = rx_wave<PS>();
  const int lr = lane & 15, lg = lane >> 4;
  const int RS = d.max_k + RX_RPAD;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* GT = reinterpret_cast<u16*>(smem + d.gt_lds_off);
  float* stats = reinterpret_cast<float*>(smem + d.stats_lds_off);
  const int ntiles = ly.out_n >> 4;
  const bool tmode = d.r_lds_off < 0;   // no R image: A operands by transposed reads of XT_l
  const AOp Aop{tmode ? reinterpret_cast<const u16*>(smem + ly.xt_off) : R, RS, tmode};
  if (nxw != nullptr && !last) nxw->issue(l + 1);   // (its latency hides behind this layer's GEMM)
  fst(0);
  // the last layer's bias moments for the in-epilogue update (persistent kernel)
  float vm_pre[T::NTW], vv_pre[T::NTW];
  if constexpr (PS && TRAIN) {
    if (last && vo.o != nullptr) {
#pragma unroll
      for (int j = 0; j < T::NTW; ++j)
        if (j * RX_NW < ntiles) ps_vec_prefetch(vo, ly, lg, min(wave + j * RX_NW, ntiles - 1) * 16 + lr, vm_pre[j], vv_pre[j]);
    }
  }

  f32x4 acc[T::NTW * MT];
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    f32x4 part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) part[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = wave + j * RX_NW;
    if (n < ntiles) {
      if (w0b != nullptr || (l == 0 && d.w0s_lds_off >= 0)) {
        // layer 0 in the k order pi (fwd_prefetch): B from the registers ps_l0_update left (the
        // persistent epoch) or from the prefetched image fragments; the A reads follow pi
        if (j < RX_W0J) {
          const bf16x8 bw = w0b != nullptr ? w0b[j] : wpre[j][0];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) part[mt] = rx_mfma16(ld_afrag_pi<MT>(Aop, mt, lane), bw, part[mt]);
        }
      } else {
        const int boff = ly.w_img + (n * 16 + lr) * ly.in_k;
        gemm_tile_pre<MT, PS>(part, Aop, lane, img, boff, ly.in_k, lg, wpre, j);
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[j * MT + mt] = part[mt];
  }
  fst(1);
  // the next layer's weights travel while this layer's epilogue runs -- issued before this
  // layer's stores (the X^T export, the saved BN inputs), so the next GEMM's wait for them does
  // not also wait for those stores
  if (!last) {
    if (nxw != nullptr) nxw->wait(l + 1);
    fwd_prefetch<PS>(nx, img, wpre);
  }
  if (TRAIN && d.wgrad_mode == 1 && w0b == nullptr) {  // X^T_l (published by the previous layer / the input load)
    if constexpr (MWT::on)
      export_rows<MT, true>(reinterpret_cast<const u16*>(smem + ly.xt_off), ly.in_n, Gr, d.act_off * 4 + ly.xg_off * 2,
                          ps_wt, mw->G * T::BP, mw->wg * T::BP);
    else
      export_rows<MT, PS>(reinterpret_cast<const u16*>(smem + ly.xt_off), ly.in_n, Gr, d.act_off * 4 + ly.xg_off * 2,
                          ps_wt);
  }

  // ---- epilogue in registers, in place on acc: bias, act, BN, loss ----
  // Phase A of a tile: bias, act, and the BatchNorm statistics of this workgroup's rows (its BN
  // input saved for the backward). Phase B: the batch statistics (stats LDS, running averages),
  // normalisation, padding, loss. One workgroup runs B right after A per tile; the
  // multi-workgroup step publishes every tile's partials, meets the other workgroups and
  // combines the batch statistics in between.
  const int n_batch = MWT::on ? mw->n_total : (FULL ? T::BP : nvalid);   // rows the statistics / loss cover
  // (a multi-workgroup step's trailing workgroups may hold no rows of a short last batch)
  const float inv_nv = FULL ? 1.f / (float)T::BP : (nvalid > 0 ? 1.f / (float)nvalid : 0.f);
  const float inv_nb = 1.f / (float)n_batch;
  // every column of the tile grid is a real one when the layer's width is a multiple of 16
  const bool cols_full = ly.out == ly.out_n;
  float bn_mean[T::NTW], bn_var[T::NTW];
  auto epi_a = [&](int j) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) return;
    const int c = n * 16 + lr;
    const bool colok = cols_full || c < ly.out;
    const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off) + ly.pr_off;
    const float bias = pr[c];
    const f32x4 b4 = f32x4{bias, bias, bias, bias};
    const bool act_first = ly.bn != 2;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      f32x4 z = acc[j * MT + mt] + b4;
      if (act_first && ly.act == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) z[r] = fmaxf(z[r], 0.f);
      }
      acc[j * MT + mt] = z;
    }
    if (TRAIN && ly.bn != 0) {
      const float s = rx_colsum16(rx_lane_sum<MT, FULL>(&acc[j * MT], lg, nvalid));
      const float mean = s * inv_nv;
      const float v = rx_colsum16(rx_lane_sqdev<MT, FULL>(&acc[j * MT], mean, lg, nvalid));
      if constexpr (MWT::on) {
        // this workgroup's (sum, centred second moment) of column c
        if (colok && lg == 0) mw_put_pair(*mw, mw_fwd(mw->part, mw->stride, ly, mw->wg) + 4 * c, s, v, mw_tag(*mw, mw->k));
      } else {
        bn_mean[j] = mean;
        bn_var[j] = v * inv_nv;
      }
      // save the BN input for the backward pass (fragment-major, see frag_off); layer 0 of a
      // persistent epoch that updates it in the step workgroup recomputes it instead
      if (w0b == nullptr) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) sv_store<MT>(ly, smem, scratch, n, mt, lane, acc[j * MT + mt]);
      }
    }
  };
  auto epi_b = [&](int j) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) return;
    const int c = n * 16 + lr;
    const bool colok = cols_full || c < ly.out;
    const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off) + ly.pr_off;
    if (ly.bn != 0) {
      float mean, invstd;
      if (TRAIN) {
        mean = bn_mean[j];
        const float var = bn_var[j];
        invstd = rsqrtf(var + ly.eps);
        if (colok && lg == 0) {
          stats[ly.stat_off + 2 * c] = mean;
          stats[ly.stat_off + 2 * c + 1] = invstd;
          const float unb = n_batch > 1 ? var * (float)n_batch / (float)(n_batch - 1) : var;
          float* prw = reinterpret_cast<float*>(smem + d.pr_lds_off) + ly.pr_off;
          prw[3 * ly.out_n + c] = fmaf(1.f - ly.momentum, prw[3 * ly.out_n + c], ly.momentum * mean);
          prw[4 * ly.out_n + c] = fmaf(1.f - ly.momentum, prw[4 * ly.out_n + c], ly.momentum * unb);
        }
      } else {
        mean = colok ? pr[3 * ly.out_n + c] : 0.f;
        invstd = colok ? rsqrtf(pr[4 * ly.out_n + c] + ly.eps) : 0.f;
      }
      const float gam = pr[ly.out_n + c];
      const float bet = pr[2 * ly.out_n + c];
      const bool act_after = ly.bn == 2;
      // gamma * (x - mean) * invstd + beta as one fma per element: x * k1 + k0
      const float k1 = invstd * gam, k0 = fmaf(-mean, k1, bet);
      const f32x4 k14 = f32x4{k1, k1, k1, k1}, k04 = f32x4{k0, k0, k0, k0};
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x4 t = __builtin_elementwise_fma(acc[j * MT + mt], k14, k04);
        if (act_after && ly.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) t[r] = fmaxf(t[r], 0.f);
        }
        acc[j * MT + mt] = t;
      }
    } else if (TRAIN && !last) {
      // ReLU mask source for the backward pass
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        if (w0b == nullptr) sv_store<MT>(ly, smem, scratch, n, mt, lane, colok ? acc[j * MT + mt] : f32x4{0.f, 0.f, 0.f, 0.f});
    }
    // padded rows / columns carry exact zeros through every GEMM
    if (!(FULL && cols_full)) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[j * MT + mt] = colok ? rx_rowmask<FULL>(acc[j * MT + mt], mt, lg, nvalid) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (last) {
      // loss, metrics and dL/dy (mean reduction over n_batch * out_dim elements)
      float lsum = 0.f, asum = 0.f, ssum = 0.f, gsum = 0.f, csum = 0.f;
      const float inv_n = inv_nb * (1.f / (float)ly.out);
      const int lcode = d.loss;
      const float beta = d.beta;
      if constexpr (!MWT::on) {
        if (d.loss_lds_off >= 0 && lcode != 4) {
          // One output column: only the 4 lanes of column 0 hold real values (MT * 4 rows
          // each), so the tile-layout loss would run its terms 4 * MT times per lane on 4 lanes.
          // Those lanes pass their rows through LDS instead, every lane takes one row (two at
          // 128 rows), and dL/dy goes back the same way into the accumulator layout.
          constexpr int RPL = T::BP > 64 ? T::BP / 64 : 1;   // rows per lane
          float* xs = reinterpret_cast<float*>(smem + d.loss_lds_off);
          if (lr == 0) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) *reinterpret_cast<f32x4*>(xs + mt * 16 + lg * 4) = acc[j * MT + mt];
          }
          const float hb = 0.5f * beta, inv_beta = 1.f / beta, h_inv_beta = 0.5f * inv_beta;
          float gv[RPL];
#pragma unroll
          for (int k = 0; k < RPL; ++k) {
            const int row = lane + 64 * k;
            const bool inb = row < T::BP;
            const bool ok = inb && (FULL || row < nvalid);
            const float x = inb ? xs[row] : 0.f;
            const float t = lab_pre != nullptr ? lab_pre[k] : rx_g(labels)[rowidx[inb ? row : 0] * d.out_dim];
            const float e = x - t;
            const float ae = fabsf(e);
            float li, gi;
            if (lcode == 3) {
              li = fmaxf(x, 0.f) - x * t + log1pf(__expf(-fabsf(x)));
              gi = 1.f / (1.f + __expf(-x)) - t;
            } else {
              const bool quad = ae < beta;
              li = quad ? e * e * h_inv_beta : ae - hb;
              const float sgn = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
              gi = lcode == 0 ? 2.f * e : (lcode == 1 && quad ? e * inv_beta : sgn);
            }
            lsum += ok ? li : 0.f;
            asum += ok ? ae : 0.f;
            ssum = ok ? fmaf(e, e, ssum) : ssum;
            if (d.acc_mode == 1) csum += (ok && (x > d.acc_thr ? 1 : 0) == (int)t) ? 1.f : 0.f;
            gv[k] = ok ? gi * inv_n : 0.f;
            gsum += gv[k];
          }
          lsum = rx_wavesum(lsum);
          asum = rx_wavesum(asum);
          ssum = rx_wavesum(ssum);
          if (d.acc_mode == 1) csum = rx_wavesum(csum);
          if (lcode == 0) lsum = ssum;
          else if (lcode == 2) lsum = asum;
          if (lane == 0) {
            atomicAdd(&metrics[0], (double)(lsum * inv_n));
            atomicAdd(&metrics[1], (double)asum);
            atomicAdd(&metrics[2], (double)ssum);
            if (d.acc_mode == 1) atomicAdd(&metrics[5], (double)csum);
            atomicAdd(&metrics[3], (double)nvalid);
            atomicAdd(&metrics[4], 1.0);
          }
          if (TRAIN) {
#pragma unroll
            for (int k = 0; k < RPL; ++k)
              if (lane + 64 * k < T::BP) xs[lane + 64 * k] = gv[k];
            if (lr == 0) {
#pragma unroll
              for (int mt = 0; mt < MT; ++mt) acc[j * MT + mt] = *reinterpret_cast<const f32x4*>(xs + mt * 16 + lg * 4);
            }
            gsum = rx_wavesum(gsum);
            if (lane == 0 && ly.b_off >= 0) Gr[ly.b_off] = gsum;
            if constexpr (PS) {
              if (vo.o != nullptr && lg == 0)
                ps_vec_update(vo, ly, reinterpret_cast<float*>(smem + d.pr_lds_off), 0, c, colok, gsum, vm_pre[j],
                              vv_pre[j]);
            }
          }
          return;
        }
      }
      // labels of all padded rows, loaded back to back (padded rows read row 0)
      const int cl = colok ? c : 0;
      float tl[MT * 4];
      if (lab_pre != nullptr && ly.out_n == 16) {  // fetched at the start of the step
#pragma unroll
        for (int q = 0; q < MT * 4; ++q) tl[q] = lab_pre[q];
      } else {
#pragma unroll
        for (int q = 0; q < MT * 4; ++q) tl[q] = rx_g(labels)[rowidx[(q >> 2) * 16 + lg * 4 + (q & 3)] * d.out_dim + cl];
      }
      const bool head_wg = !MWT::on || mw->wg == 0;   // the batch is counted once
      if (lcode == 4) {
        // Cross entropy over the out <= 16 classes of one tile (a row's logits live in the 16
        // lanes sharing lg). Labels arrive as a weighted one-hot row (t_c = w[y] at c = y,
        // else 0; an ignored row is all zeros): with W = sum of the rows' weights,
        //   loss = sum_rows (w_y * logsumexp(x) - w_y * x_y) / W
        //   dL/dx_c = (w_y * softmax(x)_c - t_c) / W      (torch's weighted mean)
        // and the row counts as correct when argmax_c x (first index on ties) is y.
        // (single workgroup only: the host never runs it multi-workgroup)
        float wsum = 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = mt * 16 + lg * 4 + r;
            const float x = acc[j * MT + mt][r];
            const float t = (colok && row < nvalid) ? tl[mt * 4 + r] : 0.f;
            float mx = colok ? x : -INFINITY;
            int bi = colok ? c : 1 << 20;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
              const float om = __shfl_xor(mx, o);
              const int oi = __shfl_xor(bi, o);
              if (om > mx || (om == mx && oi < bi)) {
                mx = om;
                bi = oi;
              }
            }
            const float ex = colok ? __expf(x - mx) : 0.f;
            float se = ex, wr = t, tx = t * (colok ? x : 0.f);
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
              se += __shfl_xor(se, o);
              wr += __shfl_xor(wr, o);
              tx += __shfl_xor(tx, o);
            }
            const bool head = lr == 0 && row < nvalid;   // one lane per row
            if (head) {
              lsum += wr * (mx + __logf(se)) - tx;
              wsum += wr;
            }
            if (t > 0.f && c == bi) csum += 1.f;          // the label's lane of a correct row
            acc[j * MT + mt][r] = (colok && row < nvalid) ? wr * (ex / se) - t : 0.f;
          }
        const float wt = rx_wavesum(wsum);
        const float invw = wt > 0.f ? 1.f / wt : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            acc[j * MT + mt][r] *= invw;
            gsum += acc[j * MT + mt][r];
          }
        lsum = rx_wavesum(lsum) * invw;
        csum = rx_wavesum(csum);
        if (lane == 0) {
          atomicAdd(&metrics[0], (double)lsum);
          atomicAdd(&metrics[5], (double)csum);
          if (n == 0) {
            atomicAdd(&metrics[3], (double)nvalid);
            atomicAdd(&metrics[4], 1.0);
          }
        }
        if (TRAIN) {
          gsum = rx_colsum16(gsum);
          if (colok && lg == 0 && ly.b_off >= 0) Gr[ly.b_off + c] = gsum;
          if constexpr (PS) {
            if (vo.o != nullptr && lg == 0)
              ps_vec_update(vo, ly, reinterpret_cast<float*>(smem + d.pr_lds_off), 0, c, colok, gsum, vm_pre[j],
                            vv_pre[j]);
          }
        }
      } else {
        // branch-free: every element computes its terms, invalid ones (padded rows / columns)
        // are selected out; per-lane sums in packed-fp32 vectors
        const float hb = 0.5f * beta, inv_beta = 1.f / beta, h_inv_beta = 0.5f * inv_beta;
        f32x4 l4 = f32x4{0.f, 0.f, 0.f, 0.f}, a4 = l4, s4 = l4, c4 = l4, g4s = l4;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x4 x4 = acc[j * MT + mt];
          f32x4 gv;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = mt * 16 + lg * 4 + r;
            const bool ok = colok && (FULL || row < nvalid);
            const float t = tl[mt * 4 + r];
            const float x = x4[r];
            const float e = x - t;
            const float ae = fabsf(e);
            float li, gi;
            if (lcode == 3) {
              // BCE with logits, softplus form (stable for either sign):
              //   l = max(x, 0) - x t + log1p(exp(-|x|)),  dl/dx = sigmoid(x) - t
              li = fmaxf(x, 0.f) - x * t + log1pf(__expf(-fabsf(x)));
              gi = 1.f / (1.f + __expf(-x)) - t;
            } else {
              const bool quad = ae < beta;
              li = quad ? e * e * h_inv_beta : ae - hb;   // smooth-L1 term
              const float sgn = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f);
              gi = lcode == 0 ? 2.f * e : (lcode == 1 && quad ? e * inv_beta : sgn);
            }
            l4[r] += ok ? li : 0.f;
            a4[r] += ok ? ae : 0.f;
            s4[r] = ok ? fmaf(e, e, s4[r]) : s4[r];
            if (d.acc_mode == 1)  // torch: (pred > thr).long() == target.long()
              c4[r] += (ok && (x > d.acc_thr ? 1 : 0) == (int)t) ? 1.f : 0.f;
            gv[r] = ok ? gi * inv_n : 0.f;
          }
          acc[j * MT + mt] = gv;  // acc now holds G_{L-1}
          g4s += gv;
        }
        lsum = (l4[0] + l4[1]) + (l4[2] + l4[3]);
        asum = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        ssum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        csum = (c4[0] + c4[1]) + (c4[2] + c4[3]);
        gsum = (g4s[0] + g4s[1]) + (g4s[2] + g4s[3]);
        lsum = rx_wavesum(lsum);
        asum = rx_wavesum(asum);
        ssum = rx_wavesum(ssum);
        if (d.acc_mode == 1) csum = rx_wavesum(csum);
        if (lcode == 0) lsum = ssum;
        else if (lcode == 2) lsum = asum;
        if (lane == 0) {
          atomicAdd(&metrics[0], (double)(lsum * inv_n));
          atomicAdd(&metrics[1], (double)asum);
          atomicAdd(&metrics[2], (double)ssum);
          if (d.acc_mode == 1) atomicAdd(&metrics[5], (double)csum);
          if (n == 0) {
            atomicAdd(&metrics[3], (double)(nvalid * ly.out));
            if (head_wg) atomicAdd(&metrics[4], 1.0);
          }
        }
        if (TRAIN) {
          gsum = rx_colsum16(gsum);
          if (colok && lg == 0 && ly.b_off >= 0) {
            if constexpr (MWT::on)
              mw_put_one(*mw, mw_bias(mw->part, mw->stride, ly, mw->wg) + 2 * c, gsum, mw_tag(*mw, 31));
            else
              Gr[ly.b_off + c] = gsum;
          }
          if constexpr (PS) {
            if (vo.o != nullptr && lg == 0)
              ps_vec_update(vo, ly, reinterpret_cast<float*>(smem + d.pr_lds_off), 0, c, colok, gsum, vm_pre[j],
                            vv_pre[j]);
          }
        }
      }  // regression / BCE losses
    }
  };
  bool split = false;
  if constexpr (MWT::on) split = TRAIN && ly.bn != 0;
  if (split) {
    if constexpr (MWT::on) {
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) epi_a(j);
      // batch statistics from every workgroup's (sum, centred second moment), workgroup order,
      // read as tagged granules (no grid barrier)
      const unsigned tag = mw_tag(*mw, mw->k);
      ++mw->k;
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) {
        const int n = wave + j * RX_NW;
        if (n >= ntiles) continue;
        const int c = n * 16 + lr;
        const int cc = c < ly.out ? c : 0;
        float mean, M2;
        mw_reduce_pairs<true>(*mw, mw_fwd(mw->part, mw->stride, ly, 0) + 4 * cc, lg, tag, n_batch, T::BP, mean, M2);
        bn_mean[j] = mean;
        bn_var[j] = M2 / (float)n_batch;
      }
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) epi_b(j);
    }
  } else {
#pragma unroll
    for (int j = 0; j < T::NTW; ++j) {
      epi_a(j);
      epi_b(j);
    }
  }
  fst(2);
  __syncthreads();  // every wave finished reading R for this layer
  fst(3);
  if (last && !TRAIN) return;

  // ---- publish y (or G_{L-1}) as bf16: row-major into R, transposed into XT_{l+1} / GT ----
  const int XS = T::XS;
  u16* dstT = last ? GT : reinterpret_cast<u16*>(smem + nx.xt_off);
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    const int n = wave + j * RX_NW;
    if (n < ntiles) {
      const int c = n * 16 + lr;
      const int tsw = T::swz(c);
      uint2 pk[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        pk[mt].x = rx_f2bf2(acc[j * MT + mt][0], acc[j * MT + mt][1]);
        pk[mt].y = rx_f2bf2(acc[j * MT + mt][2], acc[j * MT + mt][3]);
        if (TRAIN || !last)
          *reinterpret_cast<uint2*>(dstT + c * XS + ((((mt * 16 + lg * 4) >> 3) ^ tsw) << 3) + ((lg & 1) << 2)) = pk[mt];
      }
      if (!tmode) rx_publish_rows<MT>(R, RS, c, lane, pk);
    }
  }
  // zero the K padding [out_n, out_k) of the next GEMM's A operand so its K tail is exact
  const int kpad = (last ? ly.out_k : nx.in_k) - ly.out_n;
  if (tmode) {
    if (kpad > 0) zero_t_rows<MT, PS>(dstT, ly.out_n, ly.out_n + kpad);
  } else if (kpad > 0) {
    for (int idx = rx_tid<PS>(); idx < T::BP * kpad; idx += RX_THREADS) {
      const int row = idx / kpad, cc = ly.out_n + idx % kpad;
      R[rx_rix(row, cc, RS)] = 0;
    }
  }
  fst(4);
  __syncthreads();
}

// ------------------------------------------------------------------------------------------
// backward of layer l: G_l is in R (row-major) and GT (transposed).
// ------------------------------------------------------------------------------------------
// PS (persistent epoch kernel): once this layer's dgrad has read its last weight byte and its
// G^T export has drained, lane 0 publishes flag `sync[32 l] = step + 1` -- the optimizer
// workgroups of layer l may then compute dW_l and rewrite W_l / Wt_l while the backward goes on.
template <int MT, bool PS, bool FULL = false, class D, class LY, class PV, class MWT = NoMw, class VO = PsVec<>>
__device__ __forceinline__ void layer_backward(const D& d, const LY& ly, const PV& pv, int l, char* smem,
                                               const u16* __restrict__ img, const float* __restrict__ P,
                                               float* __restrict__ Gr, int nvalid, const float* __restrict__ scratch,
                                               unsigned long long* __restrict__ stamps,
                                               unsigned* __restrict__ sync = nullptr, int step = 0,
                                               bool ps_wt = true, MWT* mw = nullptr, VO vo = VO{},
                                               const bf16x8* w0b = nullptr) {
  using T = Tile<MT>;
  // persistent epoch with layer 0 updated in the step workgroup: layer 0's saved BN input is not
  // stored but recomputed here (l == 1) from the X^T_0 copy and the B fragments still in
  // registers -- the forward's very MFMAs, bias and ReLU, so the same bits -- instead of 64 KB
  // through memory each way (one CU's bandwidth: ~1.5 us a step at NYC)
  const bool rec0 = w0b != nullptr && l == 1;
  const int lane = rx_tid<PS>() & 63, wave = rx_wave<PS>();
  const int lr = lane & 15, lg = lane >> 4;
  const int RS = d.max_k + RX_RPAD;
  const int XS = T::XS;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* GT = reinterpret_cast<u16*>(smem + d.gt_lds_off);
  const u16* XT = reinterpret_cast<const u16*>(smem + ly.xt_off);
  float* stats = reinterpret_cast<float*>(smem + d.stats_lds_off);

  // ---- prefetch what the dgrad and the post-op backward read from global memory (the head of
  // every dgrad weight tile of this wave, and the saved forward values of the post-op) so both
  // round trips overlap the wgrad below instead of following it. Address-clamped, no
  // per-element branches; tiles past RX_PJ fetch in the dgrad itself.
  const int ntiles_d = ly.in_n >> 4;
  bf16x8 wpre[RX_PJ][RX_PK];
  float svp[RX_PJ][MT * 4];
  if (l != 0) {
    gemm_prefetch_flat<PS>(wpre, img, ly.wt_img, ntiles_d, ly.out_k, wave, lr, lg);
#pragma unroll
    for (int j = 0; j < RX_PJ; ++j) {
      if (j * RX_NW < ntiles_d && !rec0) {
        const int n = min(wave + j * RX_NW, ntiles_d - 1);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const f32x4 t = sv_load<MT>(pv, smem, scratch, n, mt, lane);
#pragma unroll
          for (int r = 0; r < 4; ++r) svp[j][mt * 4 + r] = t[r];
        }
      }
    }
  }
  // moments of the parameters of layer l-1 this lane updates in the post-op (persistent kernel)
  float vm_pre[T::NTW], vv_pre[T::NTW];
  if constexpr (PS) {
    if (l != 0 && vo.o != nullptr) {
#pragma unroll
      for (int j = 0; j < T::NTW; ++j)
        if (j * RX_NW < ntiles_d)
          ps_vec_prefetch(vo, pv, lg, min(wave + j * RX_NW, ntiles_d - 1) * 16 + lr, vm_pre[j], vv_pre[j]);
    }
  }

  if (d.wgrad_mode == 1) {
    // G^T_l leaves for the optimizer kernel's wgrad (GT is overwritten with G_{l-1} below)
    if constexpr (MWT::on)
      export_rows<MT, true>(GT, ly.out_n, Gr, d.act_off * 4 + ly.gg_off * 2, ps_wt, mw->G * T::BP, mw->wg * T::BP);
    else
      export_rows<MT, PS>(GT, ly.out_n, Gr, d.act_off * 4 + ly.gg_off * 2, ps_wt);
  } else
  // ---- wgrad, computed transposed: dW^T[i][o] = sum_b X[b][i] G[b][o]  (A = XT, B = GT) ----
  // each lane then holds 4 consecutive i of one o = 16 contiguous bytes of dW[o][:] ->
  // one dwordx4 store instead of four dword stores (the step is store-queue bound here).
  // Register blocking: a wave owns whole rows (or columns) of the tile grid and keeps that
  // side's fragments in registers while it streams the other side, so every XT / GT fragment
  // leaves LDS once per wave instead of once per tile (LDS bandwidth bound otherwise).
  {
    const int mo_tiles = ly.out_n >> 4, ni_tiles = ly.in_n >> 4;
    const bool vec = ((ly.w_off | ly.in) & 3) == 0;
    constexpr int KS = T::BP / 32;
    constexpr int NB = 4;  // tiles of the cached side per wave (larger grids loop)
    auto store = [&](int mo, int ni, const f32x4& a4) {
      const int o = mo * 16 + lr, i0 = ni * 16 + lg * 4;
      if (o < ly.out) {
        float* dst = Gr + ly.w_off + o * ly.in + i0;
        if (vec && i0 + 3 < ly.in) {
          *reinterpret_cast<f32x4*>(dst) = a4;   // (write-through sc1 stores measured no faster)
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (i0 + r < ly.in) dst[r] = a4[r];
        }
      }
    };
    if (ni_tiles >= mo_tiles) {
      // waves own ni tiles (XT rows cached), GT streamed once per block of NB tiles
      for (int nb0 = wave; nb0 < ni_tiles; nb0 += RX_NW * NB) {
        bf16x8 xa[NB][KS];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int ni = min(nb0 + q * RX_NW, ni_tiles - 1);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            xa[q][ks] = *reinterpret_cast<const bf16x8*>(XT + T::tix(ni * 16 + lr, ks * 32 + 8 * lg));
        }
        for (int mo = 0; mo < mo_tiles; ++mo) {
          bf16x8 gb[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            gb[ks] = *reinterpret_cast<const bf16x8*>(GT + T::tix(mo * 16 + lr, ks * 32 + 8 * lg));
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            const int ni = nb0 + q * RX_NW;
            if (ni < ni_tiles) {
              f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) a4 = rx_mfma16(xa[q][ks], gb[ks], a4);
              store(mo, ni, a4);
            }
          }
        }
      }
    } else {
      // waves own mo tiles (GT rows cached), XT streamed
      for (int mb0 = wave; mb0 < mo_tiles; mb0 += RX_NW * NB) {
        bf16x8 gb[NB][KS];
#pragma unroll
        for (int q = 0; q < NB; ++q) {
          const int mo = min(mb0 + q * RX_NW, mo_tiles - 1);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            gb[q][ks] = *reinterpret_cast<const bf16x8*>(GT + T::tix(mo * 16 + lr, ks * 32 + 8 * lg));
        }
        for (int ni = 0; ni < ni_tiles; ++ni) {
          bf16x8 xa[KS];
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            xa[ks] = *reinterpret_cast<const bf16x8*>(XT + T::tix(ni * 16 + lr, ks * 32 + 8 * lg));
#pragma unroll
          for (int q = 0; q < NB; ++q) {
            const int mo = mb0 + q * RX_NW;
            if (mo < mo_tiles) {
              f32x4 a4 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) a4 = rx_mfma16(xa[ks], gb[q][ks], a4);
              store(mo, ni, a4);
            }
          }
        }
      }
    }
  }
#ifdef RX_LAYER_STAMPS
  if (stamps != nullptr && rx_tid<PS>() == 0) rx_g(stamps)[20 + 4 * l] = __builtin_amdgcn_s_memtime();
#endif
  if (l == 0) return;   // (multi-workgroup step: layer 0 counts in with the bias gradients)

  // ---- dgrad: dX[b][i] = sum_o G[b][o] W[o][i]  (A = R or the G^T image, B = Wt, K = out_k) ----
  // pv (layer l-1) owns the post-ops between layer l-1 and l
  const int ntiles = ly.in_n >> 4;
  const bool tmode = d.r_lds_off < 0;
  const AOp Aop{tmode ? GT : R, RS, tmode};
  f32x4 acc[T::NTW * MT];
#pragma unroll
  for (int j = 0; j < T::NTW; ++j) {
    f32x4 part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) part[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int n = wave + j * RX_NW;
    if (n < ntiles) {
      const int boff = ly.wt_img + (n * 16 + lr) * ly.out_k;
      gemm_tile_pre<MT, PS>(part, Aop, lane, img, boff, ly.out_k, lg, wpre, j);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[j * MT + mt] = part[mt];
  }
#ifdef RX_LAYER_STAMPS
  if (stamps != nullptr && rx_tid<PS>() == 0) rx_g(stamps)[21 + 4 * l] = __builtin_amdgcn_s_memtime();
#endif
  bool cnt = PS;
  if constexpr (MWT::on) cnt = mw->opt.od != nullptr;
  if (cnt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's X^T / G^T exports drained
  __syncthreads();  // all reads of G_l (R, GT) are done; they are overwritten with G_{l-1}
  if constexpr (PS) {
    if (rx_tid<PS>() == 0) __hip_atomic_store(rx_g(sync) + 32 * l, (unsigned)(step + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if constexpr (MWT::on) {   // layer l's optimizer tasks may start (mlp_mwopt.h)
    if (cnt && threadIdx.x < RX_LCNT_REP)
      __hip_atomic_fetch_add(rx_g(mw->lcnt) + threadIdx.x * 32 + l, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef RX_LAYER_STAMPS
  if (stamps != nullptr && rx_tid<PS>() == 0) rx_g(stamps)[22 + 4 * l] = __builtin_amdgcn_s_memtime();
#endif

  // ---- post-op backward of layer l-1 (BN / act), producing G_{l-1} ----
  // mode 0: one workgroup, batch sums from its own rows. Multi-workgroup with BN: mode 1
  // publishes this workgroup's partial sums of dL/dy and dL/dy * x_hat, a grid barrier, then
  // mode 2 recomputes the (cheap) per-element terms and finishes with the batch sums.
  const int n_batch = MWT::on ? mw->n_total : (FULL ? T::BP : nvalid);
  const float inv_n = 1.f / (float)n_batch;
  const bool cols_full = pv.out == pv.out_n;
  float bsg[T::NTW], bsgx[T::NTW];
  auto post = [&](int j, int mode) {
    const int n = wave + j * RX_NW;
    if (n >= ntiles) return;
    const int c = n * 16 + lr;
    const bool colok = cols_full || c < pv.out;
    // The forward saved this layer's BN input / activation (fp32) for every padded row and
    // column: issue all loads back to back, unconditionally (a load under a per-element
    // branch is waited for on its own -> one dependent L2 round trip per element).
    float sv[MT * 4], g[MT * 4];
    if (rec0) {
      // layer 0's BN input: z = X_0 W_0^T (k order pi) + b, ReLU first when it precedes the BN
      const AOp X0{reinterpret_cast<const u16*>(smem + d.x0c_lds_off), 0, true};
      const float b0 = reinterpret_cast<const float*>(smem + d.pr_lds_off)[pv.pr_off + c];
      const bf16x8 bw = w0b[j < RX_W0J ? j : 0];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x4 z = rx_mfma16(ld_afrag_pi<MT>(X0, mt, lane), bw, f32x4{0.f, 0.f, 0.f, 0.f}) + f32x4{b0, b0, b0, b0};
        if (pv.bn != 2 && pv.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) z[r] = fmaxf(z[r], 0.f);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[mt * 4 + r] = z[r];
      }
    } else if (j < RX_PJ) {
#pragma unroll
      for (int q = 0; q < MT * 4; ++q) sv[q] = svp[j < RX_PJ ? j : 0][q];
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x4 t = sv_load<MT>(pv, smem, scratch, n, mt, lane);
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[mt * 4 + r] = t[r];
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const f32x4 gm = colok ? rx_rowmask<FULL>(acc[j * MT + mt], mt, lg, nvalid) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) g[mt * 4 + r] = gm[r];
    }
    float sg = 0.f, sgx = 0.f;   // batch sums of dL/dy and dL/dy * x_hat (BatchNorm)
    if (pv.bn == 0) {
      if (pv.act == 1) {
#pragma unroll
        for (int q = 0; q < MT * 4; ++q) g[q] = sv[q] > 0.f ? g[q] : 0.f;
      }
    } else {
      const float mean = colok ? stats[pv.stat_off + 2 * c] : 0.f;
      const float invstd = colok ? stats[pv.stat_off + 2 * c + 1] : 0.f;
      const float* ppr = reinterpret_cast<const float*>(smem + d.pr_lds_off) + pv.pr_off;
      const float gam = ppr[pv.out_n + c];
      const float bet = ppr[2 * pv.out_n + c];
      const bool relu_after = pv.bn == 2 && pv.act == 1;
      const bool relu_before = pv.bn == 1 && pv.act == 1;
      // x_hat = (x - mean) * invstd as one fma: x * invstd + (-mean * invstd)
      const float xb = -mean * invstd;
      f32x4 xh4[MT], g4[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x4 sv4 = f32x4{sv[mt * 4], sv[mt * 4 + 1], sv[mt * 4 + 2], sv[mt * 4 + 3]};
        xh4[mt] = __builtin_elementwise_fma(sv4, f32x4{invstd, invstd, invstd, invstd}, f32x4{xb, xb, xb, xb});
        g4[mt] = f32x4{g[mt * 4], g[mt * 4 + 1], g[mt * 4 + 2], g[mt * 4 + 3]};
        if (relu_after) {
#pragma unroll
          for (int r = 0; r < 4; ++r) g4[mt][r] = fmaf(xh4[mt][r], gam, bet) > 0.f ? g4[mt][r] : 0.f;
        }
      }
      if (mode == 2) {
        sg = bsg[j];
        sgx = bsgx[j];
      } else {
        // batch sums of dL/dy and dL/dy * x_hat: packed-fp32 trees, then across the lane groups
        f32x4 a4 = g4[0], b4 = g4[0] * xh4[0];
#pragma unroll
        for (int mt = 1; mt < MT; ++mt) {
          a4 += g4[mt];
          b4 = __builtin_elementwise_fma(g4[mt], xh4[mt], b4);
        }
        sg = rx_colsum16((a4[0] + a4[1]) + (a4[2] + a4[3]));
        sgx = rx_colsum16((b4[0] + b4[1]) + (b4[2] + b4[3]));
      }
      if (mode == 1) {
        if (colok && lg == 0) {
          if constexpr (MWT::on)
            mw_put_pair(*mw, mw_bwd(mw->part, mw->stride, pv, mw->wg) + 4 * c, sg, sgx, mw_tag(*mw, mw->k));
        }
        return;
      }
      bool owner = true;   // gamma / beta gradients are batch sums: one workgroup writes them
      if constexpr (MWT::on) owner = mw->wg == 0 && mw->ok;
      if (colok && lg == 0 && owner) {
        if constexpr (MWT::on) {   // write-through: the fused optimizer reads them in this launch
          if (pv.g_off >= 0) rx_st_sc1f(Gr + pv.g_off + c, sgx);
          if (pv.be_off >= 0) rx_st_sc1f(Gr + pv.be_off + c, sg);
        } else {
          if (pv.g_off >= 0) Gr[pv.g_off + c] = sgx;
          if (pv.be_off >= 0) Gr[pv.be_off + c] = sg;
        }
      }
      // dz = gamma * invstd * (g - sg / n - x_hat * sgx / n) = k1 * g + (c1 - x_hat * c2)
      const float k1 = gam * invstd;
      const float c1 = -k1 * (sg * inv_n), c2 = k1 * (sgx * inv_n);
      const f32x4 k14 = f32x4{k1, k1, k1, k1}, c14 = f32x4{c1, c1, c1, c1}, c24 = f32x4{-c2, -c2, -c2, -c2};
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x4 dz = __builtin_elementwise_fma(g4[mt], k14, __builtin_elementwise_fma(xh4[mt], c24, c14));
        if (relu_before) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dz[r] = sv[mt * 4 + r] > 0.f ? dz[r] : 0.f;
        }
        dz = colok ? rx_rowmask<FULL>(dz, mt, lg, nvalid) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) g[mt * 4 + r] = dz[r];
      }
    }
    // bias grad of layer l-1 (multi-workgroup: this workgroup's partial, reduced at step end)
    f32x4 bs4 = f32x4{g[0], g[1], g[2], g[3]};
#pragma unroll
    for (int mt = 1; mt < MT; ++mt) bs4 += f32x4{g[mt * 4], g[mt * 4 + 1], g[mt * 4 + 2], g[mt * 4 + 3]};
    const float bs = rx_colsum16((bs4[0] + bs4[1]) + (bs4[2] + bs4[3]));
    if (colok && lg == 0 && pv.b_off >= 0) {
      if constexpr (MWT::on)
        mw_put_one(*mw, mw_bias(mw->part, mw->stride, pv, mw->wg) + 2 * c, bs, mw_tag(*mw, 31));
      else
        Gr[pv.b_off + c] = bs;
    }
    if constexpr (PS) {
      if (vo.o != nullptr)
        ps_vec_update(vo, pv, reinterpret_cast<float*>(smem + d.pr_lds_off), lg, c, colok,
                      lg == 0 ? bs : (lg == 1 ? sgx : sg), vm_pre[j], vv_pre[j]);
    }
    // publish G_{l-1}: transposed into GT, row-major into R (quad-transposed 8-B stores)
    uint2 pk[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      pk[mt].x = rx_f2bf2(g[mt * 4 + 0], g[mt * 4 + 1]);
      pk[mt].y = rx_f2bf2(g[mt * 4 + 2], g[mt * 4 + 3]);
      *reinterpret_cast<uint2*>(GT + T::tix(c, mt * 16 + lg * 4)) = pk[mt];
    }
    if (!tmode) rx_publish_rows<MT>(R, RS, c, lane, pk);
  };
  bool split = false;
  if constexpr (MWT::on) split = pv.bn != 0;
  if (split) {
    if constexpr (MWT::on) {
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) post(j, 1);
      const unsigned tag = mw_tag(*mw, mw->k);
      ++mw->k;
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) {
        const int n = wave + j * RX_NW;
        if (n >= ntiles) continue;
        const int c = n * 16 + lr;
        const int cc = c < pv.out ? c : 0;
        float sg, sgx;
        mw_reduce_pairs<false>(*mw, mw_bwd(mw->part, mw->stride, pv, 0) + 4 * cc, lg, tag, 0, T::BP, sg, sgx);
        bsg[j] = sg;
        bsgx[j] = sgx;
      }
#pragma unroll
      for (int j = 0; j < T::NTW; ++j) post(j, 2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < T::NTW; ++j) post(j, 0);
  }
#ifdef RX_LAYER_STAMPS
  if (stamps != nullptr && rx_tid<PS>() == 0) rx_g(stamps)[23 + 4 * l] = __builtin_amdgcn_s_memtime();
#endif
  // zero the K tail [out_n, out_k) of G_{l-1} for the next dgrad
  const int kpad = pv.out_k - pv.out_n;
  if (tmode) {
    if (kpad > 0) zero_t_rows<MT, PS>(GT, pv.out_n, pv.out_k);
  } else if (kpad > 0) {
    for (int idx = rx_tid<PS>(); idx < T::BP * kpad; idx += RX_THREADS) {
      const int row = idx / kpad, cc = pv.out_n + idx % kpad;
      R[rx_rix(row, cc, RS)] = 0;
    }
  }
  __syncthreads();
}


// Stage every layer's per-column parameters (bias, BN gamma/beta, running mean/var) into LDS
// with ONE burst of independent loads per thread (column c = rx_tid() of every layer,
// address-clamped so no load sits behind a per-element branch).
template <class C, class D>
__device__ __forceinline__ void load_params(const D& d, char* smem, const float* __restrict__ P,
                                            const float* __restrict__ rstats) {
  float* pr = reinterpret_cast<float*>(smem + d.pr_lds_off);
  const int c = rx_tid<false>();
  float v[RX_MAXL][5];
  C::each_layer(d, [&](const auto& ly, int l) {
    const bool ok = c < ly.out;
    const int cc = ok ? c : 0;
    const float b = rx_g(P)[ly.b_off >= 0 ? ly.b_off + cc : 0];
    const float g = rx_g(P)[ly.g_off >= 0 ? ly.g_off + cc : 0];
    const float be = rx_g(P)[ly.be_off >= 0 ? ly.be_off + cc : 0];
    const float rm = rx_g(rstats)[ly.rs_off >= 0 ? ly.rs_off + cc : 0];
    const float rv = rx_g(rstats)[ly.rs_off >= 0 ? ly.rs_off + ly.out + cc : 0];
    v[l][0] = (ok && ly.b_off >= 0) ? b : 0.f;
    v[l][1] = (ok && ly.g_off >= 0) ? g : 1.f;
    v[l][2] = (ok && ly.be_off >= 0) ? be : 0.f;
    v[l][3] = (ok && ly.rs_off >= 0) ? rm : 0.f;
    v[l][4] = (ok && ly.rs_off >= 0) ? rv : 1.f;
  });
  C::each_layer(d, [&](const auto& ly, int l) {
    if (c < ly.out_n) {
#pragma unroll
      for (int k = 0; k < 5; ++k) pr[ly.pr_off + k * ly.out_n + c] = v[l][k];
    }
  });
}

// write the updated BatchNorm running statistics back (once per step, after the forward)
template <class C, class D>
__device__ __forceinline__ void store_running_stats(const D& d, char* smem, float* __restrict__ rstats) {
  const float* pr = reinterpret_cast<const float*>(smem + d.pr_lds_off);
  const int c = rx_tid<false>();
  C::each_layer(d, [&](const auto& ly, int) {
    if (ly.rs_off >= 0 && c < ly.out) {
      rx_g(rstats)[ly.rs_off + c] = pr[ly.pr_off + 3 * ly.out_n + c];
      rx_g(rstats)[ly.rs_off + ly.out + c] = pr[ly.pr_off + 4 * ly.out_n + c];
    }
  });
}

// The labels the loss of a single-tile output layer (out <= 16 columns: wave 0, tile 0) reads,
// fetched right after the batch's row indices are known: their dependent global round trip
// overlaps the forward instead of sitting in the last layer's epilogue.
// batch row whose label lands in slot q of this lane (-1: unused): the row-per-lane loss reads
// rows lane + 64 q, the tile layout rows (q >> 2) 16 + 4 lg + (q & 3)
template <int MT, class D>
__device__ __forceinline__ int label_row(const D& d, int lane, int q) {
  constexpr int BP = Tile<MT>::BP;
  if (d.loss_lds_off >= 0 && d.loss != 4) {
    const int r = lane + 64 * q;
    return q < (BP > 64 ? BP / 64 : 1) ? (r < BP ? r : 0) : -1;
  }
  return (q >> 2) * 16 + (lane >> 4) * 4 + (q & 3);
}

// the labels given each slot's data-row index (rix[q], from label_row through the batch's rows)
template <int MT, bool PS, class D>
__device__ __forceinline__ void prefetch_labels_rows(const D& d, const float* __restrict__ labels,
                                                     const int (&rix)[MT * 4], float (&tl)[MT * 4]) {
  const int lane = rx_tid<PS>() & 63, lr = lane & 15;
  const bool rowloss = d.loss_lds_off >= 0 && d.loss != 4;
  const int cl = !rowloss && lr < d.out_dim ? lr : 0;
#pragma unroll
  for (int q = 0; q < MT * 4; ++q)
    if (label_row<MT>(d, lane, q) >= 0) tl[q] = rx_g(labels)[rix[q] * d.out_dim + cl];
}

template <int MT, bool PS, class D>
__device__ __forceinline__ void prefetch_labels(const D& d, const float* __restrict__ labels, const int* rowidx,
                                                float (&tl)[MT * 4]) {
  const int lane = rx_tid<PS>() & 63;
  int rix[MT * 4];
#pragma unroll
  for (int q = 0; q < MT * 4; ++q) {
    const int r = label_row<MT>(d, lane, q);
    rix[q] = rowidx[r >= 0 ? r : 0];
  }
  prefetch_labels_rows<MT, PS>(d, labels, rix, tl);
}

// Embedding front: build layer 0's input [BP][in_k] from the raw feature rows -- dense columns
// copied, embedding columns gathered from the fp32 master tables in P (rounded to bf16 like
// every other activation). Ids come from bf16 features (exact for ids < 256, the host's limit);
// an id outside [0, rows) is clamped and counted in metrics[6] (the host raises on it).
template <int MT, bool PS, class D, class L0>
__device__ __forceinline__ void load_front(const D& d, const MlpDesc* __restrict__ dp, const L0& l0, char* smem,
                                           const u16* __restrict__ feats, const float* __restrict__ P,
                                           const int* __restrict__ rowidx, int nvalid, bool need_t,
                                           double* __restrict__ metrics) {
  using T = Tile<MT>;
  const int RS = d.max_k + RX_RPAD;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* XT = reinterpret_cast<u16*>(smem + l0.xt_off);
  const int in_k = l0.in_k, fn = d.front_n;
  int bad = 0;
  for (int idx = rx_tid<PS>(); idx < T::BP * in_k; idx += RX_THREADS) {
    const int row = idx / in_k, k = idx - row * in_k;
    u16 v = 0;
    if (row < nvalid && k < fn) {
      const FrontCol fc = dp->front[k];
      const u16 raw = rx_g(feats)[(size_t)rowidx[row] * d.feat_k + fc.src];
      if (fc.poff < 0) {
        v = raw;
      } else {
        int id = (int)rx_bf2f(raw);
        if (id < 0 || id >= fc.rows) {
          bad = 1;
          id = id < 0 ? 0 : fc.rows - 1;
        }
        v = rx_f2bf(rx_g(P)[fc.poff + id * fc.stride]);
      }
    }
    R[rx_rix(row, k, RS)] = v;
    if (need_t && k < l0.in_n) XT[T::tix(k, row)] = v;
  }
  if (bad && metrics != nullptr) atomicAdd(&metrics[6], 1.0);
  __syncthreads();
}

// Embedding front, backward: dX_0 = G_0 W_0 for the front's columns (one 16-column dgrad tile
// per wave), then every (column, table row) pair sums its rows' dX in row order and STORES the
// table element's gradient -- deterministic, and every element of every table is written each
// step (no zeroing, no atomics). G_0 is still in R (layer 0's backward only exported it); the
// G^T area is free and holds dX [BP][in_n] fp32 and the ids [BP][front_n] int16.
template <int MT, class D, class L0>
__device__ __forceinline__ void front_backward(const D& d, const MlpDesc* __restrict__ dp, const L0& l0, char* smem,
                                               const u16* __restrict__ img, float* __restrict__ Gr,
                                               const u16* __restrict__ feats, const int* __restrict__ rowidx,
                                               int nvalid) {
  using T = Tile<MT>;
  const int lane = rx_tid<false>() & 63, wave = rx_wave<false>();
  const int lr = lane & 15, lg = lane >> 4;
  const int RS = d.max_k + RX_RPAD;
  const u16* R = reinterpret_cast<const u16*>(smem + d.r_lds_off);
  float* dx = reinterpret_cast<float*>(smem + d.gt_lds_off);
  short* ids = reinterpret_cast<short*>(dx + T::BP * l0.in_n);
  const int fn = d.front_n;
  __syncthreads();  // layer 0's G^T export has read the G^T area
  for (int n = wave; n < (l0.in_n >> 4); n += RX_NW) {
    f32x4 part[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) part[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const AOp A{R, RS, false};   // (the embedding front always keeps the R image)
    gemm_tile<MT, false>(part, A, lane, img, l0.wt_img + (n * 16 + lr) * l0.out_k, 0, l0.out_k >> 5, lg);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) dx[(mt * 16 + lg * 4 + r) * l0.in_n + n * 16 + lr] = part[mt][r];
  }
  for (int idx = rx_tid<false>(); idx < T::BP * fn; idx += RX_THREADS) {
    const int row = idx / fn, k = idx - row * fn;
    const FrontCol fc = dp->front[k];
    int id = -1;
    if (row < nvalid && fc.poff >= 0) {
      id = (int)rx_bf2f(rx_g(feats)[(size_t)rowidx[row] * d.feat_k + fc.src]);
      id = id < 0 ? 0 : (id >= fc.rows ? fc.rows - 1 : id);
    }
    ids[row * fn + k] = (short)id;
  }
  __syncthreads();
  for (int q = rx_tid<false>(); q < d.front_q; q += RX_THREADS) {
    int k = 0;
    while (k + 1 < fn && dp->front_qbase[k + 1] <= q) ++k;
    while (k + 1 < fn && dp->front[k].poff < 0) ++k;  // a dense column shares the next one's qbase
    const FrontCol fc = dp->front[k];
    const int v = q - dp->front_qbase[k];
    float s = 0.f;
    for (int row = 0; row < nvalid; ++row) s += ids[row * fn + k] == v ? dx[row * l0.in_n + k] : 0.f;
    Gr[fc.poff + v * fc.stride] = s;
  }
}

// load the batch's feature rows (gathered through the epoch permutation) into R and XT_0
template <int MT, bool PS = false, class D, class L0>
__device__ __forceinline__ void load_inputs(const D& d, const L0& l0, char* smem, const u16* __restrict__ feats,
                                            const int* __restrict__ rowidx, int nvalid, bool need_t,
                                            const MlpDesc* __restrict__ dp = nullptr,
                                            const float* __restrict__ P = nullptr,
                                            double* __restrict__ metrics = nullptr) {
  if (d.front_n > 0) {
    load_front<MT, PS>(d, dp, l0, smem, feats, P, rowidx, nvalid, need_t, metrics);
    return;
  }
  using T = Tile<MT>;
  const int RS = d.max_k + RX_RPAD;
  const bool tmode = d.r_lds_off < 0;   // the GEMM reads XT_0 itself
  need_t = need_t || tmode;
  u16* R = reinterpret_cast<u16*>(smem + d.r_lds_off);
  u16* XT = reinterpret_cast<u16*>(smem + l0.xt_off);
  // persistent epoch with layer 0 updated in the step workgroup: a second copy of X^T_0 that
  // outlives the forward (the transposed image is reused by every later layer)
  u16* XC = d.x0c_lds_off >= 0 ? reinterpret_cast<u16*>(smem + d.x0c_lds_off) : nullptr;
  const int in_n = l0.in_n;
  const int chunks = d.feat_k >> 3;  // 8 bf16 per 16-B chunk
  if (tmode && l0.in_k > in_n) {    // K tail rows [in_n, in_k) of XT_0 (never written below)
    zero_t_rows<MT, PS>(XT, in_n, l0.in_k);
  }
  for (int idx = rx_tid<PS>(); idx < T::BP * chunks; idx += RX_THREADS) {
    const int row = idx / chunks, ch = idx % chunks;
    u32x4 v = *reinterpret_cast<const RX_GLOBAL u32x4*>(rx_g(feats) + (size_t)rowidx[row] * d.feat_k + ch * 8);
    if (row >= nvalid) v = u32x4{0u, 0u, 0u, 0u};
    if (!tmode) *reinterpret_cast<u32x4*>(R + row * RS + ((ch ^ rx_rsw(row)) << 3)) = v;
    if (need_t) {
      const u16* h = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = ch * 8 + e;
        if (k < in_n) XT[T::tix(k, row)] = h[e];
        if (XC != nullptr && k < in_n) XC[T::tix(k, row)] = h[e];
      }
    }
  }
  __syncthreads();
}

// The batch gather split in two for the persistent step's prefetch (mlp_persist.h): the global
// read of chunk `idx` (row idx / chunks, 16 B of its features; zeros past nvalid) issued during
// the previous step's backward and kept in a register, and its LDS scatter at the start of the
// step -- one chunk per thread (BP * feat_k / 8 <= RX_THREADS), no embedding front.
// Chunk idx -> (batch row, 16-B chunk of its features). QUAD (T mode): the 4 lanes of a quad hold
// 4 consecutive rows of the same chunk, so scatter_input_quads can transpose them in registers.
template <bool QUAD>
__device__ __forceinline__ void input_chunk_pos(int idx, int chunks, int& row, int& ch) {
  if (QUAD) {
    ch = (idx >> 2) % chunks;
    row = ((idx >> 2) / chunks) * 4 + (idx & 3);
  } else {
    row = idx / chunks;
    ch = idx - row * chunks;
  }
}

// `rix`: the data row of this chunk's batch row
template <int MT, bool QUAD, class D>
__device__ __forceinline__ u32x4 gather_input_chunk(const D& d, const u16* __restrict__ feats, int rix, int nvalid,
                                                   int idx) {
  int row, ch;
  input_chunk_pos<QUAD>(idx, d.feat_k >> 3, row, ch);
  const u32x4 v = *reinterpret_cast<const RX_GLOBAL u32x4*>(rx_g(feats) + (size_t)rix * d.feat_k + ch * 8);
  return row < nvalid && row < Tile<MT>::BP ? v : u32x4{0u, 0u, 0u, 0u};
}

// T-mode scatter of quad-mapped chunks: two quad transposes turn 4 rows x 8 features into 8
// features x 4 rows, written as 8-B stores into XT_0 (and the X^T_0 copy) -- 2 + 2 LDS writes per
// lane instead of 16 two-byte ones (those hit 4-way bank conflicts: 4 feature rows 1 KB apart)
template <int MT, class D, class L0>
__device__ __forceinline__ void scatter_input_quads(const D& d, const L0& l0, char* smem, int idx, const u32x4& v) {
  using T = Tile<MT>;
  int row, ch;
  input_chunk_pos<true>(idx, d.feat_k >> 3, row, ch);
  const int q = idx & 3, row0 = row - q;
  const uint2 lo = rx_quad_transpose(make_uint2(v[0], v[1]), q);   // feature ch 8 + q, rows row0 .. +3
  const uint2 hi = rx_quad_transpose(make_uint2(v[2], v[3]), q);   // feature ch 8 + 4 + q
  if (row0 >= T::BP) return;
  u16* XT = reinterpret_cast<u16*>(smem + l0.xt_off);
  u16* XC = d.x0c_lds_off >= 0 ? reinterpret_cast<u16*>(smem + d.x0c_lds_off) : nullptr;
  const int k0 = ch * 8 + q, k1 = k0 + 4;
  if (k0 < l0.in_n) {
    *reinterpret_cast<uint2*>(XT + T::tix(k0, row0)) = lo;
    if (XC != nullptr) *reinterpret_cast<uint2*>(XC + T::tix(k0, row0)) = lo;
  }
  if (k1 < l0.in_n) {
    *reinterpret_cast<uint2*>(XT + T::tix(k1, row0)) = hi;
    if (XC != nullptr) *reinterpret_cast<uint2*>(XC + T::tix(k1, row0)) = hi;
  }
}
template <int MT, class D, class L0>
__device__ __forceinline__ void scatter_input_chunk(const D& d, const L0& l0, char* smem, int idx, const u32x4& v) {
  using T = Tile<MT>;
  const int chunks = d.feat_k >> 3;
  const int row = idx / chunks, ch = idx - (idx / chunks) * chunks;
  if (row >= T::BP) return;
  const bool tmode = d.r_lds_off < 0;
  const int RS = d.max_k + RX_RPAD;
  if (!tmode) *reinterpret_cast<u32x4*>(reinterpret_cast<u16*>(smem + d.r_lds_off) + row * RS + ((ch ^ rx_rsw(row)) << 3)) = v;
  u16* XT = reinterpret_cast<u16*>(smem + l0.xt_off);
  u16* XC = d.x0c_lds_off >= 0 ? reinterpret_cast<u16*>(smem + d.x0c_lds_off) : nullptr;
  const u16* h = reinterpret_cast<const u16*>(&v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = ch * 8 + e;
    if (k < l0.in_n) {
      XT[T::tix(k, row)] = h[e];
      if (XC != nullptr) XC[T::tix(k, row)] = h[e];
    }
  }
}

// One training step (forward, loss, backward -> gradients in Gr) for rows
// perm[row0 .. row0 + nvalid) of the epoch.
template <class C, int MT>
__device__ __forceinline__ void mlp_train_step_body(
    const MlpDesc* __restrict__ dp, const u16* __restrict__ img, float* __restrict__ rstats,
    const float* __restrict__ P, float* __restrict__ Gr, const u16* __restrict__ feats,
    const float* __restrict__ labels, const int* __restrict__ perm, int row0, int nvalid,
    float* __restrict__ scratch, double* __restrict__ metrics, unsigned long long* __restrict__ stamps,
    char* smem, int* rowidx) {
  auto&& d = C::desc(dp);
  RX_GLOBAL unsigned long long* st = rx_g(stamps);
  int si = 0;
#define RX_STAMP()                                                        \
  do {                                                                    \
    if (st != nullptr && rx_tid<false>() == 0) st[si] = __builtin_amdgcn_s_memtime(); \
    ++si;                                                                 \
  } while (0)
  RX_STAMP();
  bf16x8 wpre[RX_PJ][RX_PK];
  fwd_prefetch<false>(C::first(d), img, wpre, d.w0s_lds_off >= 0);
  for (int i = rx_tid<false>(); i < Tile<MT>::BP; i += RX_THREADS)
    rowidx[i] = i < nvalid ? (perm ? rx_g(perm)[row0 + i] : row0 + i) : (perm ? rx_g(perm)[row0] : row0);
  load_params<C>(d, smem, P, rstats);
  __syncthreads();
  load_inputs<MT>(d, C::first(d), smem, feats, rowidx, nvalid, true, dp, P, metrics);
  float labp[MT * 4];
  prefetch_labels<MT, false>(d, labels, rowidx, labp);
  RX_STAMP();
  auto body = [&](auto full) {
    constexpr bool F = decltype(full)::value;
    C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
      layer_forward<MT, true, false, F>(d, ly, nx, last, smem, img, P, Gr, labels, rowidx, nvalid, scratch, metrics,
                                        wpre, true, l, stamps, labp);
      RX_STAMP();
    });
    store_running_stats<C>(d, smem, rstats);
    C::bwd_layers(d, [&](const auto& ly, const auto& pv, int l) {
      layer_backward<MT, false, F>(d, ly, pv, l, smem, img, P, Gr, nvalid, scratch, stamps);
      RX_STAMP();
    });
  };
  if (nvalid == Tile<MT>::BP)
    body(rx_bool<true>{});
  else
    body(rx_bool<false>{});
  if (d.front_n > 0) front_backward<MT>(d, dp, C::first(d), smem, img, Gr, feats, rowidx, nvalid);
#undef RX_STAMP
}

// Multi-workgroup training step (see MwCtx): workgroup blockIdx.x of mw.G runs rows
// perm[row0 + wg * BP .. ) of a batch of mw.n_total rows. `scratch` is the whole scratch
// buffer; each workgroup saves its BN inputs / masks in its own `scratch_stride` floats. Needs
// wgrad_mode 1 and no embedding front (the host checks).
template <class C, int MT>
__device__ __forceinline__ void mlp_train_step_mw_body(
    const MlpDesc* __restrict__ dp, const u16* __restrict__ img, float* __restrict__ rstats,
    const float* __restrict__ P, float* __restrict__ Gr, const u16* __restrict__ feats,
    const float* __restrict__ labels, const int* __restrict__ perm, int row0, float* __restrict__ scratch,
    long long scratch_stride, double* __restrict__ metrics, MwCtx mw, char* smem, int* rowidx) {
  if (mw.opt.od != nullptr && (int)blockIdx.x >= mw.G) {   // an optimizer workgroup (mlp_mwopt.h)
    mw_opt_role(mw, mw.opt, smem);
    return;
  }
  auto&& d = C::desc(dp);
  constexpr int BP = Tile<MT>::BP;
  mw.wg = (int)blockIdx.x;
  mw.k = 0;
  mw.ok = 1;
  // per-step device timeline (the step-time histogram of multi-workgroup epochs)
  if (mw.tstamp != nullptr && mw.wg == 0 && threadIdx.x == 0) *rx_g(mw.tstamp) = wall_clock64();
  const int nvalid = mw_rows(mw.n_total, mw.wg, BP);
  const int r0 = row0 + mw.wg * BP;
  float* sc = scratch + (size_t)mw.wg * (size_t)scratch_stride;
  bf16x8 wpre[RX_PJ][RX_PK];
  fwd_prefetch<false>(C::first(d), img, wpre, d.w0s_lds_off >= 0);
  // padded rows (and every row of a workgroup past a short last batch) read the batch's first
  // row: always inside the input, masked to zero on load
  for (int i = rx_tid<false>(); i < BP; i += RX_THREADS)
    rowidx[i] = i < nvalid ? (perm ? rx_g(perm)[r0 + i] : r0 + i) : (perm ? rx_g(perm)[row0] : row0);
  load_params<C>(d, smem, P, rstats);
  __syncthreads();
  load_inputs<MT>(d, C::first(d), smem, feats, rowidx, nvalid, true, dp, P, metrics);
  float labp[MT * 4];
  prefetch_labels<MT, false>(d, labels, rowidx, labp);
#ifdef RX_LAYER_STAMPS
  unsigned long long* lst = mw.wg == 0 ? mw.lstamp : nullptr;
#else
  unsigned long long* lst = nullptr;
#endif
  C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
    layer_forward<MT, true, false>(d, ly, nx, last, smem, img, P, Gr, labels, rowidx, nvalid, sc, metrics, wpre,
                                   true, l, lst, labp, &mw);
  });
  // every workgroup computed the same batch statistics: one stores the running averages
  if (mw.wg == 0 && mw.ok) store_running_stats<C>(d, smem, rstats);
  C::bwd_layers(d, [&](const auto& ly, const auto& pv, int l) {
    layer_backward<MT, false>(d, ly, pv, l, smem, img, P, Gr, nvalid, sc, lst, nullptr, 0, true, &mw);
  });
  if (lst != nullptr && threadIdx.x == 0) rx_g(lst)[0] = __builtin_amdgcn_s_memtime();
  // bias gradients: the workgroups' partial column sums (tagged granules, phase 31), added in
  // workgroup order, each (layer, column) by one thread of the grid -- every wave polls (the
  // granule waits are wave-collective), threads past the columns on a clamped column
  if (lst != nullptr && threadIdx.x == 0) rx_g(lst)[1] = __builtin_amdgcn_s_memtime();
  C::each_layer(d, [&](const auto& ly, int) {
    if (ly.b_off >= 0) {
      for (int c0 = (int)blockIdx.x * RX_THREADS; c0 < ly.out; c0 += mw.G * RX_THREADS) {
        const int c = c0 + rx_tid<false>();
        const int base = (int)((mw_bias(mw.part, mw.stride, ly, 0) + 2 * (c < ly.out ? c : 0) - mw.part) * 4);
        float s = 0.f;
        for (int w0 = 0; w0 < mw.G; w0 += 8) {
          u32x4 v[8];
          int off[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            off[i] = base + min(w0 + i, mw.G - 1) * mw.stride * 4;
            const uint2 y = rx_load8_sc1(mw.part, off[i]);
            v[i] = u32x4{y.x, y.y, 0u, 0u};
          }
          mw_await<8, true>(mw, v, off, mw_tag(mw, 31));
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (w0 + i < mw.G) s += __uint_as_float(v[i][0]);
        }
        if (c < ly.out && mw.ok) rx_st_sc1f(Gr + ly.b_off + c, s);   // (a timed-out wait: incomplete partials)
      }
    }
  });
  // layer 0's G^T export drained while the bias gradients were reduced: its tasks and the vector
  // parameters' chunks may start
  mw_count_in(&mw, 0, RX_LCNT_VEC);
  mw_finish(mw);
}

// Evaluation: forward + loss metrics only; one workgroup per batch.
// chunked (a batch wider than one workgroup's BP rows): ceil(batch / BP) workgroups per batch,
// each on BP rows of ONE batch, so the loss is still the mean of per-batch means (the host's
// batch count comes from each batch's first chunk).
template <class C, int MT>
__device__ __forceinline__ void mlp_eval_body(const MlpDesc* __restrict__ dp, const u16* __restrict__ img,
                                              const float* __restrict__ rstats, const float* __restrict__ P,
                                              const u16* __restrict__ feats, const float* __restrict__ labels,
                                              int n_rows, int batch, double* __restrict__ metrics, char* smem,
                                              int* rowidx, int chunked = 0) {
  auto&& d = C::desc(dp);
  constexpr int BP = Tile<MT>::BP;
  bf16x8 wpre[RX_PJ][RX_PK];
  if (chunked) {
    const int cpb = (batch + BP - 1) / BP;
    const int b = (int)blockIdx.x / cpb, q = (int)blockIdx.x % cpb;
    const int nb = min(batch, n_rows - b * batch);
    const int row0 = b * batch + q * BP;
    const int nvalid = max(0, min(BP, nb - q * BP));
    if (nvalid <= 0) return;
    for (int i = rx_tid<false>(); i < BP; i += RX_THREADS) rowidx[i] = i < nvalid ? row0 + i : row0;
    load_params<C>(d, smem, P, rstats);
    __syncthreads();
    load_inputs<MT>(d, C::first(d), smem, feats, rowidx, nvalid, false, dp, P, metrics);
    fwd_prefetch<false>(C::first(d), img, wpre, d.w0s_lds_off >= 0);
    MwCtx ev{};
    ev.n_total = nb;   // the loss mean runs over the whole batch; chunk 0 counts the batch
    ev.wg = q;
    ev.G = cpb;
    C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
      layer_forward<MT, false, false>(d, ly, nx, last, smem, img, P, nullptr, labels, rowidx, nvalid, nullptr,
                                      metrics, wpre, true, l, nullptr, nullptr, &ev);
    });
    return;
  }
  const int row0 = blockIdx.x * batch;
  const int nvalid = min(batch, n_rows - row0);
  for (int i = rx_tid<false>(); i < BP; i += RX_THREADS) rowidx[i] = i < nvalid ? row0 + i : row0;
  load_params<C>(d, smem, P, rstats);
  __syncthreads();
  load_inputs<MT>(d, C::first(d), smem, feats, rowidx, nvalid, false, dp, P, metrics);
  fwd_prefetch<false>(C::first(d), img, wpre, d.w0s_lds_off >= 0);
  C::fwd_layers(d, [&](const auto& ly, const auto& nx, int l, bool last) {
    layer_forward<MT, false, false>(d, ly, nx, last, smem, img, P, nullptr, labels, rowidx, nvalid, nullptr, metrics,
                                    wpre, true, l);
  });
}
