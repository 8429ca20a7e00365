// One-shot all-reduce over xGMI peer memory: the device-side protocol shared by the stand-alone
// reduce kernel (csrc/comm/xgmi_allreduce.hip) and the fused "reduce + optimizer" kernel of the
// NYC step loop (csrc/hip/fused_mlp.hip).
//
// Why: the reference's gradient all-reduce is DDP/Horovod over NCCL rings
// (python/raydp/torch/estimator.py:243 prepare_model; examples/horovod_nyctaxi.py:133-138). The
// NYC model's whole gradient is 194 KB, so a ring is pure latency: 2*(N-1) link hops, each a
// kernel-to-kernel hand-off. MI355X GPUs of a node are fully connected by xGMI (7 links per
// GPU), so every rank can read every peer's gradient directly: one flag exchange, then each
// rank sums the N buffers itself (N-1 reads in parallel, one per link). No staging copy.
//
// Memory: each rank owns one exchange region allocated uncached (hipDeviceMallocUncached, so
// no L2 on either side holds a stale line) and exports it with hipIpcGetMemHandle:
//   [slot 0: nf floats][slot 1: nf floats][flags: RX_XG_MAXR u32][votes: 2 x RX_XG_MAXR u32]
//   [inbox: 2 x world x nf tagged u64 granules (rx_xg_push)]
// Step s writes its gradient into slot (s & 1) of its own region, then publishes seq = s + base
// by storing it into flags[rank] of EVERY peer's region, waits until its own flags[p] >= seq for
// every peer p, and reads slot (s & 1) of every region.
// Double buffering makes one flag round per step enough: rank r overwrites slot (s & 1) at step
// s + 2 only after its kernel of step s + 1 saw every peer's seq s + 1 flag, which each peer
// publishes only after its step-s kernel (the reads of slot (s & 1)) ended.
//
// One rendezvous per LAUNCH, not per workgroup: every workgroup counts itself in on a local
// arrival word; the last one to arrive does the cross-rank flag exchange and then opens a local
// "go" word the others spin on (rx_xg_grid_rendezvous). A 1 MiB bucket is one flag round.
//
// Sequence numbers: the fused step loop takes them on the host (rx_xg_take_seq); the stand-alone
// all-reduce keeps them on the device (ctl[1], bumped by the launch's last workgroup), so its
// launch arguments never change and a HIP graph can replay it. A communicator is used in one
// of the two modes only (raydp_amd/ops/comm.py keys them apart).
//
// Every wait is bounded (spin_ticks of the 100 MHz wall clock): a missing peer sets ctl[0] and
// the kernel returns instead of hanging the GPU; the host reads it with the epoch's metrics.
#pragma once
#include <hip/hip_runtime.h>

#define RX_XG_MAXR 16

// ctl words (this rank's local device memory, zeroed at create)
enum : int { kXgErr = 0, kXgDevSeq = 1, kXgArrive = 2, kXgGo = 3, kXgDone = 4, kXgCtlWords = 16 };

struct XgDev {
  float* region[RX_XG_MAXR];  // region base of rank p, mapped into this process
  unsigned* err;              // == ctl + kXgErr
  unsigned* ctl;              // local control words (kXg*)
  unsigned long long spin_ticks;
  int world, rank, nf;        // nf: floats per slot (multiple of 64)
  unsigned layout;            // RX_XG_LAYOUT of the code that allocated the regions
};

// Region layout version. Training kernels compiled at run time (raydp_amd/ops/mlp_jit.py) index
// the regions a prebuilt library allocated: a kernel whose layout differs exchanges nothing
// (rx_xg_usable: error word set, no update) instead of writing past a region.
#define RX_XG_LAYOUT 0x58470002u

__device__ __forceinline__ unsigned* rx_xg_flags(const XgDev& x, int p) {
  return reinterpret_cast<unsigned*>(x.region[p] + 2 * (size_t)x.nf);
}

// vote words of rank p's region for a meeting of sequence seq (double-buffered by parity)
__device__ __forceinline__ unsigned* rx_xg_votes(const XgDev& x, int p, unsigned seq) {
  return rx_xg_flags(x, p) + RX_XG_MAXR * (1 + (int)(seq & 1u));
}

__device__ __forceinline__ void rx_xg_fail(const XgDev& x) {
  __hip_atomic_store(x.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Publish `seq` to every peer and wait for theirs. Call from ONE lane. Returns false on timeout
// (after setting *err).
__device__ __forceinline__ bool rx_xg_rendezvous(const XgDev& x, unsigned seq) {
  // my slot was written before this call (previous kernel, or this launch's workgroups before
  // they counted themselves in): make it visible to readers on other devices before they can
  // see the flag
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  for (int p = 0; p < x.world; ++p)
    if (p != x.rank)
      __hip_atomic_store(rx_xg_flags(x, p) + x.rank, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned* mine = rx_xg_flags(x, x.rank);
  const long long t0 = wall_clock64();
  for (int p = 0; p < x.world; ++p) {
    if (p == x.rank) continue;
    while ((int)(__hip_atomic_load(mine + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
      if ((unsigned long long)(wall_clock64() - t0) > x.spin_ticks) {
        rx_xg_fail(x);
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  return true;
}

// Launch-wide rendezvous: `nblocks` workgroups of this launch call it (all threads). The last
// workgroup to arrive meets the peers; the others wait on the local go word. Returns false on
// every workgroup when the exchange failed. All `nblocks` workgroups must be able to be
// resident together (callers launch at most a few hundred small workgroups).
__device__ __forceinline__ bool rx_xg_grid_rendezvous(const XgDev& x, unsigned seq, unsigned nblocks) {
  __shared__ int ok_s;
  __syncthreads();  // this workgroup's slot writes are done
  if (threadIdx.x == 0) {
    int ok = 1;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // (system scope) my part of the slot
    const unsigned old = __hip_atomic_fetch_add(x.ctl + kXgArrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == nblocks - 1) {
      __hip_atomic_store(x.ctl + kXgArrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = rx_xg_rendezvous(x, seq) ? 1 : 0;
      // open the gate even on failure (the others read the error word next)
      __hip_atomic_store(x.ctl + kXgGo, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const long long t0 = wall_clock64();
      while ((int)(__hip_atomic_load(x.ctl + kXgGo, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - seq) < 0) {
        if ((unsigned long long)(wall_clock64() - t0) > x.spin_ticks) {
          rx_xg_fail(x);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (system scope) the peers' slots
    }
    if (ok && __hip_atomic_load(x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) ok = 0;
    ok_s = ok;
  }
  __syncthreads();
  return ok_s != 0;
}

// 16-byte system-coherent load from a (possibly peer-mapped) region: sc0|sc1, never a stale
// line of this device's caches.
__device__ __forceinline__ float4 rx_xg_load4(const float* base, size_t idx4) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7ffffff0, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(idx4 * 16), 0, 17);
  return __builtin_bit_cast(float4, v);
}

// Sum of element idx of slot `par` over all ranks, always in rank order so every rank computes
// bit-identical sums (replicas stay identical, as under DDP).
__device__ __forceinline__ float rx_xg_sum(const XgDev& x, int par, int idx) {
  const size_t off = (size_t)par * x.nf + idx;
  float s = 0.f;
  for (int p = 0; p < x.world; ++p)
    s += p == x.rank ? x.region[p][off]
                     : __hip_atomic_load(x.region[p] + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return s;
}

// ---- gradient exchange inside a training launch (persistent epoch / multi-workgroup step) ----
// The gradient all-reduce of the fused NYC engine at world > 1 without a launch, a pass or a
// rendezvous of its own: the lanes that finish a 32x32 weight tile's gradient (or a chunk of the
// bias / BatchNorm gradients) push it into every peer's inbox and sum the world values of each of
// their elements in rank order (bit-identical on every rank) before they update (rx_xg_push /
// rx_xg_pull_sum_n below). The NYC gradient crosses each link once per step as tagged granules
// (388 KB) instead of the batch-sized X^T / G^T exports (7.8 MB at batch 4096).
struct XgStep {
  const XgDev* xd;  // the communicator's descriptor in DEVICE memory (rx_xg_devptr): read with scalar
                    // loads, so a kernel argument holding this stays small and register-resident
  unsigned seq;     // sequence number of this launch's (first) step
  int on;           // 0: one GPU (nothing exchanged)
  float gscale;     // 1 / world: the DDP average
  int pad_;
};

__device__ __forceinline__ float* rx_xg_region(const XgDev& x, int p) { return x.region[p]; }

// A specialised one-GPU code object (raydp_amd/ops/mlp_jit.py, world 1) is compiled with
// RX_XG_KERNELS 0: every exchange branch of the training kernels folds away and the kernels keep
// the one-GPU register allocation. The ahead-of-time build keeps them (1).
#ifndef RX_XG_KERNELS
#define RX_XG_KERNELS 1
#endif
__device__ __forceinline__ bool rx_xg_active(const XgStep& xs) { return RX_XG_KERNELS && xs.on; }

// (after rx_xg_active) false -- and the error word set -- when the communicator's regions were laid
// out by other code than this kernel's
__device__ __forceinline__ bool rx_xg_usable(const XgDev& x) {
  if (x.layout == RX_XG_LAYOUT) return true;
  __hip_atomic_store(x.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return false;
}

typedef __attribute__((address_space(1))) unsigned rx_xg_gu;

// ---- tagged push exchange (the persistent epoch at world > 1) ----
// Latency, not bytes, bounds the per-step exchange of a small model: the flag protocol above is
// a drain (vmcnt 0) of the slot stores, a flag store, the peer's poll of it and then its read of
// the data -- two one-way trips plus a round trip before the peer can sum. Here every element
// travels ONCE, as an 8-B granule (value bits | seq << 32) stored straight into the receiving
// rank's inbox row for this sender; the receiver polls its own (local) inbox until the tag is the
// step's seq (MI355X_MICROARCH.md R2: poll the data itself, never a flag beside it). A 64-bit
// store is single-copy atomic, so a granule whose tag matches carries that step's value. Inbox
// reuse: parity (seq & 1) rows; a sender overwrites row (seq & 1) two steps later, after its own
// step seq + 1 summed the receiver's seq + 1 values, which the receiver pushed after it read
// this step's (program order on the receiving lane).
__device__ __forceinline__ unsigned long long* rx_xg_inbox(const XgDev& x, int at, int src, unsigned seq) {
  unsigned* tail = rx_xg_flags(x, at) + 3 * RX_XG_MAXR;   // 8-B aligned: nf % 64 == 0
  return reinterpret_cast<unsigned long long*>(tail) + ((size_t)(seq & 1u) * x.world + src) * x.nf;
}

typedef __attribute__((address_space(1))) unsigned long long rx_xg_gq;

// Where a lane's granules go and come from. XgView reads the communicator's descriptor (device
// memory, scalar loads); XgRowsView reads a table of row pointers one lane of the workgroup built
// in LDS before its step loop (rx_xg_rows_init), so no descriptor load sits between a tile's
// gradient and its pushes.
struct XgView {
  const XgDev& x;
  __device__ int world() const { return x.world; }
  __device__ int rank() const { return x.rank; }
  __device__ bool usable() const { return rx_xg_usable(x); }
  __device__ unsigned long long* out(int p, unsigned seq) const { return rx_xg_inbox(x, p, x.rank, seq); }
  __device__ const unsigned long long* in(int p, unsigned seq) const { return rx_xg_inbox(x, x.rank, p, seq); }
};

struct XgRows {
  unsigned long long* out0[RX_XG_MAXR];       // peer p's inbox row for this rank, parity 0
  const unsigned long long* in0[RX_XG_MAXR];  // this rank's inbox row for peer p, parity 0
  unsigned long long par;                     // elements from a parity-0 row to its parity-1 row
  int world, rank, ok, pad_;
};

// one lane; the workgroup joins a barrier before any lane uses the table
__device__ __forceinline__ void rx_xg_rows_init(const XgDev& x, XgRows* r) {
  r->world = x.world;
  r->rank = x.rank;
  r->ok = x.layout == RX_XG_LAYOUT ? 1 : 0;
  r->par = (unsigned long long)x.world * x.nf;
  for (int p = 0; p < x.world && r->ok; ++p) {
    r->out0[p] = rx_xg_inbox(x, p, x.rank, 0u);
    r->in0[p] = rx_xg_inbox(x, x.rank, p, 0u);
  }
}

struct XgRowsView {
  const XgRows* r;
  const XgDev& x;
  __device__ int world() const { return r->world; }
  __device__ int rank() const { return r->rank; }
  __device__ bool usable() const {
    if (r->ok) return true;
    return rx_xg_usable(x);
  }
  __device__ unsigned long long* out(int p, unsigned seq) const { return r->out0[p] + (seq & 1u) * r->par; }
  __device__ const unsigned long long* in(int p, unsigned seq) const { return r->in0[p] + (seq & 1u) * r->par; }
};

// This rank's value of flat element idx at sequence seq, into every peer's inbox.
template <class V>
__device__ __forceinline__ void rx_xg_push_v(const V& w, unsigned seq, int idx, float v) {
  const unsigned long long g = ((unsigned long long)seq << 32) | __float_as_uint(v);
  const int world = w.world(), rank = w.rank();
  for (int p = 0; p < world; ++p)
    if (p != rank) __hip_atomic_store((rx_xg_gq*)(w.out(p, seq) + idx), g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void rx_xg_push(const XgDev& x, unsigned seq, int idx, float v) {
  if (x.layout != RX_XG_LAYOUT) return;
  rx_xg_push_v(XgView{x}, seq, idx, v);
}

// N elements at once: val[n] (this rank's value on entry) becomes the rank-order sum of element
// idx[n] (for valid[n]). The loads for PG peers x N elements are issued back to back before any
// tag is checked, so a lane pays one round trip per PG peers, not one per element and peer (PG
// trades registers for round trips: the multi-workgroup step kernel has none to spare).
template <int N, int PG = 1, bool SENT = false, class V>
__device__ __forceinline__ void rx_xg_pull_sum_v(const V& w, const XgDev& x, unsigned seq, const int (&idx)[N],
                                                 const bool (&valid)[N], float (&val)[N], bool& ok) {
  if (!w.usable()) {
    ok = false;
    return;
  }
  float s[N];
#pragma unroll
  for (int n = 0; n < N; ++n) s[n] = 0.f;
  const int world = w.world(), rank = w.rank();
  // SENT: one lane per wave first waits for its LAST element of each peer (a peer lane pushes its
  // N elements in order, its wave's 64 lanes in one store each): the wave's loads below then find
  // the granules in place instead of every lane polling HBM while a late peer catches up (off in
  // the multi-workgroup step kernel: the divergent loop costs it scratch)
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int il = idx[N - 1];
  if (SENT && lane == 0 && valid[N - 1] && ok) {
    const unsigned long long t0 = wall_clock64();
    for (int p = 0; p < world; ++p) {
      if (p == rank) continue;
      const rx_xg_gq* a = (const rx_xg_gq*)(w.in(p, seq) + il);
      int k = 0;
      while ((unsigned)(__hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32) != seq) {
        __builtin_amdgcn_s_sleep(1);
        if ((++k & 15) == 0 && (unsigned long long)(wall_clock64() - t0) > x.spin_ticks) break;   // (the per-element wait below decides)
      }
    }
  }
  for (int p0 = 0; p0 < world; p0 += PG) {
    unsigned long long g[PG][N];
#pragma unroll
    for (int q = 0; q < PG; ++q) {
      const int p = p0 + q;
      const bool peer = p < world && p != rank;
      const rx_xg_gq* row = peer ? (const rx_xg_gq*)w.in(p, seq) : nullptr;
#pragma unroll
      for (int n = 0; n < N; ++n)
        g[q][n] = (peer && valid[n]) ? __hip_atomic_load(row + idx[n], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0ull;
    }
#pragma unroll
    for (int q = 0; q < PG; ++q) {
      const int p = p0 + q;
      if (p >= world) break;
#pragma unroll
      for (int n = 0; n < N; ++n) {
        if (!valid[n]) continue;
        if (p == rank) {
          s[n] += val[n];
          continue;
        }
        unsigned long long gv = g[q][n];
        if ((unsigned)(gv >> 32) != seq && ok) {
          // (a per-lane poll: a lead-lane poll with wave ballots cost the multi-workgroup step
          // kernel 224 B of scratch per lane)
          const rx_xg_gq* a = (const rx_xg_gq*)(w.in(p, seq) + idx[n]);
          const unsigned long long t0 = wall_clock64();
          int k = 0;
          do {
            __builtin_amdgcn_s_sleep(2);
            gv = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if ((++k & 15) == 0 && (unsigned)(gv >> 32) != seq &&
                (__hip_atomic_load((rx_xg_gu*)x.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u ||
                 (unsigned long long)(wall_clock64() - t0) > x.spin_ticks)) {
              rx_xg_fail(x);
              ok = false;
              break;
            }
          } while ((unsigned)(gv >> 32) != seq);
        }
        s[n] += __uint_as_float((unsigned)gv);
      }
    }
  }
#pragma unroll
  for (int n = 0; n < N; ++n)
    if (valid[n]) val[n] = s[n];
}
template <int N, int PG = 1>
__device__ __forceinline__ void rx_xg_pull_sum_n(const XgDev& x, unsigned seq, const int (&idx)[N],
                                                 const bool (&valid)[N], float (&val)[N], bool& ok) {
  rx_xg_pull_sum_v<N, PG>(XgView{x}, x, seq, idx, valid, val, ok);
}
