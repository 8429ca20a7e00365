// Arrow columns in the shared-memory object store -> row-major training matrix in HBM (gfx950).
//
// Replaces the per-batch pandas/numpy -> torch conversion of Ray Data's to_torch on the
// reference's hot loop (python/raydp/torch/estimator.py:226-241; blocks come from
// python/raydp/spark/dataset.py:54-84 / :222).
//
// Data path (rx_ingest_dma):
//   * the host never touches column bytes: each Arrow block (one record batch in the store
//     arena, hipHostRegister-ed chunk by chunk, see rx_pin_range) is DMA'd with
//     hipMemcpyAsync on a dedicated COPY stream into a ring of device staging memory -- one copy
//     per block when the used columns are dense in the IPC body, one per buffer otherwise;
//   * an event hands each chunk to the COMPUTE stream, where arrow_ingest_kernel decodes it,
//     so chunk k+1's DMA overlaps chunk k's decode; ring slots are recycled only after the
//     kernel that read them has finished (event wait on the copy stream);
//   * the kernel: each wave takes whole columns (wave-uniform type -> no divergent switch),
//     16-B vector loads from the staged Arrow values (any array offset: the 16-B aligned base
//     plus a lead count), validity-bitmap -> fill value, dtype cast to f32, all into an LDS
//     column tile; then 16-B row stores of bf16 (or f32), zero padded to the MFMA K multiple
//     the fused trainer expects.
// The epoch shuffle is not materialised here: rx_feistel_perm draws a permutation on the device
// and the training kernels gather rows through it (fused into their row loads).
#include "rx_common.h"

#include <algorithm>
#include <deque>
#include <mutex>
#include <vector>

#define RX_INGEST_MAXCOLS 64
#define RX_TILE_ROWS 256

// type codes: 0 f64, 1 f32, 2 i64, 3 i32, 4 i16, 5 i8, 6 u8, 7 bool (bit-packed), 8 u16, 9 u32
struct IngestCol {
  int type;
  int pad_;
  long long vbit;        // bit index of row 0 in `valid` (bool: bit index of row 0 in `values`)
  const void* values;    // device address of row 0's value (bool: of the byte holding it)
  const uint8_t* valid;  // null: no nulls
  float fill;
  int pad2_;
};

struct IngestArgs {
  int ncols;
  int out_stride;  // elements per output row (>= ncols, zero padded)
  int out_bf16;    // output element: 0 f32, 1 bf16, 2 int64 (exact integer ids)
  int pad_;
  long long nrows;
  long long out_row0;  // first output row of this chunk
  IngestCol col[RX_INGEST_MAXCOLS];
};

// Column values converted to the tile element type E: float (training features, bf16/f32
// output) or long long (category ids: exact, no float rounding above 2^24).
template <class E, class T>
__device__ __forceinline__ E rx_cvt(T v) {
  if constexpr (sizeof(E) == 8 && (sizeof(T) == 4 || sizeof(T) == 8) && (T)0.5 != (T)0)
    return (E)(long long)v;  // float columns to int64: truncation, like a torch cast
  else
    return (E)v;
}

__device__ __forceinline__ bool rx_valid(const IngestCol& c, long long r) {
  if (c.valid == nullptr) return true;
  const long long b = c.vbit + r;
  return (c.valid[b >> 3] >> (b & 7)) & 1;
}

// One wave loads rows [row0, row0 + nr) of a fixed-width column into tile[0..nr) with 16-B
// vector loads: vector v covers elements [v*E, v*E + E) of the 16-B aligned base, element e is
// row e - lead.
template <class TE, class T>
__device__ __forceinline__ void rx_load_col(const IngestCol& c, long long row0, int nr, TE* tile, int lane) {
  constexpr int E = 16 / (int)sizeof(T);
  const uintptr_t p = reinterpret_cast<uintptr_t>(c.values);
  const uintptr_t base = p & ~(uintptr_t)15;
  const long long lead = (long long)((p - base) / sizeof(T));
  const long long e0 = lead + row0;
  const long long v0 = e0 / E, v1 = (e0 + nr - 1) / E;
  const u32x4* vp = reinterpret_cast<const u32x4*>(base);
  const TE fill = (TE)c.fill;
  for (long long v = v0 + lane; v <= v1; v += RX_WAVE) {
    const u32x4 raw = __builtin_nontemporal_load(vp + v);
    T el[E];
    __builtin_memcpy(el, &raw, 16);
#pragma unroll
    for (int q = 0; q < E; ++q) {
      const long long r = v * E + q - e0;
      if (r >= 0 && r < nr) tile[r] = rx_valid(c, row0 + r) ? rx_cvt<TE, T>(el[q]) : fill;
    }
  }
}

template <class TE>
__device__ __forceinline__ void rx_load_bool(const IngestCol& c, long long row0, int nr, TE* tile, int lane) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(c.values);
  for (int r = lane; r < nr; r += RX_WAVE) {
    const long long bit = c.vbit + row0 + r;
    const TE x = (TE)((b[bit >> 3] >> (bit & 7)) & 1);
    tile[r] = c.valid != nullptr && !rx_valid(c, row0 + r) ? (TE)c.fill : x;
  }
}

template <class TE>
__device__ __forceinline__ void rx_ingest_phase1(const IngestArgs& a, TE* tile, long long row0, int nr) {
  const int TS = RX_TILE_ROWS + 1;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int nw = blockDim.x >> 6;
  // column-major; one wave per column, the type switch is wave-uniform
  for (int c = wave; c < a.ncols; c += nw) {
    const IngestCol& col = a.col[c];
    TE* t = tile + c * TS;
    switch (col.type) {
      case 0: rx_load_col<TE, double>(col, row0, nr, t, lane); break;
      case 1: rx_load_col<TE, float>(col, row0, nr, t, lane); break;
      case 2: rx_load_col<TE, long long>(col, row0, nr, t, lane); break;
      case 3: rx_load_col<TE, int>(col, row0, nr, t, lane); break;
      case 4: rx_load_col<TE, short>(col, row0, nr, t, lane); break;
      case 5: rx_load_col<TE, signed char>(col, row0, nr, t, lane); break;
      case 6: rx_load_col<TE, unsigned char>(col, row0, nr, t, lane); break;
      case 7: rx_load_bool<TE>(col, row0, nr, t, lane); break;
      case 8: rx_load_col<TE, unsigned short>(col, row0, nr, t, lane); break;
      case 9: rx_load_col<TE, unsigned int>(col, row0, nr, t, lane); break;
      default:
        for (int r = lane; r < nr; r += RX_WAVE) t[r] = (TE)0;
    }
  }
}

__global__ __launch_bounds__(256) void arrow_ingest_kernel(IngestArgs a, void* __restrict__ out) {
  extern __shared__ float tile[];  // [ncols][RX_TILE_ROWS + 1]
  const int TS = RX_TILE_ROWS + 1;
  const long long row0 = (long long)blockIdx.x * RX_TILE_ROWS;
  const int nr = (int)min((long long)RX_TILE_ROWS, a.nrows - row0);
  rx_ingest_phase1<float>(a, tile, row0, nr);
  __syncthreads();
  // phase 2: row-major, 16-B stores along the output row (zero padded to out_stride)
  const long long obase = (a.out_row0 + row0) * a.out_stride;
  const int S = a.out_stride, nc = a.ncols;
  if (a.out_bf16 && (S & 7) == 0) {
    const int cpr = S >> 3;  // 16-B chunks per row
    uint4* o = reinterpret_cast<uint4*>(reinterpret_cast<u16*>(out) + obase);
    for (int idx = threadIdx.x; idx < nr * cpr; idx += blockDim.x) {
      const int r = idx / cpr, c0 = (idx - r * cpr) * 8;
      uint32_t w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ca = c0 + 2 * j, cb = ca + 1;
        w[j] = rx_f2bf2(ca < nc ? tile[ca * TS + r] : 0.f, cb < nc ? tile[cb * TS + r] : 0.f);
      }
      o[idx] = make_uint4(w[0], w[1], w[2], w[3]);
    }
  } else if (!a.out_bf16 && (S & 3) == 0) {
    const int cpr = S >> 2;
    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + obase);
    for (int idx = threadIdx.x; idx < nr * cpr; idx += blockDim.x) {
      const int r = idx / cpr, c0 = (idx - r * cpr) * 4;
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = c0 + j < nc ? tile[(c0 + j) * TS + r] : 0.f;
      o[idx] = make_float4(v[0], v[1], v[2], v[3]);
    }
  } else if (a.out_bf16) {
    u16* o = reinterpret_cast<u16*>(out) + obase;
    for (int idx = threadIdx.x; idx < nr * S; idx += blockDim.x) {
      const int r = idx / S, c = idx - r * S;
      o[idx] = c < nc ? rx_f2bf(tile[c * TS + r]) : (u16)0;
    }
  } else {
    float* o = reinterpret_cast<float*>(out) + obase;
    for (int idx = threadIdx.x; idx < nr * S; idx += blockDim.x) {
      const int r = idx / S, c = idx - r * S;
      o[idx] = c < nc ? tile[c * TS + r] : 0.f;
    }
  }
}

// Exact integer columns (category ids, counts) -> int64 row-major [N, stride]: same staging,
// an int64 LDS tile, 16-B row stores of two ids.
__global__ __launch_bounds__(256) void arrow_ingest_i64_kernel(IngestArgs a, long long* __restrict__ out) {
  extern __shared__ long long itile[];  // [ncols][RX_TILE_ROWS + 1]
  const int TS = RX_TILE_ROWS + 1;
  const long long row0 = (long long)blockIdx.x * RX_TILE_ROWS;
  const int nr = (int)min((long long)RX_TILE_ROWS, a.nrows - row0);
  rx_ingest_phase1<long long>(a, itile, row0, nr);
  __syncthreads();
  const int S = a.out_stride, nc = a.ncols;
  long long* o = out + (a.out_row0 + row0) * S;
  for (int idx = threadIdx.x; idx < nr * S; idx += blockDim.x) {
    const int r = idx / S, c = idx - r * S;
    o[idx] = c < nc ? itile[c * TS + r] : 0LL;
  }
}

// Row gather (sharding / explicit materialisation): out[i] = in[idx[i]] for rows of
// `row_bytes` bytes, 16-B vectorised.
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                          const int* __restrict__ idx, long long nrows,
                                                          int row_vec) {
  const long long total = nrows * row_vec;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long r = t / row_vec;
    const int v = (int)(t - r * row_vec);
    out[t] = in[(long long)idx[r] * row_vec + v];
  }
}

// ------------------------------------------------------------------ epoch permutation ------
// A keyed bijection of [0, 2^bits) (6-round unbalanced Feistel network over a murmur-style
// round function), restricted to [0, n) by cycle walking (2^bits < 2n, so < 2 steps expected).
// Every index is computed independently: one launch, no sort, no library code object to load
// lazily on the first epoch (torch.randperm's rocPRIM merge sort cost ~13 ms the first time a
// new size class was used).
__device__ __forceinline__ uint32_t rx_mix32(uint32_t x, uint32_t k) {
  x ^= k;
  x *= 0xcc9e2d51u;
  x = (x << 15) | (x >> 17);
  x *= 0x1b873593u;
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  return x;
}

__device__ __forceinline__ uint64_t rx_feistel(uint64_t x, int lbits, int rbits, const uint32_t* keys) {
  // (L, R) -> (R, L ^ F(R)): the halves swap widths every round, 6 rounds bring them back
  uint64_t L = x >> rbits, R = x & ((1ull << rbits) - 1);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const uint64_t nR = (L ^ rx_mix32((uint32_t)R, keys[i])) & ((1ull << lbits) - 1);
    L = R;
    R = nR;
    const int t = lbits;
    lbits = rbits;
    rbits = t;
  }
  return (L << rbits) | R;
}

__global__ __launch_bounds__(256) void feistel_perm_kernel(int* __restrict__ out, long long n, int lbits, int rbits,
                                                           uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                                           uint32_t k4, uint32_t k5) {
  const uint32_t keys[6] = {k0, k1, k2, k3, k4, k5};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i;
    do {
      x = rx_feistel(x, lbits, rbits, keys);
    } while (x >= (uint64_t)n);
    out[i] = (int)x;
  }
}

// ------------------------------------------------------------------ host side --------------
struct RxDmaRegion {
  unsigned long long host;  // first host byte to copy (16-B aligned down)
  long long bytes;
  long long off;            // destination byte offset inside the chunk's staging area (256-B aligned)
};

struct RxDmaCol {
  int type;
  int has_valid;
  long long vals_off;   // staging byte offset of row 0's value (bool: of its byte)
  long long valid_off;  // staging byte offset of the validity byte holding row 0
  long long vbit;       // bit of row 0 inside those bytes (Arrow: array offset % 8 for both)
  float fill;
  int pad_;
};

struct RxDmaChunk {
  long long nrows;
  long long out_row0;
  long long bytes;  // staging bytes this chunk occupies
  int first_region;
  int nregions;
  int first_col;  // ncols entries
  int pad_;
};

namespace {

std::mutex g_mu;
std::vector<hipEvent_t> g_events;  // reusable (disable-timing) events

hipEvent_t rx_event(size_t i) {
  while (g_events.size() <= i) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    g_events.push_back(e);
  }
  return g_events[i];
}

// Pinned-range registry: arenas are registered with hipHostRegister in aligned chunks, lazily,
// the first time a block inside a chunk is ingested (a 2 MiB chunk pins in tens of us; pinning
// a whole multi-GB arena up front would fault in every page of it).
// Each hipHostRegister call is its own allocation to the runtime: a copy must not straddle two
// of them, so every chunk remembers the first chunk of the run it was registered with.
struct PinnedArena {
  uintptr_t base;
  size_t cap;
  size_t chunk;
  std::vector<int64_t> run;  // -1: not registered, else the run's first chunk index
};
std::vector<PinnedArena> g_arenas;
long long g_pin_calls = 0, g_pin_bytes = 0;

// Largest n <= want such that [host, host + n) lies inside one registration run (or `want`
// when the address is in no registered arena). Caller holds g_mu.
size_t rx_contig_pinned(uintptr_t host, size_t want) {
  for (const auto& a : g_arenas) {
    if (host < a.base || host >= a.base + a.cap) continue;
    size_t c = (host - a.base) / a.chunk;
    const int64_t r = a.run[c];
    if (r < 0) return want;
    while (c + 1 < a.run.size() && a.run[c + 1] == r) ++c;
    const uintptr_t end = std::min<uintptr_t>(a.base + a.cap, a.base + (c + 1) * a.chunk);
    return std::min<size_t>(want, end - host);
  }
  return want;
}

}  // namespace

extern "C" {

int rx_ingest_args_size() { return (int)sizeof(IngestArgs); }
int rx_dma_sizes(int* out) {
  out[0] = (int)sizeof(RxDmaRegion);
  out[1] = (int)sizeof(RxDmaCol);
  out[2] = (int)sizeof(RxDmaChunk);
  return 0;
}

static int rx_ingest_launch(const IngestArgs& a, void* out, hipStream_t stream) {
  const long long blocks = (a.nrows + RX_TILE_ROWS - 1) / RX_TILE_ROWS;
  if (a.out_bf16 == 2) {
    static bool attr = false;
    if (!attr) {  // up to 64 int64 columns x 257 rows = 131.6 KB of LDS
      RX_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&arrow_ingest_i64_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr = true;
    }
    const size_t lds = (size_t)a.ncols * (RX_TILE_ROWS + 1) * sizeof(long long);
    hipLaunchKernelGGL(arrow_ingest_i64_kernel, dim3((unsigned)blocks), dim3(256), lds, stream, a,
                       reinterpret_cast<long long*>(out));
  } else {
    const size_t lds = (size_t)a.ncols * (RX_TILE_ROWS + 1) * sizeof(float);
    hipLaunchKernelGGL(arrow_ingest_kernel, dim3((unsigned)blocks), dim3(256), lds, stream, a, out);
  }
  return (int)hipGetLastError();
}

int rx_arrow_ingest(const IngestArgs* a, void* out, hipStream_t stream) {
  if (a->ncols > RX_INGEST_MAXCOLS || a->ncols > a->out_stride || a->ncols <= 0) return -1;
  if (a->nrows <= 0) return 0;
  return rx_ingest_launch(*a, out, stream);
}

// Pin [addr, addr + len) of the arena [base, base + cap) (chunk-granular, idempotent).
// Returns 0 on success, a HIP error code otherwise.
int rx_pin_range(unsigned long long base, unsigned long long cap, unsigned long long addr,
                 unsigned long long len, unsigned long long chunk) {
  if (len == 0) return 0;
  if (addr < base || addr + len > base + cap || chunk == 0) return -1;
  std::lock_guard<std::mutex> g(g_mu);
  PinnedArena* pa = nullptr;
  for (auto& a : g_arenas)
    if (a.base == base && a.cap == cap) pa = &a;
  if (pa == nullptr) {
    g_arenas.push_back(PinnedArena{(uintptr_t)base, (size_t)cap, (size_t)chunk,
                                   std::vector<int64_t>((cap + chunk - 1) / chunk, -1)});
    pa = &g_arenas.back();
  }
  const size_t c0 = (addr - base) / pa->chunk, c1 = (addr + len - 1 - base) / pa->chunk;
  size_t c = c0;
  while (c <= c1) {
    if (pa->run[c] >= 0) {
      ++c;
      continue;
    }
    size_t e = c;
    while (e + 1 <= c1 && pa->run[e + 1] < 0) ++e;
    const uintptr_t s = pa->base + c * pa->chunk;
    const size_t n = std::min(pa->cap, (e + 1) * pa->chunk) - c * pa->chunk;
    const hipError_t rc = hipHostRegister(reinterpret_cast<void*>(s), n, hipHostRegisterDefault);
    if (rc != hipSuccess && rc != hipErrorHostMemoryAlreadyRegistered) {
      (void)hipGetLastError();
      return (int)rc;
    }
    for (size_t k = c; k <= e; ++k) pa->run[k] = (int64_t)c;
    ++g_pin_calls;
    g_pin_bytes += (long long)n;
    c = e + 1;
  }
  return 0;
}

int rx_pin_stats(long long* out) {
  std::lock_guard<std::mutex> g(g_mu);
  out[0] = g_pin_calls;
  out[1] = g_pin_bytes;
  return 0;
}

// Drop every registration of the arena at `base` (store closed / unmapped).
int rx_unpin_arena(unsigned long long base) {
  std::lock_guard<std::mutex> g(g_mu);
  for (size_t i = 0; i < g_arenas.size(); ++i) {
    PinnedArena& a = g_arenas[i];
    if (a.base != base) continue;
    for (size_t c = 0; c < a.run.size(); ++c) {
      if (a.run[c] != (int64_t)c) continue;  // only run starts were registered
      (void)hipHostUnregister(reinterpret_cast<void*>(a.base + c * a.chunk));
      (void)hipGetLastError();
    }
    g_arenas.erase(g_arenas.begin() + i);
    return 0;
  }
  return 0;
}

// The whole shard: chunk k's regions are DMA'd on `copy` into the staging ring, the decode of
// chunk k runs on `compute` after an event; ring space is reused only after the kernel that
// read it has completed. stats: [pinned bytes, pageable bytes, copies issued, chunks].
int rx_ingest_dma(const RxDmaChunk* chunks, int nchunks, const RxDmaRegion* regions, const RxDmaCol* cols,
                  int ncols, int out_stride, int out_bf16, void* out, void* stage, long long stage_bytes,
                  hipStream_t compute, hipStream_t copy, long long* stats) {
  if (ncols <= 0 || ncols > RX_INGEST_MAXCOLS || ncols > out_stride) return -1;
  std::lock_guard<std::mutex> g(g_mu);
  uint8_t* ring = reinterpret_cast<uint8_t*>(stage);
  // the staging memory was just handed out by the compute stream's allocator: the copy stream
  // must not write it before the compute stream's earlier work is done
  hipEvent_t start = rx_event(0);
  if (start == nullptr) return -2;
  RX_CHECK(hipEventRecord(start, compute));
  RX_CHECK(hipStreamWaitEvent(copy, start, 0));
  struct Busy {
    long long s, e;
    size_t ev;
  };
  std::deque<Busy> busy;
  long long pos = 0;
  long long pinned = 0, pageable = 0, ncopies = 0;
  for (int k = 0; k < nchunks; ++k) {
    const RxDmaChunk& ch = chunks[k];
    if (ch.bytes > stage_bytes) return -3;
    if (pos + ch.bytes > stage_bytes) pos = 0;
    const long long s = pos, e = pos + ch.bytes;
    // wait for every earlier decode still reading [s, e) (events complete in compute-stream
    // order, so waiting on the youngest overlapping one is enough)
    long long wait_ev = -1;
    for (auto it = busy.begin(); it != busy.end();) {
      if (it->e > s && it->s < e) {
        wait_ev = (long long)it->ev;
        it = busy.erase(it);
      } else {
        ++it;
      }
    }
    if (wait_ev >= 0) RX_CHECK(hipStreamWaitEvent(copy, rx_event((size_t)wait_ev), 0));
    for (int r = 0; r < ch.nregions; ++r) {
      const RxDmaRegion& rg = regions[ch.first_region + r];
      if (rg.bytes <= 0) continue;
      hipPointerAttribute_t at;
      const bool pin = hipPointerGetAttributes(&at, reinterpret_cast<void*>(rg.host)) == hipSuccess &&
                       at.type == hipMemoryTypeHost;
      (void)hipGetLastError();
      (pin ? pinned : pageable) += rg.bytes;
      // one copy per registration run the region touches (usually exactly one)
      size_t done_b = 0;
      while (done_b < (size_t)rg.bytes) {
        const uintptr_t h = (uintptr_t)rg.host + done_b;
        const size_t n = rx_contig_pinned(h, (size_t)rg.bytes - done_b);
        RX_CHECK(hipMemcpyAsync(ring + s + rg.off + done_b, reinterpret_cast<const void*>(h), n,
                                hipMemcpyHostToDevice, copy));
        done_b += n;
        ++ncopies;
      }
    }
    const size_t ev_ready = 1 + 2 * (size_t)k, ev_done = ev_ready + 1;
    hipEvent_t ready = rx_event(ev_ready), done = rx_event(ev_done);
    if (ready == nullptr || done == nullptr) return -2;
    RX_CHECK(hipEventRecord(ready, copy));
    RX_CHECK(hipStreamWaitEvent(compute, ready, 0));
    IngestArgs a;
    a.ncols = ncols;
    a.out_stride = out_stride;
    a.out_bf16 = out_bf16;
    a.pad_ = 0;
    a.nrows = ch.nrows;
    a.out_row0 = ch.out_row0;
    for (int c = 0; c < ncols; ++c) {
      const RxDmaCol& dc = cols[ch.first_col + c];
      IngestCol& ic = a.col[c];
      ic.type = dc.type;
      ic.pad_ = 0;
      ic.values = ring + s + dc.vals_off;
      ic.valid = dc.has_valid ? ring + s + dc.valid_off : nullptr;
      ic.vbit = dc.vbit;
      ic.fill = dc.fill;
      ic.pad2_ = 0;
    }
    if (ch.nrows > 0) {
      const int lrc = rx_ingest_launch(a, out, compute);
      if (lrc) return lrc;
    }
    RX_CHECK(hipEventRecord(done, compute));
    busy.push_back(Busy{s, e, ev_done});
    pos = e;
  }
  if (stats != nullptr) {
    stats[0] += pinned;
    stats[1] += pageable;
    stats[2] += ncopies;
    stats[3] += nchunks;
  }
  return 0;
}

int rx_gather_rows(const void* in, void* out, const int* idx, long long nrows, int row_bytes,
                   hipStream_t stream) {
  if (row_bytes % 16) return -1;
  const int row_vec = row_bytes / 16;
  long long total = nrows * row_vec;
  int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
  if (blocks < 1) return 0;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(256), 0, stream,
                     reinterpret_cast<const uint4*>(in), reinterpret_cast<uint4*>(out), idx, nrows, row_vec);
  return (int)hipGetLastError();
}

// Random permutation of [0, n) into out (int32), keyed by `seed`.
int rx_feistel_perm(int* out, long long n, unsigned long long seed, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > 0x7fffffffLL) return -1;
  int bits = 1;
  while ((1ll << bits) < n) ++bits;
  if (bits < 2) bits = 2;
  const int lbits = bits / 2, rbits = bits - lbits;
  uint32_t k[6];
  uint64_t z = seed;
  for (int i = 0; i < 6; ++i) {  // splitmix64 key schedule
    z += 0x9e3779b97f4a7c15ull;
    uint64_t x = z;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    k[i] = (uint32_t)(x ^ (x >> 31));
  }
  const long long blocks = std::min<long long>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(feistel_perm_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, out, n, lbits, rbits,
                     k[0], k[1], k[2], k[3], k[4], k[5]);
  return (int)hipGetLastError();
}

}  // extern "C"
