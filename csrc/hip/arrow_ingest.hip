// Arrow columns -> row-major training matrix in HBM (gfx950).
//
// Replaces the per-batch pandas/numpy -> torch conversion of Ray Data's to_torch on the
// reference's hot loop (python/raydp/torch/estimator.py:226-241). The host hands over the raw
// Arrow buffers of every column (values + optional validity bitmap, any array offset) after ONE
// pinned H2D copy; this kernel decodes them on the GPU: dtype cast (f64/f32/i64/i32/i16/i8/u8/
// bool -> f32 or bf16), null -> fill value, and the column-major -> row-major transpose through
// an LDS tile (coalesced column reads, coalesced row writes), zero-padding the row to the
// MFMA K multiple expected by the fused trainer.
#include "rx_common.h"

#define RX_INGEST_MAXCOLS 64
#define RX_TILE_ROWS 64

struct IngestCol {
  int type;       // 0 f64, 1 f32, 2 i64, 3 i32, 4 i16, 5 i8, 6 u8, 7 bool (bit-packed), 8 u16, 9 u32
  int pad_;
  long long offset;  // Arrow array offset (elements)
  const void* values;
  const uint8_t* valid;  // null: all valid
  float fill;
  int pad2_;
};

struct IngestArgs {
  int ncols;
  int out_stride;  // elements per output row (>= ncols, zero padded)
  int out_bf16;    // 1: bf16 output, 0: f32 output
  int pad_;
  long long nrows;
  long long out_row0;  // first output row (for appending several tables)
  IngestCol col[RX_INGEST_MAXCOLS];
};

__device__ __forceinline__ float load_as_float(const IngestCol& c, long long i) {
  const long long j = c.offset + i;
  if (c.valid != nullptr && !((c.valid[j >> 3] >> (j & 7)) & 1)) return c.fill;
  switch (c.type) {
    case 0: return (float)reinterpret_cast<const double*>(c.values)[j];
    case 1: return reinterpret_cast<const float*>(c.values)[j];
    case 2: return (float)reinterpret_cast<const long long*>(c.values)[j];
    case 3: return (float)reinterpret_cast<const int*>(c.values)[j];
    case 4: return (float)reinterpret_cast<const short*>(c.values)[j];
    case 5: return (float)reinterpret_cast<const signed char*>(c.values)[j];
    case 6: return (float)reinterpret_cast<const unsigned char*>(c.values)[j];
    case 7: return (float)((reinterpret_cast<const uint8_t*>(c.values)[j >> 3] >> (j & 7)) & 1);
    case 8: return (float)reinterpret_cast<const unsigned short*>(c.values)[j];
    case 9: return (float)reinterpret_cast<const unsigned int*>(c.values)[j];
    default: return 0.f;
  }
}

__global__ __launch_bounds__(256) void arrow_ingest_kernel(IngestArgs a, void* __restrict__ out) {
  __shared__ float tile[RX_INGEST_MAXCOLS][RX_TILE_ROWS + 1];
  const long long row0 = (long long)blockIdx.x * RX_TILE_ROWS;
  const int nr = (int)min((long long)RX_TILE_ROWS, a.nrows - row0);
  // phase 1: column-major, coalesced along rows
  for (int idx = threadIdx.x; idx < a.ncols * RX_TILE_ROWS; idx += blockDim.x) {
    const int c = idx / RX_TILE_ROWS, r = idx % RX_TILE_ROWS;
    tile[c][r] = r < nr ? load_as_float(a.col[c], row0 + r) : 0.f;
  }
  __syncthreads();
  // phase 2: row-major, coalesced along the output row (zero padded to out_stride)
  const long long obase = (a.out_row0 + row0) * a.out_stride;
  if (a.out_bf16) {
    u16* o = reinterpret_cast<u16*>(out) + obase;
    for (int idx = threadIdx.x; idx < nr * a.out_stride; idx += blockDim.x) {
      const int r = idx / a.out_stride, c = idx % a.out_stride;
      o[idx] = c < a.ncols ? rx_f2bf(tile[c][r]) : (u16)0;
    }
  } else {
    float* o = reinterpret_cast<float*>(out) + obase;
    for (int idx = threadIdx.x; idx < nr * a.out_stride; idx += blockDim.x) {
      const int r = idx / a.out_stride, c = idx % a.out_stride;
      o[idx] = c < a.ncols ? tile[c][r] : 0.f;
    }
  }
}

// Row gather (epoch shuffle materialisation / sharding): out[i] = in[idx[i]] for rows of
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

extern "C" {

int rx_ingest_args_size() { return (int)sizeof(IngestArgs); }

int rx_arrow_ingest(const IngestArgs* a, void* out, hipStream_t stream) {
  if (a->ncols > RX_INGEST_MAXCOLS || a->ncols > a->out_stride) return -1;
  if (a->nrows <= 0) return 0;
  const long long blocks = (a->nrows + RX_TILE_ROWS - 1) / RX_TILE_ROWS;
  hipLaunchKernelGGL(arrow_ingest_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, *a, out);
  return (int)hipGetLastError();
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

}  // extern "C"
