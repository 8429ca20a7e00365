// Native CPU kernels of the DataFrame executor (shuffle hashing, partition scatter).
//
// Replaces the JVM-side hashing Spark does in its shuffle writer (reference: executors run
// Spark's HashPartitioner inside RayDPExecutor, core/raydp-main/.../RayDPExecutor.scala).
// Operates directly on Arrow buffers handed over from Python (no copies): fixed-width values
// and (offsets, data) string layouts, with an optional validity bitmap.
#include <cstdint>
#include <cstring>

namespace {

inline uint64_t mix64(uint64_t x) {
  // splitmix64 finalizer: full avalanche, cheap, identical on every process.
  x += 0x9e3779b97f4a7c15ULL;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ULL;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

inline uint64_t combine(uint64_t seed, uint64_t h) {
  return mix64(seed ^ (h + 0x9e3779b97f4a7c15ULL + (seed << 6) + (seed >> 2)));
}

inline bool is_valid(const uint8_t* validity, int64_t i) {
  return validity == nullptr || (validity[i >> 3] >> (i & 7)) & 1;
}

// FNV-1a over bytes, then mixed; good enough for partitioning strings.
inline uint64_t hash_bytes(const uint8_t* p, int64_t n) {
  uint64_t h = 0xcbf29ce484222325ULL;
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    std::memcpy(&w, p + i, 8);
    h = (h ^ w) * 0x100000001b3ULL;
    h ^= h >> 29;
  }
  for (; i < n; ++i) h = (h ^ p[i]) * 0x100000001b3ULL;
  return mix64(h ^ static_cast<uint64_t>(n));
}

constexpr uint64_t kNullHash = 0x5bd1e9955bd1e995ULL;

}  // namespace

extern "C" {

// width: 1, 2, 4 or 8 bytes; is_float: canonicalise -0.0 / NaN like Spark's normalisation.
void rx_hash_fixed(uint64_t* seed_inout, const void* values, const uint8_t* validity,
                   int64_t offset, int64_t n, int width, int is_float) {
  const uint8_t* base = static_cast<const uint8_t*>(values);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = offset + i;
    uint64_t v = 0;
    if (!is_valid(validity, j)) {
      seed_inout[i] = combine(seed_inout[i], kNullHash);
      continue;
    }
    if (width == 8) {
      std::memcpy(&v, base + j * 8, 8);
      if (is_float) {
        double d;
        std::memcpy(&d, &v, 8);
        if (d == 0.0) d = 0.0;
        if (d != d) v = 0x7ff8000000000000ULL; else std::memcpy(&v, &d, 8);
      }
    } else if (width == 4) {
      uint32_t w;
      std::memcpy(&w, base + j * 4, 4);
      if (is_float) {
        float f;
        std::memcpy(&f, &w, 4);
        double d = f;  // hash floats through their double value: int/float keys compare equal
        if (d == 0.0) d = 0.0;
        std::memcpy(&v, &d, 8);
      } else {
        v = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(w)));
      }
    } else if (width == 2) {
      int16_t s;
      std::memcpy(&s, base + j * 2, 2);
      v = static_cast<uint64_t>(static_cast<int64_t>(s));
    } else {
      v = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int8_t>(base[j])));
    }
    seed_inout[i] = combine(seed_inout[i], mix64(v));
  }
}

void rx_hash_binary(uint64_t* seed_inout, const int32_t* offsets, const uint8_t* data,
                    const uint8_t* validity, int64_t offset, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = offset + i;
    if (!is_valid(validity, j)) {
      seed_inout[i] = combine(seed_inout[i], kNullHash);
      continue;
    }
    const int32_t a = offsets[j], b = offsets[j + 1];
    seed_inout[i] = combine(seed_inout[i], hash_bytes(data + a, b - a));
  }
}

// Counting-sort scatter: out_order receives row indices grouped by partition (stable),
// counts[p] the number of rows of partition p. part[i] in [0, nparts).
void rx_partition_order(const int64_t* part, int64_t n, int64_t nparts, int64_t* counts,
                        int64_t* out_order) {
  std::memset(counts, 0, sizeof(int64_t) * nparts);
  for (int64_t i = 0; i < n; ++i) counts[part[i]]++;
  int64_t* cursor = new int64_t[nparts];
  int64_t acc = 0;
  for (int64_t p = 0; p < nparts; ++p) {
    cursor[p] = acc;
    acc += counts[p];
  }
  for (int64_t i = 0; i < n; ++i) out_order[cursor[part[i]]++] = i;
  delete[] cursor;
}

}  // extern "C"
