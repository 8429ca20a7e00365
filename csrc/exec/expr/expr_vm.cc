// Fused expression VM of the DataFrame executor: one native call evaluates a whole chain of
// narrow operators (filter / withColumn / select / drop) over one Arrow partition.
//
// In Spark the equivalent work is whole-stage codegen inside the executor JVM (reference:
// executors are Spark executors hosted by RayDPExecutor, core/raydp-main/src/main/scala/org/
// apache/spark/executor/RayDPExecutor.scala; the NYC ETL being run is examples/data_process.py).
// Here the Python side (raydp_amd/spark/exprc.py) compiles the operator chain into a register
// program; this file runs it chunk by chunk so every intermediate column stays in L1/L2:
//
//   * registers hold CHUNK rows of one typed column (bool as bytes, i32, i64, f32, f64) plus a
//     byte-per-row validity vector (or an all-valid flag),
//   * FILTER compacts the registers that are live after it, so later operators only touch
//     surviving rows (predicate push-through without re-materialising the table),
//   * outputs are appended to Arrow-layout buffers (values + bit-packed validity) that Python
//     wraps with pa.Array.from_buffers, and the surviving input row ids are exported so untouched
//     columns (strings etc.) are gathered once with Arrow's take.
//
// Semantics follow the single-operator Arrow path (raydp_amd/spark/column.py) bit for bit:
// the compiler inserts explicit casts so every arithmetic op runs in the type Arrow would pick,
// integer arithmetic wraps, float->int casts behave like the unchecked static_cast Arrow uses,
// and comparisons/Kleene logic propagate nulls the way pc.* kernels do.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace {

constexpr int CH = 1024;  // rows per chunk

enum Type : int32_t { T_BOOL = 0, T_I32 = 1, T_I64 = 2, T_F32 = 3, T_F64 = 4 };

enum Op : int32_t {
  OP_LOAD = 1,    // dst <- input[imm] (type)
  OP_CONST = 2,   // dst <- constant pool[imm] (type); aux=1: null constant
  OP_CAST = 3,    // dst(type) <- cast(a(aux))
  OP_BIN = 4,     // dst(type) <- a (op aux) b, both already in `type`
  OP_CMP = 5,     // dst(bool) <- a (cmp aux) b, operands in `type`
  OP_UN = 6,      // dst(type) <- unary aux (a)
  OP_AND = 7,     // Kleene and (bool)
  OP_OR = 8,      // Kleene or (bool)
  OP_IFELSE = 9,  // dst(type) <- c ? a : b ; aux=1: null condition counts as false
  OP_DT = 10,     // dst(i32) <- field aux of timestamp a (i64 in units, imm = units per second)
  OP_FILTER = 11, // keep rows where a is valid and true; compact live list at imm
  OP_ISNULL = 12, // dst(bool) <- a is null (aux=1: is not null)
  OP_FILLNULL = 13,  // dst(type) <- a if valid else b
};

enum BinKind : int32_t {
  B_ADD = 0, B_SUB = 1, B_MUL = 2, B_DIV = 3,
  B_MOD_SPARK = 4,   // floats: a - trunc(a / b) * b (column.py BinOp '%')
  B_MOD_PY = 5,      // numpy np.mod (sign of divisor)
  B_FLOORDIV_PY = 6, // numpy np.floor_divide
  B_POW = 7, B_MIN = 8, B_MAX = 9,
  B_PYMIN = 10,      // Python builtin min(a, b): b if b < a else a (NaN order-dependent, as Python)
  B_PYMAX = 11,      // Python builtin max(a, b): b if b > a else a
};

enum CmpKind : int32_t { C_LT = 0, C_LE = 1, C_GT = 2, C_GE = 3, C_EQ = 4, C_NE = 5 };

enum UnKind : int32_t {
  U_NEG = 0, U_ABS = 1, U_NOT = 2, U_SQRT = 3, U_FLOOR = 4, U_CEIL = 5, U_TRUNC = 6,
  U_ISNAN = 7, U_EXP = 8, U_SIN = 9, U_COS = 10, U_TAN = 11,
};

enum DtField : int32_t {
  D_YEAR = 0, D_MONTH = 1, D_DAY = 2, D_HOUR = 3, D_MINUTE = 4, D_SECOND = 5,
  D_DOW_SPARK = 6, D_ISOWEEK = 7, D_QUARTER = 8, D_DOY = 9,
};

struct Instr { int32_t op, dst, a, b, c, type, aux, imm; };

struct Regs {
  int nslots;
  std::vector<uint64_t> data;  // nslots * CH words (8 bytes per row, typed in place)
  std::vector<uint8_t> valid;  // nslots * CH
  std::vector<uint8_t> allvalid;
  explicit Regs(int n) : nslots(n), data(size_t(n) * CH), valid(size_t(n) * CH), allvalid(n, 1) {}
  template <typename T> T* p(int s) { return reinterpret_cast<T*>(&data[size_t(s) * CH]); }
  uint8_t* v(int s) { return &valid[size_t(s) * CH]; }
};

// ---------------------------------------------------------------- scalar helpers -----------
template <typename T> inline T wrap_add(T a, T b) {
  using U = typename std::make_unsigned<T>::type;
  return static_cast<T>(static_cast<U>(a) + static_cast<U>(b));
}
template <typename T> inline T wrap_sub(T a, T b) {
  using U = typename std::make_unsigned<T>::type;
  return static_cast<T>(static_cast<U>(a) - static_cast<U>(b));
}
template <typename T> inline T wrap_mul(T a, T b) {
  using U = typename std::make_unsigned<T>::type;
  return static_cast<T>(static_cast<U>(a) * static_cast<U>(b));
}

// x86 cvtt* semantics for out-of-range / NaN (what Arrow's unchecked static_cast compiles to),
// written without invoking C++ undefined behaviour.
template <typename I, typename F> inline I f2i(F x) {
  const F lo = static_cast<F>(std::numeric_limits<I>::min());
  const F hi = -lo;  // 2^(bits-1), exactly representable
  if (!(x >= lo && x < hi)) return std::numeric_limits<I>::min();
  return static_cast<I>(x);
}

template <typename To, typename From> inline To cvt(From x) {
  if constexpr (std::is_floating_point<From>::value && std::is_integral<To>::value &&
                !std::is_same<To, uint8_t>::value) {
    return f2i<To>(x);
  } else if constexpr (std::is_same<From, double>::value && std::is_same<To, float>::value) {
    // IEEE round-to-nearest overflows to +-inf at FLT_MAX + half an ulp (2^103); the C++
    // conversion of a value beyond float's range is undefined, so that case is spelled out
    constexpr double kOver = 3.4028235677973366e38;   // FLT_MAX + 2^103
    if (x >= kOver) return std::numeric_limits<float>::infinity();
    if (x <= -kOver) return -std::numeric_limits<float>::infinity();
    return static_cast<float>(x);
  } else if constexpr (std::is_same<To, uint8_t>::value) {
    return static_cast<uint8_t>(x != From(0));
  } else {
    return static_cast<To>(x);
  }
}

// numpy npy_divmod (numpy/_core/src/npymath/npy_math_internal.h.src) for floats
template <typename F> inline F np_fmod_py(F a, F b, F* floordiv) {
  F mod = std::fmod(a, b);
  if (b == F(0)) {
    *floordiv = a / b;
    return mod;
  }
  F div = (a - mod) / b;
  if (mod != F(0)) {
    if ((b < F(0)) != (mod < F(0))) {
      mod += b;
      div -= F(1);
    }
  } else {
    mod = std::copysign(F(0), b);
  }
  F fl;
  if (div != F(0)) {
    fl = std::floor(div);
    if (div - fl > F(0.5)) fl += F(1);
  } else {
    fl = std::copysign(F(0), a / b);
  }
  *floordiv = fl;
  return mod;
}

template <typename I> inline I np_imod(I a, I b) {
  if (b == 0) return 0;
  if (b == -1) return 0;
  I r = a % b;
  if (r != 0 && ((r < 0) != (b < 0))) r += b;
  return r;
}
template <typename I> inline I np_ifloordiv(I a, I b) {
  if (b == 0) return 0;
  if (b == -1) return wrap_sub<I>(0, a);
  I q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q -= 1;
  return q;
}

inline int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// Howard Hinnant's civil-from-days / days-from-civil (proleptic Gregorian, 1970-01-01 = 0)
inline void civil(int64_t z, int64_t* y, int* m, int* d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  *d = int(doy - (153 * mp + 2) / 5 + 1);
  *m = int(mp < 10 ? mp + 3 : mp - 9);
  *y = yoe + era * 400 + (*m <= 2);
}
inline int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

// Neri & Schneider, "Euclidean affine functions and their application to calendar
// algorithms" (2022): civil date from a day count with 32-bit multiply/shift only. With the
// shift s = 82 it is exact for days in [-K, (2^32 - 3) / 4 - K] (K = 12,699,422: about 32,800
// BC to 2.9 million AD); other values take the 64-bit routine above.
constexpr int64_t kCivil32Lo = -12699422;
constexpr int64_t kCivil32Hi = 1073741823LL - 12699422;
struct Civil { int32_t y; int32_t m; int32_t d; int32_t doy; };
inline Civil civil32(int32_t days) {
  constexpr uint32_t s = 82, K = 719468 + 146097 * s, L = 400 * s;
  const uint32_t N = uint32_t(days) + K;
  const uint32_t N1 = 4 * N + 3;
  const uint32_t C = N1 / 146097;
  const uint32_t NC = N1 % 146097 / 4;
  const uint32_t N2 = 4 * NC + 3;
  const uint64_t P2 = uint64_t(2939745) * N2;
  const uint32_t Z = uint32_t(P2 >> 32);
  const uint32_t NY = uint32_t(P2) / 2939745 / 4;  // day of the March-based year
  const uint32_t Y = 100 * C + Z;
  const uint32_t N3 = 2141 * NY + 197913;
  const uint32_t M = N3 >> 16;
  const uint32_t D = (N3 & 65535) / 2141;
  const uint32_t J = NY >= 306;                     // January or February
  Civil c;
  c.y = int32_t(Y - L + J);
  c.m = int32_t(J ? M - 12 : M);
  c.d = int32_t(D + 1);
  const int32_t leap = (c.y % 4 == 0) & ((c.y % 100 != 0) | (c.y % 400 == 0));
  c.doy = J ? int32_t(NY) - 305 : int32_t(NY) + 60 + leap;
  return c;
}

inline Civil civil_any(int64_t days) {
  if (days >= kCivil32Lo && days < kCivil32Hi) return civil32(int32_t(days));
  int64_t y; int m, d;
  civil(days, &y, &m, &d);
  return Civil{int32_t(y), m, d, int32_t(days - days_from_civil(y, 1, 1) + 1)};
}

template <int F> inline int32_t dt_field(int64_t secs) {
  const int64_t days = floor_div(secs, 86400);
  int64_t sod = secs % 86400;             // not secs - days * 86400: that overflows near INT64_MIN
  if (sod < 0) sod += 86400;
  if constexpr (F == D_HOUR) return int32_t(sod / 3600);
  if constexpr (F == D_MINUTE) return int32_t((sod / 60) % 60);
  if constexpr (F == D_SECOND) return int32_t(sod % 60);
  if constexpr (F == D_DOW_SPARK) {  // 1 = Sunday .. 7 = Saturday; 1970-01-01 was a Thursday
    int64_t w = (days + 4) % 7;
    if (w < 0) w += 7;
    return int32_t(w + 1);
  }
  if constexpr (F == D_ISOWEEK) {    // ISO-8601: the week belongs to the year of its Thursday
    int64_t wd = (days + 3) % 7;     // Monday = 0
    if (wd < 0) wd += 7;
    return (civil_any(days - wd + 3).doy - 1) / 7 + 1;
  }
  const Civil c = civil_any(days);
  if constexpr (F == D_YEAR) return c.y;
  if constexpr (F == D_MONTH) return c.m;
  if constexpr (F == D_DAY) return c.d;
  if constexpr (F == D_QUARTER) return (c.m - 1) / 3 + 1;
  if constexpr (F == D_DOY) return c.doy;
  return 0;
}

template <int F> void run_dt_field(const int64_t* a, int32_t* o, int n, int64_t ups) {
  if (ups == 1) {
    for (int i = 0; i < n; ++i) o[i] = dt_field<F>(a[i]);
  } else {
    for (int i = 0; i < n; ++i) o[i] = dt_field<F>(floor_div(a[i], ups));
  }
}

void run_dt(const int64_t* a, int32_t* o, int n, int64_t ups, int field) {
  switch (field) {
    case D_YEAR: run_dt_field<D_YEAR>(a, o, n, ups); break;
    case D_MONTH: run_dt_field<D_MONTH>(a, o, n, ups); break;
    case D_DAY: run_dt_field<D_DAY>(a, o, n, ups); break;
    case D_HOUR: run_dt_field<D_HOUR>(a, o, n, ups); break;
    case D_MINUTE: run_dt_field<D_MINUTE>(a, o, n, ups); break;
    case D_SECOND: run_dt_field<D_SECOND>(a, o, n, ups); break;
    case D_DOW_SPARK: run_dt_field<D_DOW_SPARK>(a, o, n, ups); break;
    case D_ISOWEEK: run_dt_field<D_ISOWEEK>(a, o, n, ups); break;
    case D_QUARTER: run_dt_field<D_QUARTER>(a, o, n, ups); break;
    case D_DOY: run_dt_field<D_DOY>(a, o, n, ups); break;
    default: for (int i = 0; i < n; ++i) o[i] = 0; break;
  }
}

// Sets bits [pos, pos + n) of a bitmap (whole bytes at a time where aligned).
inline void set_bits(uint8_t* bm, int64_t pos, int64_t n) {
  while (n > 0 && (pos & 7)) {
    bm[pos >> 3] |= uint8_t(1u << (pos & 7));
    ++pos;
    --n;
  }
  if (n >= 8) {
    std::memset(bm + (pos >> 3), 0xff, size_t(n >> 3));
    pos += n & ~int64_t(7);
    n &= 7;
  }
  while (n > 0) {
    bm[pos >> 3] |= uint8_t(1u << (pos & 7));
    ++pos;
    --n;
  }
}

// Packs n byte flags (0/1) into a bitmap at bit position pos; returns the number of zeros.
inline int64_t pack_bits(uint8_t* bm, int64_t pos, const uint8_t* flags, int n) {
  int64_t zeros = 0;
  int i = 0;
  while (i < n && ((pos + i) & 7)) {
    if (flags[i]) bm[(pos + i) >> 3] |= uint8_t(1u << ((pos + i) & 7));
    else ++zeros;
    ++i;
  }
  for (; i + 8 <= n; i += 8) {
    uint8_t b = 0;
    for (int k = 0; k < 8; ++k) b |= uint8_t((flags[i + k] & 1) << k);
    bm[(pos + i) >> 3] = b;
    zeros += 8 - __builtin_popcount(b);
  }
  for (; i < n; ++i) {
    if (flags[i]) bm[(pos + i) >> 3] |= uint8_t(1u << ((pos + i) & 7));
    else ++zeros;
  }
  return zeros;
}

// --------------------------------------------------------------- typed dispatch -----------
template <typename F> inline void dispatch(int type, F&& f) {
  switch (type) {
    case T_BOOL: f(uint8_t{}); break;
    case T_I32: f(int32_t{}); break;
    case T_I64: f(int64_t{}); break;
    case T_F32: f(float{}); break;
    case T_F64: f(double{}); break;
    default: break;
  }
}

inline void and_valid(Regs& R, int dst, int a, int b, int n) {
  const bool va = R.allvalid[a], vb = b < 0 || R.allvalid[b];
  if (va && vb) {
    R.allvalid[dst] = 1;
    return;
  }
  R.allvalid[dst] = 0;
  uint8_t* o = R.v(dst);
  const uint8_t* x = R.v(a);
  const uint8_t* y = b < 0 ? nullptr : R.v(b);
  for (int i = 0; i < n; ++i) o[i] = (va ? 1 : x[i]) & (vb ? 1 : y[i]);
}

template <typename T> void run_bin(Regs& R, const Instr& I, int n) {
  T* o = R.p<T>(I.dst);
  const T* a = R.p<T>(I.a);
  const T* b = R.p<T>(I.b);
  switch (I.aux) {
    case B_ADD:
      if constexpr (std::is_integral<T>::value) for (int i = 0; i < n; ++i) o[i] = wrap_add(a[i], b[i]);
      else for (int i = 0; i < n; ++i) o[i] = a[i] + b[i];
      break;
    case B_SUB:
      if constexpr (std::is_integral<T>::value) for (int i = 0; i < n; ++i) o[i] = wrap_sub(a[i], b[i]);
      else for (int i = 0; i < n; ++i) o[i] = a[i] - b[i];
      break;
    case B_MUL:
      if constexpr (std::is_integral<T>::value) for (int i = 0; i < n; ++i) o[i] = wrap_mul(a[i], b[i]);
      else for (int i = 0; i < n; ++i) o[i] = a[i] * b[i];
      break;
    case B_DIV:
      if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = a[i] / b[i];
      break;
    case B_MOD_SPARK:
      if constexpr (std::is_floating_point<T>::value)
        for (int i = 0; i < n; ++i) o[i] = a[i] - std::trunc(a[i] / b[i]) * b[i];
      break;
    case B_MOD_PY:
      if constexpr (std::is_floating_point<T>::value) {
        T fd;
        for (int i = 0; i < n; ++i) o[i] = np_fmod_py(a[i], b[i], &fd);
      } else {
        for (int i = 0; i < n; ++i) o[i] = np_imod(a[i], b[i]);
      }
      break;
    case B_FLOORDIV_PY:
      if constexpr (std::is_floating_point<T>::value) {
        for (int i = 0; i < n; ++i) { T fd; np_fmod_py(a[i], b[i], &fd); o[i] = fd; }
      } else {
        for (int i = 0; i < n; ++i) o[i] = np_ifloordiv(a[i], b[i]);
      }
      break;
    case B_POW:
      if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::pow(a[i], b[i]);
      break;
    case B_MIN:
      // numpy np.minimum: NaN in either operand propagates
      for (int i = 0; i < n; ++i) o[i] = (a[i] != a[i]) ? a[i] : (b[i] != b[i]) ? b[i] : (b[i] < a[i] ? b[i] : a[i]);
      break;
    case B_MAX:
      for (int i = 0; i < n; ++i) o[i] = (a[i] != a[i]) ? a[i] : (b[i] != b[i]) ? b[i] : (b[i] > a[i] ? b[i] : a[i]);
      break;
    case B_PYMIN:
      for (int i = 0; i < n; ++i) o[i] = b[i] < a[i] ? b[i] : a[i];
      break;
    case B_PYMAX:
      for (int i = 0; i < n; ++i) o[i] = b[i] > a[i] ? b[i] : a[i];
      break;
    default: break;
  }
  and_valid(R, I.dst, I.a, I.b, n);
}

template <typename T> void run_cmp(Regs& R, const Instr& I, int n) {
  uint8_t* o = R.p<uint8_t>(I.dst);
  const T* a = R.p<T>(I.a);
  const T* b = R.p<T>(I.b);
  switch (I.aux) {
    case C_LT: for (int i = 0; i < n; ++i) o[i] = a[i] < b[i]; break;
    case C_LE: for (int i = 0; i < n; ++i) o[i] = a[i] <= b[i]; break;
    case C_GT: for (int i = 0; i < n; ++i) o[i] = a[i] > b[i]; break;
    case C_GE: for (int i = 0; i < n; ++i) o[i] = a[i] >= b[i]; break;
    case C_EQ: for (int i = 0; i < n; ++i) o[i] = a[i] == b[i]; break;
    case C_NE: for (int i = 0; i < n; ++i) o[i] = a[i] != b[i]; break;
    default: break;
  }
  and_valid(R, I.dst, I.a, I.b, n);
}

template <typename T> void run_un(Regs& R, const Instr& I, int n) {
  T* o = R.p<T>(I.dst);
  const T* a = R.p<T>(I.a);
  switch (I.aux) {
    case U_NEG:
      if constexpr (std::is_integral<T>::value) for (int i = 0; i < n; ++i) o[i] = wrap_sub<T>(0, a[i]);
      else for (int i = 0; i < n; ++i) o[i] = -a[i];
      break;
    case U_ABS:
      if constexpr (std::is_integral<T>::value)
        for (int i = 0; i < n; ++i) o[i] = a[i] < 0 ? wrap_sub<T>(0, a[i]) : a[i];
      else for (int i = 0; i < n; ++i) o[i] = std::fabs(a[i]);
      break;
    case U_NOT:
      for (int i = 0; i < n; ++i) o[i] = !a[i];
      break;
    case U_SQRT: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::sqrt(a[i]); break;
    case U_FLOOR: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::floor(a[i]); break;
    case U_CEIL: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::ceil(a[i]); break;
    case U_TRUNC: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::trunc(a[i]); break;
    case U_EXP: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::exp(a[i]); break;
    case U_SIN: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::sin(a[i]); break;
    case U_COS: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::cos(a[i]); break;
    case U_TAN: if constexpr (std::is_floating_point<T>::value) for (int i = 0; i < n; ++i) o[i] = std::tan(a[i]); break;
    default: break;
  }
  and_valid(R, I.dst, I.a, -1, n);
}

template <typename To> void run_cast(Regs& R, const Instr& I, int n) {
  To* o = R.p<To>(I.dst);
  dispatch(I.aux, [&](auto tag) {
    using From = decltype(tag);
    const From* a = R.p<From>(I.a);
    for (int i = 0; i < n; ++i) o[i] = cvt<To, From>(a[i]);
  });
  and_valid(R, I.dst, I.a, -1, n);
}

// Loads the chunk's rows of one input column. Before any FILTER of the chunk those are the
// contiguous rows r0..r0+n; after one, `rows` (the surviving input row ids) says which.
template <typename T> void load(Regs& R, int dst, const void* vals, const uint8_t* validity,
                               int64_t off, int64_t r0, int n, const int32_t* rows) {
  T* o = R.p<T>(dst);
  if constexpr (std::is_same<T, uint8_t>::value) {
    const uint8_t* bits = static_cast<const uint8_t*>(vals);
    for (int i = 0; i < n; ++i) {
      const int64_t j = off + (rows ? rows[i] : r0 + i);
      o[i] = (bits[j >> 3] >> (j & 7)) & 1;
    }
  } else if (rows == nullptr) {
    std::memcpy(o, static_cast<const T*>(vals) + off + r0, sizeof(T) * size_t(n));
  } else {
    const T* src = static_cast<const T*>(vals) + off;
    for (int i = 0; i < n; ++i) o[i] = src[rows[i]];
  }
  if (validity == nullptr) {
    R.allvalid[dst] = 1;
    return;
  }
  R.allvalid[dst] = 0;
  uint8_t* v = R.v(dst);
  for (int i = 0; i < n; ++i) {
    const int64_t j = off + (rows ? rows[i] : r0 + i);
    v[i] = (validity[j >> 3] >> (j & 7)) & 1;
  }
}

int elem_size(int type) { return type == T_BOOL ? 1 : (type == T_I32 || type == T_F32) ? 4 : 8; }

}  // namespace

extern "C" {

// Calendar self-check (tests/test_sanitizers.py): the 32-bit civil path against the 64-bit one
// over `n` day counts spread across [lo, hi]; returns the number of mismatching fields.
int64_t rx_expr_calendar_check(int64_t lo, int64_t hi, int64_t n) {
  int64_t bad = 0;
  const double step = n > 1 ? double(hi - lo) / double(n - 1) : 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t days = lo + int64_t(step * double(k));
    int64_t y; int m, d;
    civil(days, &y, &m, &d);
    const Civil c = civil_any(days);
    const int64_t doy = days - days_from_civil(y, 1, 1) + 1;
    bad += (c.y != int32_t(y)) + (c.m != m) + (c.d != d) + (c.doy != doy);
  }
  return bad;
}

// Runs `ncode` instructions over `nrows` input rows. Returns the number of output rows, or -1
// on a malformed program. `sel_out` (nullable) receives the input row id of every output row.
int64_t rx_expr_run(const int32_t* code, int32_t ncode, const double* fconst, const int64_t* iconst,
                    const int32_t* live, int32_t nslots, int64_t nrows,
                    const void* const* in_vals, const uint8_t* const* in_valid, const int64_t* in_off,
                    const int32_t* out_slot, const int32_t* out_type, void* const* out_vals,
                    uint8_t* const* out_valid, int64_t* out_nulls, int32_t nout, int32_t* sel_out) {
  const Instr* prog = reinterpret_cast<const Instr*>(code);
  for (int k = 0; k < ncode; ++k) {
    const Instr& I = prog[k];
    if (I.dst >= nslots || I.a >= nslots || I.b >= nslots || I.c >= nslots) return -1;
  }
  Regs R(nslots);
  std::vector<int32_t> rowid(CH);
  std::vector<int32_t> keep(CH);
  for (int o = 0; o < nout; ++o) {
    out_nulls[o] = 0;
    if (out_valid[o] != nullptr) std::memset(out_valid[o], 0, size_t((nrows + 7) / 8));
    if (out_type[o] == T_BOOL) std::memset(out_vals[o], 0, size_t((nrows + 7) / 8));
  }
  int64_t pos = 0;
  for (int64_t r0 = 0; r0 < nrows; r0 += CH) {
    int n = int(nrows - r0 < CH ? nrows - r0 : CH);
    bool compacted = false;
    for (int i = 0; i < n; ++i) rowid[i] = int32_t(r0 + i);
    for (int k = 0; k < ncode && n > 0; ++k) {
      const Instr& I = prog[k];
      switch (I.op) {
        case OP_LOAD:
          dispatch(I.type, [&](auto tag) {
            load<decltype(tag)>(R, I.dst, in_vals[I.imm], in_valid[I.imm], in_off[I.imm], r0, n,
                                compacted ? rowid.data() : nullptr);
          });
          break;
        case OP_CONST:
          dispatch(I.type, [&](auto tag) {
            using T = decltype(tag);
            T c = (I.type == T_F32 || I.type == T_F64) ? T(fconst[I.imm]) : T(iconst[I.imm]);
            T* o = R.p<T>(I.dst);
            for (int i = 0; i < n; ++i) o[i] = c;
          });
          if (I.aux == 1) {
            R.allvalid[I.dst] = 0;
            std::memset(R.v(I.dst), 0, size_t(n));
          } else {
            R.allvalid[I.dst] = 1;
          }
          break;
        case OP_CAST:
          dispatch(I.type, [&](auto tag) { run_cast<decltype(tag)>(R, I, n); });
          break;
        case OP_BIN:
          dispatch(I.type, [&](auto tag) { run_bin<decltype(tag)>(R, I, n); });
          break;
        case OP_CMP:
          dispatch(I.type, [&](auto tag) { run_cmp<decltype(tag)>(R, I, n); });
          break;
        case OP_UN:
          if (I.aux == U_ISNAN) {
            uint8_t* o = R.p<uint8_t>(I.dst);
            dispatch(I.type, [&](auto tag) {
              using T = decltype(tag);
              const T* a = R.p<T>(I.a);
              for (int i = 0; i < n; ++i) o[i] = a[i] != a[i];
            });
            and_valid(R, I.dst, I.a, -1, n);
          } else {
            dispatch(I.type, [&](auto tag) { run_un<decltype(tag)>(R, I, n); });
          }
          break;
        case OP_AND:
        case OP_OR: {
          // Kleene logic: false AND null = false, true OR null = true
          const uint8_t* a = R.p<uint8_t>(I.a);
          const uint8_t* b = R.p<uint8_t>(I.b);
          uint8_t* o = R.p<uint8_t>(I.dst);
          const bool va = R.allvalid[I.a], vb = R.allvalid[I.b];
          const uint8_t* xa = R.v(I.a);
          const uint8_t* xb = R.v(I.b);
          if (va && vb) {
            if (I.op == OP_AND) for (int i = 0; i < n; ++i) o[i] = a[i] & b[i];
            else for (int i = 0; i < n; ++i) o[i] = a[i] | b[i];
            R.allvalid[I.dst] = 1;
          } else {
            uint8_t* ov = R.v(I.dst);
            for (int i = 0; i < n; ++i) {
              const uint8_t pa_ = va ? 1 : xa[i], pb = vb ? 1 : xb[i];
              if (I.op == OP_AND) {
                const bool f = (pa_ && !a[i]) || (pb && !b[i]);
                o[i] = pa_ && pb && a[i] && b[i];
                ov[i] = f || (pa_ && pb);
              } else {
                const bool t = (pa_ && a[i]) || (pb && b[i]);
                o[i] = t;
                ov[i] = t || (pa_ && pb);
              }
            }
            R.allvalid[I.dst] = 0;
          }
          break;
        }
        case OP_IFELSE: {
          const uint8_t* c = R.p<uint8_t>(I.c);
          const bool vc = R.allvalid[I.c];
          const uint8_t* xc = R.v(I.c);
          dispatch(I.type, [&](auto tag) {
            using T = decltype(tag);
            const T* a = R.p<T>(I.a);
            const T* b = R.p<T>(I.b);
            T* o = R.p<T>(I.dst);
            for (int i = 0; i < n; ++i) {
              const bool take_a = c[i] && (vc || xc[i]);
              o[i] = take_a ? a[i] : b[i];
            }
          });
          const bool va = R.allvalid[I.a], vb = R.allvalid[I.b];
          if (va && vb && (vc || I.aux == 1)) {
            R.allvalid[I.dst] = 1;
          } else {
            uint8_t* ov = R.v(I.dst);
            const uint8_t* xa = R.v(I.a);
            const uint8_t* xb = R.v(I.b);
            for (int i = 0; i < n; ++i) {
              const bool cvalid = vc || xc[i];
              const bool take_a = c[i] && cvalid;
              uint8_t v = take_a ? (va ? 1 : xa[i]) : (vb ? 1 : xb[i]);
              if (!cvalid && I.aux == 0) v = 0;
              ov[i] = v;
            }
            R.allvalid[I.dst] = 0;
          }
          break;
        }
        case OP_DT:
          run_dt(R.p<int64_t>(I.a), R.p<int32_t>(I.dst), n, I.imm > 0 ? I.imm : 1, I.aux);
          and_valid(R, I.dst, I.a, -1, n);
          break;
        case OP_ISNULL: {
          uint8_t* o = R.p<uint8_t>(I.dst);
          const bool va = R.allvalid[I.a];
          const uint8_t* xa = R.v(I.a);
          for (int i = 0; i < n; ++i) {
            const uint8_t isnull = va ? 0 : !xa[i];
            o[i] = I.aux == 1 ? !isnull : isnull;
          }
          R.allvalid[I.dst] = 1;
          break;
        }
        case OP_FILLNULL: {
          dispatch(I.type, [&](auto tag) {
            using T = decltype(tag);
            const T* a = R.p<T>(I.a);
            const T* b = R.p<T>(I.b);
            T* o = R.p<T>(I.dst);
            const bool va = R.allvalid[I.a];
            const uint8_t* xa = R.v(I.a);
            for (int i = 0; i < n; ++i) o[i] = (va || xa[i]) ? a[i] : b[i];
          });
          const bool va = R.allvalid[I.a], vb = R.allvalid[I.b];
          if (va || vb) {
            R.allvalid[I.dst] = 1;
          } else {
            uint8_t* ov = R.v(I.dst);
            const uint8_t* xa = R.v(I.a);
            const uint8_t* xb = R.v(I.b);
            for (int i = 0; i < n; ++i) ov[i] = xa[i] | xb[i];
            R.allvalid[I.dst] = 0;
          }
          break;
        }
        case OP_FILTER: {
          const uint8_t* c = R.p<uint8_t>(I.a);
          const bool vc = R.allvalid[I.a];
          const uint8_t* xc = R.v(I.a);
          int m = 0;
          for (int i = 0; i < n; ++i) {
            keep[m] = i;
            m += (c[i] && (vc || xc[i])) ? 1 : 0;
          }
          if (m != n) {
            const int32_t* lv = live + I.imm;
            const int cnt = lv[0];
            for (int q = 0; q < cnt; ++q) {
              const int s = lv[1 + 2 * q], ty = lv[2 + 2 * q];
              dispatch(ty, [&](auto tag) {
                using T = decltype(tag);
                T* d = R.p<T>(s);
                for (int i = 0; i < m; ++i) d[i] = d[keep[i]];
              });
              if (!R.allvalid[s]) {
                uint8_t* v = R.v(s);
                for (int i = 0; i < m; ++i) v[i] = v[keep[i]];
              }
            }
            for (int i = 0; i < m; ++i) rowid[i] = rowid[keep[i]];
            n = m;
            compacted = true;
          }
          break;
        }
        default:
          return -1;
      }
    }
    if (n <= 0) continue;
    // append this chunk's outputs
    for (int o = 0; o < nout; ++o) {
      const int s = out_slot[o], ty = out_type[o];
      if (ty == T_BOOL) {
        pack_bits(static_cast<uint8_t*>(out_vals[o]), pos, R.p<uint8_t>(s), n);
      } else {
        std::memcpy(static_cast<uint8_t*>(out_vals[o]) + size_t(pos) * elem_size(ty),
                    R.p<uint8_t>(s), size_t(n) * elem_size(ty));
      }
      uint8_t* vb = out_valid[o];
      if (vb == nullptr) continue;
      if (R.allvalid[s]) set_bits(vb, pos, n);
      else out_nulls[o] += pack_bits(vb, pos, R.v(s), n);
    }
    if (sel_out != nullptr) std::memcpy(sel_out + pos, rowid.data(), sizeof(int32_t) * size_t(n));
    pos += n;
  }
  return pos;
}

}  // extern "C"
