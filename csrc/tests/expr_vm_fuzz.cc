// Random-program driver for the fused expression VM (csrc/exec/expr/expr_vm.cc), built under
// AddressSanitizer+UBSan by raydp_amd/native/build.py (tests/test_sanitizers.py).
//
// Every program is well typed by construction (SSA: one register per instruction, operands
// drawn from earlier registers of the type the opcode reads), but values are adversarial:
// inputs mix nulls, NaN/inf, INT_MIN/INT_MAX, huge timestamps, zero divisors, and filters
// drop random row subsets (so later loads gather through the surviving row ids). The run
// checks memory safety / UB through the sanitizers and a few invariants: row counts, selection
// ids strictly increasing and in range, null counts consistent with the validity bitmaps.
//
//   expr_vm_fuzz <programs> <seed>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

extern "C" int64_t rx_expr_run(const int32_t* code, int32_t ncode, const double* fconst, const int64_t* iconst,
                               const int32_t* live, int32_t nslots, int64_t nrows,
                               const void* const* in_vals, const uint8_t* const* in_valid, const int64_t* in_off,
                               const int32_t* out_slot, const int32_t* out_type, void* const* out_vals,
                               uint8_t* const* out_valid, int64_t* out_nulls, int32_t nout, int32_t* sel_out);
extern "C" int64_t rx_expr_calendar_check(int64_t lo, int64_t hi, int64_t n);

namespace {

enum { T_BOOL, T_I32, T_I64, T_F32, T_F64 };
enum { OP_LOAD = 1, OP_CONST, OP_CAST, OP_BIN, OP_CMP, OP_UN, OP_AND, OP_OR, OP_IFELSE, OP_DT, OP_FILTER,
       OP_ISNULL, OP_FILLNULL };

int esize(int t) { return t == T_BOOL ? 1 : (t == T_I32 || t == T_F32) ? 4 : 8; }

struct Input {
  int type;
  int64_t off;
  std::vector<uint8_t> vals;   // values (bit-packed for bool), `off` leading rows of padding
  std::vector<uint8_t> valid;  // bitmap or empty
};

template <typename T> T pick(std::mt19937_64& g, const std::vector<T>& xs) { return xs[g() % xs.size()]; }

Input make_input(std::mt19937_64& g, int type, int64_t n) {
  Input in;
  in.type = type;
  in.off = int64_t(g() % 13);
  const int64_t tot = n + in.off;
  if (type == T_BOOL) {
    in.vals.resize(size_t((tot + 7) / 8));
    for (auto& b : in.vals) b = uint8_t(g());
  } else {
    in.vals.resize(size_t(tot) * esize(type));
    for (int64_t i = 0; i < tot; ++i) {
      uint8_t* p = in.vals.data() + i * esize(type);
      switch (type) {
        case T_I32: {
          int32_t v = pick<int32_t>(g, {0, 1, -1, 7, -13, std::numeric_limits<int32_t>::min(),
                                        std::numeric_limits<int32_t>::max(), int32_t(g())});
          std::memcpy(p, &v, 4);
          break;
        }
        case T_I64: {
          int64_t v = pick<int64_t>(g, {0, 1, -1, 86399, -86401, std::numeric_limits<int64_t>::min(),
                                        std::numeric_limits<int64_t>::max(), int64_t(g()),
                                        int64_t(g() % 4000000000ULL) - 2000000000});
          std::memcpy(p, &v, 8);
          break;
        }
        case T_F32: {
          float v = pick<float>(g, {0.f, -0.f, 1.5f, -2.25f, NAN, INFINITY, -INFINITY, 3e38f,
                                    float(int32_t(g())) * 1e-3f});
          std::memcpy(p, &v, 4);
          break;
        }
        default: {
          double v = pick<double>(g, {0.0, -0.0, 1.5, -7.75, NAN, INFINITY, -INFINITY, 1e300,
                                      9.3e18, -9.3e18, double(int64_t(g())) * 1e-6});
          std::memcpy(p, &v, 8);
        }
      }
    }
  }
  if (g() % 2) {
    in.valid.resize(size_t((tot + 7) / 8));
    for (auto& b : in.valid) b = uint8_t(g() | g());   // mostly valid
  }
  return in;
}

struct Prog {
  std::vector<int32_t> code;   // 8 ints per instruction
  std::vector<int32_t> live;
  std::vector<int> type;       // register type
  std::vector<double> f;
  std::vector<int64_t> i;
};

void emit(Prog& P, int op, int dst, int a, int b, int c, int ty, int aux, int imm) {
  P.code.insert(P.code.end(), {op, dst, a, b, c, ty, aux, imm});
}

int new_reg(Prog& P, int ty) {
  P.type.push_back(ty);
  return int(P.type.size()) - 1;
}

int any_of(std::mt19937_64& g, const Prog& P, int ty) {
  std::vector<int> c;
  for (size_t r = 0; r < P.type.size(); ++r)
    if (P.type[r] == ty) c.push_back(int(r));
  return c.empty() ? -1 : c[g() % c.size()];
}

bool is_float(int t) { return t == T_F32 || t == T_F64; }

Prog make_prog(std::mt19937_64& g, const std::vector<Input>& ins, int len) {
  Prog P;
  // load every input once, up front (some after filters too, below)
  for (size_t k = 0; k < ins.size(); ++k) emit(P, OP_LOAD, new_reg(P, ins[k].type), -1, -1, -1, ins[k].type, 0, int(k));
  for (int t = 0; t < 5; ++t) {  // one constant per type
    const int r = new_reg(P, t);
    if (is_float(t)) {
      P.f.push_back(pick<double>(g, {0.0, 2.0, -1.0, NAN}));
      emit(P, OP_CONST, r, -1, -1, -1, t, g() % 5 == 0 ? 1 : 0, int(P.f.size()) - 1);
    } else {
      P.i.push_back(pick<int64_t>(g, {0, 1, -1, 3}));
      emit(P, OP_CONST, r, -1, -1, -1, t, g() % 5 == 0 ? 1 : 0, int(P.i.size()) - 1);
    }
  }
  for (int s = 0; s < len; ++s) {
    const int op = pick<int>(g, {OP_CAST, OP_BIN, OP_BIN, OP_CMP, OP_UN, OP_AND, OP_OR, OP_IFELSE, OP_DT,
                                 OP_FILTER, OP_ISNULL, OP_FILLNULL, OP_LOAD});
    const int t = int(g() % 5);
    switch (op) {
      case OP_LOAD: {
        const int k = int(g() % ins.size());
        emit(P, OP_LOAD, new_reg(P, ins[k].type), -1, -1, -1, ins[k].type, 0, k);
        break;
      }
      case OP_CAST: {
        const int a = any_of(g, P, t);
        const int to = int(g() % 5);
        emit(P, OP_CAST, new_reg(P, to), a, -1, -1, to, t, 0);
        break;
      }
      case OP_BIN: {
        if (t == T_BOOL) break;
        const int a = any_of(g, P, t), b = any_of(g, P, t);
        int kind = int(g() % 10);
        if (!is_float(t) && (kind == 3 || kind == 4 || kind == 7)) kind = 0;  // float-only kinds
        emit(P, OP_BIN, new_reg(P, t), a, b, -1, t, kind, 0);
        break;
      }
      case OP_CMP: {
        const int a = any_of(g, P, t), b = any_of(g, P, t);
        emit(P, OP_CMP, new_reg(P, T_BOOL), a, b, -1, t, int(g() % 6), 0);
        break;
      }
      case OP_UN: {
        int kind;
        if (t == T_BOOL) kind = 2;
        else if (is_float(t)) kind = pick<int>(g, {0, 1, 3, 4, 5, 6, 7});
        else kind = pick<int>(g, {0, 1});
        const int a = any_of(g, P, t);
        const int dt = kind == 7 ? T_BOOL : t;
        emit(P, OP_UN, new_reg(P, dt), a, -1, -1, kind == 7 ? t : t, kind, 0);
        break;
      }
      case OP_AND:
      case OP_OR: {
        const int a = any_of(g, P, T_BOOL), b = any_of(g, P, T_BOOL);
        emit(P, op, new_reg(P, T_BOOL), a, b, -1, T_BOOL, 0, 0);
        break;
      }
      case OP_IFELSE: {
        const int c = any_of(g, P, T_BOOL), a = any_of(g, P, t), b = any_of(g, P, t);
        emit(P, OP_IFELSE, new_reg(P, t), a, b, c, t, int(g() % 2), 0);
        break;
      }
      case OP_DT: {
        const int a = any_of(g, P, T_I64);
        emit(P, OP_DT, new_reg(P, T_I32), a, -1, -1, T_I64, int(g() % 10),
             pick<int>(g, {1, 1000, 1000000}));
        break;
      }
      case OP_FILTER: {
        if (g() % 3) break;   // keep most rows alive
        const int a = any_of(g, P, T_BOOL);
        const int at = int(P.live.size());
        P.live.push_back(int32_t(P.type.size()));
        for (size_t r = 0; r < P.type.size(); ++r) {
          P.live.push_back(int32_t(r));
          P.live.push_back(P.type[r]);
        }
        emit(P, OP_FILTER, -1, a, -1, -1, T_BOOL, 0, at);
        break;
      }
      case OP_ISNULL: {
        const int a = any_of(g, P, t);
        emit(P, OP_ISNULL, new_reg(P, T_BOOL), a, -1, -1, t, int(g() % 2), 0);
        break;
      }
      case OP_FILLNULL: {
        const int a = any_of(g, P, t), b = any_of(g, P, t);
        emit(P, OP_FILLNULL, new_reg(P, t), a, b, -1, t, 0, 0);
        break;
      }
    }
  }
  P.live.push_back(0);
  P.f.push_back(0);
  P.i.push_back(0);
  return P;
}

}  // namespace

int main(int argc, char** argv) {
  const int programs = argc > 1 ? std::atoi(argv[1]) : 300;
  std::mt19937_64 g(argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 1);
  int64_t total_rows = 0, kept_rows = 0;
  for (int p = 0; p < programs; ++p) {
    const int64_t n = int64_t(g() % 3000);   // spans several 1024-row chunks
    std::vector<Input> ins;
    for (int t = 0; t < 5; ++t) ins.push_back(make_input(g, t, n));
    ins.push_back(make_input(g, T_I64, n));
    Prog P = make_prog(g, ins, 10 + int(g() % 60));
    const int nslots = int(P.type.size());
    std::vector<const void*> iv;
    std::vector<const uint8_t*> ivd;
    std::vector<int64_t> io;
    for (auto& in : ins) {
      iv.push_back(in.vals.data());
      ivd.push_back(in.valid.empty() ? nullptr : in.valid.data());
      io.push_back(in.off);
    }
    // outputs: a handful of registers of every type
    std::vector<int32_t> os, ot;
    for (int k = 0; k < 6; ++k) {
      const int r = int(g() % nslots);
      os.push_back(r);
      ot.push_back(P.type[size_t(r)]);
    }
    std::vector<std::vector<uint8_t>> ov(os.size()), ovd(os.size());
    std::vector<void*> ovp;
    std::vector<uint8_t*> ovdp;
    for (size_t k = 0; k < os.size(); ++k) {
      ov[k].resize(ot[k] == T_BOOL ? size_t((n + 7) / 8 + 1) : size_t(n) * esize(ot[k]) + 8);
      ovd[k].resize(size_t((n + 7) / 8 + 1));
      ovp.push_back(ov[k].data());
      ovdp.push_back(ovd[k].data());
    }
    std::vector<int64_t> nulls(os.size());
    std::vector<int32_t> sel(size_t(n > 0 ? n : 1));
    const int64_t m = rx_expr_run(P.code.data(), int32_t(P.code.size() / 8), P.f.data(), P.i.data(), P.live.data(),
                                  nslots, n, iv.data(), ivd.data(), io.data(), os.data(), ot.data(), ovp.data(),
                                  ovdp.data(), nulls.data(), int32_t(os.size()), sel.data());
    if (m < 0 || m > n) {
      std::printf("program %d: bad row count %lld of %lld\n", p, (long long)m, (long long)n);
      return 1;
    }
    for (int64_t r = 1; r < m; ++r)
      if (sel[size_t(r)] <= sel[size_t(r - 1)] || sel[size_t(r)] >= n) {
        std::printf("program %d: selection not increasing / out of range\n", p);
        return 1;
      }
    for (size_t k = 0; k < os.size(); ++k) {
      int64_t zeros = 0;
      for (int64_t r = 0; r < m; ++r) zeros += !((ovd[k][size_t(r >> 3)] >> (r & 7)) & 1);
      if (zeros != nulls[k]) {
        std::printf("program %d: null count %lld vs bitmap %lld\n", p, (long long)nulls[k], (long long)zeros);
        return 1;
      }
    }
    total_rows += n;
    kept_rows += m;
  }
  const int64_t cal = rx_expr_calendar_check(-12699422, 1073741823LL - 12699422 - 1, 200001) +
                      rx_expr_calendar_check(-4000000000LL, 4000000000LL, 20001);
  std::printf("programs %d rows %lld kept %lld calendar mismatches %lld\n", programs, (long long)total_rows,
              (long long)kept_rows, (long long)cal);
  return cal == 0 ? 0 : 1;
}
