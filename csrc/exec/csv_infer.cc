// Small-file CSV read with schema inference, natively (SURVEY §2.9 exec: the executor's data
// path; reference role: Spark's `spark.read.csv(..., inferSchema=true)` in
// examples/pytorch_nyctaxi.py / data_process.py).
//
// raydp_amd/spark/sources.py CsvSource._infer parses the head of the first file with pyarrow's
// reader (inference over every value, null token "" only) and, for a file that fits in that
// head, ships the parse as the partition. For the few-thousand-row files of the NYC pipeline
// that read is ~1 ms of fixed reader cost. This is the same read done in one pass over the bytes
// -- and it gives exactly Arrow's answer or none:
//
//   * every field is classified with ARROW'S OWN value parsers (arrow::internal::ParseValue /
//     StringToFloat, the functions the CSV converters call): int64, double, or "surely text" (a
//     value that no numeric / boolean / ISO date, time or timestamp parser can accept because it
//     holds a character none of them consumes);
//   * a column is int64 when all its values are ints, double when ints and reals, string when it
//     has at least one surely-text value -- the type Arrow's inference ladder ends on;
//   * anything else (booleans, temporal-looking values, hex ints, NaN/inf words, leading
//     whitespace, '+' signs, quotes inside fields, CR line ends, non-ASCII bytes, ragged rows,
//     all-null columns) returns "not handled" and the caller reads with pyarrow.
#include <arrow/api.h>
#include <arrow/c/bridge.h>
#include <arrow/util/value_parsing.h>

#include <emmintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

namespace {

struct Field {
  const char* p;
  int32_t n;
};

enum Kind : uint8_t { kNull = 0, kInt = 1, kReal = 2, kText = 3, kAmbiguous = 4 };

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// -?[0-9]+ (at most 18 digits: always within int64)
bool int_shape(const char* s, int32_t n) {
  int i = 0;
  if (n > 0 && s[0] == '-') i = 1;
  if (i == n || n - i > 18) return false;
  for (; i < n; ++i)
    if (!is_digit(s[i])) return false;
  return true;
}

// -?[0-9]+(.[0-9]+)?([eE]-?[0-9]+)?. On a match, *fast says whether the value is exactly
// w * 10^e10 with w < 2^53 and |e10| <= 22 (decimal mantissa digits accumulated on the way):
// then one IEEE multiply or divide of two exact doubles is the correctly rounded result
// (Clinger's fast path) -- the same double any correctly rounding parser, Arrow's
// StringToFloat included, returns -- and the library parser runs only for the rest.
bool real_shape(const char* s, int32_t n, bool* fast, double* dv) {
  int i = 0;
  bool neg = false;
  if (i < n && s[i] == '-') neg = true, ++i;
  uint64_t w = 0;
  int nd = 0, frac = 0;
  const int d0 = i;
  while (i < n && is_digit(s[i])) w = w * 10 + static_cast<uint64_t>(s[i++] - '0'), ++nd;
  if (i == d0) return false;
  if (i < n && s[i] == '.') {
    ++i;
    const int f0 = i;
    while (i < n && is_digit(s[i])) w = w * 10 + static_cast<uint64_t>(s[i++] - '0'), ++nd;
    frac = i - f0;
    if (frac == 0) return false;
  }
  int e = 0, ed = 0;
  bool eneg = false;
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    if (i < n && s[i] == '-') eneg = true, ++i;
    const int e0 = i;
    while (i < n && is_digit(s[i])) {
      if (ed < 6) e = e * 10 + (s[i] - '0');
      ++i, ++ed;
    }
    if (i == e0) return false;
  }
  if (i != n) return false;
  static const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  const int e10 = (eneg ? -e : e) - frac;
  *fast = nd <= 19 && ed <= 5 && w <= (uint64_t{1} << 53) && e10 >= -22 && e10 <= 22;
  if (*fast) {
    const double m = static_cast<double>(w);
    const double v = e10 < 0 ? m / kPow10[-e10] : m * kPow10[e10];
    *dv = neg ? -v : v;
  }
  return true;
}

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? static_cast<char>(c - 'A' + 'a') : c; }

bool word_is(const char* s, int32_t n, const char* w) {
  const int32_t m = static_cast<int32_t>(std::strlen(w));
  if (n != m) return false;
  for (int32_t i = 0; i < n; ++i)
    if (lower(s[i]) != w[i]) return false;
  return true;
}

// Classify one field; a number is parsed once, into *iv / *dv.
Kind classify(const Field& f, int64_t* iv, double* dv) {
  const char* s = f.p;
  const int32_t n = f.n;
  if (n == 0) return kNull;
  if (s[0] == ' ' || s[0] == '\t' || s[n - 1] == ' ' || s[n - 1] == '\t') return kAmbiguous;
  if (int_shape(s, n)) {
    // -?[0-9]{1,18}: the exact value (what Arrow's integer parser returns for it)
    const bool neg = s[0] == '-';
    int64_t v = 0;
    for (int32_t i = neg; i < n; ++i) v = v * 10 + (s[i] - '0');
    *iv = neg ? -v : v;
    return kInt;
  }
  bool fast = false;
  if (real_shape(s, n, &fast, dv))
    return fast || arrow::internal::StringToFloat(s, static_cast<size_t>(n), '.', dv) ? kReal : kAmbiguous;
  // not a vetted number shape: ambiguous if Arrow would still read it as one (both parsers
  // need a sign, a digit, '.', or the first letter of inf / nan up front)
  const char c0 = (s[0] == '-' || s[0] == '+') && n > 1 ? s[1] : s[0];
  if ((is_digit(c0) || c0 == '.' || c0 == 'i' || c0 == 'I' || c0 == 'n' || c0 == 'N') &&
      (arrow::internal::ParseValue<arrow::Int64Type>(s, static_cast<size_t>(n), iv) ||
       arrow::internal::StringToFloat(s, static_cast<size_t>(n), '.', dv)))
    return kAmbiguous;
  // boolean / special float words
  const char* t = s;
  int32_t m = n;
  if (m > 0 && (t[0] == '-' || t[0] == '+')) ++t, --m;
  static const char* kWords[] = {"true", "false", "inf", "infinity", "nan"};
  for (const char* w : kWords)
    if (word_is(t, m, w)) return kAmbiguous;
  // characters an ISO-8601 date / time / timestamp (with zone) can consist of
  for (int32_t i = 0; i < n; ++i) {
    const char c = s[i];
    if (static_cast<unsigned char>(c) >= 0x80) return kAmbiguous;   // utf8 validity: leave to Arrow
    if (!(is_digit(c) || c == '-' || c == ':' || c == '.' || c == ' ' || c == '+' || c == 'T' || c == 't' ||
          c == 'Z' || c == 'z' || c == 'W'))
      return kText;
  }
  return kAmbiguous;
}

// First byte at or after k that is the delimiter, a quote, CR or LF (len if none): 16 bytes per
// compare (SSE2, part of x86-64) -- fields are short, so mostly one load per field.
inline int64_t next_special(const char* d, int64_t k, int64_t len, char delim) {
  const __m128i vd = _mm_set1_epi8(delim), vq = _mm_set1_epi8('"'), vr = _mm_set1_epi8('\r'),
                vn = _mm_set1_epi8('\n');
  while (k + 16 <= len) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(d + k));
    const __m128i m = _mm_or_si128(_mm_or_si128(_mm_cmpeq_epi8(x, vd), _mm_cmpeq_epi8(x, vq)),
                                   _mm_or_si128(_mm_cmpeq_epi8(x, vr), _mm_cmpeq_epi8(x, vn)));
    const int bits = _mm_movemask_epi8(m);
    if (bits) return k + __builtin_ctz(static_cast<unsigned>(bits));
    k += 16;
  }
  while (k < len && d[k] != delim && d[k] != '"' && d[k] != '\r' && d[k] != '\n') ++k;
  return k;
}

// Tokenise `data` into a row-major field grid (`ncol` fields per row, header included).
// Returns false on anything the simple grammar does not cover (the caller falls back to Arrow's
// reader) or on a row whose field count differs from the header's (Arrow raises on it).
// Empty lines are skipped (Arrow's ignore_empty_lines); a delimiter ending a line adds one empty
// field; a quoted field must close on its line and be followed by the delimiter or the line end;
// an unquoted field holding a quote or a CR is not handled.
bool tokenize(const char* data, int64_t len, char delim, std::vector<Field>* cells, size_t* ncol) {
  int64_t i = 0;
  *ncol = 0;
  cells->reserve(static_cast<size_t>(len / 8 + 16));
  while (i < len) {
    if (data[i] == '\n') {  // empty line
      ++i;
      continue;
    }
    const size_t row_start = cells->size();
    int64_t k = i;
    for (;;) {
      if (k >= len || data[k] == '\n') {  // after a delimiter that ended the line
        cells->push_back(Field{data + k, 0});
        break;
      }
      if (data[k] == '"') {
        int64_t q = k + 1;
        while (q < len && data[q] != '"' && data[q] != '\n') ++q;
        if (q >= len || data[q] != '"') return false;                                  // unterminated on this line
        if (q + 1 < len && data[q + 1] != delim && data[q + 1] != '\n') return false;  // "" escape or text after quote
        cells->push_back(Field{data + k + 1, static_cast<int32_t>(q - k - 1)});
        k = q + 1;
      } else {
        const int64_t q = next_special(data, k, len, delim);
        if (q < len && (data[q] == '"' || data[q] == '\r')) return false;
        cells->push_back(Field{data + k, static_cast<int32_t>(q - k)});
        k = q;
      }
      if (k >= len || data[k] == '\n') break;
      ++k;  // delimiter
    }
    const size_t nf = cells->size() - row_start;
    if (*ncol == 0) *ncol = nf;
    else if (nf != *ncol) return false;
    i = k + 1;
  }
  return *ncol > 0;
}

// Type and build column c (1), or say the column is not decided here (0) / an Arrow error (-1).
int build_column(const std::vector<Field>& cells, size_t ncol, size_t nrow, size_t c,
                 std::shared_ptr<arrow::Array>* out) {
  std::vector<Kind> kinds(nrow);
  std::vector<int64_t> ivals(nrow);
  std::vector<double> dvals(nrow);
  const Field& h = cells[c];
  for (int32_t j = 0; j < h.n; ++j)
    if (static_cast<unsigned char>(h.p[j]) >= 0x80) return 0;
  bool any_real = false, any_text = false, any_value = false;
  for (size_t r = 0; r < nrow; ++r) {
    // one surely-text value decides the column (Arrow's ladder ends on string whatever the
    // other values are; "" stays the only null): the rest need no classification -- only a
    // check that they are ASCII (a byte >= 0x80 may be invalid UTF-8, which Arrow types as
    // binary: then the column is Arrow's to decide)
    if (any_text) {
      const Field& f = cells[(r + 1) * ncol + c];
      for (int32_t j = 0; j < f.n; ++j)
        if (static_cast<unsigned char>(f.p[j]) >= 0x80) return 0;
      continue;
    }
    const Kind k = classify(cells[(r + 1) * ncol + c], &ivals[r], &dvals[r]);
    if (k == kAmbiguous) return 0;
    kinds[r] = k;
    any_value |= k != kNull;
    any_real |= k == kReal;
    any_text |= k == kText;
  }
  if (!any_value) return 0;                                // null-typed column: Arrow decides
  std::shared_ptr<arrow::Array> arr;
  arrow::Status st;
  if (any_text) {
    arrow::StringBuilder b;
    st = b.Reserve(static_cast<int64_t>(nrow));
    for (size_t r = 0; r < nrow && st.ok(); ++r) {
      const Field& f = cells[(r + 1) * ncol + c];
      st = f.n == 0 ? b.AppendNull() : b.Append(f.p, f.n);
    }
    if (st.ok()) st = b.Finish(&arr);
  } else if (any_real) {
    // ints inside a double column: Arrow's real decoder parses their text as a double
    // (at most 18 digits: exact as a double below 2^53, the correctly rounded double above)
    for (size_t r = 0; r < nrow; ++r) {
      if (kinds[r] != kInt) continue;
      const int64_t a = ivals[r] < 0 ? -ivals[r] : ivals[r];
      if (a <= (int64_t{1} << 53)) {
        dvals[r] = static_cast<double>(ivals[r]);
        continue;
      }
      const Field& f = cells[(r + 1) * ncol + c];
      if (!arrow::internal::StringToFloat(f.p, static_cast<size_t>(f.n), '.', &dvals[r])) return 0;
    }
    arrow::DoubleBuilder b;
    st = b.Reserve(static_cast<int64_t>(nrow));
    for (size_t r = 0; r < nrow && st.ok(); ++r) {
      if (kinds[r] == kNull) b.UnsafeAppendNull();
      else b.UnsafeAppend(dvals[r]);
    }
    if (st.ok()) st = b.Finish(&arr);
  } else {
    arrow::Int64Builder b;
    st = b.Reserve(static_cast<int64_t>(nrow));
    for (size_t r = 0; r < nrow && st.ok(); ++r) {
      if (kinds[r] == kNull) b.UnsafeAppendNull();
      else b.UnsafeAppend(ivals[r]);
    }
    if (st.ok()) st = b.Finish(&arr);
  }
  if (!st.ok()) return -1;
  *out = arr;
  return 1;
}

}  // namespace

extern "C" {

// Parse a CSV held in memory (first line = header, null token "") the way pyarrow's reader with
// type inference would. Returns 1 and exports the table as an ArrowArrayStream into `out`, 0 when
// the input holds anything this reader does not decide (read it with Arrow), -1 on an error.
int rx_csv_infer(const char* data, int64_t len, char delim, void* out) {
  std::vector<Field> cells;
  size_t ncol = 0;
  if (len <= 0 || !tokenize(data, len, delim, &cells, &ncol)) return 0;
  const size_t nrow = cells.size() / ncol - 1;
  if (nrow == 0) return 0;
  // one column after the other on the calling thread (typing them on 4 threads measured slower
  // on the GPU box: thread start-up on a shared 256-core host outweighed ~60 us of parsing)
  std::vector<std::shared_ptr<arrow::Array>> cols(ncol);
  std::vector<int> rc(ncol, 1);
  for (size_t c = 0; c < ncol; ++c) {
    rc[c] = build_column(cells, ncol, nrow, c, &cols[c]);
    if (rc[c] != 1) return rc[c];
  }
  std::vector<std::shared_ptr<arrow::Field>> fields;
  for (size_t c = 0; c < ncol; ++c) {
    if (rc[c] != 1) return rc[c];   // the first undecided / failed column, as a column-order scan
    const Field& h = cells[c];
    fields.push_back(arrow::field(std::string(h.p, static_cast<size_t>(h.n)), cols[c]->type()));
  }
  auto table = arrow::Table::Make(arrow::schema(fields), cols, static_cast<int64_t>(nrow));
  auto reader = std::make_shared<arrow::TableBatchReader>(table);
  if (!arrow::ExportRecordBatchReader(reader, static_cast<struct ArrowArrayStream*>(out)).ok()) return -1;
  return 1;
}

}  // extern "C"
