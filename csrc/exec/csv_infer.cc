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

// -?[0-9]+(.[0-9]+)?([eE]-?[0-9]+)?
bool real_shape(const char* s, int32_t n) {
  int i = 0;
  if (i < n && s[i] == '-') ++i;
  const int d0 = i;
  while (i < n && is_digit(s[i])) ++i;
  if (i == d0) return false;
  if (i < n && s[i] == '.') {
    ++i;
    const int f0 = i;
    while (i < n && is_digit(s[i])) ++i;
    if (i == f0) return false;
  }
  if (i < n && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    if (i < n && s[i] == '-') ++i;
    const int e0 = i;
    while (i < n && is_digit(s[i])) ++i;
    if (i == e0) return false;
  }
  return i == n;
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
  if (int_shape(s, n))
    return arrow::internal::ParseValue<arrow::Int64Type>(s, static_cast<size_t>(n), iv) ? kInt : kAmbiguous;
  if (real_shape(s, n))
    return arrow::internal::StringToFloat(s, static_cast<size_t>(n), '.', dv) ? kReal : kAmbiguous;
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

// Tokenise `data` into a row-major field grid (`ncol` fields per row, header included).
// Returns false on anything the simple grammar does not cover (the caller falls back to Arrow's
// reader) or on a row whose field count differs from the header's (Arrow raises on it).
bool tokenize(const char* data, int64_t len, char delim, std::vector<Field>* cells, size_t* ncol) {
  int64_t i = 0;
  size_t row_start = 0;
  *ncol = 0;
  cells->reserve(static_cast<size_t>(len / 8 + 16));
  while (i < len) {
    int64_t e = i;
    const void* nl = std::memchr(data + i, '\n', static_cast<size_t>(len - i));
    e = nl ? static_cast<const char*>(nl) - data : len;
    if (e == i) {  // empty line: Arrow's ignore_empty_lines
      i = e + 1;
      continue;
    }
    row_start = cells->size();
    int64_t k = i;
    for (;;) {
      if (k < e && data[k] == '"') {
        int64_t q = k + 1;
        while (q < e && data[q] != '"') ++q;
        if (q >= e) return false;                              // unterminated on this line
        if (q + 1 < e && data[q + 1] != delim) return false;   // "" escape or text after quote
        cells->push_back(Field{data + k + 1, static_cast<int32_t>(q - k - 1)});
        k = q + 1;
      } else {
        int64_t q = k;
        while (q < e && data[q] != delim) {
          if (data[q] == '"' || data[q] == '\r') return false;
          ++q;
        }
        cells->push_back(Field{data + k, static_cast<int32_t>(q - k)});
        k = q;
      }
      if (k >= e) break;
      ++k;  // delimiter
      if (k == e) {  // trailing delimiter: one more empty field
        cells->push_back(Field{data + k, 0});
        break;
      }
    }
    const size_t nf = cells->size() - row_start;
    if (*ncol == 0) *ncol = nf;
    else if (nf != *ncol) return false;
    i = e + 1;
  }
  return *ncol > 0;
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
  std::vector<std::shared_ptr<arrow::Field>> fields;
  std::vector<std::shared_ptr<arrow::Array>> cols;
  std::vector<Kind> kinds(nrow);
  std::vector<int64_t> ivals(nrow);
  std::vector<double> dvals(nrow);
  for (size_t c = 0; c < ncol; ++c) {
    const Field& h = cells[c];
    for (int32_t j = 0; j < h.n; ++j)
      if (static_cast<unsigned char>(h.p[j]) >= 0x80) return 0;
    bool any_real = false, any_text = false, any_value = false;
    for (size_t r = 0; r < nrow; ++r) {
      // one surely-text value decides the column (Arrow's ladder ends on string whatever the
      // other values are; "" stays the only null): the rest need no classification
      if (any_text) break;
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
      for (size_t r = 0; r < nrow; ++r) {
        if (kinds[r] != kInt) continue;
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
    fields.push_back(arrow::field(std::string(h.p, static_cast<size_t>(h.n)), arr->type()));
    cols.push_back(arr);
  }
  auto table = arrow::Table::Make(arrow::schema(fields), cols, static_cast<int64_t>(nrow));
  auto reader = std::make_shared<arrow::TableBatchReader>(table);
  if (!arrow::ExportRecordBatchReader(reader, static_cast<struct ArrowArrayStream*>(out)).ok()) return -1;
  return 1;
}

}  // extern "C"
