// Native executor core (reference: core/raydp-main/src/main/scala/org/apache/
// spark/executor/RayDPExecutor.scala -- the JVM executor process that runs Spark tasks, caches
// converted RDD blocks (:312-355 getRDDPartition / cacheRDD), reports block locations and asks
// the master to recache a lost block (:289-310)).
//
// The Python actor (raydp_amd/spark/executor.py) owns registration, payload decoding and the
// generic Python task path. This library owns what the reference's executor does natively:
//
//   * the TASK LOOP: a pool of `cores` worker threads fed by a queue. A native task is one
//     partition of a lowered stage -- source -> fused expression-VM segments -> sink -- executed
//     with no Python on the hot path (the caller's ctypes call drops the GIL while it waits, so
//     the executor's cores really run in parallel);
//   * the SOURCE: a byte split of a CSV file parsed by Arrow's C++ reader with the stage's
//     schema (the same split/line-ownership rule as raydp_amd/spark/sources.py CsvSource.load),
//     or a table handed over through the Arrow C stream interface;
//   * the SEGMENTS: register programs of csrc/exec/expr/expr_vm.cc, with string -> timestamp
//     inputs parsed natively and the untouched columns gathered by the surviving row ids;
//   * the PYTHON-UDF BRIDGE: a segment that inlines Python UDFs calls back into Python once,
//     after its VM run, with the exported outputs, so the UDF guards / sampled verification of
//     raydp_amd/spark/exprc.py decide exactly as on the Python path;
//   * the SINK: the result is serialised as an Arrow IPC stream STRAIGHT into an object-store
//     allocation (size measured with a mock stream, written through a fixed-size writer over the
//     mapped bytes, sealed) -- no intermediate copy, no Python objects;
//   * the PARTITION CACHE: (rdd id, partition) -> object id with block listing and unpersist.
//
// Anything a task cannot execute exactly like the Python path (an unexpected column type, a
// timestamp string outside the strict ISO shape, a UDF guard trip) returns FALLBACK and the
// caller runs that partition through Python: results are identical either way.
#include <arrow/api.h>
#include <arrow/array/concatenate.h>
#include <arrow/c/bridge.h>
#include <arrow/csv/api.h>
#include <arrow/io/api.h>
#include <arrow/ipc/api.h>
#include <arrow/util/bitmap_ops.h>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

extern "C" {
int64_t rx_expr_run(const int32_t* code, int32_t ncode, const double* fconst, const int64_t* iconst,
                    const int32_t* live, int32_t nslots, int64_t nrows, const void* const* in_vals,
                    const uint8_t* const* in_valid, const int64_t* in_off, const int32_t* out_slot,
                    const int32_t* out_type, void* const* out_vals, uint8_t* const* out_valid,
                    int64_t* out_nulls, int32_t nout, int32_t* sel_out);
// csrc/runtime/objstore.cc (libraydp_runtime.so)
uint8_t* rt_store_data(void* hs);
int64_t rt_obj_create(void* hs, const char* id, uint64_t size, int32_t kind, int64_t pid);
int rt_obj_seal(void* hs, const char* id);
int rt_obj_abort(void* hs, const char* id);
int rt_obj_delete(void* hs, const char* id);
}

namespace {

enum Status : int { kOk = 0, kFallback = 1, kRetry = 2, kError = -1 };
enum SrcKind : int { kSrcCsv = 1, kSrcStream = 2 };
enum InKind : int { kInCol = 0, kInTs = 1 };
enum ColKind : int { kColVm = 0, kColIn = 1 };
constexpr int kStoreKindArrow = 1;   // raydp_amd/runtime/store.py KIND_ARROW
constexpr int kVmBool = 0;           // expr_vm.cc T_BOOL

// UDF bridge: (user, segment, rows, out values, out validity, out null counts) -> Status
typedef int (*TapFn)(void*, int32_t, int64_t, void* const*, uint8_t* const*, const int64_t*);

// ------------------------------------------------------------------ stage description ------
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  template <typename T> T get() {
    T v{};
    if (end - p < static_cast<ptrdiff_t>(sizeof(T))) { ok = false; return v; }
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint32_t n = get<uint32_t>();
    if (!ok || end - p < static_cast<ptrdiff_t>(n)) { ok = false; return {}; }
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  template <typename T> std::vector<T> vec() {
    uint32_t n = get<uint32_t>();
    std::vector<T> v;
    if (!ok || (end - p) / static_cast<ptrdiff_t>(sizeof(T)) < static_cast<ptrdiff_t>(n)) { ok = false; return v; }
    v.resize(n);
    if (n) std::memcpy(v.data(), p, sizeof(T) * n);
    p += sizeof(T) * n;
    return v;
  }
};

std::shared_ptr<arrow::DataType> type_of(const std::string& s) {
  static const std::unordered_map<std::string, std::shared_ptr<arrow::DataType>> m = {
      {"bool", arrow::boolean()},       {"int8", arrow::int8()},
      {"int16", arrow::int16()},        {"int32", arrow::int32()},
      {"int64", arrow::int64()},        {"uint8", arrow::uint8()},
      {"uint16", arrow::uint16()},      {"uint32", arrow::uint32()},
      {"uint64", arrow::uint64()},      {"float", arrow::float32()},
      {"double", arrow::float64()},     {"string", arrow::utf8()},
      {"large_string", arrow::large_utf8()}, {"binary", arrow::binary()},
      {"large_binary", arrow::large_binary()}, {"date32[day]", arrow::date32()},
      {"timestamp[s]", arrow::timestamp(arrow::TimeUnit::SECOND)},
      {"timestamp[ms]", arrow::timestamp(arrow::TimeUnit::MILLI)},
      {"timestamp[us]", arrow::timestamp(arrow::TimeUnit::MICRO)},
      {"timestamp[ns]", arrow::timestamp(arrow::TimeUnit::NANO)},
      {"null", arrow::null()},
  };
  auto it = m.find(s);
  return it == m.end() ? nullptr : it->second;
}

struct InputSpec { int kind; int col; std::shared_ptr<arrow::DataType> type; };
struct ColSpec { std::string name; int kind; int idx; };

struct Segment {
  std::vector<int32_t> code;   // ncode x 8
  std::vector<double> fconst;
  std::vector<int64_t> iconst;
  std::vector<int32_t> live;
  int32_t nslots = 1;
  std::vector<InputSpec> inputs;
  std::vector<int32_t> out_ct;
  std::vector<std::shared_ptr<arrow::DataType>> out_types;
  std::vector<int32_t> out_slots;
  bool has_filter = false;
  bool taps = false;
  std::vector<ColSpec> cols;
};

struct Stage {
  std::shared_ptr<arrow::Schema> src_schema;   // CSV column names + types
  std::vector<bool> src_needed;                // source columns the first segment reads or passes
  bool header = true;
  char delim = ',';
  std::string null_token;
  std::vector<Segment> segs;
};

// Spec layout (little endian; raydp_amd/spark/native_exec.py _StageSpec writes it):
//   u32 'RXS1' | u8 header | u8 delim | str null | u32 nfields {str name, str type}
//   u32 nseg { vec<i32> code | vec<f64> fconst | vec<i64> iconst | vec<i32> live | i32 nslots
//              u32 nin {u8 kind, i32 col, str type} | u32 nout {i32 ct, str type, i32 slot}
//              u8 has_filter | u8 taps | u32 ncol {str name, u8 kind, i32 idx} }
Stage* parse_stage(const uint8_t* data, int64_t len, std::string* err) {
  Reader r{data, data + len};
  if (r.get<uint32_t>() != 0x31535852u) { *err = "bad stage magic"; return nullptr; }
  auto st = std::make_unique<Stage>();
  st->header = r.get<uint8_t>() != 0;
  st->delim = static_cast<char>(r.get<uint8_t>());
  st->null_token = r.str();
  uint32_t nf = r.get<uint32_t>();
  std::vector<std::shared_ptr<arrow::Field>> fields;
  for (uint32_t i = 0; i < nf && r.ok; ++i) {
    std::string name = r.str(), ty = r.str();
    auto t = type_of(ty);
    if (!t) { *err = "unsupported source type " + ty; return nullptr; }
    fields.push_back(arrow::field(name, t));
  }
  st->src_schema = arrow::schema(fields);
  uint32_t ns = r.get<uint32_t>();
  for (uint32_t s = 0; s < ns && r.ok; ++s) {
    Segment g;
    g.code = r.vec<int32_t>();
    g.fconst = r.vec<double>();
    g.iconst = r.vec<int64_t>();
    g.live = r.vec<int32_t>();
    g.nslots = r.get<int32_t>();
    uint32_t nin = r.get<uint32_t>();
    for (uint32_t i = 0; i < nin && r.ok; ++i) {
      InputSpec in;
      in.kind = r.get<uint8_t>();
      in.col = r.get<int32_t>();
      std::string ty = r.str();
      in.type = type_of(ty);
      if (!in.type) { *err = "unsupported input type " + ty; return nullptr; }
      g.inputs.push_back(in);
    }
    uint32_t nout = r.get<uint32_t>();
    for (uint32_t i = 0; i < nout && r.ok; ++i) {
      g.out_ct.push_back(r.get<int32_t>());
      std::string ty = r.str();
      auto t = type_of(ty);
      if (!t) { *err = "unsupported output type " + ty; return nullptr; }
      g.out_types.push_back(t);
      g.out_slots.push_back(r.get<int32_t>());
    }
    g.has_filter = r.get<uint8_t>() != 0;
    g.taps = r.get<uint8_t>() != 0;
    uint32_t nc = r.get<uint32_t>();
    for (uint32_t i = 0; i < nc && r.ok; ++i) {
      ColSpec c;
      c.name = r.str();
      c.kind = r.get<uint8_t>();
      c.idx = r.get<int32_t>();
      g.cols.push_back(c);
    }
    if (g.code.size() % 8 != 0) { *err = "ragged program"; return nullptr; }
    st->segs.push_back(std::move(g));
  }
  if (!r.ok || r.p != r.end) { *err = "truncated or oversized stage spec"; return nullptr; }
  // projection: a CSV column no VM input reads and no output passes through (the NYC chain's
  // "key", dropped unread) is not converted at all
  const int nsrc = st->src_schema->num_fields();
  st->src_needed.assign(static_cast<size_t>(nsrc), st->segs.empty());
  if (!st->segs.empty()) {
    for (const auto& in : st->segs[0].inputs)
      if (in.col >= 0 && in.col < nsrc) st->src_needed[static_cast<size_t>(in.col)] = true;
    for (const auto& c : st->segs[0].cols)
      if (c.kind != 0 && c.idx >= 0 && c.idx < nsrc) st->src_needed[static_cast<size_t>(c.idx)] = true;
  }
  return st.release();
}

// ------------------------------------------------------------------ source ----------------
// The byte range [lo, hi) of a CSV file, extended to whole lines: a split owns every line
// that STARTS inside it (the line straddling `lo` belongs to the previous split).
arrow::Result<std::shared_ptr<arrow::Table>> read_csv_split(const Stage& st, const std::string& path,
                                                           int64_t lo, int64_t hi) {
  // Only this split's bytes are read (plus the line straddling `hi`, and the header line when
  // the split starts the file): a 1 GB file cut into 16 splits costs 16 x 1/16 of it, not 16 x
  // the whole file.
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return arrow::Status::IOError("cannot open ", path);
  struct stat sb;
  if (fstat(fd, &sb) != 0) { ::close(fd); return arrow::Status::IOError("cannot stat ", path); }
  const int64_t size = sb.st_size;
  // position just past the '\n' ending the line that contains byte `pos` (size at EOF)
  auto line_end = [&](int64_t pos) -> int64_t {
    char chunk[4096];
    while (pos < size) {
      const ssize_t k = ::pread(fd, chunk, sizeof(chunk), pos);
      if (k <= 0) return size;
      const void* nl = memchr(chunk, '\n', static_cast<size_t>(k));
      if (nl != nullptr) return pos + (static_cast<const char*>(nl) - chunk) + 1;
      pos += k;
    }
    return size;
  };
  auto byte_at = [&](int64_t pos) -> char {
    char c = 0;
    return ::pread(fd, &c, 1, pos) == 1 ? c : '\n';
  };
  const int64_t header_len = st.header ? line_end(0) : 0;
  int64_t pos = header_len;
  if (lo > 0) {
    pos = lo;
    if (byte_at(lo - 1) != '\n') pos = line_end(lo);
  }
  const int64_t start = std::max(pos, header_len);
  if (start >= hi && lo > 0) { ::close(fd); return arrow::Table::MakeEmpty(st.src_schema); }
  int64_t stop = std::min<int64_t>(std::max<int64_t>(hi, start), size);
  if (stop > start && byte_at(stop - 1) != '\n') stop = line_end(stop);
  const int64_t n = stop - start;
  ARROW_ASSIGN_OR_RAISE(std::shared_ptr<arrow::ResizableBuffer> bufr, arrow::AllocateResizableBuffer(std::max<int64_t>(n, 1)));
  char* all_p = reinterpret_cast<char*>(bufr->mutable_data());
  int64_t got = 0;
  while (got < n) {
    const ssize_t k = ::pread(fd, all_p + got, static_cast<size_t>(n - got), start + got);
    if (k <= 0) break;
    got += k;
  }
  ::close(fd);
  if (got != n) return arrow::Status::IOError("short read of ", path);
  ARROW_RETURN_NOT_OK(bufr->Resize(n, false));
  bool blank = true;
  for (int64_t i = 0; i < n && blank; ++i) {
    const char c = all_p[i];
    blank = c == ' ' || c == '\n' || c == '\r' || c == '\t' || c == '\v' || c == '\f';
  }
  if (blank) return arrow::Table::MakeEmpty(st.src_schema);
  std::shared_ptr<arrow::Buffer> buf = std::move(bufr);
  auto ro = arrow::csv::ReadOptions::Defaults();
  ro.use_threads = n > (4 << 20);
  ro.block_size = static_cast<int32_t>(std::max<int64_t>(1 << 20, std::min<int64_t>(n + 1, INT32_MAX)));
  for (const auto& f : st.src_schema->fields()) ro.column_names.push_back(f->name());
  auto po = arrow::csv::ParseOptions::Defaults();
  po.delimiter = st.delim;
  auto co = arrow::csv::ConvertOptions::Defaults();
  for (const auto& f : st.src_schema->fields()) co.column_types[f->name()] = f->type();
  co.strings_can_be_null = true;
  co.null_values = {st.null_token};
  bool all_needed = true;
  for (size_t i = 0; i < st.src_needed.size(); ++i) all_needed = all_needed && st.src_needed[i];
  if (!all_needed) {   // include_columns selects by name: only with unique column names
    std::unordered_set<std::string> names;
    for (const auto& f : st.src_schema->fields()) all_needed = all_needed || !names.insert(f->name()).second;
  }
  if (!all_needed) {
    for (size_t i = 0; i < st.src_needed.size(); ++i)
      if (st.src_needed[i]) co.include_columns.push_back(st.src_schema->field(static_cast<int>(i))->name());
  }
  auto in = std::make_shared<arrow::io::BufferReader>(buf);
  ARROW_ASSIGN_OR_RAISE(auto rd, arrow::csv::TableReader::Make(arrow::io::default_io_context(), in, ro, po, co));
  ARROW_ASSIGN_OR_RAISE(auto t, rd->Read());
  if (all_needed) return t;
  // back to the source layout (column indices of the stage program): skipped columns all-null
  std::vector<std::shared_ptr<arrow::ChunkedArray>> cols;
  int k = 0;
  for (int i = 0; i < st.src_schema->num_fields(); ++i) {
    if (st.src_needed[static_cast<size_t>(i)]) {
      cols.push_back(t->column(k++));
    } else {
      ARROW_ASSIGN_OR_RAISE(auto nul, arrow::MakeArrayOfNull(st.src_schema->field(i)->type(), t->num_rows()));
      cols.push_back(std::make_shared<arrow::ChunkedArray>(nul));
    }
  }
  return arrow::Table::Make(st.src_schema, cols, t->num_rows());
}

// ------------------------------------------------------------------ inputs ----------------
inline bool digits(const char* s, int n, int* out) {
  int v = 0;
  for (int i = 0; i < n; ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = v;
  return true;
}

inline int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = static_cast<unsigned>(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + static_cast<int64_t>(doe) - 719468;
}

// "YYYY-MM-DD HH:MM:SS" (or 'T'), optionally followed by " UTC": the shape the Python path
// parses with Arrow's ISO-8601 cast (raydp_amd/spark/column.py _parse_ts fast path). Any other
// value -> false (the partition falls back to Python, which tries its other formats).
bool parse_ts(const char* s, int64_t n, int64_t* out) {
  if (!(n == 19 || (n == 23 && std::memcmp(s + 19, " UTC", 4) == 0))) return false;
  int Y, M, D, h, mi, se;
  if (!digits(s, 4, &Y) || s[4] != '-' || !digits(s + 5, 2, &M) || s[7] != '-' || !digits(s + 8, 2, &D) ||
      (s[10] != ' ' && s[10] != 'T') || !digits(s + 11, 2, &h) || s[13] != ':' || !digits(s + 14, 2, &mi) ||
      s[16] != ':' || !digits(s + 17, 2, &se))
    return false;
  if (Y < 1 || M < 1 || M > 12 || D < 1 || h > 23 || mi > 59 || se > 59) return false;
  static const int mdays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  const bool leap = (Y % 4 == 0 && Y % 100 != 0) || Y % 400 == 0;
  if (D > mdays[M - 1] + (M == 2 && leap ? 1 : 0)) return false;
  *out = days_from_civil(Y, static_cast<unsigned>(M), static_cast<unsigned>(D)) * 86400 + h * 3600 + mi * 60 + se;
  return true;
}

template <typename Offset>
arrow::Result<std::shared_ptr<arrow::Array>> parse_ts_column(const arrow::ArrayData& a, bool* fallback) {
  const int64_t n = a.length;
  const uint8_t* valid = a.buffers[0] ? a.buffers[0]->data() : nullptr;
  const Offset* off = a.GetValues<Offset>(1);
  const char* chars = a.buffers[2] ? reinterpret_cast<const char*>(a.buffers[2]->data()) : "";
  ARROW_ASSIGN_OR_RAISE(auto vals, arrow::AllocateBuffer(n * 8 + 8));
  int64_t* o = reinterpret_cast<int64_t*>(vals->mutable_data());
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = a.offset + i;
    if (valid && !((valid[j >> 3] >> (j & 7)) & 1)) { o[i] = 0; continue; }
    if (!parse_ts(chars + off[i], static_cast<int64_t>(off[i + 1] - off[i]), &o[i])) {
      *fallback = true;
      return nullptr;
    }
  }
  std::shared_ptr<arrow::Buffer> vb;
  if (a.GetNullCount() > 0) {
    ARROW_ASSIGN_OR_RAISE(vb, arrow::AllocateBitmap(n));
    arrow::internal::CopyBitmap(valid, a.offset, n, vb->mutable_data(), 0);
  }
  return arrow::MakeArray(arrow::ArrayData::Make(arrow::timestamp(arrow::TimeUnit::SECOND), n,
                                                 {vb, std::shared_ptr<arrow::Buffer>(std::move(vals))},
                                                 a.GetNullCount()));
}

// ------------------------------------------------------------------ gather ----------------
// rows `sel[0..m)` of `a` (the untouched columns of a filtering segment), for the layouts
// Arrow's take would handle here; nullptr = unsupported layout (fallback).
arrow::Result<std::shared_ptr<arrow::Array>> gather(const std::shared_ptr<arrow::Array>& arr,
                                                    const int32_t* sel, int64_t m) {
  const arrow::ArrayData& a = *arr->data();
  const auto id = a.type->id();
  const uint8_t* valid = (a.buffers.size() > 0 && a.buffers[0]) ? a.buffers[0]->data() : nullptr;
  std::shared_ptr<arrow::Buffer> vb;
  int64_t nulls = 0;
  if (id == arrow::Type::NA) return arrow::MakeArrayOfNull(a.type, m);
  if (valid && a.GetNullCount() > 0) {
    ARROW_ASSIGN_OR_RAISE(vb, arrow::AllocateBitmap(m));
    uint8_t* o = vb->mutable_data();
    std::memset(o, 0, static_cast<size_t>((m + 7) / 8));
    for (int64_t i = 0; i < m; ++i) {
      const int64_t j = a.offset + sel[i];
      if ((valid[j >> 3] >> (j & 7)) & 1) o[i >> 3] |= static_cast<uint8_t>(1u << (i & 7));
      else ++nulls;
    }
    if (nulls == 0) vb.reset();
  }
  if (id == arrow::Type::BOOL) {
    ARROW_ASSIGN_OR_RAISE(auto b, arrow::AllocateBitmap(m));
    uint8_t* o = b->mutable_data();
    std::memset(o, 0, static_cast<size_t>((m + 7) / 8));
    const uint8_t* v = a.buffers[1]->data();
    for (int64_t i = 0; i < m; ++i) {
      const int64_t j = a.offset + sel[i];
      if ((v[j >> 3] >> (j & 7)) & 1) o[i >> 3] |= static_cast<uint8_t>(1u << (i & 7));
    }
    return arrow::MakeArray(arrow::ArrayData::Make(a.type, m, {vb, std::shared_ptr<arrow::Buffer>(std::move(b))}, nulls));
  }
  if (arrow::is_fixed_width(id) && id != arrow::Type::DICTIONARY && id != arrow::Type::FIXED_SIZE_LIST &&
      id != arrow::Type::EXTENSION) {
    const int w = a.type->byte_width();
    if (w <= 0) return nullptr;
    ARROW_ASSIGN_OR_RAISE(auto b, arrow::AllocateBuffer(m * w + 8));
    const uint8_t* v = a.buffers[1]->data() + a.offset * w;
    uint8_t* o = b->mutable_data();
    for (int64_t i = 0; i < m; ++i) std::memcpy(o + i * w, v + static_cast<int64_t>(sel[i]) * w, w);
    return arrow::MakeArray(arrow::ArrayData::Make(a.type, m, {vb, std::shared_ptr<arrow::Buffer>(std::move(b))}, nulls));
  }
  auto var = [&](auto tag) -> arrow::Result<std::shared_ptr<arrow::Array>> {
    using Off = decltype(tag);
    const Off* off = a.GetValues<Off>(1);
    const uint8_t* chars = a.buffers[2] ? a.buffers[2]->data() : nullptr;
    int64_t total = 0;
    for (int64_t i = 0; i < m; ++i) total += static_cast<int64_t>(off[sel[i] + 1] - off[sel[i]]);
    if (sizeof(Off) == 4 && total > INT32_MAX) return nullptr;
    ARROW_ASSIGN_OR_RAISE(auto ob, arrow::AllocateBuffer((m + 1) * static_cast<int64_t>(sizeof(Off))));
    ARROW_ASSIGN_OR_RAISE(auto cb, arrow::AllocateBuffer(total + 8));
    Off* oo = reinterpret_cast<Off*>(ob->mutable_data());
    uint8_t* oc = cb->mutable_data();
    Off pos = 0;
    for (int64_t i = 0; i < m; ++i) {
      oo[i] = pos;
      const Off s = off[sel[i]], e = off[sel[i] + 1];
      if (e > s) std::memcpy(oc + pos, chars + s, static_cast<size_t>(e - s));
      pos += e - s;
    }
    oo[m] = pos;
    return arrow::MakeArray(arrow::ArrayData::Make(
        a.type, m, {vb, std::shared_ptr<arrow::Buffer>(std::move(ob)), std::shared_ptr<arrow::Buffer>(std::move(cb))},
        nulls));
  };
  if (id == arrow::Type::STRING || id == arrow::Type::BINARY) return var(int32_t{});
  if (id == arrow::Type::LARGE_STRING || id == arrow::Type::LARGE_BINARY) return var(int64_t{});
  return nullptr;
}

// One contiguous array of a column (what the VM and the gather read).
arrow::Result<std::shared_ptr<arrow::Array>> whole(const std::shared_ptr<arrow::ChunkedArray>& c) {
  if (c->num_chunks() == 1) return c->chunk(0);
  if (c->num_chunks() == 0) return arrow::MakeEmptyArray(c->type());
  return arrow::Concatenate(c->chunks());
}

// ------------------------------------------------------------------ one segment -----------
struct TaskCtx {
  TapFn tap = nullptr;
  void* user = nullptr;
};

arrow::Result<std::shared_ptr<arrow::Table>> run_segment(const Segment& g, int seg_index,
                                                        const std::shared_ptr<arrow::Table>& t,
                                                        const TaskCtx& ctx, int* status) {
  const int64_t n = t->num_rows();
  std::vector<std::shared_ptr<arrow::Array>> ins;
  for (const auto& in : g.inputs) {
    if (in.col < 0 || in.col >= t->num_columns()) { *status = kError; return nullptr; }
    ARROW_ASSIGN_OR_RAISE(auto a, whole(t->column(in.col)));
    if (in.kind == kInTs) {
      const auto id = a->type_id();
      bool fb = false;
      if (id == arrow::Type::STRING) {
        ARROW_ASSIGN_OR_RAISE(a, parse_ts_column<int32_t>(*a->data(), &fb));
      } else if (id == arrow::Type::LARGE_STRING) {
        ARROW_ASSIGN_OR_RAISE(a, parse_ts_column<int64_t>(*a->data(), &fb));
      } else if (!a->type()->Equals(*arrow::timestamp(arrow::TimeUnit::SECOND))) {
        fb = true;    // dates / other units / zones: Arrow's casts on the Python path
      }
      if (fb) { *status = kFallback; return nullptr; }
    }
    if (!a->type()->Equals(*in.type)) { *status = kFallback; return nullptr; }
    ins.push_back(a);
  }
  const size_t nin = std::max<size_t>(1, ins.size());
  std::vector<const void*> in_vals(nin, nullptr);
  std::vector<const uint8_t*> in_valid(nin, nullptr);
  std::vector<int64_t> in_off(nin, 0);
  for (size_t j = 0; j < ins.size(); ++j) {
    const auto& d = *ins[j]->data();
    in_valid[j] = (d.buffers[0] && d.GetNullCount() > 0) ? d.buffers[0]->data() : nullptr;
    in_vals[j] = d.buffers.size() > 1 && d.buffers[1] ? d.buffers[1]->data() : nullptr;
    in_off[j] = d.offset;
  }
  const int32_t nout = static_cast<int32_t>(g.out_ct.size());
  const int64_t nbits = (n + 7) / 8;
  std::vector<std::shared_ptr<arrow::Buffer>> vals, valids;
  std::vector<void*> o_vals(std::max(1, nout), nullptr);
  std::vector<uint8_t*> o_valid(std::max(1, nout), nullptr);
  for (int32_t j = 0; j < nout; ++j) {
    const int ct = g.out_ct[j];
    const int64_t bytes = ct == kVmBool ? nbits + 1 : n * ((ct == 1 || ct == 3) ? 4 : 8) + 8;
    ARROW_ASSIGN_OR_RAISE(auto vb, arrow::AllocateBuffer(bytes));
    ARROW_ASSIGN_OR_RAISE(auto mb, arrow::AllocateBuffer(nbits + 1));
    o_vals[j] = vb->mutable_data();
    o_valid[j] = mb->mutable_data();
    vals.push_back(std::shared_ptr<arrow::Buffer>(std::move(vb)));
    valids.push_back(std::shared_ptr<arrow::Buffer>(std::move(mb)));
  }
  std::vector<int64_t> nulls(std::max(1, nout), 0);
  std::vector<int32_t> sel;
  if (g.has_filter) sel.resize(static_cast<size_t>(std::max<int64_t>(1, n)));
  const int64_t m = rx_expr_run(g.code.data(), static_cast<int32_t>(g.code.size() / 8), g.fconst.data(),
                                g.iconst.data(), g.live.data(), g.nslots, n, in_vals.data(), in_valid.data(),
                                in_off.data(), g.out_slots.data(), g.out_ct.data(), o_vals.data(), o_valid.data(),
                                nulls.data(), nout, g.has_filter ? sel.data() : nullptr);
  if (m < 0) { *status = kError; return arrow::Status::Invalid("expression VM rejected the program"); }
  if (g.taps) {
    if (ctx.tap == nullptr) { *status = kFallback; return nullptr; }
    const int rc = ctx.tap(ctx.user, seg_index, m, o_vals.data(), o_valid.data(), nulls.data());
    if (rc != kOk) { *status = rc; return nullptr; }
  }
  std::vector<std::shared_ptr<arrow::Field>> fields;
  std::vector<std::shared_ptr<arrow::Array>> cols;
  std::unordered_map<int, std::shared_ptr<arrow::Array>> passed;
  for (const auto& c : g.cols) {
    std::shared_ptr<arrow::Array> col;
    if (c.kind == kColVm) {
      if (c.idx < 0 || c.idx >= nout) { *status = kError; return nullptr; }
      std::shared_ptr<arrow::Buffer> vb = nulls[c.idx] ? valids[c.idx] : nullptr;
      col = arrow::MakeArray(arrow::ArrayData::Make(g.out_types[c.idx], m, {vb, vals[c.idx]}, nulls[c.idx]));
    } else {
      if (c.idx < 0 || c.idx >= t->num_columns()) { *status = kError; return nullptr; }
      auto hit = passed.find(c.idx);
      if (hit != passed.end()) {
        col = hit->second;
      } else {
        ARROW_ASSIGN_OR_RAISE(auto src, whole(t->column(c.idx)));
        if (g.has_filter) {
          ARROW_ASSIGN_OR_RAISE(col, gather(src, sel.data(), m));
          if (!col) { *status = kFallback; return nullptr; }
        } else {
          col = src;
        }
        passed[c.idx] = col;
      }
    }
    fields.push_back(arrow::field(c.name, col->type()));
    cols.push_back(col);
  }
  return arrow::Table::Make(arrow::schema(fields), cols, m);
}

// ------------------------------------------------------------------ sink ------------------
arrow::Status write_ipc(const std::shared_ptr<arrow::Table>& t, void* store, const char* oid, int64_t* nbytes) {
  auto mock = std::make_shared<arrow::io::MockOutputStream>();
  {
    ARROW_ASSIGN_OR_RAISE(auto w, arrow::ipc::MakeStreamWriter(mock, t->schema()));
    ARROW_RETURN_NOT_OK(w->WriteTable(*t));
    ARROW_RETURN_NOT_OK(w->Close());
  }
  const int64_t size = mock->GetExtentBytesWritten();
  const int64_t off = rt_obj_create(store, oid, static_cast<uint64_t>(size), kStoreKindArrow, getpid());
  if (off == -2) return arrow::Status::AlreadyExists("object ", oid, " already exists");
  if (off < 0) return arrow::Status::OutOfMemory("object store full (", size, " bytes requested)");
  auto region = std::make_shared<arrow::MutableBuffer>(rt_store_data(store) + off, size);
  arrow::Status st;
  {
    auto sink = std::make_shared<arrow::io::FixedSizeBufferWriter>(region);
    auto w = arrow::ipc::MakeStreamWriter(sink, t->schema());
    st = w.status();
    if (st.ok()) st = (*w)->WriteTable(*t);
    if (st.ok()) st = (*w)->Close();
  }
  if (!st.ok()) {
    rt_obj_abort(store, oid);
    return st;
  }
  rt_obj_seal(store, oid);
  *nbytes = size;
  return arrow::Status::OK();
}

// ------------------------------------------------------------------ task loop -------------
struct Task {
  const Stage* stage = nullptr;
  int src_kind = 0;
  std::string path;
  int64_t lo = 0, hi = 0;
  std::shared_ptr<arrow::Table> table;    // kSrcStream, imported by the submitter
  void* store = nullptr;
  std::string oid;
  TaskCtx ctx;
  // results
  int64_t t0_ns = 0, t1_ns = 0;   // wall clock (CLOCK_REALTIME, as Python's time.time_ns)
  int worker = 0;
  bool done = false;
  int status = kOk;
  int64_t rows = 0, bytes = 0;
  std::string err;
};

struct Executor {
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<Task*> queue;
  std::unordered_map<int64_t, std::unique_ptr<Task>> tasks;
  int64_t next_id = 1;
  bool stopping = false;
  std::vector<std::thread> workers;
  // partition cache: (rdd id, partition) -> object id
  std::mutex cmu;
  std::map<std::pair<std::string, int32_t>, std::string> cache;
  std::atomic<int64_t> n_ok{0}, n_fallback{0}, n_error{0}, rows_out{0}, bytes_out{0};

  explicit Executor(int threads) {
    for (int i = 0; i < std::max(1, threads); ++i) workers.emplace_back([this, i] { loop(i); });
  }
  ~Executor() {
    {
      std::lock_guard<std::mutex> g(mu);
      stopping = true;
    }
    cv_work.notify_all();
    for (auto& w : workers) w.join();
  }
  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::system_clock::now().time_since_epoch()).count();
  }
  void loop(int wid) {
    for (;;) {
      Task* t = nullptr;
      {
        std::unique_lock<std::mutex> g(mu);
        cv_work.wait(g, [this] { return stopping || !queue.empty(); });
        if (queue.empty()) return;
        t = queue.front();
        queue.pop_front();
      }
      t->worker = wid;
      t->t0_ns = now_ns();
      run(t);
      t->t1_ns = now_ns();
      {
        std::lock_guard<std::mutex> g(mu);
        t->done = true;
      }
      cv_done.notify_all();
    }
  }
  void run(Task* t) {
    auto r = execute(t);
    if (!r.ok()) {
      if (t->status == kOk) t->status = kError;
      t->err = r.ToString();
    }
    if (t->status == kOk) {
      n_ok++;
      rows_out += t->rows;
      bytes_out += t->bytes;
    } else if (t->status == kError) {
      n_error++;
    } else {
      n_fallback++;
    }
  }
  arrow::Status execute(Task* t) {
    const Stage& st = *t->stage;
    std::shared_ptr<arrow::Table> cur;
    if (t->src_kind == kSrcCsv) {
      ARROW_ASSIGN_OR_RAISE(cur, read_csv_split(st, t->path, t->lo, t->hi));
    } else {
      cur = t->table;
    }
    for (size_t k = 0; k < st.segs.size(); ++k) {
      int status = kOk;
      auto next = run_segment(st.segs[k], static_cast<int>(k), cur, t->ctx, &status);
      if (!next.ok()) {
        t->status = kError;
        return next.status();
      }
      if (status != kOk) {
        t->status = status;
        return arrow::Status::OK();
      }
      cur = *next;
    }
    t->rows = cur->num_rows();
    return write_ipc(cur, t->store, t->oid.c_str(), &t->bytes);
  }
};

void put_err(const std::string& e, char* err, int errlen) {
  if (err && errlen > 0) {
    std::strncpy(err, e.c_str(), static_cast<size_t>(errlen - 1));
    err[errlen - 1] = '\0';
  }
}

}  // namespace

extern "C" {

void* rx_exec_create(int threads) { return new Executor(threads); }

void rx_exec_destroy(void* ex) { delete static_cast<Executor*>(ex); }

void* rx_stage_create(const uint8_t* spec, int64_t len, char* err, int errlen) {
  std::string e;
  Stage* st = parse_stage(spec, len, &e);
  if (!st) put_err(e, err, errlen);
  return st;
}

void rx_stage_destroy(void* st) { delete static_cast<Stage*>(st); }

// Queue one partition of `stage`. Source: `path` [lo, hi) of a CSV file, or (`stream` != null)
// an ArrowArrayStream, consumed here on the caller's thread. Returns the task id (> 0), or -1
// when the stream could not be imported (`err` says why).
int64_t rx_exec_submit(void* exp, void* stage, const char* path, int64_t lo, int64_t hi, void* stream, void* store,
                       const char* oid, TapFn tap, void* user, char* err, int errlen) {
  auto* ex = static_cast<Executor*>(exp);
  auto t = std::make_unique<Task>();
  t->stage = static_cast<const Stage*>(stage);
  t->store = store;
  t->oid = oid;
  t->ctx.tap = tap;
  t->ctx.user = user;
  if (stream != nullptr) {
    t->src_kind = kSrcStream;
    auto rd = arrow::ImportRecordBatchReader(static_cast<struct ArrowArrayStream*>(stream));
    if (!rd.ok()) { put_err(rd.status().ToString(), err, errlen); return -1; }
    auto tab = (*rd)->ToTable();
    if (!tab.ok()) { put_err(tab.status().ToString(), err, errlen); return -1; }
    t->table = *tab;
  } else {
    t->src_kind = kSrcCsv;
    t->path = path ? path : "";
    t->lo = lo;
    t->hi = hi;
  }
  int64_t id;
  {
    std::lock_guard<std::mutex> g(ex->mu);
    id = ex->next_id++;
    ex->queue.push_back(t.get());
    ex->tasks[id] = std::move(t);
  }
  ex->cv_work.notify_one();
  return id;
}

// Block until task `id` finished; returns its status (0 ok, 1 fallback, 2 retry, -1 error).
// `times` (nullable) receives {start ns, end ns, worker index}.
int rx_exec_wait(void* exp, int64_t id, int64_t* rows, int64_t* bytes, int64_t* times, char* err, int errlen) {
  auto* ex = static_cast<Executor*>(exp);
  std::unique_ptr<Task> t;
  {
    std::unique_lock<std::mutex> g(ex->mu);
    auto it = ex->tasks.find(id);
    if (it == ex->tasks.end()) { put_err("unknown task", err, errlen); return kError; }
    Task* p = it->second.get();
    // a task no pool thread has picked up yet runs here, on the waiting thread: a one-partition
    // stage (every small refit) then skips the hand-off to a pool thread and back (two wake-ups,
    // 0.05-0.07 ms each on the box, profiles/r4_headline_timeline.txt "native tasks" vs "task")
    auto qi = std::find(ex->queue.begin(), ex->queue.end(), p);
    if (qi != ex->queue.end()) {
      ex->queue.erase(qi);
      g.unlock();
      p->worker = -1;
      p->t0_ns = Executor::now_ns();
      ex->run(p);
      p->t1_ns = Executor::now_ns();
      g.lock();
      p->done = true;
    }
    ex->cv_done.wait(g, [p] { return p->done; });
    // `mu` was released above (inline run, cv wait): a concurrent rx_exec_submit may have
    // inserted into `tasks` and rehashed it, so the iterator from before is stale -- look the
    // task up again by its id.
    auto it2 = ex->tasks.find(id);
    t = std::move(it2->second);
    ex->tasks.erase(it2);
  }
  *rows = t->rows;
  *bytes = t->bytes;
  if (times != nullptr) {
    times[0] = t->t0_ns;
    times[1] = t->t1_ns;
    times[2] = t->worker;
  }
  if (!t->err.empty()) put_err(t->err, err, errlen);
  return t->status;
}

// stats: [ok tasks, fallback tasks, failed tasks, rows written, bytes written]
void rx_exec_stats(void* exp, int64_t* out) {
  auto* ex = static_cast<Executor*>(exp);
  out[0] = ex->n_ok;
  out[1] = ex->n_fallback;
  out[2] = ex->n_error;
  out[3] = ex->rows_out;
  out[4] = ex->bytes_out;
}

// ---- partition cache (ids are at most 32 chars; `old` receives a replaced id or "") ----------
void rx_cache_put(void* exp, const char* rdd, int32_t idx, const char* oid, char* old) {
  auto* ex = static_cast<Executor*>(exp);
  std::lock_guard<std::mutex> g(ex->cmu);
  auto& slot = ex->cache[{rdd, idx}];
  std::strncpy(old, slot.c_str(), 33);
  old[32] = '\0';
  slot = oid;
}

int rx_cache_get(void* exp, const char* rdd, int32_t idx, char* oid) {
  auto* ex = static_cast<Executor*>(exp);
  std::lock_guard<std::mutex> g(ex->cmu);
  auto it = ex->cache.find({rdd, idx});
  if (it == ex->cache.end()) return 0;
  std::strncpy(oid, it->second.c_str(), 33);
  oid[32] = '\0';
  return 1;
}

// Remove (rdd, idx) and return its id in `oid` (1) or 0 when absent.
int rx_cache_pop(void* exp, const char* rdd, int32_t idx, char* oid) {
  auto* ex = static_cast<Executor*>(exp);
  std::lock_guard<std::mutex> g(ex->cmu);
  auto it = ex->cache.find({rdd, idx});
  if (it == ex->cache.end()) return 0;
  std::strncpy(oid, it->second.c_str(), 33);
  oid[32] = '\0';
  ex->cache.erase(it);
  return 1;
}

// Partitions of `rdd` cached here (up to `max`, ascending); returns how many exist.
int rx_cache_list(void* exp, const char* rdd, int32_t* out, int max) {
  auto* ex = static_cast<Executor*>(exp);
  std::lock_guard<std::mutex> g(ex->cmu);
  int n = 0;
  for (auto it = ex->cache.lower_bound({rdd, INT32_MIN}); it != ex->cache.end() && it->first.first == rdd; ++it) {
    if (n < max) out[n] = it->first.second;
    ++n;
  }
  return n;
}

// Drop every block of `rdd` (`rdd` == nullptr: of every RDD), deleting the objects from
// `store`; returns the number of blocks dropped.
int rx_cache_unpersist(void* exp, const char* rdd, void* store) {
  auto* ex = static_cast<Executor*>(exp);
  std::vector<std::string> oids;
  {
    std::lock_guard<std::mutex> g(ex->cmu);
    for (auto it = ex->cache.begin(); it != ex->cache.end();) {
      if (rdd == nullptr || it->first.first == rdd) {
        oids.push_back(it->second);
        it = ex->cache.erase(it);
      } else {
        ++it;
      }
    }
  }
  if (store != nullptr)
    for (const auto& o : oids) rt_obj_delete(store, o.c_str());
  return static_cast<int>(oids.size());
}

// Distinct RDD ids with cached blocks, '\n'-separated into `out` (NUL-terminated); returns
// the bytes needed.
int rx_cache_rdds(void* exp, char* out, int cap) {
  auto* ex = static_cast<Executor*>(exp);
  std::string s;
  {
    std::lock_guard<std::mutex> g(ex->cmu);
    std::string last;
    for (const auto& kv : ex->cache) {
      if (kv.first.first != last) {
        s += kv.first.first;
        s += '\n';
        last = kv.first.first;
      }
    }
  }
  put_err(s, out, cap);
  return static_cast<int>(s.size()) + 1;
}

}  // extern "C"
