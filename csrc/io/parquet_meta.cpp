// Parquet footer / page-header decoding (Thrift compact protocol), the column
// page planner and the positional reader. See parquet_meta.h.
#include "io/parquet_meta.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <climits>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>

#include "kernels/kernels.h"

namespace igloo {
namespace io {

namespace {

// ---- Thrift compact protocol -------------------------------------------------
enum TType : int { T_STOP = 0, T_TRUE = 1, T_FALSE = 2, T_BYTE = 3, T_I16 = 4, T_I32 = 5, T_I64 = 6, T_DOUBLE = 7,
                   T_BINARY = 8, T_LIST = 9, T_SET = 10, T_MAP = 11, T_STRUCT = 12 };

class TReader {
 public:
  TReader(const uint8_t* p, const uint8_t* end) : p_(p), begin_(p), end_(end) {}

  size_t consumed() const { return (size_t)(p_ - begin_); }

  uint8_t byte() {
    if (p_ >= end_) throw ParquetError("thrift: unexpected end of input");
    return *p_++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      uint8_t b = byte();
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    throw ParquetError("thrift: varint too long");
  }
  int64_t zigzag() {
    uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  int32_t i32() { return (int32_t)zigzag(); }
  int64_t i64() { return zigzag(); }
  std::string binary() {
    uint64_t n = varint();
    if (n > (uint64_t)(end_ - p_)) throw ParquetError("thrift: binary length past end of input");
    std::string s((const char*)p_, (size_t)n);
    p_ += n;
    return s;
  }
  // Next field of the current struct; false at STOP. `last` is the previous field id.
  bool field(int16_t& last, int& type, int16_t& id) {
    uint8_t b = byte();
    if (b == 0) return false;
    type = b & 0x0f;
    int delta = b >> 4;
    id = delta ? (int16_t)(last + delta) : (int16_t)zigzag();
    last = id;
    return true;
  }
  // List/set header: returns the element count, element type in `et`.
  int64_t list(int& et) {
    uint8_t b = byte();
    et = b & 0x0f;
    int64_t n = b >> 4;
    if (n == 15) n = (int64_t)varint();
    if (n < 0 || n > (int64_t)(end_ - p_) + 1) throw ParquetError("thrift: bad list size");
    return n;
  }
  bool boolean(int type) {
    if (type == T_TRUE) return true;
    if (type == T_FALSE) return false;
    throw ParquetError("thrift: expected a bool field");
  }
  void skip(int type, int depth = 0) {
    if (depth > 64) throw ParquetError("thrift: nesting too deep");
    switch (type) {
      case T_TRUE:
      case T_FALSE:
        return;
      case T_BYTE:
        byte();
        return;
      case T_I16:
      case T_I32:
      case T_I64:
        varint();
        return;
      case T_DOUBLE:
        if (end_ - p_ < 8) throw ParquetError("thrift: truncated double");
        p_ += 8;
        return;
      case T_BINARY:
        binary();
        return;
      case T_LIST:
      case T_SET: {
        int et;
        int64_t n = list(et);
        for (int64_t i = 0; i < n; ++i) {
          if (et == T_TRUE || et == T_FALSE)
            byte();
          else
            skip(et, depth + 1);
        }
        return;
      }
      case T_MAP: {
        int64_t n = (int64_t)varint();
        if (n == 0) return;
        uint8_t kv = byte();
        for (int64_t i = 0; i < n; ++i) {
          int kt = kv >> 4, vt = kv & 0x0f;
          if (kt == T_TRUE || kt == T_FALSE) byte(); else skip(kt, depth + 1);
          if (vt == T_TRUE || vt == T_FALSE) byte(); else skip(vt, depth + 1);
        }
        return;
      }
      case T_STRUCT: {
        int16_t last = 0;
        int t;
        int16_t id;
        while (field(last, t, id)) skip(t, depth + 1);
        return;
      }
      default:
        throw ParquetError("thrift: unknown field type " + std::to_string(type));
    }
  }
  // Iterate the fields of a struct: fn(id, type) must consume or skip each field.
  void each(const std::function<void(int16_t, int)>& fn) {
    int16_t last = 0;
    int t;
    int16_t id;
    while (field(last, t, id)) fn(id, t);
  }

 private:
  const uint8_t* p_;
  const uint8_t* begin_;
  const uint8_t* end_;
};

struct SchemaEl {
  int type = -1, type_length = 0, repetition = 0, num_children = 0, converted = -1, scale = 0, precision = 0;
  std::string name, logical;
  int lscale = -1, lprecision = -1;
};

std::string time_unit(TReader& r) {
  std::string u = "us";
  r.each([&](int16_t id, int t) {
    if (id == 1) u = "ms";
    else if (id == 2) u = "us";
    else if (id == 3) u = "ns";
    r.skip(t);
  });
  return u;
}

void parse_logical(TReader& r, SchemaEl& e) {
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1:   // STRING
      case 4:   // ENUM
      case 12:  // JSON
        e.logical = "string";
        r.skip(t);
        break;
      case 5:
        e.logical = "decimal";
        r.each([&](int16_t f, int ft) {
          if (f == 1) e.lscale = r.i32();
          else if (f == 2) e.lprecision = r.i32();
          else r.skip(ft);
        });
        break;
      case 6:
        e.logical = "date";
        r.skip(t);
        break;
      case 8: {
        std::string unit = "us";
        r.each([&](int16_t f, int ft) {
          if (f == 2) unit = time_unit(r);
          else r.skip(ft);
        });
        e.logical = "timestamp_" + unit;
        break;
      }
      case 10: {
        int bits = 64;
        bool sign = true;
        r.each([&](int16_t f, int ft) {
          if (f == 1) bits = (int8_t)r.byte();
          else if (f == 2) sign = r.boolean(ft);
          else r.skip(ft);
        });
        e.logical = std::string(sign ? "int" : "uint") + std::to_string(bits);
        break;
      }
      default:
        e.logical = "other";
        r.skip(t);
    }
  });
}

SchemaEl parse_schema_element(TReader& r) {
  SchemaEl e;
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1: e.type = r.i32(); break;
      case 2: e.type_length = r.i32(); break;
      case 3: e.repetition = r.i32(); break;
      case 4: e.name = r.binary(); break;
      case 5: e.num_children = r.i32(); break;
      case 6: e.converted = r.i32(); break;
      case 7: e.scale = r.i32(); break;
      case 8: e.precision = r.i32(); break;
      case 10: parse_logical(r, e); break;
      default: r.skip(t);
    }
  });
  return e;
}

std::string logical_from_converted(int c) {
  switch (c) {
    case 0: case 4: case 19: return "string";  // UTF8, ENUM, JSON
    case 5: return "decimal";
    case 6: return "date";
    case 9: return "timestamp_ms";
    case 10: return "timestamp_us";
    case 11: return "uint8";
    case 12: return "uint16";
    case 13: return "uint32";
    case 14: return "uint64";
    case 15: return "int8";
    case 16: return "int16";
    case 17: return "int32";
    case 18: return "int64";
    case -1: return "";
    default: return "other";
  }
}

PqStats parse_stats(TReader& r) {
  PqStats s;
  std::string min_old, max_old;
  bool has_min_old = false, has_max_old = false;
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1: max_old = r.binary(); has_max_old = true; break;
      case 2: min_old = r.binary(); has_min_old = true; break;
      case 3: s.null_count = r.i64(); s.has_nulls = true; break;
      case 5: s.max = r.binary(); s.has_max = true; break;
      case 6: s.min = r.binary(); s.has_min = true; break;
      default: r.skip(t);
    }
  });
  if (!s.has_max && has_max_old) { s.max = max_old; s.has_max = true; }
  if (!s.has_min && has_min_old) { s.min = min_old; s.has_min = true; }
  return s;
}

void parse_column_meta(TReader& r, PqChunk& c) {
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1: c.type = r.i32(); break;
      case 2: {
        int et;
        int64_t n = r.list(et);
        for (int64_t i = 0; i < n; ++i) c.encodings.push_back(r.i32());
        break;
      }
      case 4: c.codec = r.i32(); break;
      case 5: c.num_values = r.i64(); break;
      case 6: c.total_uncompressed = r.i64(); break;
      case 7: c.total_compressed = r.i64(); break;
      case 9: c.data_page_offset = r.i64(); break;
      case 11: c.dictionary_page_offset = r.i64(); break;
      case 12: c.stats = parse_stats(r); break;
      default: r.skip(t);
    }
  });
}

PqChunk parse_column_chunk(TReader& r) {
  PqChunk c;
  r.each([&](int16_t id, int t) {
    if (id == 1) c.external = !r.binary().empty();
    else if (id == 3) parse_column_meta(r, c);
    else r.skip(t);
  });
  return c;
}

PqRowGroup parse_row_group(TReader& r) {
  PqRowGroup g;
  r.each([&](int16_t id, int t) {
    if (id == 1) {
      int et;
      int64_t n = r.list(et);
      for (int64_t i = 0; i < n; ++i) g.chunks.push_back(parse_column_chunk(r));
    } else if (id == 3) {
      g.num_rows = r.i64();
    } else {
      r.skip(t);
    }
  });
  return g;
}

// Depth-first walk of the flattened schema tree -> leaves with def/rep levels.
size_t flatten(const std::vector<SchemaEl>& s, size_t i, int def, int rep, const std::string& prefix,
               std::vector<PqLeaf>& out) {
  const SchemaEl& e = s[i];
  const int d = def + (e.repetition != 0 ? 1 : 0);
  const int rr = rep + (e.repetition == 2 ? 1 : 0);
  const std::string name = prefix.empty() ? e.name : prefix + "." + e.name;
  size_t next = i + 1;
  if (e.num_children > 0) {
    for (int c = 0; c < e.num_children; ++c) {
      if (next >= s.size()) throw ParquetError("schema: truncated element list");
      next = flatten(s, next, d, rr, name, out);
    }
    return next;
  }
  PqLeaf l;
  l.name = name;
  l.type = e.type;
  l.type_length = e.type_length;
  l.max_def = d;
  l.max_rep = rr;
  l.converted_type = e.converted;
  l.logical = e.logical.empty() ? logical_from_converted(e.converted) : e.logical;
  l.scale = e.lscale >= 0 ? e.lscale : e.scale;
  l.precision = e.lprecision >= 0 ? e.lprecision : e.precision;
  out.push_back(std::move(l));
  return next;
}

int64_t align_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

struct Fd {
  int fd = -1;
  explicit Fd(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw ParquetError("cannot open " + path + ": " + std::strerror(errno));
  }
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

void pread_all(int fd, uint8_t* dst, int64_t len, int64_t off, const std::string& path) {
  while (len > 0) {
    ssize_t got = ::pread(fd, dst, (size_t)len, (off_t)off);
    if (got < 0) {
      if (errno == EINTR) continue;
      throw ParquetError("read error in " + path + ": " + std::strerror(errno));
    }
    if (got == 0) throw ParquetError("unexpected end of file in " + path);
    dst += got;
    len -= got;
    off += got;
  }
}

}  // namespace

PqFileMeta parse_file_meta(const uint8_t* p, size_t n) {
  TReader r(p, p + n);
  PqFileMeta m;
  std::vector<SchemaEl> schema;
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1: m.version = r.i32(); break;
      case 2: {
        int et;
        int64_t k = r.list(et);
        for (int64_t i = 0; i < k; ++i) schema.push_back(parse_schema_element(r));
        break;
      }
      case 3: m.num_rows = r.i64(); break;
      case 4: {
        int et;
        int64_t k = r.list(et);
        for (int64_t i = 0; i < k; ++i) m.row_groups.push_back(parse_row_group(r));
        break;
      }
      case 6: m.created_by = r.binary(); break;
      default: r.skip(t);
    }
  });
  if (schema.empty()) throw ParquetError("footer: empty schema");
  // schema[0] is the root group: its children are the top-level fields
  size_t next = 1;
  for (int c = 0; c < schema[0].num_children; ++c) {
    if (next >= schema.size()) throw ParquetError("schema: truncated element list");
    next = flatten(schema, next, 0, 0, "", m.leaves);
  }
  for (auto& g : m.row_groups)
    if (g.chunks.size() != m.leaves.size()) throw ParquetError("footer: row group column count != schema leaves");
  return m;
}

PqFileMeta read_file_meta(const std::string& path) {
  Fd f(path);
  struct stat st;
  if (fstat(f.fd, &st) != 0) throw ParquetError("cannot stat " + path);
  const int64_t size = st.st_size;
  if (size < 12) throw ParquetError(path + ": file too small to be Parquet");
  uint8_t tail[8], head[4];
  pread_all(f.fd, head, 4, 0, path);
  pread_all(f.fd, tail, 8, size - 8, path);
  if (std::memcmp(head, "PAR1", 4) != 0 || std::memcmp(tail + 4, "PAR1", 4) != 0)
    throw ParquetError(path + ": not a Parquet file (bad magic)");
  const uint32_t flen = (uint32_t)tail[0] | ((uint32_t)tail[1] << 8) | ((uint32_t)tail[2] << 16) |
                        ((uint32_t)tail[3] << 24);
  if ((int64_t)flen + 12 > size) throw ParquetError(path + ": bad footer length");
  std::vector<uint8_t> buf(flen);
  pread_all(f.fd, buf.data(), flen, size - 8 - flen, path);
  return parse_file_meta(buf.data(), buf.size());
}

PqPageHeader parse_page_header(const uint8_t* p, size_t n) {
  TReader r(p, p + n);
  PqPageHeader h;
  r.each([&](int16_t id, int t) {
    switch (id) {
      case 1: h.type = r.i32(); break;
      case 2: h.uncompressed = r.i32(); break;
      case 3: h.compressed = r.i32(); break;
      case 5:
        r.each([&](int16_t f, int ft) {
          if (f == 1) h.num_values = r.i32();
          else if (f == 2) h.encoding = r.i32();
          else if (f == 3) h.def_encoding = r.i32();
          else if (f == 4) h.rep_encoding = r.i32();
          else r.skip(ft);
        });
        break;
      case 7:
        r.each([&](int16_t f, int ft) {
          if (f == 1) h.num_values = r.i32();
          else if (f == 2) h.encoding = r.i32();
          else r.skip(ft);
        });
        break;
      case 8:
        r.each([&](int16_t f, int ft) {
          switch (f) {
            case 1: h.num_values = r.i32(); break;
            case 2: h.num_nulls = r.i32(); break;
            case 3: h.num_rows = r.i32(); break;
            case 4: h.encoding = r.i32(); break;
            case 5: h.def_len = r.i32(); break;
            case 6: h.rep_len = r.i32(); break;
            case 7: h.is_compressed = r.boolean(ft); break;
            default: r.skip(ft);
          }
        });
        break;
      default: r.skip(t);
    }
  });
  h.header_len = (int32_t)r.consumed();
  if (h.compressed < 0 || h.uncompressed < 0 || h.num_values < 0) throw ParquetError("page header: negative size");
  return h;
}

std::vector<PqPageHeader> parse_chunk_pages(const uint8_t* p, size_t n) {
  std::vector<PqPageHeader> out;
  size_t pos = 0;
  while (pos < n) {
    PqPageHeader h = parse_page_header(p + pos, n - pos);
    if ((size_t)h.header_len + (size_t)h.compressed > n - pos) throw ParquetError("column chunk: truncated page");
    out.push_back(h);
    pos += (size_t)h.header_len + (size_t)h.compressed;
  }
  return out;
}

void pread_ranges(const std::string& path, const std::vector<ReadRange>& ranges, int threads) {
  // <= 8 MiB pieces so the threads share big chunks evenly
  constexpr int64_t kPiece = 8 << 20;
  std::vector<ReadRange> pieces;
  for (auto& r : ranges)
    for (int64_t o = 0; o < r.length; o += kPiece)
      pieces.push_back({r.file_offset + o, std::min(kPiece, r.length - o), r.dst + o});
  if (pieces.empty()) return;
  Fd f(path);
  threads = std::max(1, std::min<int>(threads, (int)pieces.size()));
  std::atomic<size_t> next{0};
  std::mutex mu;
  std::string err;
  auto work = [&]() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= pieces.size()) return;
      try {
        pread_all(f.fd, pieces[i].dst, pieces[i].length, pieces[i].file_offset, path);
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> g(mu);
        if (err.empty()) err = e.what();
        next.store(pieces.size());
        return;
      }
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  if (!err.empty()) throw ParquetError(err);
}

PqPlan plan_column(const uint8_t* host, const std::vector<PqChunkIn>& chunks, int phys, int max_def, int max_rep,
                   int64_t dec_base, int type_len) {
  PqPlan plan;
  plan.dec_bytes = align_up(dec_base, 16);
  if (max_rep > 0) {
    plan.unsupported = "repeated (nested) column";
    return plan;
  }
  if (max_def > 1) {
    plan.unsupported = "nested optional column (max definition level > 1)";
    return plan;
  }
  if (phys == PQ_INT96 || phys < 0 || phys > PQ_FLBA) {
    plan.unsupported = "physical type " + std::to_string(phys);
    return plan;
  }
  std::vector<kern::PqPage> pages;
  std::vector<kern::PqSnappyJob> jobs;
  int64_t dict_base = 0;
  int codec = PQ_UNCOMPRESSED;
  auto add_job = [&](int64_t src, int64_t src_len, int64_t dst_len) -> int64_t {
    const int64_t dst = plan.dec_bytes;
    jobs.push_back(kern::PqSnappyJob{src, dst, (int32_t)src_len, (int32_t)dst_len, codec, 0});
    if (codec == PQ_ZSTD) ++plan.num_zstd_jobs;
    plan.dec_bytes = align_up(plan.dec_bytes + dst_len, 16);
    return dst;
  };
  for (const auto& ch : chunks) {
    if (ch.codec != PQ_UNCOMPRESSED && ch.codec != PQ_SNAPPY && ch.codec != PQ_ZSTD) {
      plan.unsupported = "codec " + std::to_string(ch.codec);
      return plan;
    }
    codec = ch.codec;
    const bool snappy = ch.codec != PQ_UNCOMPRESSED;   // a decompression job per page (snappy or zstd)
    int64_t pos = ch.buf_off;
    const int64_t end = ch.buf_off + ch.length;
    int64_t rows = 0;
    int64_t dict_off = -1;
    int32_t dict_count = 0, dict_flags = 0;
    while (pos < end && rows < ch.num_rows) {
      const PqPageHeader h = parse_page_header(host + pos, (size_t)(end - pos));
      const int64_t payload = pos + h.header_len;
      if (payload + h.compressed > end) throw ParquetError("column chunk: truncated page");
      pos = payload + h.compressed;
      if (h.type == PQ_INDEX_PAGE) continue;
      kern::PqPage pg{};
      pg.levels_off = -1;
      pg.dict_off = -1;
      pg.aux_off = -1;
      if (h.type == PQ_DICTIONARY_PAGE) {
        if (h.encoding != PQ_PLAIN && h.encoding != PQ_PLAIN_DICTIONARY) {
          plan.unsupported = "dictionary page encoding " + std::to_string(h.encoding);
          return plan;
        }
        if (dict_count) throw ParquetError("column chunk: two dictionary pages");
        if (snappy && h.compressed > 0) {
          dict_off = add_job(payload, h.compressed, h.uncompressed);
          dict_flags = kern::PQ_DICT_IN_DEC;
          pg.flags = kern::PQ_DATA_IN_DEC;
        } else {
          dict_off = payload;
          dict_flags = 0;
        }
        dict_count = h.num_values;
        pg.kind = kern::PQ_PAGE_DICT;
        pg.data_off = dict_off;
        pg.size = h.uncompressed;
        pg.num_values = h.num_values;
        pg.encoding = PQ_PLAIN;
        pg.dict_base = (int32_t)dict_base;
        pg.dict_count = dict_count;
        pages.push_back(pg);
        ++plan.num_dict_pages;
        continue;
      }
      if (h.type != PQ_DATA_PAGE && h.type != PQ_DATA_PAGE_V2) throw ParquetError("unknown page type");
      const int enc = h.encoding;
      const bool dict_enc = enc == PQ_PLAIN_DICTIONARY || enc == PQ_RLE_DICTIONARY;
      // DELTA_BINARY_PACKED ints, DELTA_LENGTH_BYTE_ARRAY strings and
      // BYTE_STREAM_SPLIT values decode on the device into an aux slot of the
      // decompression buffer (values, or string lengths), then read as PLAIN
      const bool fixed = phys == PQ_INT32 || phys == PQ_INT64 || phys == PQ_FLOAT || phys == PQ_DOUBLE || phys == PQ_FLBA;
      const bool delta = (enc == PQ_DELTA_BINARY_PACKED && (phys == PQ_INT32 || phys == PQ_INT64)) ||
                         (enc == PQ_DELTA_LENGTH_BYTE_ARRAY && phys == PQ_BYTE_ARRAY) ||
                         (enc == PQ_BYTE_STREAM_SPLIT && fixed);
      if (!(enc == PQ_PLAIN || dict_enc || (enc == PQ_RLE && phys == PQ_BOOLEAN) || delta)) {
        plan.unsupported = "data page encoding " + std::to_string(enc);
        return plan;
      }
      if (dict_enc && dict_count == 0 && h.num_values > 0 && h.num_values != h.num_nulls)
        throw ParquetError("dictionary-encoded page without a dictionary page");
      if (!dict_enc) ++plan.plain_pages;
      int64_t nrows;
      if (h.type == PQ_DATA_PAGE) {
        if (max_def > 0 && h.def_encoding != PQ_RLE) {
          plan.unsupported = "bit-packed definition levels";
          return plan;
        }
        pg.kind = kern::PQ_PAGE_DATA_V1;
        if (snappy && h.compressed > 0) {
          pg.data_off = add_job(payload, h.compressed, h.uncompressed);
          pg.flags = kern::PQ_DATA_IN_DEC;
        } else {
          pg.data_off = payload;
        }
        pg.size = h.uncompressed;
        nrows = h.num_values;
      } else {
        if (h.rep_len != 0) throw ParquetError("repetition levels in a flat column");
        pg.kind = kern::PQ_PAGE_DATA_V2;
        pg.levels_off = payload;
        pg.levels_len = h.def_len;
        const int64_t vsrc = payload + h.def_len + h.rep_len;
        const int64_t vcomp = (int64_t)h.compressed - h.def_len - h.rep_len;
        const int64_t vunc = (int64_t)h.uncompressed - h.def_len - h.rep_len;
        if (vcomp < 0 || vunc < 0) throw ParquetError("v2 page: level lengths exceed page size");
        if (snappy && h.is_compressed && vcomp > 0) {
          pg.data_off = add_job(vsrc, vcomp, vunc);
          pg.flags = kern::PQ_DATA_IN_DEC;
        } else {
          pg.data_off = vsrc;
        }
        pg.size = (int32_t)vunc;
        nrows = h.num_rows ? h.num_rows : h.num_values;
      }
      pg.num_values = (int32_t)nrows;
      pg.encoding = enc;
      if (delta) {
        const int64_t w = enc == PQ_DELTA_LENGTH_BYTE_ARRAY ? 4
                          : phys == PQ_INT32 || phys == PQ_FLOAT ? 4
                          : phys == PQ_FLBA ? (int64_t)type_len
                          : 8;
        pg.aux_off = plan.dec_bytes;
        plan.dec_bytes = align_up(plan.dec_bytes + std::max<int64_t>(nrows, 1) * w, 16);
      }
      pg.out_row = ch.first_row + rows;
      pg.dict_off = dict_count ? dict_off : -1;
      pg.flags |= dict_flags;
      pg.dict_base = (int32_t)dict_base;
      pg.dict_count = dict_count;
      pages.push_back(pg);
      plan.max_page_values = std::max<int64_t>(plan.max_page_values, nrows);
      rows += nrows;
    }
    if (rows != ch.num_rows)
      throw ParquetError("column chunk holds " + std::to_string(rows) + " rows, row group says " +
                         std::to_string(ch.num_rows));
    dict_base += dict_count;
    plan.dict_entries += dict_count;
    if (dict_base > INT32_MAX) {
      plan.unsupported = "dictionary too large";
      return plan;
    }
  }
  plan.num_pages = (int64_t)pages.size();
  plan.num_jobs = (int64_t)jobs.size();
  plan.pages.resize(pages.size() * sizeof(kern::PqPage));
  if (!pages.empty()) std::memcpy(plan.pages.data(), pages.data(), plan.pages.size());
  plan.jobs.resize(jobs.size() * sizeof(kern::PqSnappyJob));
  if (!jobs.empty()) std::memcpy(plan.jobs.data(), jobs.data(), plan.jobs.size());
  return plan;
}

}  // namespace io
}  // namespace igloo
