// GPU NDJSON (newline-delimited JSON) parsing for gfx950.
//
// DataFusion reads ``STORED AS JSON`` tables with arrow-json on the CPU
// (reference Cargo.lock:947 datafusion-datasource-json). Here the file is
// staged in HBM once and:
//
//   rows          csv_rows (csv.hip) with no quote character: a raw newline
//                 cannot occur inside a JSON string, so every '\n' ends a
//                 record (empty lines skipped).
//   json_parse    one lane per record: walks the top-level object, matches
//                 each key against the schema's field names (packed in
//                 global memory, compared length-first), and parses the
//                 value straight into its typed column (int32/int64, exact
//                 decimal, float64, bool, date from a "YYYY-MM-DD" string),
//                 or records (address, unescaped length | escape flag) for
//                 string fields. Nested objects / arrays are skipped by
//                 bracket depth (strings honoured); a string column receives
//                 their raw JSON text. Absent keys and ``null`` are NULL.
//   json_str_copy one wave per 64 strings: plain strings copied lane-
//                 parallel, strings with escapes decoded by lane 0
//                 (\" \\ \/ \b \f \n \r \t and \uXXXX with surrogate pairs,
//                 written as UTF-8).
#include "common.h"
#include "kernels.h"
#include "textparse.h"

namespace igloo {
namespace kern {

namespace {

enum : int { JSON_ERR_SYNTAX = 1, JSON_ERR_VALUE = 2, JSON_ERR_FIELDS = 3 };

__device__ inline void jset_err(int* err, int code) { atomicCAS(err, 0, code); }

__device__ inline bool is_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }

__device__ inline int hexv(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

__device__ inline int utf8_bytes(uint32_t cp) { return cp < 0x80 ? 1 : cp < 0x800 ? 2 : cp < 0x10000 ? 3 : 4; }

// \uXXXX at p (p points at 'u'); returns the code point or -1
__device__ inline int64_t u4(const uint8_t* p, const uint8_t* e) {
  if (e - p < 5) return -1;
  int64_t v = 0;
  for (int k = 1; k <= 4; ++k) {
    const int h = hexv(p[k]);
    if (h < 0) return -1;
    v = v * 16 + h;
  }
  return v;
}

// Scans a JSON string whose opening quote is at p. Returns the position of the
// closing quote (or -1), the decoded UTF-8 length and whether escapes occur.
__device__ inline const uint8_t* scan_string(const uint8_t* p, const uint8_t* e, int64_t* out_len, bool* esc) {
  int64_t len = 0;
  bool any = false;
  for (const uint8_t* q = p + 1; q < e; ++q) {
    const uint8_t c = *q;
    if (c == '"') {
      *out_len = len;
      *esc = any;
      return q;
    }
    if (c != '\\') {
      ++len;
      continue;
    }
    any = true;
    if (q + 1 >= e) return nullptr;
    const uint8_t x = q[1];
    if (x == 'u') {
      int64_t cp = u4(q + 1, e);
      if (cp < 0) return nullptr;
      q += 5;
      if (cp >= 0xD800 && cp < 0xDC00 && q + 2 < e && q[1] == '\\' && q[2] == 'u') {
        const int64_t lo = u4(q + 2, e);
        if (lo >= 0xDC00 && lo < 0xE000) {
          cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          q += 6;
        }
      }
      len += utf8_bytes((uint32_t)cp);
    } else {
      ++q;
      ++len;
    }
  }
  return nullptr;
}

// end of a nested object / array starting at p ('{' or '['), or null
__device__ inline const uint8_t* skip_nested(const uint8_t* p, const uint8_t* e) {
  int depth = 0;
  for (const uint8_t* q = p; q < e; ++q) {
    const uint8_t c = *q;
    if (c == '"') {
      int64_t l;
      bool x;
      q = scan_string(q, e, &l, &x);
      if (!q) return nullptr;
    } else if (c == '{' || c == '[') {
      ++depth;
    } else if (c == '}' || c == ']') {
      if (--depth == 0) return q + 1;
    }
  }
  return nullptr;
}

__device__ inline int find_field(const uint8_t* k, int64_t kl, const uint8_t* names, const int32_t* name_off,
                                 int nf) {
  for (int f = 0; f < nf; ++f) {
    const int32_t a = name_off[f], b = name_off[f + 1];
    if (b - a != kl) continue;
    bool eq = true;
    for (int64_t j = 0; j < kl && eq; ++j) eq = names[a + j] == k[j];
    if (eq) return f;
  }
  return -1;
}

__global__ __launch_bounds__(kBlock) void json_parse_kernel(const uint8_t* __restrict__ buf, int64_t start,
                                                          const int64_t* __restrict__ rows_end, int64_t nrows,
                                                          const CsvColumn* __restrict__ cols, int ncols,
                                                          const uint8_t* __restrict__ names,
                                                          const int32_t* __restrict__ name_off,
                                                          int* __restrict__ err) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* p = buf + (r == 0 ? start : rows_end[r - 1] + 1);
    const uint8_t* e = buf + rows_end[r];
    uint64_t seen = 0;
    while (p < e && is_ws(*p)) ++p;
    if (p >= e || *p != '{') {
      jset_err(err, JSON_ERR_SYNTAX);
      continue;
    }
    ++p;
    bool bad = false;
    for (;;) {
      while (p < e && is_ws(*p)) ++p;
      if (p < e && *p == '}') break;
      if (p >= e || *p != '"') { bad = true; break; }
      int64_t kl;
      bool kesc;
      const uint8_t* kq = scan_string(p, e, &kl, &kesc);
      if (!kq) { bad = true; break; }
      const uint8_t* ks = p + 1;
      const int f = kesc ? -1 : find_field(ks, kq - ks, names, name_off, ncols);
      p = kq + 1;
      while (p < e && is_ws(*p)) ++p;
      if (p >= e || *p != ':') { bad = true; break; }
      ++p;
      while (p < e && is_ws(*p)) ++p;
      if (p >= e) { bad = true; break; }
      // ---- value [vs, ve): kind 's' string (content span), 'n' null, 'x' nested, 'l' literal
      const uint8_t* vs = p;
      const uint8_t* ve;
      char vk;
      int64_t slen = 0;
      bool sesc = false;
      if (*p == '"') {
        const uint8_t* q = scan_string(p, e, &slen, &sesc);
        if (!q) { bad = true; break; }
        vs = p + 1;
        ve = q;
        p = q + 1;
        vk = 's';
      } else if (*p == '{' || *p == '[') {
        const uint8_t* q = skip_nested(p, e);
        if (!q) { bad = true; break; }
        ve = q;
        p = q;
        vk = 'x';
      } else {
        const uint8_t* q = p;
        while (q < e && *q != ',' && *q != '}' && !is_ws(*q)) ++q;
        ve = q;
        p = q;
        vk = (ve - vs == 4 && vs[0] == 'n' && vs[1] == 'u' && vs[2] == 'l' && vs[3] == 'l') ? 'n' : 'l';
      }
      if (f >= 0) {
        seen |= 1ull << (f & 63);
        const CsvColumn& c = cols[f];
        bool ok = true, valid = vk != 'n';
        switch (c.kind) {
          case CSV_SKIP:
            break;
          case CSV_UTF8:
            reinterpret_cast<int64_t*>(c.out)[r] = (int64_t)vs;
            if (vk == 's') c.len[r] = slen | (sesc ? ((int64_t)1 << 62) : 0);
            else c.len[r] = valid ? (ve - vs) : 0;   // raw text of a number / literal / nested value
            break;
          case CSV_INT32:
          case CSV_INT64: {
            int64_t v = 0;
            if (valid) ok = vk == 'l' && parse_int(vs, ve, &v) &&
                            (c.kind == CSV_INT64 || (v >= INT32_MIN && v <= INT32_MAX));
            if (c.kind == CSV_INT32) reinterpret_cast<int32_t*>(c.out)[r] = (int32_t)v;
            else reinterpret_cast<int64_t*>(c.out)[r] = v;
            break;
          }
          case CSV_DECIMAL: {
            int64_t v = 0;
            if (valid) ok = (vk == 'l' || (vk == 's' && !sesc)) && parse_decimal(vs, ve, c.scale, &v);
            reinterpret_cast<int64_t*>(c.out)[r] = v;
            break;
          }
          case CSV_FLOAT64: {
            double v = 0;
            if (valid) ok = vk == 'l' && parse_f64(vs, ve, &v);
            reinterpret_cast<double*>(c.out)[r] = v;
            break;
          }
          case CSV_DATE: {
            int32_t v = 0;
            if (valid) ok = vk == 's' && parse_date(vs, ve, &v);
            reinterpret_cast<int32_t*>(c.out)[r] = v;
            break;
          }
          case CSV_BOOL: {
            uint8_t v = 0;
            if (valid) {
              if (ve - vs == 4 && vs[0] == 't' && vs[1] == 'r' && vs[2] == 'u' && vs[3] == 'e') v = 1;
              else ok = ve - vs == 5 && vs[0] == 'f' && vs[1] == 'a' && vs[2] == 'l' && vs[3] == 's' && vs[4] == 'e';
            }
            reinterpret_cast<uint8_t*>(c.out)[r] = v;
            break;
          }
        }
        if (!ok) jset_err(err, JSON_ERR_VALUE);
        if (c.valid) c.valid[r] = valid;
        else if (!valid) jset_err(err, JSON_ERR_VALUE);
      }
      while (p < e && is_ws(*p)) ++p;
      if (p < e && *p == ',') {
        ++p;
        continue;
      }
      if (p < e && *p == '}') break;
      bad = true;
      break;
    }
    if (bad) jset_err(err, JSON_ERR_SYNTAX);
    // keys the record does not have are NULL
    for (int f = 0; f < ncols; ++f) {
      if (seen & (1ull << (f & 63))) continue;
      const CsvColumn& c = cols[f];
      if (c.kind == CSV_SKIP) continue;
      if (c.kind == CSV_UTF8) {
        reinterpret_cast<int64_t*>(c.out)[r] = (int64_t)buf;
        c.len[r] = 0;
      } else if (c.kind == CSV_INT64 || c.kind == CSV_DECIMAL) {
        reinterpret_cast<int64_t*>(c.out)[r] = 0;
      } else if (c.kind == CSV_FLOAT64) {
        reinterpret_cast<double*>(c.out)[r] = 0;
      } else if (c.kind == CSV_INT32 || c.kind == CSV_DATE) {
        reinterpret_cast<int32_t*>(c.out)[r] = 0;
      } else {
        reinterpret_cast<uint8_t*>(c.out)[r] = 0;
      }
      if (c.valid) c.valid[r] = 0;
      else jset_err(err, JSON_ERR_FIELDS);
    }
  }
}

__device__ inline int put_utf8(uint8_t* o, uint32_t cp) {
  if (cp < 0x80) {
    o[0] = (uint8_t)cp;
    return 1;
  }
  if (cp < 0x800) {
    o[0] = (uint8_t)(0xC0 | (cp >> 6));
    o[1] = (uint8_t)(0x80 | (cp & 0x3F));
    return 2;
  }
  if (cp < 0x10000) {
    o[0] = (uint8_t)(0xE0 | (cp >> 12));
    o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
    o[2] = (uint8_t)(0x80 | (cp & 0x3F));
    return 3;
  }
  o[0] = (uint8_t)(0xF0 | (cp >> 18));
  o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
  o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
  o[3] = (uint8_t)(0x80 | (cp & 0x3F));
  return 4;
}

// out[off[r] .. off[r+1]): plain strings copied by the whole wave, escaped
// ones decoded by lane 0 (bounded by the row's output length)
__global__ __launch_bounds__(kBlock) void json_str_copy_kernel(const int64_t* __restrict__ pos,
                                                             const int64_t* __restrict__ len_flag,
                                                             const int64_t* __restrict__ off, int64_t n,
                                                             uint8_t* __restrict__ out) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t r0 = wave * kWave; r0 < n; r0 += nwaves * kWave) {
    const int64_t r1 = r0 + kWave < n ? r0 + kWave : n;
    for (int64_t r = r0; r < r1; ++r) {
      const uint8_t* sp = reinterpret_cast<const uint8_t*>(pos[r]);
      const int64_t o = off[r], len = off[r + 1] - o;
      if (!(len_flag[r] >> 62)) {
        for (int64_t k = lane; k < len; k += kWave) out[o + k] = sp[k];
      } else if (lane == 0) {
        int64_t j = 0;
        uint8_t tmp[4];
        for (int64_t k = 0; j < len;) {
          const uint8_t c = sp[k];
          if (c != '\\') {
            out[o + j++] = c;
            ++k;
            continue;
          }
          const uint8_t x = sp[k + 1];
          if (x == 'u') {
            int64_t cp = 0;
            for (int q = 2; q < 6; ++q) cp = cp * 16 + hexv(sp[k + q]);
            k += 6;
            if (cp >= 0xD800 && cp < 0xDC00 && sp[k] == '\\' && sp[k + 1] == 'u') {
              int64_t lo = 0;
              bool okh = true;
              for (int q = 2; q < 6; ++q) {
                const int h = hexv(sp[k + q]);
                okh &= h >= 0;
                lo = lo * 16 + h;
              }
              if (okh && lo >= 0xDC00 && lo < 0xE000) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                k += 6;
              }
            }
            const int m = put_utf8(tmp, (uint32_t)cp);
            for (int q = 0; q < m && j < len; ++q) out[o + j++] = tmp[q];
          } else {
            const uint8_t d = x == 'b' ? '\b' : x == 'f' ? '\f' : x == 'n' ? '\n' : x == 'r' ? '\r'
                            : x == 't' ? '\t' : x;
            out[o + j++] = d;
            k += 2;
          }
        }
      }
    }
  }
}

}  // namespace

void json_parse(const uint8_t* buf, int64_t start, const int64_t* rows_end, int64_t nrows, const CsvColumn* cols,
                int ncols, const uint8_t* names, const int32_t* name_off, int* err, hipStream_t stream) {
  if (nrows == 0) return;
  hipLaunchKernelGGL(json_parse_kernel, dim3(grid_for(nrows, kBlock, 1 << 14)), dim3(kBlock), 0, stream, buf, start,
                     rows_end, nrows, cols, ncols, names, name_off, err);
  check_launch("json_parse", stream);
}

void json_str_copy(const int64_t* pos, const int64_t* len_flag, const int64_t* off, int64_t n, uint8_t* out,
                   hipStream_t stream) {
  if (n == 0) return;
  const int64_t waves = (n + kWave - 1) / kWave;
  const int64_t blocks = std::min<int64_t>((waves * kWave + kBlock - 1) / kBlock, 1 << 14);
  hipLaunchKernelGGL(json_str_copy_kernel, dim3(blocks), dim3(kBlock), 0, stream, pos, len_flag, off, n, out);
  check_launch("json_str_copy", stream);
}

}  // namespace kern
}  // namespace igloo
