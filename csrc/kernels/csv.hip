// GPU CSV parsing for gfx950.
//
// Replaces the reference's row-at-a-time csv-crate reader that materialises
// every field as a String (crates/connectors/filesystem/src/lib.rs:34-45) and
// DataFusion's CsvFormat (crates/coordinator/src/main.rs:38-41). The file is
// staged in HBM once; then:
//
//   csv_quote_parity  one wave per 16 KiB tile: parity of quote characters.
//                     (host: exclusive XOR-scan of the tile parities = quote
//                     state at every tile start)
//   csv_rows          pass 0 counts, pass 1 writes the positions of the row
//                     terminators ('\n' outside quotes, empty lines skipped).
//                     Lanes own 16 consecutive bytes of a 1 KiB wave chunk;
//                     each lane's starting quote state is the chunk state XOR
//                     the parity of the quotes below it (ballot + mbcnt), so
//                     loads stay coalesced and no lane walks another's bytes.
//   csv_parse         one lane per row: splits the row into fields (RFC 4180
//                     quoting, "" escapes, CRLF) and parses each field straight
//                     into its typed column (int32/int64, exact decimal,
//                     float64, date, bool) or records (position, length) of
//                     string fields; csv_str_copy then writes the Arrow chars
//                     (un-escaping quoted fields) after an offset scan.
#include "common.h"
#include "kernels.h"
#include "textparse.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kChunk = kWave * 16;          // bytes per wave step
constexpr int kTileChunks = kCsvTile / kChunk;

enum : int { CSV_ERR_FIELDS = 1, CSV_ERR_VALUE = 2, CSV_ERR_QUOTE = 3 };

__device__ inline void set_err(int* err, int code) { atomicCAS(err, 0, code); }

// 16 bytes at p (p 16-byte aligned inside the padded buffer); bytes past n read as 0
__device__ inline uint4 load16(const uint8_t* buf, int64_t pos, int64_t n) {
  if (pos + 16 <= n) return *reinterpret_cast<const uint4*>(buf + pos);
  uint8_t t[16];
  for (int k = 0; k < 16; ++k) t[k] = pos + k < n ? buf[pos + k] : 0;
  uint4 v;
  __builtin_memcpy(&v, t, 16);
  return v;
}

__device__ inline int count_byte(uint4 v, uint8_t c) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  int n = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int b = 0; b < 4; ++b) n += ((w[k] >> (8 * b)) & 0xff) == c;
  return n;
}

__global__ __launch_bounds__(kWave) void csv_quote_parity_kernel(const uint8_t* __restrict__ buf, int64_t n,
                                                               uint8_t quote, uint8_t* __restrict__ tile_par) {
  const int64_t base = (int64_t)blockIdx.x * kCsvTile;
  int c = 0;
  for (int s = 0; s < kTileChunks; ++s) {
    const int64_t pos = base + (int64_t)s * kChunk + threadIdx.x * 16;
    if (pos < n) c += count_byte(load16(buf, pos, n), quote);
  }
  c = (int)wave_reduce_sum((int64_t)c);
  if (threadIdx.x == 0) tile_par[blockIdx.x] = (uint8_t)(c & 1);
}

// WRITE = false: tile_rows[tile] = row terminators in the tile.
// WRITE = true: rows_end[tile_off[tile] + k] = position of the k-th terminator.
template <bool WRITE>
__global__ __launch_bounds__(kWave) void csv_rows_kernel(const uint8_t* __restrict__ buf, int64_t n, int64_t start,
                                                       uint8_t quote, const uint8_t* __restrict__ tile_state,
                                                       int64_t* __restrict__ tile_rows,
                                                       const int64_t* __restrict__ tile_off,
                                                       int64_t* __restrict__ rows_end) {
  const int lane = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kCsvTile;
  int state = tile_state[blockIdx.x];
  int64_t out = WRITE ? tile_off[blockIdx.x] : 0;
  int64_t total = 0;
  for (int s = 0; s < kTileChunks; ++s) {
    const int64_t pos = base + (int64_t)s * kChunk + lane * 16;
    uint8_t b[16];
    const uint4 v = pos < n ? load16(buf, pos, n) : make_uint4(0, 0, 0, 0);
    __builtin_memcpy(b, &v, 16);
    int q = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) q += b[k] == quote;
    const uint64_t qmask = __ballot(q & 1);
    int st = state ^ (lane_prefix(qmask) & 1);
    // the two bytes before this lane's 16 (bytes before `start` read as '\n'):
    // a '\n' right after '\n' or "\n\r" ends an empty line, which is skipped
    uint8_t prev = pos - 1 >= start && pos - 1 < n ? buf[pos - 1] : '\n';
    uint8_t prev2 = pos - 2 >= start && pos - 2 < n ? buf[pos - 2] : '\n';
    int cnt = 0;
    uint32_t hits = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint8_t c = b[k];
      if (c == quote) {
        st ^= 1;
      } else if (c == '\n' && st == 0 && pos + k < n && pos + k >= start &&
                 !(prev == '\n' || (prev == '\r' && prev2 == '\n'))) {
        hits |= 1u << k;
        ++cnt;
      }
      prev2 = prev;
      prev = c;
    }
    if (WRITE) {
      const int64_t inc = wave_inclusive_scan(cnt);
      int64_t o = out + inc - cnt;
      for (int k = 0; k < 16; ++k)
        if (hits & (1u << k)) rows_end[o++] = pos + k;
      out += __shfl(inc, kWave - 1, kWave);
    } else {
      total += cnt;
    }
    state ^= __popcll(qmask) & 1;
  }
  if (!WRITE) {
    total = wave_reduce_sum(total);
    if (lane == 0) tile_rows[blockIdx.x] = total;
  }
}


__global__ __launch_bounds__(kBlock) void csv_parse_kernel(const uint8_t* __restrict__ buf, int64_t start,
                                                         const int64_t* __restrict__ rows_end, int64_t nrows,
                                                         const CsvColumn* __restrict__ cols, int ncols,
                                                         uint8_t delim, uint8_t quote, int* __restrict__ err) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t p = r == 0 ? start : rows_end[r - 1] + 1;
    int64_t end = rows_end[r];
    while (p < end && (buf[p] == '\n' || buf[p] == '\r')) ++p;  // skipped empty lines before the row
    if (end > p && buf[end - 1] == '\r') --end;
    int f = 0;
    for (;;) {
      // ---- one field [fs, fe), quoted or not
      int64_t fs, fe, next;
      int escapes = 0;
      bool quoted = false;
      if (p < end && buf[p] == quote) {
        quoted = true;
        int64_t q = p + 1;
        for (;;) {
          if (q >= end) {
            set_err(err, CSV_ERR_QUOTE);
            q = end;
            break;
          }
          if (buf[q] == quote) {
            if (q + 1 < end && buf[q + 1] == quote) {
              ++escapes;
              q += 2;
              continue;
            }
            break;
          }
          ++q;
        }
        fs = p + 1;
        fe = q;
        next = q + 1;
        if (next < end && buf[next] != delim) set_err(err, CSV_ERR_QUOTE);
      } else {
        int64_t q = p;
        while (q < end && buf[q] != delim) ++q;
        fs = p;
        fe = q;
        next = q;
      }
      if (f < ncols) {
        const CsvColumn& c = cols[f];
        const uint8_t* a = buf + fs;
        const uint8_t* b = buf + fe;
        const bool empty = fe == fs;
        bool ok = true, valid = true;
        switch (c.kind) {
          case CSV_SKIP:
            break;
          case CSV_UTF8:
            reinterpret_cast<int64_t*>(c.out)[r] = (int64_t)a;
            c.len[r] = (fe - fs - escapes) | (escapes ? ((int64_t)1 << 62) : 0);
            break;
          case CSV_INT32:
          case CSV_INT64: {
            int64_t v = 0;
            if (empty) valid = false;
            else ok = parse_int(a, b, &v) && (c.kind == CSV_INT64 || (v >= INT32_MIN && v <= INT32_MAX));
            if (c.kind == CSV_INT32) reinterpret_cast<int32_t*>(c.out)[r] = (int32_t)v;
            else reinterpret_cast<int64_t*>(c.out)[r] = v;
            break;
          }
          case CSV_DECIMAL: {
            int64_t v = 0;
            if (empty) valid = false;
            else ok = parse_decimal(a, b, c.scale, &v);
            reinterpret_cast<int64_t*>(c.out)[r] = v;
            break;
          }
          case CSV_FLOAT64: {
            double v = 0;
            if (empty) valid = false;
            else ok = parse_f64(a, b, &v);
            reinterpret_cast<double*>(c.out)[r] = v;
            break;
          }
          case CSV_DATE: {
            int32_t v = 0;
            if (empty) valid = false;
            else ok = parse_date(a, b, &v);
            reinterpret_cast<int32_t*>(c.out)[r] = v;
            break;
          }
          case CSV_BOOL: {
            uint8_t v = 0;
            if (empty) valid = false;
            else if (ieq(a, b, "true") || ieq(a, b, "1")) v = 1;
            else if (!(ieq(a, b, "false") || ieq(a, b, "0"))) ok = false;
            reinterpret_cast<uint8_t*>(c.out)[r] = v;
            break;
          }
        }
        if (!ok) set_err(err, CSV_ERR_VALUE);
        if (c.valid) c.valid[r] = valid;
        else if (!valid) set_err(err, CSV_ERR_VALUE);  // NULL where the caller expects none
      }
      ++f;
      if (next >= end) break;
      p = next + 1;  // skip the delimiter
      if (p == end) {  // trailing delimiter: one more (empty) field
        if (f < ncols) {
          const CsvColumn& c = cols[f];
          if (c.kind == CSV_UTF8) {
            reinterpret_cast<int64_t*>(c.out)[r] = (int64_t)(buf + p);
            c.len[r] = 0;
          } else if (c.kind != CSV_SKIP) {
            if (c.valid) c.valid[r] = 0;
            else set_err(err, CSV_ERR_VALUE);
          }
        }
        ++f;
        break;
      }
    }
    if (f != ncols) set_err(err, CSV_ERR_FIELDS);
  }
}

// One wave copies 64 consecutive strings; quoted fields with "" escapes are
// copied by lane 0 with the escapes collapsed.
__global__ __launch_bounds__(kBlock) void csv_str_copy_kernel(const int64_t* __restrict__ pos,
                                                            const int64_t* __restrict__ len_flag,
                                                            const int64_t* __restrict__ off, int64_t n,
                                                            uint8_t quote, uint8_t* __restrict__ out) {
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
        for (int64_t k = 0; j < len; ++k) {
          out[o + j++] = sp[k];
          if (sp[k] == quote) ++k;  // "" -> "
        }
      }
    }
  }
}

__global__ void csv_len_kernel(const int64_t* __restrict__ len_flag, int64_t n, int64_t* __restrict__ len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    len[i] = len_flag[i] & (((int64_t)1 << 62) - 1);
}

}  // namespace

int64_t csv_num_tiles(int64_t n) { return (n + kCsvTile - 1) / kCsvTile; }

void csv_quote_parity(const uint8_t* buf, int64_t n, uint8_t quote, uint8_t* tile_par, hipStream_t stream) {
  const int64_t t = csv_num_tiles(n);
  if (t == 0) return;
  hipLaunchKernelGGL(csv_quote_parity_kernel, dim3((unsigned)t), dim3(kWave), 0, stream, buf, n, quote, tile_par);
  check_launch("csv_quote_parity", stream);
}

void csv_rows(const uint8_t* buf, int64_t n, int64_t start, uint8_t quote, const uint8_t* tile_state,
              int64_t* tile_rows, const int64_t* tile_off, int64_t* rows_end, hipStream_t stream) {
  const int64_t t = csv_num_tiles(n);
  if (t == 0) return;
  if (rows_end)
    hipLaunchKernelGGL(csv_rows_kernel<true>, dim3((unsigned)t), dim3(kWave), 0, stream, buf, n, start, quote,
                       tile_state, tile_rows, tile_off, rows_end);
  else
    hipLaunchKernelGGL(csv_rows_kernel<false>, dim3((unsigned)t), dim3(kWave), 0, stream, buf, n, start, quote,
                       tile_state, tile_rows, tile_off, rows_end);
  check_launch("csv_rows", stream);
}

void csv_parse(const uint8_t* buf, int64_t start, const int64_t* rows_end, int64_t nrows, const CsvColumn* cols,
               int ncols, uint8_t delim, uint8_t quote, int* err, hipStream_t stream) {
  if (nrows <= 0) return;
  hipLaunchKernelGGL(csv_parse_kernel, dim3(grid_for(nrows, kBlock, 1 << 16)), dim3(kBlock), 0, stream, buf, start,
                     rows_end, nrows, cols, ncols, delim, quote, err);
  check_launch("csv_parse", stream);
}

void csv_str_lengths(const int64_t* len_flag, int64_t n, int64_t* len, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(csv_len_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, stream, len_flag, n, len);
  check_launch("csv_str_lengths", stream);
}

void csv_str_copy(const int64_t* pos, const int64_t* len_flag, const int64_t* off, int64_t n, uint8_t quote,
                  uint8_t* out, hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(csv_str_copy_kernel, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, stream, pos, len_flag,
                     off, n, quote, out);
  check_launch("csv_str_copy", stream);
}

}  // namespace kern
}  // namespace igloo
