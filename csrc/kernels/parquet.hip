// GPU Parquet page decoding for gfx950.
//
// Replaces the reference's host-side parquet-rs reader (crates/engine/src/
// operators/parquet_scan.rs:47-58: 1024-row record batches on a blocking
// thread) with device decoding of whole column chunks that were staged into
// HBM with one H2D copy (host side: csrc/io/parquet_meta.cpp plans the pages).
//
// Kernels (one launch for every page of every column of a scan, one workgroup
// per page; page_col[] selects the page's column spec):
//   pq_snappy_kernel       raw snappy -> dec buffer. One wave per compressed
//                          page; every lane parses the same tag from an LDS
//                          input window (broadcast reads), copies are spread
//                          over the 64 lanes, back-references are served from
//                          a 64 KiB LDS history ring (snappy offsets < 64 KiB).
//   pq_dict_strings_kernel BYTE_ARRAY dictionary pages -> (position, length)
//                          of every dictionary entry.
//   pq_decode_kernel       data pages: RLE/bit-packed definition levels ->
//                          validity; PLAIN / dictionary values -> typed output
//                          (conversion fused: decimal widening, FLBA big-endian
//                          decimals, timestamp units, booleans); strings ->
//                          per-row (position, length) or global dictionary code.
//   pq_str_copy_kernel     string bytes into the Arrow chars buffer once the
//                          offsets are known (exclusive scan of the lengths).
//
// RLE / bit-packed hybrid streams are decoded block-cooperatively: lane 0 of
// the workgroup parses up to kRunCap run headers into LDS, then all 256 lanes
// decode values by binary search over the run starts.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kRunCap = 512;
constexpr int kWalkWin = 8192;
constexpr int kItems = 4;  // rows per lane per mapping step
constexpr int kSnapRing = 65536;
constexpr int kSnapIn = 4096;

enum : int {
  PQ_ERR_RLE = 1,
  PQ_ERR_DICT_INDEX = 2,
  PQ_ERR_BYTE_ARRAY = 3,
  PQ_ERR_SNAPPY = 4,
  PQ_ERR_SNAPPY_SIZE = 5,
  PQ_ERR_DECIMAL = 6,
  PQ_ERR_ENCODING = 7,
  PQ_ERR_NULLS = 8,
  PQ_ERR_TRUNCATED = 9,
};

__device__ inline void set_error(int* err, int code) { atomicCAS(err, 0, code); }

__device__ inline uint32_t ld_u32(const uint8_t* p) {
  if ((((uintptr_t)p) & 3) == 0) return *reinterpret_cast<const uint32_t*>(p);
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ inline uint64_t ld_u64(const uint8_t* p) {
  if ((((uintptr_t)p) & 7) == 0) return *reinterpret_cast<const uint64_t*>(p);
  return (uint64_t)ld_u32(p) | ((uint64_t)ld_u32(p + 4) << 32);
}

struct RleTable {
  int32_t start[kRunCap + 1];
  uint32_t val[kRunCap];
  int64_t ptr[kRunCap];  // bit-packed run: data address; RLE run: 0
  int64_t cur;
  int32_t done;
  int32_t nruns;
  int32_t err;
};

// Decode `count` values of an RLE / bit-packed hybrid stream [p, end) with bit
// width bw (0..32). sink(i, v) runs once per value index i in [0, count), on
// some lane of the block. Must be called by every lane; ends synchronised.
template <typename Sink>
__device__ bool rle_decode(const uint8_t* p, const uint8_t* end, int bw, int count, RleTable& t, Sink sink) {
  const int nbytes = (bw + 7) >> 3;
  const uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1u);
  if (threadIdx.x == 0) {
    t.cur = (int64_t)p;
    t.done = 0;
    t.err = 0;
  }
  __syncthreads();
  for (;;) {
    if (threadIdx.x == 0) {
      const uint8_t* q = (const uint8_t*)t.cur;
      int done = t.done, nr = 0;
      while (nr < kRunCap && done < count) {
        uint32_t h = 0;
        int sh = 0;
        bool ok = false;
        while (q < end && sh <= 28) {
          const uint8_t b = *q++;
          h |= (uint32_t)(b & 0x7f) << sh;
          if (!(b & 0x80)) {
            ok = true;
            break;
          }
          sh += 7;
        }
        if (!ok) {
          t.err = 1;
          break;
        }
        const int64_t left = count - done;
        int64_t n;
        t.start[nr] = done;
        if (h & 1) {
          const int64_t groups = h >> 1;
          n = groups * 8;
          const int64_t bytes = groups * bw;
          const int64_t need = left < n ? left : n;
          if (bw > 0 && (int64_t)(end - q) * 8 < need * bw) {  // truncated run
            t.err = 1;
            break;
          }
          t.ptr[nr] = bw > 0 ? (int64_t)q : 0;
          t.val[nr] = 0;
          q += bytes < (int64_t)(end - q) ? bytes : (int64_t)(end - q);
        } else {
          n = h >> 1;
          if (n == 0 || q + nbytes > end) {
            t.err = 1;
            break;
          }
          uint32_t v = 0;
          for (int b = 0; b < nbytes; ++b) v |= (uint32_t)q[b] << (8 * b);
          q += nbytes;
          t.ptr[nr] = 0;
          t.val[nr] = v & mask;
        }
        done += (int)(left < n ? left : n);
        ++nr;
      }
      t.start[nr] = done;
      t.nruns = nr;
      t.cur = (int64_t)q;
      t.done = done;
    }
    __syncthreads();
    const int nr = t.nruns;
    const int lo = t.start[0], hi = t.start[nr];
    if (t.err) return false;
    for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) {
      int a = 0, b = nr - 1;
      while (a < b) {
        const int m = (a + b + 1) >> 1;
        if (t.start[m] <= i) a = m;
        else b = m - 1;
      }
      uint32_t v;
      if (t.ptr[a] == 0) {
        v = t.val[a];
      } else {
        const int64_t bit = (int64_t)(i - t.start[a]) * bw;
        const uint8_t* q = (const uint8_t*)t.ptr[a] + (bit >> 3);
        const int sh = (int)(bit & 7);
        const int nb = (sh + bw + 7) >> 3;
        uint64_t w = 0;
        for (int k = 0; k < nb; ++k) w |= (uint64_t)q[k] << (8 * k);
        v = (uint32_t)(w >> sh) & mask;
      }
      sink(i, v);
    }
    const bool fin = hi >= count || nr == 0;
    __syncthreads();
    if (fin) return true;
  }
}

struct WalkState {
  int64_t pos;
  int32_t j;
  int32_t err;
};

// Positions of `count` PLAIN BYTE_ARRAY values (4-byte little-endian length +
// bytes) in [p, end). The stream is walked by lane 0 over 8 KiB LDS windows
// the whole block stages. sink(j, offset_of_bytes, length) runs on lane 0.
template <typename Sink>
__device__ bool walk_byte_array(const uint8_t* p, const uint8_t* end, int count, uint8_t* win, WalkState& w,
                                Sink sink) {
  const int64_t size = end - p;
  if (threadIdx.x == 0) {
    w.pos = 0;
    w.j = 0;
    w.err = 0;
  }
  __syncthreads();
  for (;;) {
    const int64_t wbeg = w.pos;
    const int j0 = w.j;
    if (w.err || j0 >= count) break;
    if (wbeg + 4 > size) {
      __syncthreads();
      return false;
    }
    const int64_t wlen = size - wbeg < kWalkWin ? size - wbeg : kWalkWin;
    for (int64_t k = threadIdx.x; k < wlen; k += blockDim.x) win[k] = p[wbeg + k];
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t pos = wbeg;
      int j = j0;
      while (j < count && pos + 4 <= wbeg + wlen) {
        const uint8_t* q = win + (pos - wbeg);
        const uint32_t len =
            (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        if ((int64_t)len > size - pos - 4) {
          w.err = 1;
          break;
        }
        sink(j, (uint32_t)(pos + 4), len);
        pos += 4 + (int64_t)len;
        ++j;
      }
      w.pos = pos;
      w.j = j;
    }
    __syncthreads();
  }
  const bool ok = w.err == 0;
  __syncthreads();
  return ok;
}

// DELTA_BINARY_PACKED (parquet Encodings.md): a header <block size> <miniblocks
// per block> <value count> <first value>, then per block a zigzag min delta,
// one bit width per miniblock and the bit-packed miniblocks. Thread 0 walks
// the block headers (up to kDbpCap miniblocks per round) into LDS; then every
// lane unpacks one delta (binary search for its miniblock) and a block-wide
// scan turns deltas into values, carried from round to round.
constexpr int kDbpCap = 256;
struct DbpTable {
  int64_t mb_ptr[kDbpCap];
  uint64_t mb_min[kDbpCap];
  int32_t mb_first[kDbpCap + 1];
  uint8_t mb_bw[kDbpCap];
  int64_t cur, bw_ptr, end;
  uint64_t first, blk_min;
  int32_t mpb, vpm, total, in_block, done, nmb, err;
};

__device__ inline bool uleb(const uint8_t*& q, const uint8_t* end, uint64_t* v) {
  uint64_t x = 0;
  for (int sh = 0; sh < 64 && q < end; sh += 7) {
    const uint8_t b = *q++;
    x |= (uint64_t)(b & 0x7f) << sh;
    if (!(b & 0x80)) {
      *v = x;
      return true;
    }
  }
  return false;
}

__device__ inline uint64_t unpack_bits(const uint8_t* p, int64_t bit, int bw) {
  if (bw == 0) return 0;
  const uint8_t* q = p + (bit >> 3);
  const int sh = (int)(bit & 7);
  const int nb = (sh + bw + 7) >> 3;
  uint64_t lo = 0;
  for (int k = 0; k < nb && k < 8; ++k) lo |= (uint64_t)q[k] << (8 * k);
  uint64_t v = lo >> sh;
  if (nb > 8) v |= (uint64_t)q[8] << (64 - sh);
  return bw >= 64 ? v : v & ((1ull << bw) - 1ull);
}

// Decodes `count` values of a DELTA_BINARY_PACKED stream at [p, end):
// out(i, value) once per value (some lane); returns the end of the stream (or
// nullptr when malformed). Call with every thread of the block.
template <typename Out>
__device__ const uint8_t* dbp_decode(const uint8_t* p, const uint8_t* end, int count, DbpTable& d, int64_t* scan_ws,
                                     Out out) {
  if (threadIdx.x == 0) {
    const uint8_t* q = p;
    uint64_t bs = 0, mpb = 0, total = 0, first = 0;
    d.err = !(uleb(q, end, &bs) && uleb(q, end, &mpb) && uleb(q, end, &total) && uleb(q, end, &first));
    // mpb <= bs keeps values-per-miniblock >= 1 (0 % 32 == 0 would pass);
    // the caps keep both in int32 (a negative mpb would move q backwards)
    if (!d.err && (mpb == 0 || bs == 0 || mpb > bs || bs > (1u << 20) || mpb > kDbpCap || bs % 128 != 0 ||
                   bs / mpb == 0 || (bs / mpb) % 32 != 0 || (int64_t)total != count))
      d.err = 1;
    d.mpb = (int32_t)mpb;
    d.vpm = mpb ? (int32_t)(bs / mpb) : 0;
    d.total = (int32_t)total;
    d.first = (first >> 1) ^ (0 - (first & 1));   // zigzag
    d.cur = (int64_t)q;
    d.end = (int64_t)end;
    d.in_block = d.mpb;
    d.done = 0;
  }
  __syncthreads();
  if (d.err) return nullptr;
  if (count > 0 && threadIdx.x == 0) out(0, d.first);
  const int nd = count > 0 ? count - 1 : 0;
  uint64_t carry = d.first;
  while (d.done < nd) {
    if (threadIdx.x == 0) {
      const uint8_t* q = (const uint8_t*)d.cur;
      int done = d.done, nmb = 0;
      while (nmb < kDbpCap && done < nd && !d.err) {
        if (d.in_block == d.mpb) {
          uint64_t z;
          if (!uleb(q, end, &z) || q + d.mpb > end) {
            d.err = 1;
            break;
          }
          d.blk_min = (z >> 1) ^ (0 - (z & 1));
          d.bw_ptr = (int64_t)q;
          q += d.mpb;
          d.in_block = 0;
        }
        const int bw = ((const uint8_t*)d.bw_ptr)[d.in_block];
        const int n = nd - done < d.vpm ? nd - done : d.vpm;
        if (bw > 64 || q + (((int64_t)n * bw + 7) >> 3) > end) {
          d.err = 1;
          break;
        }
        d.mb_ptr[nmb] = (int64_t)q;
        d.mb_min[nmb] = d.blk_min;
        d.mb_bw[nmb] = (uint8_t)bw;
        d.mb_first[nmb] = done;
        const int64_t full = ((int64_t)d.vpm * bw) >> 3;
        q = q + full <= end ? q + full : end;   // the last miniblock may stop at the stream end
        ++d.in_block;
        done += n;
        ++nmb;
      }
      d.mb_first[nmb] = done;
      d.nmb = nmb;
      d.cur = (int64_t)q;
    }
    __syncthreads();
    if (d.err) return nullptr;
    const int nmb = d.nmb, lo = d.mb_first[0], hi = d.mb_first[nmb];
    for (int base = lo; base < hi; base += kBlock) {
      const int i = base + (int)threadIdx.x;
      uint64_t dl = 0;
      if (i < hi) {
        int a = 0, b = nmb - 1;
        while (a < b) {
          const int m = (a + b + 1) >> 1;
          if (d.mb_first[m] <= i) a = m;
          else b = m - 1;
        }
        const int bw = d.mb_bw[a];
        dl = d.mb_min[a] + unpack_bits((const uint8_t*)d.mb_ptr[a], (int64_t)(i - d.mb_first[a]) * bw, bw);
      }
      int64_t tot;
      const uint64_t ex = (uint64_t)block_exclusive_scan((int64_t)dl, scan_ws, &tot);
      if (i < hi) out(i + 1, carry + ex + dl);
      carry += (uint64_t)tot;
    }
    __syncthreads();
    if (threadIdx.x == 0) d.done = hi;
    __syncthreads();
  }
  return (const uint8_t*)d.cur;
}

__device__ inline int block_sum_int(int v, int* red) {
  v = (int)wave_reduce_sum((int64_t)v);
  if (lane_id() == 0) red[threadIdx.x / kWave] = v;
  __syncthreads();
  int t = 0;
  for (int w = 0; w < kWavesPerBlock; ++w) t += red[w];
  __syncthreads();
  return t;
}

__device__ inline const uint8_t* data_ptr(const PqPage& pg, const PqDecodeSpec& s) {
  return ((pg.flags & PQ_DATA_IN_DEC) ? s.dec : s.raw) + pg.data_off;
}
__device__ inline const uint8_t* dict_ptr(const PqPage& pg, const PqDecodeSpec& s) {
  return ((pg.flags & PQ_DICT_IN_DEC) ? s.dec : s.raw) + pg.dict_off;
}

// big-endian two's complement (FIXED_LEN_BYTE_ARRAY decimal) -> int64
__device__ inline int64_t flba_to_i64(const uint8_t* p, int len, bool* ovf) {
  if (len <= 8) {
    uint64_t u = 0;
    for (int k = 0; k < len; ++k) u = (u << 8) | p[k];
    const int sh = 64 - 8 * len;
    return sh >= 64 ? 0 : (int64_t)(u << sh) >> sh;
  }
  uint64_t u = 0;
  for (int k = len - 8; k < len; ++k) u = (u << 8) | p[k];
  const int64_t v = (int64_t)u;
  const uint8_t sign = v < 0 ? 0xff : 0;
  for (int k = 0; k < len - 8; ++k)
    if (p[k] != sign) *ovf = true;
  return v;
}

// One output row of a fixed-width column from its source bytes.
__device__ inline void store_fixed(const PqDecodeSpec& s, int64_t row, const uint8_t* src, int* err) {
  switch (s.conv) {
    case PQ_CONV_COPY:
      if (s.out_width == 4) reinterpret_cast<uint32_t*>(s.out)[row] = ld_u32(src);
      else reinterpret_cast<uint64_t*>(s.out)[row] = ld_u64(src);
      break;
    case PQ_CONV_NARROW: {
      const uint32_t v = ld_u32(src);
      if (s.out_width == 1) reinterpret_cast<uint8_t*>(s.out)[row] = (uint8_t)v;
      else reinterpret_cast<uint16_t*>(s.out)[row] = (uint16_t)v;
      break;
    }
    case PQ_CONV_SEXT:
      reinterpret_cast<int64_t*>(s.out)[row] = (int64_t)(int32_t)ld_u32(src);
      break;
    case PQ_CONV_ZEXT:
      reinterpret_cast<int64_t*>(s.out)[row] = (int64_t)ld_u32(src);
      break;
    case PQ_CONV_F2D: {
      const uint32_t b = ld_u32(src);
      float f;
      __builtin_memcpy(&f, &b, 4);
      reinterpret_cast<double*>(s.out)[row] = (double)f;
      break;
    }
    case PQ_CONV_FLBA: {
      bool ovf = false;
      const int64_t v = flba_to_i64(src, s.type_len, &ovf);
      if (ovf) set_error(err, PQ_ERR_DECIMAL);
      reinterpret_cast<int64_t*>(s.out)[row] = v;
      break;
    }
    case PQ_CONV_MUL:
      reinterpret_cast<int64_t*>(s.out)[row] = (int64_t)ld_u64(src) * s.conv_k;
      break;
    case PQ_CONV_DIV:
      reinterpret_cast<int64_t*>(s.out)[row] = (int64_t)ld_u64(src) / s.conv_k;
      break;
    default:
      set_error(err, PQ_ERR_ENCODING);
  }
}

__device__ inline void store_zero(const PqDecodeSpec& s, int64_t row) {
  if (s.phys == PQ_PHYS_BYTE_ARRAY) {
    if (s.codes) {
      s.codes[row] = 0;
    } else {
      s.str_len[row] = 0;
      s.str_pos[row] = 0;
    }
    return;
  }
  switch (s.out_width) {
    case 1: reinterpret_cast<uint8_t*>(s.out)[row] = 0; break;
    case 2: reinterpret_cast<uint16_t*>(s.out)[row] = 0; break;
    case 4: reinterpret_cast<uint32_t*>(s.out)[row] = 0; break;
    default: reinterpret_cast<uint64_t*>(s.out)[row] = 0;
  }
}

__global__ __launch_bounds__(kBlock) void pq_decode_kernel(const PqPage* __restrict__ pages,
                                                           const int32_t* __restrict__ page_col,
                                                           const PqDecodeSpec* __restrict__ specs) {
  __shared__ RleTable rt;
  __shared__ WalkState ws;
  __shared__ uint8_t win[kWalkWin];
  __shared__ int64_t scan_ws[kWavesPerBlock + 1];
  __shared__ int red[kWavesPerBlock];
  __shared__ DbpTable dbp;

  const PqPage pg = pages[blockIdx.x];
  if (pg.kind == PQ_PAGE_DICT) return;
  const PqDecodeSpec s = specs[page_col[blockIdx.x]];
  const int n = pg.num_values;
  const int64_t row0 = pg.out_row;
  const uint8_t* p = data_ptr(pg, s);
  const uint8_t* end = p + pg.size;

  // ---- definition levels -> validity
  int nnz = n;
  if (s.max_def > 0) {
    const uint8_t* lv;
    const uint8_t* lend;
    if (pg.kind == PQ_PAGE_DATA_V2) {
      lv = s.raw + pg.levels_off;
      lend = lv + pg.levels_len;
    } else {
      if (p + 4 > end) {
        if (threadIdx.x == 0) set_error(s.error, PQ_ERR_TRUNCATED);
        return;
      }
      const uint32_t len = ld_u32(p);
      lv = p + 4;
      lend = lv + len;
      if (lend > end) {
        if (threadIdx.x == 0) set_error(s.error, PQ_ERR_TRUNCATED);
        return;
      }
      p = lend;
    }
    const int bw = 32 - __clz(s.max_def);
    int local = 0;
    uint8_t* valid = s.valid ? s.valid + row0 : nullptr;
    const uint32_t md = (uint32_t)s.max_def;
    const bool ok = rle_decode(lv, lend, bw, n, rt, [&](int i, uint32_t v) {
      const uint8_t f = v == md;
      if (valid) valid[i] = f;
      local += f;
    });
    if (!ok) {
      if (threadIdx.x == 0) set_error(s.error, PQ_ERR_RLE);
      return;
    }
    nnz = block_sum_int(local, red);
    if (!s.valid && nnz != n) {
      if (threadIdx.x == 0) set_error(s.error, PQ_ERR_NULLS);
      return;
    }
  }
  const bool has_nulls = nnz != n;

  // ---- values -> compact index j (dictionary index / bool / byte-array offset)
  const int enc = pg.encoding;
  const bool dict = enc == 2 || enc == 8;
  const bool bool_rle = s.phys == PQ_PHYS_BOOLEAN && enc == 3;
  const bool str_plain = s.phys == PQ_PHYS_BYTE_ARRAY && !dict;
  const bool dlba = enc == 6;
  uint32_t* idx = s.scratch + row0;
  const int w_in = (s.phys == PQ_PHYS_INT32 || s.phys == PQ_PHYS_FLOAT) ? 4
                   : s.phys == PQ_PHYS_FLBA                             ? s.type_len
                                                                        : 8;
  uint8_t* aux = pg.aux_off >= 0 ? const_cast<uint8_t*>(s.dec) + pg.aux_off : nullptr;   // this page's own slot
  if (nnz > 0) {
    bool ok = true;
    if ((enc == 5 || enc == 6 || enc == 9) && !aux) {
      ok = false;
    } else if (enc == 5) {
      // DELTA_BINARY_PACKED ints -> plain little-endian values in the aux slot
      const bool w4 = w_in == 4;
      ok = dbp_decode(p, end, nnz, dbp, scan_ws, [&](int i, uint64_t v) {
             if (w4) reinterpret_cast<uint32_t*>(aux)[i] = (uint32_t)v;
             else reinterpret_cast<uint64_t*>(aux)[i] = v;
           }) != nullptr;
      __syncthreads();
      p = aux;
      end = aux + (int64_t)nnz * w_in;
    } else if (enc == 6) {
      // DELTA_LENGTH_BYTE_ARRAY: lengths (DELTA_BINARY_PACKED) -> aux, then the
      // concatenated bytes; idx[j] = offset of value j's bytes from p
      const uint8_t* bytes = dbp_decode(p, end, nnz, dbp, scan_ws, [&](int i, uint64_t v) {
        reinterpret_cast<uint32_t*>(aux)[i] = (uint32_t)v;
      });
      __syncthreads();
      ok = bytes != nullptr;
      if (ok) {
        int64_t carry = bytes - p;
        for (int b0 = 0; b0 < nnz; b0 += kBlock) {
          const int j = b0 + (int)threadIdx.x;
          const int64_t len = j < nnz ? (int64_t)reinterpret_cast<const int32_t*>(aux)[j] : 0;
          int64_t tot;
          const int64_t ex = block_exclusive_scan(len < 0 ? 0 : len, scan_ws, &tot);
          if (j < nnz) idx[j] = (uint32_t)(carry + ex);
          carry += tot;
          if (len < 0) ok = false;
        }
        ok = __syncthreads_and(ok) && carry <= end - p;
      }
    } else if (enc == 9) {
      // BYTE_STREAM_SPLIT: byte k of value j at p[k * nnz + j] -> plain values in aux
      ok = p + (int64_t)w_in * nnz <= end;
      if (ok)
        for (int64_t t = threadIdx.x; t < (int64_t)w_in * nnz; t += kBlock) {
          const int64_t j = t / w_in, k = t - j * w_in;
          aux[t] = p[k * nnz + j];
        }
      __syncthreads();
      p = aux;
      end = aux + (int64_t)nnz * w_in;
    } else if (dict) {
      if (p >= end) {
        ok = false;
      } else {
        const int bw = *p;
        ok = bw <= 32 && rle_decode(p + 1, end, bw, nnz, rt, [&](int j, uint32_t v) { idx[j] = v; });
      }
    } else if (bool_rle) {
      if (p + 4 > end) {
        ok = false;
      } else {
        const uint32_t len = ld_u32(p);
        ok = p + 4 + len <= end &&
             rle_decode(p + 4, p + 4 + len, 1, nnz, rt, [&](int j, uint32_t v) { idx[j] = v; });
      }
    } else if (enc != 0) {
      if (threadIdx.x == 0) set_error(s.error, PQ_ERR_ENCODING);
      return;
    } else if (str_plain && !dlba) {
      if (!walk_byte_array(p, end, nnz, win, ws, [&](int j, uint32_t off, uint32_t) { idx[j] = off; })) {
        if (threadIdx.x == 0) set_error(s.error, PQ_ERR_BYTE_ARRAY);
        return;
      }
    }
    if (!ok) {
      if (threadIdx.x == 0) set_error(s.error, PQ_ERR_RLE);
      return;
    }
  }
  __syncthreads();

  // ---- rows: compact value index j = number of valid rows before row i
  const uint8_t* dp = dict ? dict_ptr(pg, s) : nullptr;
  const uint32_t dcount = (uint32_t)pg.dict_count;
  int64_t carry = 0;
  for (int base = 0; base < n; base += kBlock * kItems) {
    const int i0 = base + (int)threadIdx.x * kItems;
    int f[kItems];
    int cnt = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int i = i0 + k;
      f[k] = i < n ? (has_nulls ? (int)s.valid[row0 + i] : 1) : 0;
      cnt += f[k];
    }
    int64_t j;
    if (has_nulls) {
      int64_t tot;
      j = carry + block_exclusive_scan(cnt, scan_ws, &tot);
      carry += tot;
    } else {
      j = i0;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int i = i0 + k;
      if (i >= n) break;
      const int64_t row = row0 + i;
      if (!f[k]) {
        store_zero(s, row);
        continue;
      }
      if (s.phys == PQ_PHYS_BYTE_ARRAY) {
        if (dict) {
          const uint32_t d = idx[j];
          if (d >= dcount) {
            set_error(s.error, PQ_ERR_DICT_INDEX);
            store_zero(s, row);
          } else if (s.codes) {
            s.codes[row] = pg.dict_base + (int32_t)d;
          } else {
            s.str_len[row] = s.dict_len[pg.dict_base + d];
            s.str_pos[row] = s.dict_pos[pg.dict_base + d];
          }
        } else {
          const uint32_t off = idx[j];
          s.str_len[row] = dlba ? (int64_t)reinterpret_cast<const int32_t*>(aux)[j] : (int64_t)ld_u32(p + off - 4);
          s.str_pos[row] = (int64_t)(p + off);
        }
      } else if (s.phys == PQ_PHYS_BOOLEAN) {
        uint8_t v;
        if (bool_rle) v = (uint8_t)(idx[j] & 1);
        else v = (p + (j >> 3) < end) ? (uint8_t)((p[j >> 3] >> (j & 7)) & 1) : 0;
        reinterpret_cast<uint8_t*>(s.out)[row] = v;
      } else if (dict) {
        const uint32_t d = idx[j];
        if (d >= dcount) {
          set_error(s.error, PQ_ERR_DICT_INDEX);
          store_zero(s, row);
        } else {
          store_fixed(s, row, dp + (int64_t)d * w_in, s.error);
        }
      } else {
        const uint8_t* src = p + j * w_in;
        if (src + w_in > end) {
          set_error(s.error, PQ_ERR_TRUNCATED);
          store_zero(s, row);
        } else {
          store_fixed(s, row, src, s.error);
        }
      }
      ++j;
    }
  }
}

__global__ __launch_bounds__(kBlock) void pq_dict_strings_kernel(const PqPage* __restrict__ pages,
                                                                 const int32_t* __restrict__ page_col,
                                                                 const PqDecodeSpec* __restrict__ specs) {
  __shared__ WalkState ws;
  __shared__ uint8_t win[kWalkWin];
  const PqPage pg = pages[blockIdx.x];
  if (pg.kind != PQ_PAGE_DICT) return;
  const PqDecodeSpec s = specs[page_col[blockIdx.x]];
  if (s.phys != PQ_PHYS_BYTE_ARRAY || !s.dict_len) return;
  const uint8_t* p = data_ptr(pg, s);
  const uint8_t* end = p + pg.size;
  int64_t* dl = s.dict_len + pg.dict_base;
  int64_t* dpos = s.dict_pos + pg.dict_base;
  const bool ok = walk_byte_array(p, end, pg.num_values, win, ws, [&](int j, uint32_t off, uint32_t len) {
    dl[j] = len;
    dpos[j] = (int64_t)(p + off);
  });
  if (!ok && threadIdx.x == 0) set_error(s.error, PQ_ERR_BYTE_ARRAY);
}

// One wave per compressed page, decoding a BATCH of snappy elements per step:
//   1. speculative parse: lane k assumes an element starts k bytes into the
//      64-byte step window and computes its size, output length and offset
//      from the LDS input window;
//   2. scalar walk: starting at lane 0, the true element starts are chained
//      with readlane (SALU), giving a 64-bit mask of element lanes;
//   3. output offsets: wave prefix sum of the element lengths;
//   4. copy: literals and matches whose source lies before the batch are
//      independent -> every such lane copies its own element in parallel;
//      matches that read output of this batch are then copied in order, each
//      by the whole wave (64 bytes per step).
// Back-references read a 16 KiB LDS history ring, or — beyond it — the
// already written output (ordered after this wave's stores by a wait).
// A literal too long for the window streams through it on its own. Page
// sizes are < 2 GiB, so positions are 32-bit.
constexpr int kSnapRingS = 16384;
constexpr int kSnapInS = 4096;
// a batch writes at most one window-sized literal plus 32 short matches:
// independent ring reads closer than this never alias the batch's own writes
constexpr int kSnapFarRing = kSnapRingS - kSnapInS - 2048 - 64;

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__global__ __launch_bounds__(64) void pq_snappy_kernel(const PqSnappyJob* __restrict__ jobs,
                                                       const uint8_t* __restrict__ raw, uint8_t* __restrict__ dec,
                                                       int* __restrict__ err) {
  __shared__ uint8_t ring[kSnapRingS];
  __shared__ uint8_t inw[kSnapInS + 8];
  const PqSnappyJob jb = jobs[blockIdx.x];
  if (jb.codec != PQ_CODEC_SNAPPY) return;   // (ZSTD pages: pq_zstd)
  const uint8_t* src = raw + jb.src_off;
  const int slen = uni(jb.src_len);
  uint8_t* dst = dec + jb.dst_off;
  const int dlen = uni(jb.dst_len);
  const int lane = threadIdx.x;
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  int wbeg = 0, wend = 0;

  auto refill = [&](int at) {
    __syncthreads();
    wbeg = at;
    wend = slen < at + kSnapInS ? slen : at + kSnapInS;
    const int cnt = wend - wbeg;
    if (((((uintptr_t)(src + wbeg)) & 3) == 0)) {
      for (int k = 4 * lane; k < cnt; k += 256) {
        if (k + 4 <= cnt) {
          *reinterpret_cast<uint32_t*>(inw + k) = *reinterpret_cast<const uint32_t*>(src + wbeg + k);
        } else {
          for (int t = k; t < cnt; ++t) inw[t] = src[wbeg + t];
        }
      }
    } else {
      for (int k = lane; k < cnt; k += 64) inw[k] = src[wbeg + k];
    }
    __syncthreads();
  };
  auto fail = [&](int code) {
    if (lane == 0) set_error(err, code);
  };
  refill(0);
  int ip = 0;
  uint32_t ulen = 0;
  for (int sh = 0;; sh += 7) {
    if (ip >= wend || sh > 28) return fail(PQ_ERR_SNAPPY);
    const uint32_t b = (uint32_t)uni(inw[ip++ - wbeg]);
    ulen |= (b & 0x7f) << sh;
    if (!(b & 0x80)) break;
  }
  if ((int)ulen != dlen) return fail(PQ_ERR_SNAPPY_SIZE);
  int op = 0;
  while (ip < slen) {
    if (ip + 128 > wend && wend < slen) refill(ip);
    // ---- 1. speculative parse at ip + lane
    const int P = ip + lane;                 // absolute input position of this lane's candidate
    const int avail = wend - P;              // window bytes from P on
    int sz = 1 << 30, olen = 0, off = 0, lsrc = 0;
    bool lit = false;
    if (avail > 0) {
      const uint8_t* w = inw + (P - wbeg);
      const uint32_t t = w[0];
      const uint32_t b1 = avail > 1 ? w[1] : 0, b2 = avail > 2 ? w[2] : 0;
      const uint32_t b3 = avail > 3 ? w[3] : 0, b4 = avail > 4 ? w[4] : 0;
      const int kind = t & 3;
      if (kind == 0) {
        int L = (int)(t >> 2) + 1, hdr = 1;
        if (L > 60) {
          const int nb = L - 60;
          uint32_t l = b1;
          if (nb > 1) l |= b2 << 8;
          if (nb > 2) l |= b3 << 16;
          if (nb > 3) l |= b4 << 24;
          L = (int)l + 1;
          hdr = 1 + nb;
        }
        lit = true;
        olen = L;
        lsrc = P + hdr;
        sz = (L > 0 && L < (1 << 29)) ? hdr + L : (1 << 30);
      } else if (kind == 1) {
        olen = (int)((t >> 2) & 7) + 4;
        off = (int)(((t >> 5) << 8) | b1);
        sz = 2;
      } else if (kind == 2) {
        olen = (int)(t >> 2) + 1;
        off = (int)(b1 | (b2 << 8));
        sz = 3;
      } else {
        olen = (int)(t >> 2) + 1;
        const uint32_t o = b1 | (b2 << 8) | (b3 << 16) | (b4 << 24);
        off = o > 0x7fffffffu ? 0 : (int)o;
        sz = 5;
      }
      if (sz > avail) sz = 1 << 30;   // not entirely inside the window
    }
    // ---- 2. scalar walk over the true element starts
    uint64_t starts = 0;
    int pos = 0;
    while (pos < 64) {
      const int s = __builtin_amdgcn_readlane(sz, pos);
      if (s >= (1 << 30) || ip + pos + s > slen) break;
      starts |= 1ull << pos;
      pos += s;
    }
    if (starts == 0) {
      // the element at ip does not fit the window: a long literal, streamed
      const uint32_t t = (uint32_t)uni(inw[ip - wbeg]);
      if ((t & 3) != 0 || !uni((int)lit)) return fail(PQ_ERR_SNAPPY);
      const int L = uni(olen), hdr = uni(lsrc) - ip;
      if (L <= 0 || ip + hdr + L > slen || op + L > dlen) return fail(PQ_ERR_SNAPPY);
      ip += hdr;
      int done = 0;
      while (done < L) {
        if (ip + done >= wend) refill(ip + done);
        const int av = uni((wend - (ip + done)) < (L - done) ? (wend - (ip + done)) : (L - done));
        const uint8_t* w = inw + (ip + done - wbeg);
        for (int k = lane; k < av; k += 64) {
          const uint8_t v = w[k];
          dst[op + done + k] = v;
          ring[(op + done + k) & (kSnapRingS - 1)] = v;
        }
        done += av;
      }
      ip += L;
      op += L;
      continue;
    }
    // ---- 3. output offsets of the element lanes
    const bool is_el = (starts >> lane) & 1ull;
    int mylen = is_el ? olen : 0;
    int inc = mylen;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    const int total = __builtin_amdgcn_readlane(inc, 63);
    const int o = op + inc - mylen;          // this element's output position
    bool bad = is_el && (o + olen > dlen || (!lit && (off <= 0 || off > o)));
    if (__ballot(bad)) return fail(PQ_ERR_SNAPPY);
    // ---- 4a. independent elements, one lane each
    const bool dep = is_el && !lit && (o - off + olen > op);
    const bool far = is_el && !lit && !dep && off > kSnapFarRing;
    if (__ballot(far)) {
      __builtin_amdgcn_s_waitcnt(0);
      __threadfence_block();
    }
    if (is_el && !dep) {
      if (lit) {
        const uint8_t* w = inw + (lsrc - wbeg);
        for (int b = 0; b < olen; ++b) {
          const uint8_t v = w[b];
          dst[o + b] = v;
          ring[(o + b) & (kSnapRingS - 1)] = v;
        }
      } else if (!far) {
        for (int b = 0; b < olen; ++b) {
          const uint8_t v = ring[(o - off + b) & (kSnapRingS - 1)];
          dst[o + b] = v;
          ring[(o + b) & (kSnapRingS - 1)] = v;
        }
      } else {
        for (int b = 0; b < olen; ++b) {
          const uint8_t v = __builtin_nontemporal_load(dst + (o - off + b));
          dst[o + b] = v;
          ring[(o + b) & (kSnapRingS - 1)] = v;
        }
      }
    }
    // ---- 4b. elements that read this batch's output, in order, whole wave each
    uint64_t deps = __ballot(dep);
    while (deps) {
      const int k = __builtin_ctzll(deps);
      deps &= deps - 1;
      const int eo = __builtin_amdgcn_readlane(o, k);
      const int el = __builtin_amdgcn_readlane(olen, k);
      const int eoff = __builtin_amdgcn_readlane(off, k);
      if (lane < el) {
        const int from = eo - eoff + (eoff >= el ? lane : lane % eoff);
        const uint8_t v = ring[from & (kSnapRingS - 1)];
        dst[eo + lane] = v;
        ring[(eo + lane) & (kSnapRingS - 1)] = v;
      }
    }
    ip += pos;
    op += total;
  }
  if (op != dlen) fail(PQ_ERR_SNAPPY_SIZE);
}

__global__ __launch_bounds__(kBlock) void pq_str_copy_kernel(const int64_t* __restrict__ pos,
                                                             const int64_t* __restrict__ off, int64_t n,
                                                             uint8_t* __restrict__ out) {
  // one wave copies 64 consecutive strings, its lanes striding over each string's bytes
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
  for (int64_t r0 = wave * kWave; r0 < n; r0 += nwaves * kWave) {
    const int64_t r1 = r0 + kWave < n ? r0 + kWave : n;
    for (int64_t r = r0; r < r1; ++r) {
      const uint8_t* sp = reinterpret_cast<const uint8_t*>(pos[r]);
      const int64_t o = off[r], len = off[r + 1] - o;
      for (int64_t k = lane; k < len; k += kWave) out[o + k] = sp[k];
    }
  }
}

}  // namespace

void pq_snappy(const PqSnappyJob* jobs, int64_t njobs, const uint8_t* raw, uint8_t* dec, int* error,
               hipStream_t stream) {
  if (njobs <= 0) return;
  hipLaunchKernelGGL(pq_snappy_kernel, dim3((unsigned)njobs), dim3(64), 0, stream, jobs, raw, dec, error);
  check_launch("pq_snappy", stream);
}

void pq_dict_strings(const PqPage* pages, int64_t npages, const int32_t* page_col, const PqDecodeSpec* specs,
                     hipStream_t stream) {
  if (npages <= 0) return;
  hipLaunchKernelGGL(pq_dict_strings_kernel, dim3((unsigned)npages), dim3(kBlock), 0, stream, pages, page_col, specs);
  check_launch("pq_dict_strings", stream);
}

void pq_decode(const PqPage* pages, int64_t npages, const int32_t* page_col, const PqDecodeSpec* specs,
               hipStream_t stream) {
  if (npages <= 0) return;
  hipLaunchKernelGGL(pq_decode_kernel, dim3((unsigned)npages), dim3(kBlock), 0, stream, pages, page_col, specs);
  check_launch("pq_decode", stream);
}

void pq_str_copy(const int64_t* pos, const int64_t* off, int64_t n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return;
  const unsigned grid = grid_for(n, kBlock, 8192);
  hipLaunchKernelGGL(pq_str_copy_kernel, dim3(grid), dim3(kBlock), 0, stream, pos, off, n, out);
  check_launch("pq_str_copy", stream);
}

}  // namespace kern
}  // namespace igloo
