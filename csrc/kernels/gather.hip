// Index gathers for late materialisation after joins, filters and sorts.
//
// Replaces the reference's per-pair RecordBatch concatenation
// (reference crates/engine/src/operators/hash_join.rs:221-240 combine_batches,
// :242-280 combine_with_nulls) with one launch that reads the index vector
// once and gathers up to kMaxGatherCols fixed-width columns. A negative index
// produces a NULL row (outer-join padding).
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

struct GatherParams {
  int ncols;
  GatherDesc d[kMaxGatherCols];
};

// Read by the loads of a column whose source is empty (null pointer): every
// index of such a column is negative, and the kernel loads unconditionally.
__device__ __attribute__((aligned(16))) uint8_t g_gather_zero[64];

constexpr int kGatherRows = 4;   // rows per lane

template <typename T, int kRows>
__device__ inline void gather_col(const void* src_, void* dst_, const int64_t (&s)[kRows], const int64_t (&i)[kRows],
                                  int64_t n, int64_t rows) {
  const T* __restrict__ src = static_cast<const T*>(src_);
  T* __restrict__ dst = static_cast<T*>(dst_);
  T v[kRows];
#pragma unroll
  for (int r = 0; r < kRows; ++r) v[r] = (uint64_t)s[r] < (uint64_t)rows ? src[s[r]] : T{};
#pragma unroll
  for (int r = 0; r < kRows; ++r)
    if (i[r] < n) dst[i[r]] = v[r];
}

// Rows base + r * blockDim (r < kGatherRows) per lane, every column in one
// launch: every store of a column follows all of that column's loads, so a
// lane keeps kGatherRows random reads in flight instead of one load->store
// round trip per value. (A variant grouping up to 4 columns of one element
// type per launch, every load unconditional, measured within 1% over the
// SF100 suite -- profiles/r3_ab_gather_grouped.txt -- and was removed.)
template <typename I, int kGatherRows>
__global__ __launch_bounds__(kBlock) void gather_percol_kernel(const I* __restrict__ idx, int64_t n, GatherParams p) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * kGatherRows;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * kGatherRows + threadIdx.x; base < n; base += step) {
    int64_t i[kGatherRows], s[kGatherRows];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r) {
      i[r] = base + (int64_t)r * blockDim.x;
      s[r] = i[r] < n ? (int64_t)idx[i[r]] : -1;
    }
    for (int c = 0; c < p.ncols; ++c) {
      const GatherDesc& d = p.d[c];
      switch (d.elem_bytes) {
        case 1: gather_col<uint8_t, kGatherRows>(d.src, d.dst, s, i, n, d.src_rows); break;
        case 2: gather_col<uint16_t, kGatherRows>(d.src, d.dst, s, i, n, d.src_rows); break;
        case 4: gather_col<uint32_t, kGatherRows>(d.src, d.dst, s, i, n, d.src_rows); break;
        case 8: gather_col<uint64_t, kGatherRows>(d.src, d.dst, s, i, n, d.src_rows); break;
        case 16: gather_col<uint4, kGatherRows>(d.src, d.dst, s, i, n, d.src_rows); break;
      }
      if (d.dst_valid) {
        const uint8_t* __restrict__ sv = d.src_valid;
        uint8_t* __restrict__ dv = d.dst_valid;
        uint8_t v[kGatherRows];
#pragma unroll
        for (int r = 0; r < kGatherRows; ++r) v[r] = (uint64_t)s[r] < (uint64_t)d.src_rows && (!sv || sv[s[r]]);
#pragma unroll
        for (int r = 0; r < kGatherRows; ++r)
          if (i[r] < n) dv[i[r]] = v[r];
      }
    }
  }
}

struct PackedParams {
  const uint8_t* src;
  int64_t rows;
  int nf;
  PackedField f[kMaxPackedFields];
};

// word k of a row held in registers (compare-select: no dynamic register indexing)
template <int W>
__device__ inline uint64_t pick_word(const uint64_t (&w)[W], int k) {
  uint64_t x = w[0];
#pragma unroll
  for (int j = 1; j < W; ++j) x = k == j ? w[j] : x;
  return x;
}

// kGatherRows rows per lane, each row's W words loaded before any field is
// split out (16-byte loads for 16/32-byte rows), then every field of every
// row stored: one cache line per gathered row for all its fields.
template <typename I, int W>
__global__ __launch_bounds__(kBlock) void gather_packed_kernel(const I* __restrict__ idx, int64_t n, PackedParams p) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x * kGatherRows;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * kGatherRows + threadIdx.x; base < n; base += step) {
    int64_t i[kGatherRows];
    bool ok[kGatherRows];
    uint64_t w[kGatherRows][W];
#pragma unroll
    for (int r = 0; r < kGatherRows; ++r) {
      i[r] = base + (int64_t)r * blockDim.x;
      const int64_t s = i[r] < n ? (int64_t)idx[i[r]] : -1;
      ok[r] = (uint64_t)s < (uint64_t)p.rows;
      const int64_t at = ok[r] ? s : 0;
      if constexpr (W % 2 == 0) {
        const ulonglong2* row = reinterpret_cast<const ulonglong2*>(p.src) + at * (W / 2);
#pragma unroll
        for (int k = 0; k < W / 2; ++k) {
          const ulonglong2 v = ok[r] ? row[k] : ulonglong2{0, 0};
          w[r][2 * k] = v.x;
          w[r][2 * k + 1] = v.y;
        }
      } else {
        const uint64_t* row = reinterpret_cast<const uint64_t*>(p.src) + at * W;
#pragma unroll
        for (int k = 0; k < W; ++k) w[r][k] = ok[r] ? row[k] : 0;
      }
    }
    for (int f = 0; f < p.nf; ++f) {
      const PackedField d = p.f[f];
      const int word = d.off >> 3, sh = (d.off & 7) * 8, bits = d.width * 8;
      uint64_t v[kGatherRows];
#pragma unroll
      for (int r = 0; r < kGatherRows; ++r) {
        uint64_t x = pick_word<W>(w[r], word) >> sh;
        if (bits < 64) {
          x &= (1ull << bits) - 1;
          if (d.flags & kPackedSigned) x = (uint64_t)((int64_t)(x << (64 - bits)) >> (64 - bits));
        }
        v[r] = (d.flags & kPackedInRange) ? (uint64_t)ok[r] : x;
      }
#pragma unroll
      for (int r = 0; r < kGatherRows; ++r) {
        if (i[r] >= n) continue;
        switch (d.out_bytes) {
          case 1: static_cast<uint8_t*>(d.dst)[i[r]] = (uint8_t)v[r]; break;
          case 2: static_cast<uint16_t*>(d.dst)[i[r]] = (uint16_t)v[r]; break;
          case 4: static_cast<uint32_t*>(d.dst)[i[r]] = (uint32_t)v[r]; break;
          default: static_cast<uint64_t*>(d.dst)[i[r]] = v[r]; break;
        }
      }
    }
  }
}

template <typename I>
__global__ __launch_bounds__(kBlock) void str_lengths_kernel(const int64_t* __restrict__ off, int64_t rows,
                                                            const I* __restrict__ idx, int64_t n,
                                                            int64_t* __restrict__ len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = idx ? (int64_t)idx[i] : i;
    len[i] = (uint64_t)s < (uint64_t)rows ? off[s + 1] - off[s] : 0;
  }
}

// 8 lanes cooperate on one string: each step moves 8 bytes per lane.
// out_cap: bytes the output holds (sized by a possibly replayed total): a
// string that would end past it is skipped, never written out of bounds
template <typename I>
__global__ __launch_bounds__(kBlock) void str_copy_kernel(const int64_t* __restrict__ off, int64_t rows,
                                                         const uint8_t* __restrict__ chars,
                                                         const I* __restrict__ idx, int64_t n,
                                                         const int64_t* __restrict__ new_off, uint8_t* __restrict__ out,
                                                         int64_t out_cap) {
  const int sub = threadIdx.x & 7;
  const int64_t rows_per_block = kBlock / 8;
  for (int64_t r = blockIdx.x * rows_per_block + threadIdx.x / 8; r < n; r += (int64_t)gridDim.x * rows_per_block) {
    int64_t s = idx ? (int64_t)idx[r] : r;
    if ((uint64_t)s >= (uint64_t)rows) continue;
    int64_t src = off[s], len = off[s + 1] - src, dst = new_off[r];
    if (dst < 0 || len < 0 || dst + len > out_cap) continue;
    for (int64_t b = sub; b < len; b += 8) out[dst + b] = chars[src + b];
  }
}

}  // namespace

void gather_multi(const void* idx, bool idx64, int64_t n, const GatherDesc* descs, int ncols, hipStream_t stream) {
  if (n == 0 || ncols == 0) return;
  for (int c = 0; c < ncols; ++c) {
    const int eb = descs[c].elem_bytes;
    if (eb != 1 && eb != 2 && eb != 4 && eb != 8 && eb != 16)
      throw std::runtime_error("gather_multi: unsupported element size " + std::to_string(eb));
  }
  // every column of the request in one launch (kMaxGatherCols per launch)
  for (int base = 0; base < ncols; base += kMaxGatherCols) {
    GatherParams p;
    p.ncols = ncols - base < kMaxGatherCols ? ncols - base : kMaxGatherCols;
    for (int c = 0; c < p.ncols; ++c) p.d[c] = descs[base + c];
    const dim3 g(grid_for(n, kBlock * kGatherRows, 65536)), b(kBlock);
    if (idx64)
      hipLaunchKernelGGL((gather_percol_kernel<int64_t, kGatherRows>), g, b, 0, stream, (const int64_t*)idx, n, p);
    else
      hipLaunchKernelGGL((gather_percol_kernel<int32_t, kGatherRows>), g, b, 0, stream, (const int32_t*)idx, n, p);
    check_launch("gather_multi", stream);
  }
}

template <typename I>
static void launch_packed(const I* idx, int64_t n, const PackedParams& p, int words, hipStream_t stream) {
  const dim3 g(grid_for(n, kBlock * kGatherRows, 65536)), b(kBlock);
  switch (words) {
    case 1: hipLaunchKernelGGL((gather_packed_kernel<I, 1>), g, b, 0, stream, idx, n, p); break;
    case 2: hipLaunchKernelGGL((gather_packed_kernel<I, 2>), g, b, 0, stream, idx, n, p); break;
    case 3: hipLaunchKernelGGL((gather_packed_kernel<I, 3>), g, b, 0, stream, idx, n, p); break;
    default: hipLaunchKernelGGL((gather_packed_kernel<I, 4>), g, b, 0, stream, idx, n, p); break;
  }
}

void gather_packed(const void* idx, bool idx64, int64_t n, const uint8_t* src, int64_t src_rows, int row_bytes,
                   const PackedField* fields, int nf, hipStream_t stream) {
  if (n == 0 || nf == 0) return;
  if (row_bytes <= 0 || row_bytes > 32 || row_bytes % 8 != 0)
    throw std::runtime_error("gather_packed: row bytes must be 8, 16, 24 or 32, got " + std::to_string(row_bytes));
  if (nf > kMaxPackedFields) throw std::runtime_error("gather_packed: too many fields");
  if (src_rows > 0 && (src == nullptr || (reinterpret_cast<uintptr_t>(src) & 15) != 0))
    throw std::runtime_error("gather_packed: source must be 16-byte aligned");
  PackedParams p;
  p.src = src;
  p.rows = src == nullptr ? 0 : src_rows;
  p.nf = nf;
  for (int f = 0; f < nf; ++f) {
    const PackedField& d = fields[f];
    const bool w_ok = d.width == 1 || d.width == 2 || d.width == 4 || d.width == 8;
    const bool o_ok = d.out_bytes == 1 || d.out_bytes == 2 || d.out_bytes == 4 || d.out_bytes == 8;
    if (!d.dst || !w_ok || !o_ok || d.off < 0 || d.off % d.width != 0 || d.off + d.width > row_bytes)
      throw std::runtime_error("gather_packed: bad field " + std::to_string(f));
    p.f[f] = d;
  }
  if (idx64)
    launch_packed(static_cast<const int64_t*>(idx), n, p, row_bytes / 8, stream);
  else
    launch_packed(static_cast<const int32_t*>(idx), n, p, row_bytes / 8, stream);
  check_launch("gather_packed", stream);
}

void str_gather_lengths(const int64_t* off, int64_t src_rows, const void* idx, bool idx64, int64_t n, int64_t* len,
                        hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (idx64)
    hipLaunchKernelGGL(str_lengths_kernel<int64_t>, g, b, 0, stream, off, src_rows, (const int64_t*)idx, n, len);
  else
    hipLaunchKernelGGL(str_lengths_kernel<int32_t>, g, b, 0, stream, off, src_rows, (const int32_t*)idx, n, len);
  check_launch("str_gather_lengths", stream);
}

void str_gather_copy(const int64_t* off, int64_t src_rows, const uint8_t* chars, const void* idx, bool idx64,
                     int64_t n, const int64_t* new_off, uint8_t* out, int64_t out_cap, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock / 8, 65536)), b(kBlock);
  if (idx64)
    hipLaunchKernelGGL(str_copy_kernel<int64_t>, g, b, 0, stream, off, src_rows, chars, (const int64_t*)idx, n, new_off,
                       out, out_cap);
  else
    hipLaunchKernelGGL(str_copy_kernel<int32_t>, g, b, 0, stream, off, src_rows, chars, (const int32_t*)idx, n, new_off,
                       out, out_cap);
  check_launch("str_gather_copy", stream);
}

}  // namespace kern
}  // namespace igloo
