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
