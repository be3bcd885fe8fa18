// Index gathers for late materialisation after joins, filters and sorts.
//
// Replaces the reference's per-pair RecordBatch concatenation
// (reference crates/engine/src/operators/hash_join.rs:221-240 combine_batches,
// :242-280 combine_with_nulls) with one launch that reads the index vector
// once and gathers up to kMaxGatherCols fixed-width columns. A negative index
// produces a NULL row (outer-join padding).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

struct GatherParams {
  int ncols;
  GatherDesc d[kMaxGatherCols];
};

template <typename I>
__global__ __launch_bounds__(kBlock) void gather_multi_kernel(const I* __restrict__ idx, int64_t n, GatherParams p) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = (int64_t)idx[i];
    bool ok = s >= 0;
    for (int c = 0; c < p.ncols; ++c) {
      const GatherDesc& d = p.d[c];
      switch (d.elem_bytes) {
        case 1: ((uint8_t*)d.dst)[i] = ok ? ((const uint8_t*)d.src)[s] : 0; break;
        case 2: ((uint16_t*)d.dst)[i] = ok ? ((const uint16_t*)d.src)[s] : 0; break;
        case 4: ((uint32_t*)d.dst)[i] = ok ? ((const uint32_t*)d.src)[s] : 0; break;
        case 8: ((uint64_t*)d.dst)[i] = ok ? ((const uint64_t*)d.src)[s] : 0; break;
        case 16: {
          uint4 z = {0, 0, 0, 0};
          ((uint4*)d.dst)[i] = ok ? ((const uint4*)d.src)[s] : z;
          break;
        }
      }
      if (d.dst_valid) d.dst_valid[i] = ok && (!d.src_valid || d.src_valid[s]);
    }
  }
}

template <typename I>
__global__ __launch_bounds__(kBlock) void str_lengths_kernel(const int64_t* __restrict__ off, const I* __restrict__ idx,
                                                            int64_t n, int64_t* __restrict__ len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = idx ? (int64_t)idx[i] : i;
    len[i] = s >= 0 ? off[s + 1] - off[s] : 0;
  }
}

// 8 lanes cooperate on one string: each step moves 8 bytes per lane.
template <typename I>
__global__ __launch_bounds__(kBlock) void str_copy_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                         const I* __restrict__ idx, int64_t n,
                                                         const int64_t* __restrict__ new_off, uint8_t* __restrict__ out) {
  const int sub = threadIdx.x & 7;
  const int64_t rows_per_block = kBlock / 8;
  for (int64_t r = blockIdx.x * rows_per_block + threadIdx.x / 8; r < n; r += (int64_t)gridDim.x * rows_per_block) {
    int64_t s = idx ? (int64_t)idx[r] : r;
    if (s < 0) continue;
    int64_t src = off[s], len = off[s + 1] - src, dst = new_off[r];
    for (int64_t b = sub; b < len; b += 8) out[dst + b] = chars[src + b];
  }
}

}  // namespace

void gather_multi(const void* idx, bool idx64, int64_t n, const GatherDesc* descs, int ncols, hipStream_t stream) {
  if (n == 0 || ncols == 0) return;
  for (int base = 0; base < ncols; base += kMaxGatherCols) {
    GatherParams p;
    p.ncols = ncols - base < kMaxGatherCols ? ncols - base : kMaxGatherCols;
    for (int c = 0; c < p.ncols; ++c) p.d[c] = descs[base + c];
    dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
    if (idx64)
      hipLaunchKernelGGL(gather_multi_kernel<int64_t>, g, b, 0, stream, (const int64_t*)idx, n, p);
    else
      hipLaunchKernelGGL(gather_multi_kernel<int32_t>, g, b, 0, stream, (const int32_t*)idx, n, p);
    check_launch("gather_multi", stream);
  }
}

void str_gather_lengths(const int64_t* off, const void* idx, bool idx64, int64_t n, int64_t* len, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (idx64)
    hipLaunchKernelGGL(str_lengths_kernel<int64_t>, g, b, 0, stream, off, (const int64_t*)idx, n, len);
  else
    hipLaunchKernelGGL(str_lengths_kernel<int32_t>, g, b, 0, stream, off, (const int32_t*)idx, n, len);
  check_launch("str_gather_lengths", stream);
}

void str_gather_copy(const int64_t* off, const uint8_t* chars, const void* idx, bool idx64, int64_t n,
                     const int64_t* new_off, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock / 8, 65536)), b(kBlock);
  if (idx64)
    hipLaunchKernelGGL(str_copy_kernel<int64_t>, g, b, 0, stream, off, chars, (const int64_t*)idx, n, new_off, out);
  else
    hipLaunchKernelGGL(str_copy_kernel<int32_t>, g, b, 0, stream, off, chars, (const int32_t*)idx, n, new_off, out);
  check_launch("str_gather_copy", stream);
}

}  // namespace kern
}  // namespace igloo
