// LIST / STRUCT column helpers (DataFusion's datafusion-functions-nested,
// reference Cargo.lock:1125, reached through SessionContext::sql at
// crates/engine/src/lib.rs:54-57).
//
// A LIST row is an (start, length) pair into a child column, so most list
// work is index arithmetic followed by one gather of the child (gather.hip):
//   list_element_idx  child row of element i (1-based; negative counts from
//                     the end) per row, -1 = NULL (out of range / NULL row)
//   interleave_idx    make_array(c0..ck-1): child row r*k+j is c_j[r], read
//                     from the columns concatenated end to end (j*n + r)
//   list_slots        per-row (start, length) of a fixed-arity list
// Unnest uses expand_ranges (ranges.hip) over (start, length).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__global__ __launch_bounds__(kBlock) void list_element_idx_kernel(const int64_t* __restrict__ se,
                                                                const uint8_t* __restrict__ valid,
                                                                const int64_t* __restrict__ pos,
                                                                const uint8_t* __restrict__ pos_valid,
                                                                int64_t pos_const, int64_t n, int64_t child_n,
                                                                int64_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t start = se[2 * r], len = se[2 * r + 1];
    const int64_t i = pos ? pos[r] : pos_const;
    int64_t k = i > 0 ? i - 1 : len + i;          // 1-based from the front, -1 = last
    const bool ok = (!valid || valid[r]) && (!pos_valid || pos_valid[r]) && i != 0 && k >= 0 && k < len &&
                    start >= 0 && start + k < child_n;
    out[r] = ok ? start + k : -1;
  }
}

__global__ __launch_bounds__(kBlock) void interleave_idx_kernel(int64_t n, int k, int64_t* __restrict__ out) {
  const int64_t total = n * k;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / k, j = t - r * k;
    out[t] = j * n + r;
  }
}

__global__ __launch_bounds__(kBlock) void list_slots_kernel(int64_t n, int64_t k, int64_t* __restrict__ se) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    se[2 * r] = r * k;
    se[2 * r + 1] = k;
  }
}

}  // namespace

void list_element_idx(const int64_t* se, const uint8_t* valid, const int64_t* pos, const uint8_t* pos_valid,
                      int64_t pos_const, int64_t n, int64_t child_n, int64_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(list_element_idx_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, s, se, valid, pos,
                     pos_valid, pos_const, n, child_n, out);
  check_launch("list_element_idx", s);
}

void interleave_idx(int64_t n, int k, int64_t* out, hipStream_t s) {
  if (n == 0 || k == 0) return;
  hipLaunchKernelGGL(interleave_idx_kernel, dim3(grid_for(n * k, kBlock, 1 << 16)), dim3(kBlock), 0, s, n, k, out);
  check_launch("interleave_idx", s);
}

void list_slots(int64_t n, int64_t k, int64_t* se, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(list_slots_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, s, n, k, se);
  check_launch("list_slots", s);
}

}  // namespace kern
}  // namespace igloo
