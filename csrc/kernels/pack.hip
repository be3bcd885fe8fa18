// Row packing for exchanges: ONE all-to-all-v per shuffle instead of one per
// column (SURVEY §5.8 step 5 "all fixed-width columns packed into one buffer
// to cut call count").
//
//   pack_rows:   out[i * row_bytes + off_c .. + w_c] = col_c[perm[i]]  (the
//                destination-grouping permutation of the hash partitioner is
//                fused in, so the gather and the pack are one pass);
//   unpack_rows: col_c[i] = in[i * row_bytes + off_c ..]  after the exchange.
//
// Fields are laid out widest first and rows padded to 8 bytes by the host,
// so every field access is naturally aligned. One lane per row: a wave writes
// 64 consecutive rows (one contiguous 64 x row_bytes span) per column.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__device__ inline void copy_field(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int w) {
  switch (w) {
    case 1: *d = *s; break;
    case 2: *reinterpret_cast<uint16_t*>(d) = *reinterpret_cast<const uint16_t*>(s); break;
    case 4: *reinterpret_cast<uint32_t*>(d) = *reinterpret_cast<const uint32_t*>(s); break;
    case 8: *reinterpret_cast<uint64_t*>(d) = *reinterpret_cast<const uint64_t*>(s); break;
    case 16:
      reinterpret_cast<uint64_t*>(d)[0] = reinterpret_cast<const uint64_t*>(s)[0];
      reinterpret_cast<uint64_t*>(d)[1] = reinterpret_cast<const uint64_t*>(s)[1];
      break;
    default:
      for (int b = 0; b < w; ++b) d[b] = s[b];
  }
}

template <typename P>
__global__ __launch_bounds__(kBlock) void pack_rows_kernel(PackSpec spec, const P* __restrict__ perm, int64_t n,
                                                           uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int64_t r = perm ? (int64_t)perm[i] : i;
    uint8_t* row = out + i * spec.row_bytes;
    for (int c = 0; c < spec.ncols; ++c) {
      const PackCol& col = spec.cols[c];
      copy_field(reinterpret_cast<const uint8_t*>(col.src) + r * col.width, row + col.offset, col.width);
    }
  }
}

__global__ __launch_bounds__(kBlock) void unpack_rows_kernel(PackSpec spec, const uint8_t* __restrict__ in, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint8_t* row = in + i * spec.row_bytes;
    for (int c = 0; c < spec.ncols; ++c) {
      const PackCol& col = spec.cols[c];
      copy_field(row + col.offset, reinterpret_cast<uint8_t*>(col.dst) + i * col.width, col.width);
    }
  }
}

}  // namespace

void pack_rows(const PackSpec& spec, const void* perm, bool perm64, int64_t n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock, 8192);
  if (perm64)
    hipLaunchKernelGGL(pack_rows_kernel<int64_t>, dim3(g), dim3(kBlock), 0, stream, spec, (const int64_t*)perm, n, out);
  else
    hipLaunchKernelGGL(pack_rows_kernel<int32_t>, dim3(g), dim3(kBlock), 0, stream, spec, (const int32_t*)perm, n, out);
  check_launch("pack.rows", stream);
}

void unpack_rows(const PackSpec& spec, const uint8_t* in, int64_t n, hipStream_t stream) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock, 8192);
  hipLaunchKernelGGL(unpack_rows_kernel, dim3(g), dim3(kBlock), 0, stream, spec, in, n);
  check_launch("pack.unpack", stream);
}

}  // namespace kern
}  // namespace igloo
