// Device-wide exclusive prefix sum (int32/int64 -> int64), used for join
// output offsets, string offset construction and partition offsets.
// Three-phase tile scan: tile reduce -> scan of tile sums -> tile rescan.
// Tiles are 256 lanes x 8 items so a 600M-row input still launches ~290k
// workgroups, and each phase streams the input once.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kItems = 8;
constexpr int kTile = kBlock * kItems;

template <typename T>
__global__ __launch_bounds__(kBlock) void tile_sum_kernel(const T* __restrict__ in, int64_t n,
                                                         int64_t* __restrict__ sums) {
  __shared__ int64_t red[kWavesPerBlock];
  int64_t base = (int64_t)blockIdx.x * kTile + threadIdx.x;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    int64_t i = base + (int64_t)j * kBlock;
    if (i < n) s += (int64_t)in[i];
  }
  s = wave_reduce_sum(s);
  if (lane_id() == 0) red[threadIdx.x / kWave] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) t += red[w];
    sums[blockIdx.x] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void tile_scan_kernel(const T* __restrict__ in, int64_t n,
                                                          const int64_t* __restrict__ tile_off,
                                                          int64_t* __restrict__ out) {
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  // each lane owns kItems consecutive rows, moved with 16-byte loads and
  // stores when whole and aligned (8 scalar accesses at a 32/64-byte lane
  // stride otherwise)
  static_assert(kItems == 8, "vector path assumes 8 items per lane");
  const int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  const bool whole = base + kItems <= n && (((uintptr_t)(in + base)) & 15) == 0 &&
                     (((uintptr_t)(out + base)) & 15) == 0;
  int64_t v[kItems];
  if (whole) {
    if (sizeof(T) == 4) {
      const uint4 a = reinterpret_cast<const uint4*>(in + base)[0], b = reinterpret_cast<const uint4*>(in + base)[1];
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
      for (int j = 0; j < kItems; ++j) v[j] = (int64_t)(int32_t)w[j];
    } else {
#pragma unroll
      for (int q = 0; q < kItems / 2; ++q) {
        const longlong2 x = reinterpret_cast<const longlong2*>(in + base)[q];
        v[2 * q] = x.x;
        v[2 * q + 1] = x.y;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kItems; ++j) v[j] = base + j < n ? (int64_t)in[base + j] : 0;
  }
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) s += v[j];
  int64_t total;
  int64_t run = tile_off[blockIdx.x] + block_exclusive_scan(s, scratch, &total);
  if (whole) {
#pragma unroll
    for (int q = 0; q < kItems / 2; ++q) {
      longlong2 x;
      x.x = run;
      run += v[2 * q];
      x.y = run;
      run += v[2 * q + 1];
      reinterpret_cast<longlong2*>(out + base)[q] = x;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kItems; ++j) {
      if (base + j < n) out[base + j] = run;
      run += v[j];
    }
  }
}

// Inputs of at most kSmall values (the common case: per-group counts, the
// string lengths of a top-k, small joins): the whole scan in ONE workgroup,
// one launch instead of three. Each lane owns kSmallItems consecutive values.
constexpr int kSmallItems = 32;
constexpr int64_t kSmall = (int64_t)kBlock * kSmallItems;

template <typename T>
__global__ __launch_bounds__(kBlock) void small_scan_kernel(const T* __restrict__ in, int64_t n,
                                                           int64_t* __restrict__ out, int64_t* __restrict__ total) {
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  const int64_t base = (int64_t)threadIdx.x * kSmallItems;
  // every load issued before any is used: one memory latency, not 32
  int64_t v[kSmallItems];
#pragma unroll
  for (int j = 0; j < kSmallItems; ++j) v[j] = base + j < n ? (int64_t)in[base + j] : 0;
  int64_t s = 0;
#pragma unroll
  for (int j = 0; j < kSmallItems; ++j) s += v[j];
  int64_t tot;
  int64_t run = block_exclusive_scan(s, scratch, &tot);
#pragma unroll
  for (int j = 0; j < kSmallItems; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 0 && total) *total = tot;
}

template <typename T>
void exclusive_scan_impl(const T* in, int64_t n, int64_t* out, int64_t* tile_ws, int64_t* total,
                         hipStream_t stream) {
  int64_t tiles = (n + kTile - 1) / kTile;
  if (tiles == 0) {
    IGLOO_HIP_CHECK(hipMemsetAsync(total, 0, sizeof(int64_t), stream));
    return;
  }
  if (n <= kSmall) {
    hipLaunchKernelGGL(small_scan_kernel<T>, dim3(1), dim3(kBlock), 0, stream, in, n, out, total);
    check_launch("scan.small", stream);
    return;
  }
  hipLaunchKernelGGL(tile_sum_kernel<T>, dim3((unsigned)tiles), dim3(kBlock), 0, stream, in, n, tile_ws);
  check_launch("scan.tile_sum", stream);
  scan_counts(tile_ws, tiles, total, stream);
  hipLaunchKernelGGL(tile_scan_kernel<T>, dim3((unsigned)tiles), dim3(kBlock), 0, stream, in, n, tile_ws, out);
  check_launch("scan.tile_scan", stream);
}

}  // namespace

int64_t scan_workspace_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

void exclusive_scan(const void* in, bool in64, int64_t n, int64_t* out, int64_t* tile_ws, int64_t* total,
                    hipStream_t stream) {
  if (in64)
    exclusive_scan_impl((const int64_t*)in, n, out, tile_ws, total, stream);
  else
    exclusive_scan_impl((const int32_t*)in, n, out, tile_ws, total, stream);
}

}  // namespace kern
}  // namespace igloo
