// Hash partitioning for exchanges (shuffle before RCCL all-to-all-v) and
// date-part extraction.
//
// The reference declares but never implements a shuffle
// (reference crates/coordinator/src/fragment.rs:12 FragmentType::Shuffle,
// crates/api/proto/coordinator.proto:50-58). Here rows are routed to the
// rank owning hash(key) % nparts with a stable counting sort:
//   1. per-workgroup histograms -> counts[part][block]  (part-major),
//   2. exclusive scan of that matrix (one contiguous send range per part),
//   3. per-workgroup scatter in row order (wave ballot per part gives each
//      row's rank inside its wave; LDS carries the per-part running offset).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kPartBlocks = 1024;

template <typename K>
__device__ inline int part_of(const K* keys, int64_t i, int nparts) {
  return (int)(mix64((uint64_t)(int64_t)keys[i]) % (uint64_t)nparts);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void part_hist_kernel(const K* __restrict__ keys, int64_t n, int nparts,
                                                          int64_t rows_per_block, int64_t* __restrict__ counts) {
  __shared__ int64_t h[kMaxParts];
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) h[p] = 0;
  __syncthreads();
  int64_t lo = blockIdx.x * rows_per_block, hi = lo + rows_per_block < n ? lo + rows_per_block : n;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd((unsigned long long*)&h[part_of(keys, i, nparts)], 1ULL);
  __syncthreads();
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) counts[(int64_t)p * gridDim.x + blockIdx.x] = h[p];
}

template <typename K, typename I>
__global__ __launch_bounds__(kBlock) void part_scatter_kernel(const K* __restrict__ keys, int64_t n, int nparts,
                                                             int64_t rows_per_block, const int64_t* __restrict__ offsets,
                                                             I* __restrict__ perm) {
  __shared__ int64_t base[kMaxParts];
  __shared__ int wave_cnt[kWavesPerBlock][kMaxParts];
  for (int p = threadIdx.x; p < nparts; p += blockDim.x) base[p] = offsets[(int64_t)p * gridDim.x + blockIdx.x];
  __syncthreads();
  const int wave = threadIdx.x / kWave, lane = lane_id();
  int64_t lo = blockIdx.x * rows_per_block, hi = lo + rows_per_block < n ? lo + rows_per_block : n;
  for (int64_t t = lo; t < hi; t += blockDim.x) {
    int64_t i = t + threadIdx.x;
    int my = i < hi ? part_of(keys, i, nparts) : -1;
    int my_rank = 0;
    for (int p = 0; p < nparts; ++p) {
      uint64_t m = __ballot(my == p);
      if (my == p) my_rank = lane_prefix(m);
      if (lane == 0) wave_cnt[wave][p] = __popcll(m);
    }
    __syncthreads();
    if (my >= 0) {
      int64_t pos = base[my] + my_rank;
      for (int w = 0; w < wave; ++w) pos += wave_cnt[w][my];
      perm[pos] = (I)i;
    }
    __syncthreads();
    for (int p = threadIdx.x; p < nparts; p += blockDim.x) {
      int64_t s = 0;
      for (int w = 0; w < kWavesPerBlock; ++w) s += wave_cnt[w][p];
      base[p] += s;
    }
    __syncthreads();
  }
}

template <typename K>
__global__ __launch_bounds__(kBlock) void part_ids_kernel(const K* __restrict__ keys, int64_t n, int nparts,
                                                         int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = part_of(keys, i, nparts);
}

// civil-from-days (proleptic Gregorian), days since 1970-01-01
__device__ inline void civil(int32_t z0, int* y, int* m, int* d) {
  int64_t z = (int64_t)z0 + 719468;
  int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  int64_t doe = z - era * 146097;
  int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t yy = yoe + era * 400;
  int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int64_t mp = (5 * doy + 2) / 153;
  int64_t dd = doy - (153 * mp + 2) / 5 + 1;
  int64_t mm = mp < 10 ? mp + 3 : mp - 9;
  *y = (int)(yy + (mm <= 2));
  *m = (int)mm;
  *d = (int)dd;
}

__device__ inline int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

__global__ __launch_bounds__(kBlock) void date_part_kernel(const int32_t* __restrict__ days, int64_t n, int field,
                                                          int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int y, m, d;
    int32_t z = days[i];
    civil(z, &y, &m, &d);
    int32_t r;
    switch (field) {
      case 0: r = y; break;
      case 1: r = m; break;
      case 2: r = d; break;
      case 3: r = (m - 1) / 3 + 1; break;
      case 4: r = (int32_t)(((int64_t)z % 7 + 7 + 4) % 7); break;  // dow, 0 = Sunday (1970-01-01 was Thursday)
      default:  // day of year
        r = (int32_t)((int64_t)z - days_from_civil(y, 1, 1) + 1);
    }
    out[i] = r;
  }
}

}  // namespace

int64_t partition_blocks(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  return b < kPartBlocks ? (b < 1 ? 1 : b) : kPartBlocks;
}

void partition_hist(const void* keys, bool key64, int64_t n, int nparts, int64_t* counts, hipStream_t stream) {
  if (nparts > kMaxParts) throw std::runtime_error("partition_hist: too many partitions");
  int64_t blocks = partition_blocks(n);
  int64_t rpb = (n + blocks - 1) / blocks;
  if (key64)
    hipLaunchKernelGGL(part_hist_kernel<int64_t>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, (const int64_t*)keys, n, nparts, rpb, counts);
  else
    hipLaunchKernelGGL(part_hist_kernel<int32_t>, dim3((unsigned)blocks), dim3(kBlock), 0, stream, (const int32_t*)keys, n, nparts, rpb, counts);
  check_launch("partition_hist", stream);
}

void partition_run(const void* keys, bool key64, int64_t n, int nparts, int64_t* counts_ws, int64_t* total,
                   void* perm, bool perm64, hipStream_t stream) {
  if (nparts > kMaxParts) throw std::runtime_error("partition: too many partitions");
  int64_t blocks = partition_blocks(n);
  int64_t rpb = (n + blocks - 1) / blocks;
  rpb = (rpb + kBlock - 1) / kBlock * kBlock;
  blocks = n > 0 ? (n + rpb - 1) / rpb : 1;
  dim3 g((unsigned)blocks), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(part_hist_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, n, nparts, rpb, counts_ws);
  else
    hipLaunchKernelGGL(part_hist_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, n, nparts, rpb, counts_ws);
  check_launch("partition_hist", stream);
  scan_counts(counts_ws, (int64_t)nparts * blocks, total, stream);
  if (key64) {
    if (perm64) hipLaunchKernelGGL((part_scatter_kernel<int64_t, int64_t>), g, b, 0, stream, (const int64_t*)keys, n, nparts, rpb, counts_ws, (int64_t*)perm);
    else hipLaunchKernelGGL((part_scatter_kernel<int64_t, int32_t>), g, b, 0, stream, (const int64_t*)keys, n, nparts, rpb, counts_ws, (int32_t*)perm);
  } else {
    if (perm64) hipLaunchKernelGGL((part_scatter_kernel<int32_t, int64_t>), g, b, 0, stream, (const int32_t*)keys, n, nparts, rpb, counts_ws, (int64_t*)perm);
    else hipLaunchKernelGGL((part_scatter_kernel<int32_t, int32_t>), g, b, 0, stream, (const int32_t*)keys, n, nparts, rpb, counts_ws, (int32_t*)perm);
  }
  check_launch("partition_scatter", stream);
}

int64_t partition_run_blocks(int64_t n) {
  int64_t blocks = partition_blocks(n);
  int64_t rpb = (n + blocks - 1) / blocks;
  rpb = (rpb + kBlock - 1) / kBlock * kBlock;
  return n > 0 ? (n + rpb - 1) / rpb : 1;
}

void partition_ids(const void* keys, bool key64, int64_t n, int nparts, int32_t* out, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(part_ids_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, n, nparts, out);
  else
    hipLaunchKernelGGL(part_ids_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, n, nparts, out);
  check_launch("partition_ids", stream);
}

void date_part(const int32_t* days, int64_t n, int field, int32_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(date_part_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, days, n, field, out);
  check_launch("date_part", stream);
}

}  // namespace kern
}  // namespace igloo
