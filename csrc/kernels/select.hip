// Stream compaction: boolean mask -> ordered row indices.
//
// Replaces arrow's filter_record_batch / DataFusion FilterExec compaction
// (reference crates/engine/src/operators/filter.rs:57). Three launches:
//   1. per-tile popcount of the mask (32 bytes per lane, two uint4 loads),
//   2. exclusive scan of the tile counts (one workgroup),
//   3. per-tile rewrite: each wave writes its rows' indices in rounds of
//      256 rows, one contiguous output run per round (ballot prefix of the
//      per-lane counts); output order equals input order (stable).
// A tile is kBlock*32 = 8192 rows, so SF100 lineitem (600M rows) launches
// ~73k workgroups: far more than 256 CUs x occupancy, as the HBM stream wants.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kItems = 32;
constexpr int kTile = kBlock * kItems;

// flags of rows [base, base + kItems) as 0/1 bytes (bool bytes are 0/1)
__device__ inline void load_flags(const uint8_t* mask, int64_t base, int64_t n, uint32_t (&w)[kItems / 4]) {
  if (base + kItems <= n && (((uintptr_t)(mask + base)) & 15) == 0) {
#pragma unroll
    for (int q = 0; q < kItems / 16; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(mask + base)[q];
      w[4 * q] = v.x;
      w[4 * q + 1] = v.y;
      w[4 * q + 2] = v.z;
      w[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kItems / 4; ++q) {
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b)
        if (base + 4 * q + b < n && mask[base + 4 * q + b]) x |= 1u << (8 * b);
      w[q] = x;
    }
  }
}

__device__ inline int count_flags(const uint8_t* mask, int64_t base, int64_t n) {
  uint32_t w[kItems / 4];
  load_flags(mask, base, n, w);
  int c = 0;
#pragma unroll
  for (int q = 0; q < kItems / 4; ++q) c += __popc(w[q]);
  return c;
}

__global__ __launch_bounds__(kBlock) void tile_count_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                           int64_t* __restrict__ counts) {
  __shared__ int64_t red[kWavesPerBlock];
  int64_t base = (int64_t)blockIdx.x * kTile + (int64_t)threadIdx.x * kItems;
  int64_t c = count_flags(mask, base, n);
  c = wave_reduce_sum(c);
  if (lane_id() == 0) red[threadIdx.x / kWave] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t t = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) t += red[w];
    counts[blockIdx.x] = t;
  }
}

}  // namespace

// Exclusive scan of `n` int64 counts in place with one workgroup of 1024
// lanes; writes the grand total to *total. Used for tile offsets everywhere.
__global__ __launch_bounds__(1024) void scan_counts_kernel(int64_t* __restrict__ counts, int64_t n,
                                                          int64_t* __restrict__ total) {
  __shared__ int64_t part[1024 / kWave + 1];
  const int t = threadIdx.x;
  int64_t per = (n + 1023) / 1024;
  int64_t lo = t * per, hi = lo + per < n ? lo + per : n;
  int64_t s = 0;
  for (int64_t i = lo; i < hi; ++i) s += counts[i];
  // block scan over 1024 threads (16 waves)
  int64_t inc = wave_inclusive_scan(s);
  if (lane_id() == kWave - 1) part[t / kWave] = inc;
  __syncthreads();
  if (t == 0) {
    int64_t run = 0;
    for (int w = 0; w < 1024 / kWave; ++w) {
      int64_t x = part[w];
      part[w] = run;
      run += x;
    }
    part[1024 / kWave] = run;
  }
  __syncthreads();
  int64_t run = inc - s + part[t / kWave];
  for (int64_t i = lo; i < hi; ++i) {
    int64_t c = counts[i];
    counts[i] = run;
    run += c;
  }
  if (t == 0 && total) *total = part[1024 / kWave];
}

namespace {

// Each wave owns 2048 consecutive rows of the tile and reads them as 8 rounds
// of one 4-flag word per lane (round q, lane l: rows q*256 + 4l .. +3), so
// row order is (round, lane, byte). A lane's position inside the round is the
// wave prefix of the per-lane counts (0..4), taken with three ballots of the
// count's bits; every round then writes one contiguous run of output. No LDS
// staging: the earlier per-lane scatter into a uint16 LDS buffer spent ~40%
// of the kernel in bank conflicts (profiles/r3_sf100_pmc_roofline.txt).
constexpr int kWaveRows = kTile / kWavesPerBlock;     // 2048
constexpr int kRounds = kWaveRows / (4 * kWave);      // 8

template <typename IdxT>
__global__ __launch_bounds__(kBlock) void tile_write_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                           const int64_t* __restrict__ offsets,
                                                           IdxT* __restrict__ out, int64_t cap) {
  __shared__ int64_t wcount[kWavesPerBlock];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t wbase_row = (int64_t)blockIdx.x * kTile + (int64_t)wave * kWaveRows;
  uint32_t w[kRounds];
  if (wbase_row + kWaveRows <= n && (((uintptr_t)mask) & 3) == 0) {
#pragma unroll
    for (int q = 0; q < kRounds; ++q)
      w[q] = *reinterpret_cast<const uint32_t*>(mask + wbase_row + q * 4 * kWave + 4 * lane);
  } else {
#pragma unroll
    for (int q = 0; q < kRounds; ++q) {
      uint32_t x = 0;
      const int64_t r0 = wbase_row + q * 4 * kWave + 4 * lane;
      for (int bb = 0; bb < 4; ++bb)
        if (r0 + bb < n && mask[r0 + bb]) x |= 1u << (8 * bb);
      w[q] = x;
    }
  }
  int64_t c = 0;
#pragma unroll
  for (int q = 0; q < kRounds; ++q) c += __popc(w[q]);
  c = wave_reduce_sum(c);
  if (lane == 0) wcount[wave] = c;
  __syncthreads();
  int64_t run = offsets[blockIdx.x];
  for (int v = 0; v < wave; ++v) run += wcount[v];
  // writes stay inside the caller's buffer of ``cap`` entries, and the last
  // tile zero-fills [total, cap): a size the host replayed instead of reading
  // (ops/_lib.py Speculation) can then never make this kernel or a consumer of
  // the indices touch memory out of bounds before the replay is validated
#pragma unroll
  for (int q = 0; q < kRounds; ++q) {
    const int cq = __popc(w[q]);
    const uint64_t b1 = __ballot(cq & 1), b2 = __ballot(cq & 2), b4 = __ballot(cq & 4);
    int64_t p = run + lane_prefix(b1) + 2 * lane_prefix(b2) + 4 * lane_prefix(b4);
    const int64_t r0 = wbase_row + q * 4 * kWave + 4 * lane;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
      if ((w[q] >> (8 * bb)) & 1u) {
        if (p < cap) out[p] = (IdxT)(r0 + bb);
        ++p;
      }
    run += __popcll(b1) + 2 * __popcll(b2) + 4 * __popcll(b4);
  }
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t p = offsets[gridDim.x] + threadIdx.x; p < cap; p += kBlock) out[p] = (IdxT)0;
}

}  // namespace

int64_t select_num_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

void select_count(const uint8_t* mask, int64_t n, int64_t* tile_counts, int64_t* total,
                  hipStream_t stream) {
  int64_t tiles = select_num_tiles(n);
  if (tiles == 0) {
    IGLOO_HIP_CHECK(hipMemsetAsync(total, 0, sizeof(int64_t), stream));
    return;
  }
  hipLaunchKernelGGL(tile_count_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, stream, mask, n,
                     tile_counts);
  check_launch("select.tile_count", stream);
  hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(1024), 0, stream, tile_counts, tiles, total);
  check_launch("select.scan", stream);
}

void select_write(const uint8_t* mask, int64_t n, const int64_t* tile_offsets, void* out, bool idx64, int64_t cap,
                  hipStream_t stream) {
  int64_t tiles = select_num_tiles(n);
  if (tiles == 0) return;
  if (idx64)
    hipLaunchKernelGGL(tile_write_kernel<int64_t>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                       mask, n, tile_offsets, (int64_t*)out, cap);
  else
    hipLaunchKernelGGL(tile_write_kernel<int32_t>, dim3((unsigned)tiles), dim3(kBlock), 0, stream,
                       mask, n, tile_offsets, (int32_t*)out, cap);
  check_launch("select.tile_write", stream);
}

void scan_counts(int64_t* counts, int64_t n, int64_t* total, hipStream_t stream) {
  hipLaunchKernelGGL(scan_counts_kernel, dim3(1), dim3(1024), 0, stream, counts, n, total);
  check_launch("scan_counts", stream);
}

}  // namespace kern
}  // namespace igloo
