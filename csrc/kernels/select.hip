// Stream compaction: boolean mask -> ordered row indices.
//
// Replaces arrow's filter_record_batch / DataFusion FilterExec compaction
// (reference crates/engine/src/operators/filter.rs:57). Three launches:
//   1. per-tile popcount of the mask (32 bytes per lane, two uint4 loads),
//   2. exclusive scan of the tile counts (one workgroup),
//   3. per-tile rewrite: each lane expands its 32 flags at its block-scan
//      offset into an LDS staging buffer, then the workgroup streams the
//      tile's indices out with contiguous (coalesced) stores; output order
//      equals input order (stable). (A variant without the LDS stage — one
//      ballot-ranked output run per 256 rows, no bank conflicts — measured
//      56 us/call against 35 us: its per-lane scattered stores cost more than
//      the staging conflicts, profiles/r3_sf100_pmc_roofline.txt. A
//      conflict-free LDS stage -- one row per lane per step, ballot-ranked
//      into consecutive words -- took the conflicts from 150M to 0 but needs
//      byte loads of the mask and ran 12-28 % slower: 0.445 vs 0.357 ms for
//      a 600M-row mask at 1 %, profiles/r4_select_like_ab.txt. The staging
//      conflicts are not on this kernel's critical path; the mask stream is.)
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

// Masks of at most kSmallTiles tiles: ONE workgroup counts every tile in turn
// and writes the tiles' exclusive offsets and the total directly (one launch
// instead of tile counts + a scan of them).
constexpr int kSmallTiles = 8;

__global__ __launch_bounds__(kBlock) void small_count_kernel(const uint8_t* __restrict__ mask, int64_t n, int tiles,
                                                            int64_t* __restrict__ offsets, int64_t* __restrict__ total) {
  __shared__ int64_t red[kWavesPerBlock];
  int64_t run = 0;
  for (int t = 0; t < tiles; ++t) {
    const int64_t base = (int64_t)t * kTile + (int64_t)threadIdx.x * kItems;
    int64_t c = wave_reduce_sum((int64_t)count_flags(mask, base, n));
    if (lane_id() == 0) red[threadIdx.x / kWave] = c;
    __syncthreads();
    int64_t tile_total = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) tile_total += red[w];
    if (threadIdx.x == 0) offsets[t] = run;
    run += tile_total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = run;
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
  // eight independent loads in flight per step (a 600M-row mask has 73K
  // tiles: 72 counts per lane, which one load at a time left latency-bound)
  constexpr int kU = 8;
  int64_t s = 0;
  int64_t i = lo;
  for (; i + kU <= hi; i += kU) {
    int64_t v[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) v[k] = counts[i + k];
#pragma unroll
    for (int k = 0; k < kU; ++k) s += v[k];
  }
  for (; i < hi; ++i) s += counts[i];
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
  for (i = lo; i + kU <= hi; i += kU) {
    int64_t v[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) v[k] = counts[i + k];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      counts[i + k] = run;
      run += v[k];
    }
  }
  for (; i < hi; ++i) {
    int64_t c = counts[i];
    counts[i] = run;
    run += c;
  }
  if (t == 0 && total) *total = part[1024 / kWave];
}

namespace {

template <typename IdxT>
__global__ __launch_bounds__(kBlock) void tile_write_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                           const int64_t* __restrict__ offsets,
                                                           IdxT* __restrict__ out, int64_t cap) {
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  __shared__ uint16_t stage[kTile];  // row offsets inside the tile, in output order
  const int64_t tile_base = (int64_t)blockIdx.x * kTile;
  const int first = threadIdx.x * kItems;
  uint32_t w[kItems / 4];
  load_flags(mask, tile_base + first, n, w);
  int64_t c = 0;
#pragma unroll
  for (int q = 0; q < kItems / 4; ++q) c += __popc(w[q]);
  int64_t total;
  int pos = (int)block_exclusive_scan(c, scratch, &total);
#pragma unroll
  for (int q = 0; q < kItems / 4; ++q)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if ((w[q] >> (8 * b)) & 1u) stage[pos++] = (uint16_t)(first + 4 * q + b);
  __syncthreads();
  // writes stay inside the caller's buffer of ``cap`` entries, and the last
  // tile zero-fills [total, cap): a size the host replayed instead of reading
  // (ops/_lib.py Speculation) can then never make this kernel or a consumer of
  // the indices touch memory out of bounds before the replay is validated
  const int64_t o = offsets[blockIdx.x];
  for (int k = threadIdx.x; k < (int)total; k += kBlock)
    if (o + k < cap) out[o + k] = (IdxT)(tile_base + stage[k]);
  if (blockIdx.x == gridDim.x - 1)
    for (int64_t p = offsets[gridDim.x] + threadIdx.x; p < cap; p += kBlock) out[p] = (IdxT)0;
}

template <typename IdxT>
__device__ __forceinline__ void compact_idx(IdxT* __restrict__ out, const uint16_t* stage, int total,
                                            int64_t tile_base, int64_t o, int64_t cap) {
  for (int k = threadIdx.x; k < total; k += kBlock)
    if (o + k < cap) out[o + k] = (IdxT)(tile_base + stage[k]);
}

// Fused stream compaction of whole columns: the tile's surviving row
// offsets are staged in LDS once (as in tile_write) and every column of the
// batch is copied through them -- one pass over each column with the writes
// coalesced, and no index vector written to and read back from HBM per
// column (mask -> indices -> gather). Reads stay inside the tile's 8192-row
// window of each column, so the lines a sparse tile touches are fetched once.
template <typename T>
__device__ __forceinline__ void compact_copy(const T* __restrict__ src, T* __restrict__ dst, const uint16_t* stage,
                                             int total, int64_t tile_base, int64_t o, int64_t cap) {
  for (int k = threadIdx.x; k < total; k += kBlock)
    if (o + k < cap) dst[o + k] = src[tile_base + stage[k]];
}

struct U128 {
  uint64_t lo, hi;
};

__global__ __launch_bounds__(kBlock) void tile_compact_kernel(const uint8_t* __restrict__ mask, int64_t n,
                                                             const int64_t* __restrict__ offsets, CompactArgs a,
                                                             int64_t cap) {
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  __shared__ uint16_t stage[kTile];
  const int64_t tile_base = (int64_t)blockIdx.x * kTile;
  const int first = threadIdx.x * kItems;
  uint32_t w[kItems / 4];
  load_flags(mask, tile_base + first, n, w);
  int64_t c = 0;
#pragma unroll
  for (int q = 0; q < kItems / 4; ++q) c += __popc(w[q]);
  int64_t total64;
  int pos = (int)block_exclusive_scan(c, scratch, &total64);
#pragma unroll
  for (int q = 0; q < kItems / 4; ++q)
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if ((w[q] >> (8 * b)) & 1u) stage[pos++] = (uint16_t)(first + 4 * q + b);
  __syncthreads();
  const int total = (int)total64;
  const int64_t o = offsets[blockIdx.x];
  if (a.idx != nullptr) {
    if (a.idx64) compact_idx<int64_t>((int64_t*)a.idx, stage, total, tile_base, o, cap);
    else compact_idx<int32_t>((int32_t*)a.idx, stage, total, tile_base, o, cap);
  }
  for (int j = 0; j < a.ncols; ++j) {
    const CompactCol& cc = a.cols[j];
    switch (cc.esz) {
      case 1: compact_copy((const uint8_t*)cc.src, (uint8_t*)cc.dst, stage, total, tile_base, o, cap); break;
      case 2: compact_copy((const uint16_t*)cc.src, (uint16_t*)cc.dst, stage, total, tile_base, o, cap); break;
      case 4: compact_copy((const uint32_t*)cc.src, (uint32_t*)cc.dst, stage, total, tile_base, o, cap); break;
      case 8: compact_copy((const uint64_t*)cc.src, (uint64_t*)cc.dst, stage, total, tile_base, o, cap); break;
      default: compact_copy((const U128*)cc.src, (U128*)cc.dst, stage, total, tile_base, o, cap); break;
    }
    if (cc.sv != nullptr) compact_copy(cc.sv, cc.dv, stage, total, tile_base, o, cap);
  }
  // as in tile_write: a row count the host replayed instead of reading back
  // may exceed the real one; the tail [real total, cap) is zeroed so no
  // consumer of these outputs (row indices, join keys) sees garbage
  if (blockIdx.x == gridDim.x - 1) {
    for (int64_t p = offsets[gridDim.x] + threadIdx.x; p < cap; p += kBlock) {
      if (a.idx != nullptr) {
        if (a.idx64) ((int64_t*)a.idx)[p] = 0;
        else ((int32_t*)a.idx)[p] = 0;
      }
      for (int j = 0; j < a.ncols; ++j) {
        const CompactCol& cc = a.cols[j];
        uint8_t* d = (uint8_t*)cc.dst + p * cc.esz;
        for (int q = 0; q < cc.esz; ++q) d[q] = 0;
        if (cc.dv != nullptr) cc.dv[p] = 0;
      }
    }
  }
}

}  // namespace

void select_compact(const uint8_t* mask, int64_t n, const int64_t* tile_offsets, const CompactArgs& a, int64_t cap,
                    hipStream_t stream) {
  int64_t tiles = select_num_tiles(n);
  if (tiles == 0) return;
  hipLaunchKernelGGL(tile_compact_kernel, dim3((unsigned)tiles), dim3(kBlock), 0, stream, mask, n, tile_offsets, a,
                     cap);
  check_launch("select.compact", stream);
}

int64_t select_num_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

void select_count(const uint8_t* mask, int64_t n, int64_t* tile_counts, int64_t* total,
                  hipStream_t stream) {
  int64_t tiles = select_num_tiles(n);
  if (tiles == 0) {
    IGLOO_HIP_CHECK(hipMemsetAsync(total, 0, sizeof(int64_t), stream));
    return;
  }
  if (tiles <= kSmallTiles) {
    hipLaunchKernelGGL(small_count_kernel, dim3(1), dim3(kBlock), 0, stream, mask, n, (int)tiles, tile_counts, total);
    check_launch("select.small_count", stream);
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
