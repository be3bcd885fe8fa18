// LSD radix sort of (key, row id) pairs, key packing for multi-column ORDER
// BY, and radix-select helpers for ORDER BY ... LIMIT k (top-k).
//
// Replaces DataFusion SortExec / TopK (reference crates/engine/src/lib.rs:205
// ORDER BY ... NULLS FIRST, crates/engine/tests/integration_test.rs:59 ORDER
// BY age, coordinator LIMIT 5) and the secondary-index build of a resident
// key column. Design for CDNA4 (wave64, 160 KB LDS per CU):
//
// * keys are unsigned 32/64-bit, already range-compressed by the packer, so a
//   sort runs only ceil(bits / 8) passes of 8-bit digits;
// * one pass = histogram (per-tile digit counts, digit-major [256][tiles])
//   -> exclusive scan (scan.hip) -> scatter. A tile is 256 lanes x 16 items;
//   wave w owns a contiguous quarter of the tile and walks it in rounds of 64
//   consecutive rows, so (round, lane) order IS row order;
// * stable in-tile ranking without atomics: 8 ballots give each lane the
//   64-bit mask of lanes holding the same digit ("match" mask); the lane's
//   rank is popc(mask below it) plus the wave's running count of that digit,
//   which only the lowest matching lane updates. Per-wave counts are then
//   scanned across waves and digits in LDS;
// * the tile is placed in LDS in sorted order and streamed out with
//   consecutive lanes writing consecutive positions of each digit's run;
// * n <= one tile (4096 rows, typical post-aggregation ORDER BY) sorts in ONE
//   workgroup launch doing every pass in LDS.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kRsItems = 16;
constexpr int kRsTile = kBlock * kRsItems;  // 4096 rows per workgroup
constexpr int kRadix = 256;
static_assert(kBlock == kRadix, "one lane per digit in the per-tile scans");

template <typename K>
__device__ inline uint32_t digit_of(K k, int shift) {
  return (uint32_t)(k >> shift) & (kRadix - 1);
}

// mask of active lanes whose digit equals this lane's
__device__ inline uint64_t match_digit(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

// Rank this wave's items (registers k[], valid when row < n) by digit:
// r[j] = number of earlier items of the wave with the same digit.
// wcnt: this wave's 256 running counters in LDS (zeroed by the caller).
template <typename K>
__device__ inline void rank_wave(const K (&k)[kRsItems], const bool (&ok)[kRsItems], int shift, int32_t* wcnt,
                                 int32_t (&r)[kRsItems]) {
  const int lane = lane_id();
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const uint32_t d = digit_of(k[j], shift);
    const uint64_t m = match_digit(d, ok[j]);
    const int pre = __popcll(m & below);
    int32_t base = 0;
    if (ok[j]) base = wcnt[d];
    r[j] = base + pre;
    // the read of the old count above precedes this store in program order
    // (one wave, in-order LDS), so every matching lane saw the same base
    if (ok[j] && pre == 0) wcnt[d] = base + __popcll(m);
  }
}

// After rank_wave in every wave: turn wcnt[w][d] into the wave's base inside
// digit d's run, and dstart[d] into the run's start inside the tile.
__device__ inline void tile_digit_scan(int32_t (*wcnt)[kRadix], int32_t* dstart, int64_t* scratch) {
  const int d = threadIdx.x;  // kBlock == kRadix
  int32_t tot = 0;
#pragma unroll
  for (int w = 0; w < kWavesPerBlock; ++w) {
    const int32_t c = wcnt[w][d];
    wcnt[w][d] = tot;
    tot += c;
  }
  int64_t all;
  dstart[d] = (int32_t)block_exclusive_scan(tot, scratch, &all);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void rs_hist_kernel(const K* __restrict__ keys, int64_t n, int shift,
                                                         int32_t* __restrict__ counts, int64_t tiles) {
  __shared__ int32_t wh[kWavesPerBlock][kRadix];
  const int w = threadIdx.x / kWave, lane = lane_id();
  for (int i = threadIdx.x; i < kWavesPerBlock * kRadix; i += kBlock) (&wh[0][0])[i] = 0;
  __syncthreads();
  const int64_t wbase = (int64_t)blockIdx.x * kRsTile + (int64_t)w * kRsItems * kWave;
  K k[kRsItems];
  bool ok[kRsItems];
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const int64_t i = wbase + j * kWave + lane;
    ok[j] = i < n;
    k[j] = ok[j] ? keys[i] : K(0);
  }
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const uint32_t d = digit_of(k[j], shift);
    const uint64_t m = match_digit(d, ok[j]);
    if (ok[j] && __popcll(m & below) == 0) wh[w][d] += __popcll(m);
  }
  __syncthreads();
  const int d = threadIdx.x;
  int32_t t = 0;
#pragma unroll
  for (int ww = 0; ww < kWavesPerBlock; ++ww) t += wh[ww][d];
  counts[(int64_t)d * tiles + blockIdx.x] = t;
}

template <typename K, typename V>
__global__ __launch_bounds__(kBlock) void rs_scatter_kernel(const K* __restrict__ kin, const V* __restrict__ vin,
                                                            K* __restrict__ kout, V* __restrict__ vout, int64_t n,
                                                            int shift, const int64_t* __restrict__ offsets,
                                                            int64_t tiles) {
  __shared__ int32_t wcnt[kWavesPerBlock][kRadix];
  __shared__ int32_t dstart[kRadix];
  __shared__ int64_t gofs[kRadix];
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  __shared__ K sk[kRsTile];
  __shared__ V sv[kRsTile];
  const int w = threadIdx.x / kWave, lane = lane_id();
  for (int i = threadIdx.x; i < kWavesPerBlock * kRadix; i += kBlock) (&wcnt[0][0])[i] = 0;
  __syncthreads();
  const int64_t tile0 = (int64_t)blockIdx.x * kRsTile;
  const int64_t wbase = tile0 + (int64_t)w * kRsItems * kWave;
  K k[kRsItems];
  V v[kRsItems];
  bool ok[kRsItems];
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const int64_t i = wbase + j * kWave + lane;
    ok[j] = i < n;
    k[j] = ok[j] ? kin[i] : K(0);
    v[j] = ok[j] ? vin[i] : V(0);
  }
  int32_t r[kRsItems];
  rank_wave(k, ok, shift, wcnt[w], r);
  __syncthreads();
  tile_digit_scan(wcnt, dstart, scratch);
  {
    const int d = threadIdx.x;
    gofs[d] = offsets[(int64_t)d * tiles + blockIdx.x] - dstart[d];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    if (!ok[j]) continue;
    const uint32_t d = digit_of(k[j], shift);
    const int pos = dstart[d] + wcnt[w][d] + r[j];
    sk[pos] = k[j];
    sv[pos] = v[j];
  }
  __syncthreads();
  const int cnt = (int)((n - tile0) < kRsTile ? (n - tile0) : kRsTile);
  for (int i = threadIdx.x; i < cnt; i += kBlock) {
    const K key = sk[i];
    const int64_t g = gofs[digit_of(key, shift)] + i;
    kout[g] = key;
    vout[g] = sv[i];
  }
}

// n <= kRsTile: one workgroup. The keys' OR and AND over the sorted bit
// range show which 8-bit digits vary at all; passes over constant digits are
// skipped (ORDER BY keys packed at full field width leave most high digits
// constant). Up to kRankMax rows sort in one step instead: every item's
// stable rank (keys below it + equal keys before it) from the keys in LDS.
constexpr int kRankMax = 512;

template <typename K>
__device__ inline K bit_range_mask(int begin_bit, int end_bit) {
  constexpr int kBits = 8 * (int)sizeof(K);
  const K hi = end_bit >= kBits ? ~K(0) : ((K(1) << end_bit) - K(1));
  const K lo = begin_bit <= 0 ? K(0) : ((K(1) << begin_bit) - K(1));
  return hi & ~lo;
}

template <typename K>
__device__ inline K wave_or(K v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v |= (K)__shfl_xor(v, off, kWave);
  return v;
}

template <typename K>
__device__ inline K wave_and(K v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v &= (K)__shfl_xor(v, off, kWave);
  return v;
}

template <typename K, typename V>
__global__ __launch_bounds__(kBlock) void rs_small_kernel(K* __restrict__ keys, V* __restrict__ vals, int64_t n,
                                                          int begin_bit, int end_bit) {
  __shared__ int32_t wcnt[kWavesPerBlock][kRadix];
  __shared__ int32_t dstart[kRadix];
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  __shared__ K sk[kRsTile];
  __shared__ V sv[kRsTile];
  __shared__ K red[2][kWavesPerBlock];
  const int w = threadIdx.x / kWave, lane = lane_id();
  const int wbase = w * kRsItems * kWave;
  const K mask = bit_range_mask<K>(begin_bit, end_bit);
  if (n <= kRankMax) {
    // stable rank sort: stage the masked keys, rank every item against all of them
    for (int i = threadIdx.x; i < n; i += kBlock) sk[i] = keys[i] & mask;
    K mk[kRankMax / kBlock];
    K fk[kRankMax / kBlock];
    V fv[kRankMax / kBlock];
    int64_t pos[kRankMax / kBlock];
#pragma unroll
    for (int j = 0; j < kRankMax / kBlock; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < n) {
        fk[j] = keys[i];
        fv[j] = vals[i];
      }
      pos[j] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRankMax / kBlock; ++j) mk[j] = sk[threadIdx.x + j * kBlock < n ? threadIdx.x + j * kBlock : 0];
    for (int t = 0; t < n; ++t) {
      const K o = sk[t];  // one address for the whole wave: an LDS broadcast
#pragma unroll
      for (int j = 0; j < kRankMax / kBlock; ++j) {
        const int i = threadIdx.x + j * kBlock;
        pos[j] += (o < mk[j]) || (o == mk[j] && t < i);
      }
    }
    __syncthreads();  // every item was read before any is overwritten
#pragma unroll
    for (int j = 0; j < kRankMax / kBlock; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < n) {
        keys[pos[j]] = fk[j];
        vals[pos[j]] = fv[j];
      }
    }
    return;
  }
  K k[kRsItems];
  V v[kRsItems];
  bool ok[kRsItems];
  K kor = K(0), kand = ~K(0);
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const int i = wbase + j * kWave + lane;
    ok[j] = i < n;
    k[j] = ok[j] ? keys[i] : K(0);
    v[j] = ok[j] ? vals[i] : V(0);
    if (ok[j]) {
      kor |= k[j];
      kand &= k[j];
    }
  }
  kor = wave_or(kor);
  kand = wave_and(kand);
  if (lane == 0) {
    red[0][w] = kor;
    red[1][w] = kand;
  }
  __syncthreads();
  K diff = K(0);
  {
    K o = K(0), a = ~K(0);
#pragma unroll
    for (int x = 0; x < kWavesPerBlock; ++x) {
      o |= red[0][x];
      a &= red[1][x];
    }
    diff = (o ^ a) & mask;  // bits that differ between some two keys
  }
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    if (((diff >> shift) & K(kRadix - 1)) == K(0)) continue;  // every key has the same digit here
    for (int i = threadIdx.x; i < kWavesPerBlock * kRadix; i += kBlock) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    int32_t r[kRsItems];
    rank_wave(k, ok, shift, wcnt[w], r);
    __syncthreads();
    tile_digit_scan(wcnt, dstart, scratch);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
      if (!ok[j]) continue;
      const uint32_t d = digit_of(k[j], shift);
      const int pos = dstart[d] + wcnt[w][d] + r[j];
      sk[pos] = k[j];
      sv[pos] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kRsItems; ++j) {
      const int i = wbase + j * kWave + lane;
      if (ok[j]) {
        k[j] = sk[i];
        v[j] = sv[i];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const int i = wbase + j * kWave + lane;
    if (ok[j]) {
      keys[i] = k[j];
      vals[i] = v[j];
    }
  }
}

template <typename K, typename V>
int radix_sort_impl(K* k0, K* k1, V* v0, V* v1, int64_t n, int begin_bit, int end_bit, uint8_t* ws,
                    hipStream_t stream) {
  if (n <= 1 || begin_bit >= end_bit) return 0;
  if (n <= kRsTile) {
    hipLaunchKernelGGL((rs_small_kernel<K, V>), dim3(1), dim3(kBlock), 0, stream, k0, v0, n, begin_bit, end_bit);
    check_launch("sort.small", stream);
    return 0;
  }
  const int64_t tiles = (n + kRsTile - 1) / kRsTile;
  const int64_t m = tiles * kRadix;
  int32_t* counts = reinterpret_cast<int32_t*>(ws);
  int64_t* offsets = reinterpret_cast<int64_t*>(ws + ((m * 4 + 255) / 256) * 256);
  int64_t* scan_ws = offsets + m;
  const int64_t scan_tiles = scan_workspace_tiles(m);
  int cur = 0;
  K* kb[2] = {k0, k1};
  V* vb[2] = {v0, v1};
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    hipLaunchKernelGGL((rs_hist_kernel<K>), dim3((unsigned)tiles), dim3(kBlock), 0, stream, kb[cur], n, shift,
                       counts, tiles);
    check_launch("sort.hist", stream);
    exclusive_scan(counts, false, m, offsets, scan_ws, scan_ws + scan_tiles, stream);
    hipLaunchKernelGGL((rs_scatter_kernel<K, V>), dim3((unsigned)tiles), dim3(kBlock), 0, stream, kb[cur], vb[cur],
                       kb[cur ^ 1], vb[cur ^ 1], n, shift, offsets, tiles);
    check_launch("sort.scatter", stream);
    cur ^= 1;
  }
  return cur;
}

// ---------------------------------------------------------------- key packing
__device__ inline uint64_t ordered_bits(const SortKeyCol& c, int64_t row) {
  switch (c.kind) {
    case 0: {  // signed integer of c.width bytes
      int64_t v;
      if (c.width == 8) v = reinterpret_cast<const int64_t*>(c.ptr)[row];
      else if (c.width == 4) v = reinterpret_cast<const int32_t*>(c.ptr)[row];
      else if (c.width == 2) v = reinterpret_cast<const int16_t*>(c.ptr)[row];
      else v = reinterpret_cast<const int8_t*>(c.ptr)[row];
      return (uint64_t)v ^ 0x8000000000000000ull;
    }
    case 1: {  // float64: total order (-0.0 folded onto +0.0 by the host bounds)
      double d = reinterpret_cast<const double*>(c.ptr)[row];
      if (d == 0.0) d = 0.0;
      uint64_t b;
      __builtin_memcpy(&b, &d, 8);
      return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    }
    case 2:  // unsigned byte / bool
      return reinterpret_cast<const uint8_t*>(c.ptr)[row];
    default: {  // float32
      float f = reinterpret_cast<const float*>(c.ptr)[row];
      if (f == 0.0f) f = 0.0f;
      uint32_t b;
      __builtin_memcpy(&b, &f, 4);
      return (b >> 31) ? (uint64_t)(~b) : (uint64_t)(b | 0x80000000u);
    }
  }
}

template <typename P, typename O>
__global__ __launch_bounds__(kBlock) void sort_key_pack_kernel(SortKeySpec spec, const P* __restrict__ perm, int64_t n,
                                                               O* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const int64_t row = perm ? (int64_t)perm[i] : i;
    uint64_t key = 0;
    for (int c = 0; c < spec.ncols; ++c) {
      const SortKeyCol& col = spec.cols[c];
      const bool valid = col.valid == nullptr || col.valid[row];
      uint64_t f = 0;
      if (valid) {
        f = ordered_bits(col, row) - col.lo;
        if (col.desc) f = col.span - f;
      }
      const int width = col.bits + (col.valid != nullptr ? 1 : 0);
      key = width >= 64 ? 0ull : (key << width);
      if (col.valid != nullptr) {
        // NULL flag ABOVE the value field: NULLS FIRST -> nulls 0, values 1
        const uint64_t nf = col.nulls_first ? (valid ? 1ull : 0ull) : (valid ? 0ull : 1ull);
        f |= nf << col.bits;
      }
      key |= f;
    }
    out[i] = (O)key;
  }
}

// Zeroes the digit histogram. A kernel rather than hipMemsetAsync: inside a
// captured query graph (igloo_amd/exec/graphs.py) the memset node did not
// reliably clear the buffer before the histogram kernel ran on replay (the
// replayed counts came back offset by the buffer's previous contents).
__global__ void rs_zero_hist_kernel(unsigned long long* __restrict__ hist, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) hist[i] = 0ull;
}

template <typename K>
__global__ __launch_bounds__(kBlock) void rs_digit_hist_kernel(const K* __restrict__ keys, int64_t n, int shift,
                                                               uint64_t prefix, int pshift,
                                                               unsigned long long* __restrict__ hist) {
  __shared__ int32_t h[kRadix];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint64_t k = (uint64_t)keys[i];
    if (pshift >= 64 || (k >> pshift) == prefix) atomicAdd(&h[(k >> shift) & (kRadix - 1)], 1);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void rs_le_mask_kernel(const K* __restrict__ keys, int64_t n, uint64_t bound,
                                                            uint8_t* __restrict__ mask) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    mask[i] = (uint64_t)keys[i] <= bound;
}

}  // namespace

int64_t radix_sort_ws_bytes(int64_t n) {
  const int64_t tiles = (n + kRsTile - 1) / kRsTile;
  const int64_t m = tiles * kRadix;
  return ((m * 4 + 255) / 256) * 256 + 8 * m + 8 * (scan_workspace_tiles(m) + 1) + 256;
}

int radix_sort_pairs(void* k0, void* k1, bool key64, void* v0, void* v1, bool val64, int64_t n, int begin_bit,
                     int end_bit, void* ws, hipStream_t stream) {
  uint8_t* w = reinterpret_cast<uint8_t*>(ws);
  if (key64) {
    if (val64)
      return radix_sort_impl((uint64_t*)k0, (uint64_t*)k1, (int64_t*)v0, (int64_t*)v1, n, begin_bit, end_bit, w, stream);
    return radix_sort_impl((uint64_t*)k0, (uint64_t*)k1, (int32_t*)v0, (int32_t*)v1, n, begin_bit, end_bit, w, stream);
  }
  if (val64)
    return radix_sort_impl((uint32_t*)k0, (uint32_t*)k1, (int64_t*)v0, (int64_t*)v1, n, begin_bit, end_bit, w, stream);
  return radix_sort_impl((uint32_t*)k0, (uint32_t*)k1, (int32_t*)v0, (int32_t*)v1, n, begin_bit, end_bit, w, stream);
}

void sort_key_pack(const SortKeySpec& spec, const void* perm, bool perm64, int64_t n, void* out, bool out32,
                   hipStream_t stream) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock, 8192);
#define IGLOO_PACK(P, O) \
  hipLaunchKernelGGL((sort_key_pack_kernel<P, O>), dim3(g), dim3(kBlock), 0, stream, spec, (const P*)perm, n, (O*)out)
  if (perm64) {
    if (out32) IGLOO_PACK(int64_t, uint32_t); else IGLOO_PACK(int64_t, uint64_t);
  } else {
    if (out32) IGLOO_PACK(int32_t, uint32_t); else IGLOO_PACK(int32_t, uint64_t);
  }
#undef IGLOO_PACK
  check_launch("sort.key_pack", stream);
}

void radix_digit_hist(const void* keys, bool key64, int64_t n, int shift, uint64_t prefix, int pshift,
                      unsigned long long* hist, hipStream_t stream) {
  hipLaunchKernelGGL(rs_zero_hist_kernel, dim3(1), dim3(kRadix), 0, stream, hist, kRadix);
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock * 8, 2048);
  if (key64)
    hipLaunchKernelGGL(rs_digit_hist_kernel<uint64_t>, dim3(g), dim3(kBlock), 0, stream, (const uint64_t*)keys, n,
                       shift, prefix, pshift, hist);
  else
    hipLaunchKernelGGL(rs_digit_hist_kernel<uint32_t>, dim3(g), dim3(kBlock), 0, stream, (const uint32_t*)keys, n,
                       shift, prefix, pshift, hist);
  check_launch("sort.digit_hist", stream);
}

void radix_le_mask(const void* keys, bool key64, int64_t n, uint64_t bound, uint8_t* mask, hipStream_t stream) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock * 8, 8192);
  if (key64)
    hipLaunchKernelGGL(rs_le_mask_kernel<uint64_t>, dim3(g), dim3(kBlock), 0, stream, (const uint64_t*)keys, n, bound,
                       mask);
  else
    hipLaunchKernelGGL(rs_le_mask_kernel<uint32_t>, dim3(g), dim3(kBlock), 0, stream, (const uint32_t*)keys, n, bound,
                       mask);
  check_launch("sort.le_mask", stream);
}

}  // namespace kern
}  // namespace igloo
