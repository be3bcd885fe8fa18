// Whole-column checks the planner asks for before choosing a join / group-by
// strategy, as single-pass bandwidth kernels (they replaced ATen compare +
// reduce pairs that each read the column twice and launched 2-3 kernels):
//
//   column_stats  -> {min, max, sorted flag} of an int32/int64 key column
//                    (NULL rows skipped) in ONE read: every lane checks its
//                    run of 64 bytes plus the row before it; block min/max via
//                    wave shuffles into a per-block partial, reduced by a
//                    one-block second kernel (same-address device atomics from
//                    thousands of blocks serialise at the memory side: they
//                    held the SF100 calls at ~1 TB/s);
//   run_bounds    -> bound[i] = (i == 0 || k[i] != k[i-1]) for run-id group-by
//                    over clustered keys.
#include <limits>

#include <stdexcept>

#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {


__device__ inline int64_t wave_min(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    int64_t o = __shfl_xor(v, off, kWave);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline int64_t wave_max(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    int64_t o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

// 64 bytes per lane per iteration (4 x dwordx4), min/max in the column's own
// type; the NULL-free path (HAS_VALID = false, the common case: resident key
// columns and join outputs) has no per-row branches: the sortedness check
// compares each row with its neighbour inside the run plus one load of the
// row before it. (SF100 PMC: the previous 8-row, per-row-checked loop ran at
// 1.7 TB/s over 77 calls per suite.)
template <typename T, bool HAS_VALID>
__global__ __launch_bounds__(kBlock) void column_stats_kernel(const T* __restrict__ k, const uint8_t* __restrict__ valid,
                                                              int64_t n, long long* __restrict__ part) {
  constexpr int kRun = 64 / sizeof(T);
  __shared__ int64_t smin[kWavesPerBlock], smax[kWavesPerBlock];
  __shared__ int sbad;
  if (threadIdx.x == 0) sbad = 0;
  __syncthreads();
  T tmn = std::numeric_limits<T>::max(), tmx = std::numeric_limits<T>::min();
  bool any = false;
  bool bad = false;
  const int64_t stride = (int64_t)gridDim.x * kBlock * kRun;
  const bool aligned = (((uintptr_t)k) & 15) == 0;
  for (int64_t base = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kRun; base < n; base += stride) {
    T v[kRun];
    if (!HAS_VALID && aligned && base + kRun <= n) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 w = reinterpret_cast<const uint4*>(k + base)[q];
        __builtin_memcpy(&v[q * 16 / sizeof(T)], &w, 16);
      }
      // unconditional (clamped) load: a conditional one would make the branch
      // merge wait for the four vector loads above
      const T before = k[base > 0 ? base - 1 : 0];
      bad |= base > 0 && v[0] < before;
#pragma unroll
      for (int j = 0; j < kRun; ++j) {
        tmn = v[j] < tmn ? v[j] : tmn;
        tmx = v[j] > tmx ? v[j] : tmx;
        if (j) bad |= v[j] < v[j - 1];
      }
      any = true;
      continue;
    }
    // tail / NULL-aware path
    T prev = base > 0 ? k[base - 1] : T(0);
    bool prev_ok = base > 0 && (!HAS_VALID || valid[base - 1]);
    for (int j = 0; j < kRun && base + j < n; ++j) {
      const T x = k[base + j];
      if (!HAS_VALID || valid[base + j]) {
        tmn = x < tmn ? x : tmn;
        tmx = x > tmx ? x : tmx;
        any = true;
        if (prev_ok && x < prev) bad = true;
        prev = x;
        prev_ok = true;
      }
    }
  }
  int64_t mn = any ? (int64_t)tmn : INT64_MAX, mx = any ? (int64_t)tmx : INT64_MIN;
  mn = wave_min(mn);
  mx = wave_max(mx);
  const uint64_t anybad = __ballot(bad);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    smin[w] = mn;
    smax[w] = mx;
    if (anybad) sbad = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t a = smin[0], b = smax[0];
    for (int i = 1; i < kWavesPerBlock; ++i) {
      a = smin[i] < a ? smin[i] : a;
      b = smax[i] > b ? smax[i] : b;
    }
    part[blockIdx.x * 3 + 0] = a;
    part[blockIdx.x * 3 + 1] = b;
    part[blockIdx.x * 3 + 2] = sbad;
  }
}

// out[0..2] from the g per-block partials (one block)
__global__ __launch_bounds__(kBlock) void stats_reduce_kernel(const long long* __restrict__ part, int g,
                                                              long long* __restrict__ out) {
  __shared__ int64_t smin[kWavesPerBlock], smax[kWavesPerBlock];
  __shared__ int sbad;
  if (threadIdx.x == 0) sbad = 0;
  __syncthreads();
  int64_t mn = INT64_MAX, mx = INT64_MIN;
  bool bad = false;
  for (int i = threadIdx.x; i < g; i += kBlock) {
    const int64_t a = part[i * 3], b = part[i * 3 + 1];
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
    bad |= part[i * 3 + 2] != 0;
  }
  mn = wave_min(mn);
  mx = wave_max(mx);
  const uint64_t anybad = __ballot(bad);
  const int w = threadIdx.x / kWave;
  if (lane_id() == 0) {
    smin[w] = mn;
    smax[w] = mx;
    if (anybad) sbad = 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t a = smin[0], b = smax[0];
    for (int i = 1; i < kWavesPerBlock; ++i) {
      a = smin[i] < a ? smin[i] : a;
      b = smax[i] > b ? smax[i] : b;
    }
    out[0] = a;
    out[1] = b;
    out[2] = sbad;
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void run_bounds_kernel(const T* __restrict__ k, int64_t n, uint8_t* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    out[i] = (i == 0 || k[i] != k[i - 1]) ? 1 : 0;
}

}  // namespace

void column_stats(const void* keys, bool key64, const uint8_t* valid, int64_t n, long long* out, hipStream_t stream) {
  // out[0] = min, out[1] = max over non-NULL rows; out[2] = 1 if some row is
  // below its predecessor (only meaningful without NULLs). out holds
  // kStatsSlots int64: out[3..] takes the per-block partials.
  const int run = key64 ? 8 : 16;
  const unsigned g = n > 0 ? grid_for(n, kBlock * run, kStatsMaxBlocks) : 0;
  long long* part = out + 3;
  if (g == 0) {
    hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(kBlock), 0, stream, part, 0, out);
    check_launch("util.column_stats", stream);
    return;
  }
  if (key64) {
    if (valid)
      hipLaunchKernelGGL((column_stats_kernel<int64_t, true>), dim3(g), dim3(kBlock), 0, stream, (const int64_t*)keys,
                         valid, n, part);
    else
      hipLaunchKernelGGL((column_stats_kernel<int64_t, false>), dim3(g), dim3(kBlock), 0, stream, (const int64_t*)keys,
                         valid, n, part);
  } else {
    if (valid)
      hipLaunchKernelGGL((column_stats_kernel<int32_t, true>), dim3(g), dim3(kBlock), 0, stream, (const int32_t*)keys,
                         valid, n, part);
    else
      hipLaunchKernelGGL((column_stats_kernel<int32_t, false>), dim3(g), dim3(kBlock), 0, stream, (const int32_t*)keys,
                         valid, n, part);
  }
  hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(kBlock), 0, stream, part, (int)g, out);
  check_launch("util.column_stats", stream);
}

void run_bounds(const void* keys, bool key64, int64_t n, uint8_t* out, hipStream_t stream) {
  if (n <= 0) return;
  const unsigned g = grid_for(n, kBlock * 4, 8192);
  if (key64)
    hipLaunchKernelGGL(run_bounds_kernel<int64_t>, dim3(g), dim3(kBlock), 0, stream, (const int64_t*)keys, n, out);
  else
    hipLaunchKernelGGL(run_bounds_kernel<int32_t>, dim3(g), dim3(kBlock), 0, stream, (const int32_t*)keys, n, out);
  check_launch("util.run_bounds", stream);
}

namespace {

// Exact decimal AVG finaliser: out[i] = round_half_away(sum[i] * up / max(cnt[i], 1))
// for 128-bit sums stored as (lo, hi) int64 pairs (or plain int64 when hi is
// null). Keeps the whole aggregation on the device (no host round trip for
// the int128 division), so AVG over wide sums can live inside a query graph.
__global__ __launch_bounds__(kBlock) void avg_wide_kernel(const int64_t* __restrict__ sums, bool wide,
                                                          const int64_t* __restrict__ cnt, int64_t n, int64_t up,
                                                          int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    __int128 v = wide ? (((__int128)sums[2 * i + 1]) << 64) | (unsigned __int128)(uint64_t)sums[2 * i]
                      : (__int128)sums[i];
    const bool neg = v < 0;
    unsigned __int128 num = (unsigned __int128)(neg ? -v : v) * (unsigned __int128)up;
    const uint64_t k = (uint64_t)(cnt[i] > 0 ? cnt[i] : 1);
    // schoolbook 128 / 64 division (the divisor fits 64 bits): two 64-bit steps
    const uint64_t hi = (uint64_t)(num >> 64), lo = (uint64_t)num;
    const uint64_t qh = hi / k, rh = hi % k;
    unsigned __int128 rest = ((unsigned __int128)rh << 64) | lo;
    // rest < k * 2^64: long division bit by bit over the low word
    uint64_t ql = 0;
    unsigned __int128 r = 0;
    for (int b = 127; b >= 0; --b) {
      r = (r << 1) | (uint64_t)((rest >> b) & 1);
      if (r >= k) {
        r -= k;
        if (b < 64) ql |= (uint64_t)1 << b;
      }
    }
    unsigned __int128 q = ((unsigned __int128)qh << 64) | ql;
    if (2 * r >= (unsigned __int128)k) q += 1;   // half away from zero
    const int64_t res = (int64_t)(uint64_t)q;
    out[i] = neg ? -res : res;
  }
}

__global__ void zero_flag_kernel(int* __restrict__ flag) { *flag = 0; }

__global__ __launch_bounds__(kBlock) void wide_fits_kernel(const int64_t* __restrict__ lo,
                                                           const int64_t* __restrict__ hi, int64_t n,
                                                           int* __restrict__ flag) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= hi[i] != (lo[i] >> 63);
  if (__any(bad) && lane_id() == 0) atomicOr(flag, 1);
}

// flag = 1 when some row's value differs from its group representative's
// (a[i] != a[rep[i]]): the functional-dependency check of a GROUP BY key,
// one pass with no gathered copy or difference temporary.
template <typename T, typename R>
__global__ __launch_bounds__(kBlock) void differs_from_rep_kernel(const T* __restrict__ a, const R* __restrict__ rep,
                                                                 int64_t n, int* __restrict__ flag) {
  bool bad = false;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bad |= a[i] != a[rep[i]];
  if (__any(bad) && lane_id() == 0) atomicOr(flag, 1);
}

}  // namespace

void differs_from_rep(const void* a, int elem_bytes, const void* rep, bool rep64, int64_t n, int* flag,
                      hipStream_t stream) {
  hipLaunchKernelGGL(zero_flag_kernel, dim3(1), dim3(1), 0, stream, flag);
  if (n > 0) {
    const dim3 g(grid_for(n, kBlock * 4, 8192)), b(kBlock);
#define IGLOO_DIFF(T)                                                                                      \
  if (rep64)                                                                                               \
    hipLaunchKernelGGL((differs_from_rep_kernel<T, int64_t>), g, b, 0, stream, (const T*)a, (const int64_t*)rep, n, \
                       flag);                                                                              \
  else                                                                                                     \
    hipLaunchKernelGGL((differs_from_rep_kernel<T, int32_t>), g, b, 0, stream, (const T*)a, (const int32_t*)rep, n, flag);
    switch (elem_bytes) {
      case 1: IGLOO_DIFF(uint8_t) break;
      case 2: IGLOO_DIFF(uint16_t) break;
      case 4: IGLOO_DIFF(uint32_t) break;
      default: IGLOO_DIFF(uint64_t) break;
    }
#undef IGLOO_DIFF
  }
  check_launch("util.differs_from_rep", stream);
}

// flag = 1 when some 128-bit (lo, hi) sum does not fit int64 (hi is not the
// sign extension of lo). Replaces a torch `.all()` over the groups: a torch
// multi-block reduction zeroes its semaphores with a memset, and inside a
// captured query graph that memset was not reliably ordered.
void wide_fits(const int64_t* lo, const int64_t* hi, int64_t n, int* flag, hipStream_t stream) {
  hipLaunchKernelGGL(zero_flag_kernel, dim3(1), dim3(1), 0, stream, flag);
  if (n > 0)
    hipLaunchKernelGGL(wide_fits_kernel, dim3(grid_for(n, kBlock * 4, 8192)), dim3(kBlock), 0, stream, lo, hi, n,
                       flag);
  check_launch("util.wide_fits", stream);
}

void avg_wide(const int64_t* sums, bool wide, const int64_t* cnt, int64_t n, int64_t up, int64_t* out,
              hipStream_t stream) {
  if (n <= 0) return;
  hipLaunchKernelGGL(avg_wide_kernel, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, stream, sums, wide, cnt, n,
                     up, out);
  check_launch("util.avg_wide", stream);
}

// Small host constants written by a kernel whose arguments carry the values:
// a graph-capturable "upload" (a host-to-device copy inside a captured HIP
// graph is refused by the runtime, and would read host memory at replay).
constexpr int kConstInts = 64;
struct ConstInts {
  int64_t v[kConstInts];
};

__global__ void const_ints_kernel(int64_t* __restrict__ out, int n, ConstInts vals) {
  const int i = threadIdx.x;
  if (i < n) out[i] = vals.v[i];
}

void const_ints(int64_t* out, const int64_t* vals, int64_t n, hipStream_t stream) {
  for (int64_t base = 0; base < n; base += kConstInts) {
    ConstInts c{};
    const int k = (int)(n - base < kConstInts ? n - base : kConstInts);
    for (int i = 0; i < k; ++i) c.v[i] = vals[base + i];
    hipLaunchKernelGGL(const_ints_kernel, dim3(1), dim3(kConstInts), 0, stream, out + base, k, c);
  }
  check_launch("const_ints", stream);
}

// Composite integer keys bit-packed into one int64 per row (GROUP BY / join
// on several columns whose ranges fit in 62 bits): one pass over all key
// columns instead of a subtract, shift and OR per column in ATen.
struct PackBitsParams {
  int ncols;
  const void* col[kMaxPackBits];
  int is64[kMaxPackBits];
  long long lo[kMaxPackBits];
  int shift[kMaxPackBits];
};

__global__ __launch_bounds__(kBlock) void pack_bits_kernel(PackBitsParams p, int64_t n, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    uint64_t acc = 0;
    for (int c = 0; c < p.ncols; ++c) {
      const int64_t v = p.is64[c] ? ((const int64_t*)p.col[c])[i] : (int64_t)((const int32_t*)p.col[c])[i];
      acc = (acc << p.shift[c]) | (uint64_t)(v - p.lo[c]);
    }
    out[i] = (int64_t)acc;
  }
}

// 4 rows per lane: one 16-byte load per int32 column (two per int64 column)
// and two 16-byte stores (all pointers 16-byte aligned; the host checks)
__global__ __launch_bounds__(kBlock) void pack_bits4_kernel(PackBitsParams p, int64_t n, int64_t* __restrict__ out) {
  const int64_t n4 = n >> 2;
  for (int64_t q = blockIdx.x * (int64_t)kBlock + threadIdx.x; q < n4; q += (int64_t)gridDim.x * kBlock) {
    const int64_t i = q << 2;
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (int c = 0; c < p.ncols; ++c) {
      int64_t v0, v1, v2, v3;
      if (p.is64[c]) {
        const longlong2* src = (const longlong2*)((const int64_t*)p.col[c] + i);
        const longlong2 x = src[0], y = src[1];
        v0 = x.x; v1 = x.y; v2 = y.x; v3 = y.y;
      } else {
        const int4 x = *(const int4*)((const int32_t*)p.col[c] + i);
        v0 = x.x; v1 = x.y; v2 = x.z; v3 = x.w;
      }
      const uint64_t lo = (uint64_t)p.lo[c];
      const int sh = p.shift[c];
      a0 = (a0 << sh) | ((uint64_t)v0 - lo);
      a1 = (a1 << sh) | ((uint64_t)v1 - lo);
      a2 = (a2 << sh) | ((uint64_t)v2 - lo);
      a3 = (a3 << sh) | ((uint64_t)v3 - lo);
    }
    longlong2* o = (longlong2*)(out + i);
    o[0] = longlong2{(long long)a0, (long long)a1};
    o[1] = longlong2{(long long)a2, (long long)a3};
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const int64_t i = (n4 << 2) + threadIdx.x;
    uint64_t acc = 0;
    for (int c = 0; c < p.ncols; ++c) {
      const int64_t v = p.is64[c] ? ((const int64_t*)p.col[c])[i] : (int64_t)((const int32_t*)p.col[c])[i];
      acc = (acc << p.shift[c]) | (uint64_t)(v - p.lo[c]);
    }
    out[i] = (int64_t)acc;
  }
}

// Dense key marks (range-sliced SEMI / ANTI joins, parallel/exchange.py):
// marks[k - kmin] = 1 for every valid key k in [kmin, kmin + dom) -- one
// pass over the keys, plain byte stores (racing stores all write 1).
template <typename T>
__global__ __launch_bounds__(kBlock) void mark_keys_kernel(const T* __restrict__ k, const uint8_t* __restrict__ valid,
                                                          int64_t n, int64_t kmin, int64_t dom,
                                                          uint8_t* __restrict__ marks) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int64_t d = (int64_t)k[i] - kmin;
    if (d >= 0 && d < dom && (!valid || valid[i])) marks[d] = 1;
  }
}

// out[i] = (key i has a mark in [base, base + dom)) != negate; a NULL or
// out-of-domain key has none.
template <typename T>
__global__ __launch_bounds__(kBlock) void probe_marks_kernel(const T* __restrict__ k, const uint8_t* __restrict__ valid,
                                                            int64_t n, int64_t base, int64_t dom,
                                                            const uint8_t* __restrict__ marks, bool negate,
                                                            uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const int64_t d = (int64_t)k[i] - base;
    const bool hit = d >= 0 && d < dom && (!valid || valid[i]) && marks[d] != 0;
    out[i] = hit != negate;
  }
}

void pack_bits(const void* const* cols, const bool* is64, const int64_t* lo, const int* shift, int ncols, int64_t n,
               int64_t* out, hipStream_t stream) {
  if (n == 0) return;
  if (ncols < 1 || ncols > kMaxPackBits) throw std::runtime_error("pack_bits: column count");
  PackBitsParams p{};
  p.ncols = ncols;
  for (int c = 0; c < ncols; ++c) {
    p.col[c] = cols[c];
    p.is64[c] = is64[c] ? 1 : 0;
    p.lo[c] = lo[c];
    p.shift[c] = shift[c];
  }
  static const bool scalar = debug_flag("pack_bits_scalar");
  bool vec = ((uintptr_t)out & 15) == 0 && !scalar;
  for (int c = 0; c < ncols; ++c) vec = vec && ((uintptr_t)cols[c] & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(pack_bits4_kernel, dim3(grid_for((n + 3) / 4, kBlock, 65536)), dim3(kBlock), 0, stream, p, n, out);
  else
    hipLaunchKernelGGL(pack_bits_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, p, n, out);
  check_launch("util.pack_bits", stream);
}

// mark[trow[s]] = 1 for every occupied slot of a group-by table: the first
// row of every group (COUNT/SUM(DISTINCT) keep exactly those rows) without
// assigning group ids or counting the groups.
__global__ __launch_bounds__(kBlock) void mark_slot_rows_kernel(const int32_t* __restrict__ trow, int64_t cap,
                                                               int64_t n, uint8_t* __restrict__ mark) {
  for (int64_t s = blockIdx.x * (int64_t)kBlock + threadIdx.x; s < cap; s += (int64_t)gridDim.x * kBlock) {
    const int32_t r = trow[s];
    if (r >= 0 && (int64_t)r < n) mark[r] = 1;
  }
}

void mark_slot_rows(const int32_t* trow, int64_t cap, int64_t n, uint8_t* mark, hipStream_t stream) {
  if (cap == 0) return;
  hipLaunchKernelGGL(mark_slot_rows_kernel, dim3(grid_for(cap, kBlock, 65536)), dim3(kBlock), 0, stream, trow, cap, n,
                     mark);
  check_launch("util.mark_slot_rows", stream);
}

void mark_keys(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin, int64_t dom,
               uint8_t* marks, hipStream_t stream) {
  if (n == 0) return;
  const dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(mark_keys_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, valid, n, kmin, dom, marks);
  else
    hipLaunchKernelGGL(mark_keys_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, valid, n, kmin, dom, marks);
  check_launch("mark_keys", stream);
}

void probe_marks(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t base, int64_t dom,
                 const uint8_t* marks, bool negate, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  const dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(probe_marks_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, valid, n, base, dom, marks,
                       negate, out);
  else
    hipLaunchKernelGGL(probe_marks_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, valid, n, base, dom, marks,
                       negate, out);
  check_launch("probe_marks", stream);
}

// End a stream capture the runtime invalidated (the failed capture's graph
// is discarded), so the thread can launch again.
void end_capture(hipStream_t stream) {
  hipStreamCaptureStatus st;
  if (hipStreamIsCapturing(stream, &st) == hipSuccess && st != hipStreamCaptureStatusNone) {
    hipGraph_t g = nullptr;
    (void)hipStreamEndCapture(stream, &g);
    if (g) (void)hipGraphDestroy(g);
  }
  (void)hipGetLastError();
}

}  // namespace kern
}  // namespace igloo