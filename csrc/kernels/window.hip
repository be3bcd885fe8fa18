// Window-function kernels (SQL `f(...) OVER (PARTITION BY ... ORDER BY ... frame)`).
//
// The window operator (igloo_amd/exec/window.py) sorts the rows once by
// (partition, order) keys and hands these kernels the sorted segment ids.
// Everything a window function needs is then a scan or an elementwise pass
// over that order:
//   * win_seg_scan: segmented inclusive scan (sum / min / max over int64 or
//     f64, counts, nearest-head index, head counts), forward or reverse. Three
//     phases (tile reduce -> carry scan over tiles -> tile rescan) with the
//     segmented operator (f1,v1)+(f2,v2) = (f1|f2, f2 ? v2 : v1 op v2) carried
//     through wave64 shuffles, so it is exact for any segment layout.
//   * win_bounds: per-row frame [lo, hi] for ROWS / RANGE / GROUPS frames;
//     RANGE offsets binary-search the sorted ORDER BY key inside the
//     partition's non-NULL block.
//   * win_frame_sum: framed sum + count as a difference of global prefixes.
//   * win_frame_minmax: framed min / max by a loop over the frame.
//   * win_rank / win_index: ranking functions and the source row of
//     lag / lead / first_value / last_value / nth_value.
// Parity: DataFusion's WindowAggExec / BoundedWindowAggExec, reached by the
// reference through SessionContext::sql (reference crates/engine/src/lib.rs:54-57,
// Cargo.lock datafusion-functions-window 48.0.0).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kWItems = 8;
constexpr int kWTile = kBlock * kWItems;

template <int OP>
struct WOp;
// 0 sum int64 (wrapping, overflow flagged), 1 sum f64, 2 min i64, 3 max i64, 4 min f64, 5 max f64
template <>
struct WOp<0> {
  static __device__ int64_t id() { return 0; }
  static __device__ int64_t ap(int64_t a, int64_t b, bool& ovf) {
    int64_t r;
    ovf |= __builtin_add_overflow(a, b, &r);
    return r;
  }
};
template <>
struct WOp<1> {
  static __device__ int64_t id() { return __builtin_bit_cast(int64_t, 0.0); }
  static __device__ int64_t ap(int64_t a, int64_t b, bool&) {
    return __builtin_bit_cast(int64_t, __builtin_bit_cast(double, a) + __builtin_bit_cast(double, b));
  }
};
template <>
struct WOp<2> {
  static __device__ int64_t id() { return INT64_MAX; }
  static __device__ int64_t ap(int64_t a, int64_t b, bool&) { return a < b ? a : b; }
};
template <>
struct WOp<3> {
  static __device__ int64_t id() { return INT64_MIN; }
  static __device__ int64_t ap(int64_t a, int64_t b, bool&) { return a > b ? a : b; }
};
template <>
struct WOp<4> {
  static __device__ int64_t id() { return __builtin_bit_cast(int64_t, __builtin_huge_val()); }
  static __device__ int64_t ap(int64_t a, int64_t b, bool&) {
    double x = __builtin_bit_cast(double, a), y = __builtin_bit_cast(double, b);
    return __builtin_bit_cast(int64_t, y < x ? y : x);
  }
};
template <>
struct WOp<5> {
  static __device__ int64_t id() { return __builtin_bit_cast(int64_t, -__builtin_huge_val()); }
  static __device__ int64_t ap(int64_t a, int64_t b, bool&) {
    double x = __builtin_bit_cast(double, a), y = __builtin_bit_cast(double, b);
    return __builtin_bit_cast(int64_t, y > x ? y : x);
  }
};

struct ScanArgs {
  const void* ids;    // sorted segment ids (nullptr: one segment)
  bool ids64;
  const void* ids2;   // second id array (head index / head count values)
  bool ids2_64;
  const void* vals;
  int vkind;          // WinVal
  const uint8_t* valid;
  int64_t n;
  bool reverse;
};

__device__ __forceinline__ int64_t ld_id(const void* p, bool is64, int64_t i) {
  return is64 ? ((const int64_t*)p)[i] : (int64_t)((const int32_t*)p)[i];
}

// head flag of scan position k (row r) with respect to `ids`
__device__ __forceinline__ bool head_at(const void* ids, bool is64, int64_t n, bool rev, int64_t k, int64_t r) {
  if (k == 0) return true;
  if (ids == nullptr) return false;
  int64_t prev = rev ? r + 1 : r - 1;
  return ld_id(ids, is64, r) != ld_id(ids, is64, prev);
}

template <int OP>
__device__ __forceinline__ int64_t value_at(const ScanArgs& a, int64_t k, int64_t r) {
  if (a.valid != nullptr && !a.valid[r]) {
    if (a.vkind == kWinOne || a.vkind == kWinHead2) return 0;
    return WOp<OP>::id();
  }
  switch (a.vkind) {
    case kWinI64: return ((const int64_t*)a.vals)[r];
    case kWinI32: return (int64_t)((const int32_t*)a.vals)[r];
    case kWinF64: return ((const int64_t*)a.vals)[r];
    case kWinOne: return 1;
    case kWinHeadIdx: return head_at(a.ids2, a.ids2_64, a.n, a.reverse, k, r) ? r : WOp<OP>::id();
    default: return head_at(a.ids2, a.ids2_64, a.n, a.reverse, k, r) ? 1 : 0;  // kWinHead2
  }
}

// inclusive wave scan of (flag, value) pairs with the segmented operator
template <int OP>
__device__ __forceinline__ void wave_seg_scan(int& f, int64_t& v, bool& ovf) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int of = __shfl_up(f, off, kWave);
    int64_t ov = __shfl_up(v, off, kWave);
    if (lane >= off) {
      if (!f) v = WOp<OP>::ap(ov, v, ovf);
      f |= of;
    }
  }
}

// per-thread aggregate of its kWItems rows -> block-inclusive pair per thread.
// Returns the thread's EXCLUSIVE prefix pair within the block in (ef, ev) and
// the block total in (tf, tv).
template <int OP>
__device__ void block_seg_scan(int f, int64_t v, int& ef, int64_t& ev, int& tf, int64_t& tv, bool& ovf,
                               int* sf, int64_t* sv) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int incf = f;
  int64_t incv = v;
  wave_seg_scan<OP>(incf, incv, ovf);
  if (lane == kWave - 1) {
    sf[wave] = incf;
    sv[wave] = incv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int rf = 0;
    int64_t rv = WOp<OP>::id();
    for (int w = 0; w < kWavesPerBlock; ++w) {
      int wf = sf[w];
      int64_t wv = sv[w];
      sf[w] = rf;
      sv[w] = rv;
      rv = wf ? wv : WOp<OP>::ap(rv, wv, ovf);
      rf |= wf;
    }
    sf[kWavesPerBlock] = rf;
    sv[kWavesPerBlock] = rv;
  }
  __syncthreads();
  // exclusive within the wave: the previous lane's inclusive pair
  int pf = __shfl_up(incf, 1, kWave);
  int64_t pv = __shfl_up(incv, 1, kWave);
  if (lane == 0) {
    pf = 0;
    pv = WOp<OP>::id();
  }
  const int wf = sf[wave];
  const int64_t wv = sv[wave];
  ef = wf | pf;
  ev = pf ? pv : WOp<OP>::ap(wv, pv, ovf);
  tf = sf[kWavesPerBlock];
  tv = sv[kWavesPerBlock];
  __syncthreads();
}

template <int OP>
__global__ __launch_bounds__(kBlock) void seg_scan_reduce(ScanArgs a, int* tflag, int64_t* tval) {
  __shared__ int sf[kWavesPerBlock + 1];
  __shared__ int64_t sv[kWavesPerBlock + 1];
  const int64_t base = (int64_t)blockIdx.x * kWTile + (int64_t)threadIdx.x * kWItems;
  bool ovf = false;
  int f = 0;
  int64_t v = WOp<OP>::id();
#pragma unroll
  for (int j = 0; j < kWItems; ++j) {
    const int64_t k = base + j;
    if (k < a.n) {
      const int64_t r = a.reverse ? a.n - 1 - k : k;
      const bool h = head_at(a.ids, a.ids64, a.n, a.reverse, k, r);
      const int64_t x = value_at<OP>(a, k, r);
      v = h ? x : WOp<OP>::ap(v, x, ovf);
      f |= h;
    }
  }
  int ef, tf;
  int64_t ev, tv;
  block_seg_scan<OP>(f, v, ef, ev, tf, tv, ovf, sf, sv);
  if (threadIdx.x == 0) {
    tflag[blockIdx.x] = tf;
    tval[blockIdx.x] = tv;
  }
}

// one workgroup: exclusive carry per tile, in chunks of kWTile tiles
template <int OP>
__global__ __launch_bounds__(kBlock) void seg_scan_carry(int* tflag, int64_t* tval, int64_t tiles) {
  __shared__ int sf[kWavesPerBlock + 1];
  __shared__ int64_t sv[kWavesPerBlock + 1];
  __shared__ int cf;
  __shared__ int64_t cv;
  bool ovf = false;
  if (threadIdx.x == 0) {
    cf = 0;
    cv = WOp<OP>::id();
  }
  __syncthreads();
  for (int64_t c0 = 0; c0 < tiles; c0 += kWTile) {
    const int64_t base = c0 + (int64_t)threadIdx.x * kWItems;
    int lf[kWItems];
    int64_t lv[kWItems];
    int f = 0;
    int64_t v = WOp<OP>::id();
#pragma unroll
    for (int j = 0; j < kWItems; ++j) {
      const int64_t t = base + j;
      lf[j] = t < tiles ? tflag[t] : 0;
      lv[j] = t < tiles ? tval[t] : WOp<OP>::id();
      v = lf[j] ? lv[j] : WOp<OP>::ap(v, lv[j], ovf);
      f |= lf[j];
    }
    int ef, tf;
    int64_t ev, tv;
    block_seg_scan<OP>(f, v, ef, ev, tf, tv, ovf, sf, sv);
    // running carry = chunk carry (+) exclusive prefix
    int rf = cf | ef;
    int64_t rv = ef ? ev : WOp<OP>::ap(cv, ev, ovf);
#pragma unroll
    for (int j = 0; j < kWItems; ++j) {
      const int64_t t = base + j;
      if (t < tiles) {
        tflag[t] = rf;
        tval[t] = rv;
      }
      rv = lf[j] ? lv[j] : WOp<OP>::ap(rv, lv[j], ovf);
      rf |= lf[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      cv = tf ? tv : WOp<OP>::ap(cv, tv, ovf);
      cf |= tf;
    }
    __syncthreads();
  }
}

template <int OP>
__global__ __launch_bounds__(kBlock) void seg_scan_down(ScanArgs a, const int* tflag, const int64_t* tval,
                                                        bool use_carry, int64_t* out, int* err) {
  __shared__ int sf[kWavesPerBlock + 1];
  __shared__ int64_t sv[kWavesPerBlock + 1];
  const int64_t base = (int64_t)blockIdx.x * kWTile + (int64_t)threadIdx.x * kWItems;
  bool ovf = false;
  bool hs[kWItems];
  int64_t xs[kWItems];
  int f = 0;
  int64_t v = WOp<OP>::id();
#pragma unroll
  for (int j = 0; j < kWItems; ++j) {
    const int64_t k = base + j;
    hs[j] = false;
    xs[j] = WOp<OP>::id();
    if (k < a.n) {
      const int64_t r = a.reverse ? a.n - 1 - k : k;
      hs[j] = head_at(a.ids, a.ids64, a.n, a.reverse, k, r);
      xs[j] = value_at<OP>(a, k, r);
      v = hs[j] ? xs[j] : WOp<OP>::ap(v, xs[j], ovf);
      f |= hs[j];
    }
  }
  int ef, tf;
  int64_t ev, tv;
  block_seg_scan<OP>(f, v, ef, ev, tf, tv, ovf, sf, sv);
  int64_t acc = ev;
  if (use_carry && !ef) acc = WOp<OP>::ap(tval[blockIdx.x], ev, ovf);
#pragma unroll
  for (int j = 0; j < kWItems; ++j) {
    const int64_t k = base + j;
    if (k < a.n) {
      acc = hs[j] ? xs[j] : WOp<OP>::ap(acc, xs[j], ovf);
      out[a.reverse ? a.n - 1 - k : k] = acc;
    }
  }
  if (OP == 0 && ovf && err != nullptr) *err = 1;
}

template <int OP>
void seg_scan_impl(const ScanArgs& a, int* tflag, int64_t* tval, int64_t* out, int* err, hipStream_t s) {
  const int64_t tiles = (a.n + kWTile - 1) / kWTile;
  if (tiles == 0) return;
  if (tiles > 1) {
    hipLaunchKernelGGL(seg_scan_reduce<OP>, dim3((unsigned)tiles), dim3(kBlock), 0, s, a, tflag, tval);
    check_launch("win.scan_reduce", s);
    hipLaunchKernelGGL(seg_scan_carry<OP>, dim3(1), dim3(kBlock), 0, s, tflag, tval, tiles);
    check_launch("win.scan_carry", s);
  }
  hipLaunchKernelGGL(seg_scan_down<OP>, dim3((unsigned)tiles), dim3(kBlock), 0, s, a, tflag, tval, tiles > 1, out,
                     err);
  check_launch("win.scan_down", s);
}

// ----------------------------------------------------------------- frame bounds
struct BoundArgs {
  int64_t n;
  const int64_t* seg_start;
  const int64_t* seg_end;
  const int64_t* peer_start;
  const int64_t* peer_end;
  int unit;  // 0 rows, 1 range, 2 groups
  int skind, ekind;  // 0 unbounded preceding, 1 preceding, 2 current, 3 following, 4 unbounded following
  int64_t soff_i, eoff_i;
  double soff_f, eoff_f;
  const void* key;  // RANGE with offsets: sorted ORDER BY key (int64 or f64)
  bool key_f64;
  const uint8_t* key_valid;
  bool desc;
  const int64_t* gnum;  // GROUPS: global peer-group number per row
  const int64_t* gpos;  // GROUPS: first row of each global peer group
  int64_t ngroups;
};

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
  int64_t r;
  if (__builtin_add_overflow(a, b, &r)) return b > 0 ? INT64_MAX : INT64_MIN;
  return r;
}

// first index in [lo, hi] whose key is at-or-after `t` in the sort direction
// (asc: key >= t; desc: key <= t); hi + 1 when none
template <typename K>
__device__ int64_t lower_idx(const K* key, int64_t lo, int64_t hi, K t, bool desc) {
  int64_t a = lo, b = hi + 1;
  while (a < b) {
    int64_t m = a + ((b - a) >> 1);
    bool before = desc ? (key[m] > t) : (key[m] < t);
    if (before) a = m + 1;
    else b = m;
  }
  return a;
}
// last index in [lo, hi] whose key is at-or-before `t` (asc: key <= t; desc: key >= t); lo - 1 when none
template <typename K>
__device__ int64_t upper_idx(const K* key, int64_t lo, int64_t hi, K t, bool desc) {
  int64_t a = lo, b = hi + 1;
  while (a < b) {
    int64_t m = a + ((b - a) >> 1);
    bool after = desc ? (key[m] < t) : (key[m] > t);
    if (after) b = m;
    else a = m + 1;
  }
  return a - 1;
}

template <typename K>
__device__ void range_bounds(const BoundArgs& a, int64_t r, int64_t ss, int64_t se, int64_t& lo, int64_t& hi) {
  const K* key = (const K*)a.key;
  // offsets apply inside the partition's non-NULL block (NULL keys sort
  // together at one end; a NULL row's offset frame is its peer group)
  int64_t nb = ss, ne = se;
  if (a.key_valid != nullptr) {
    if (!a.key_valid[r]) {
      if (a.skind != 0) lo = a.peer_start[r];
      if (a.ekind != 4) hi = a.peer_end[r];
      return;
    }
    if (!a.key_valid[ss]) nb = a.peer_end[ss] + 1;
    if (!a.key_valid[se]) ne = a.peer_start[se] - 1;
  }
  const K x = key[r];
  // "preceding" moves against the sort direction, "following" with it
  auto shift = [&](bool forward, int64_t oi, double of) -> K {
    bool up = forward != a.desc;  // value increases
    if constexpr (sizeof(K) == 8 && K(0.5) != K(0)) {
      return up ? x + (K)of : x - (K)of;
    } else {
      return up ? (K)sat_add((int64_t)x, oi) : (K)sat_add((int64_t)x, -oi);
    }
  };
  if (a.skind == 1) lo = lower_idx<K>(key, nb, ne, shift(false, a.soff_i, a.soff_f), a.desc);
  else if (a.skind == 3) lo = lower_idx<K>(key, nb, ne, shift(true, a.soff_i, a.soff_f), a.desc);
  if (a.ekind == 1) hi = upper_idx<K>(key, nb, ne, shift(false, a.eoff_i, a.eoff_f), a.desc);
  else if (a.ekind == 3) hi = upper_idx<K>(key, nb, ne, shift(true, a.eoff_i, a.eoff_f), a.desc);
}

__global__ __launch_bounds__(kBlock) void win_bounds_kernel(BoundArgs a, int64_t* lo_out, int64_t* hi_out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= a.n) return;
  const int64_t ss = a.seg_start ? a.seg_start[r] : 0;
  const int64_t se = a.seg_end ? a.seg_end[r] : a.n - 1;
  int64_t lo = ss, hi = se;
  if (a.skind == 2) lo = a.unit == 0 ? r : a.peer_start[r];
  if (a.ekind == 2) hi = a.unit == 0 ? r : a.peer_end[r];
  if (a.unit == 0) {
    if (a.skind == 1) lo = sat_add(r, -a.soff_i);
    else if (a.skind == 3) lo = sat_add(r, a.soff_i);
    if (a.ekind == 1) hi = sat_add(r, -a.eoff_i);
    else if (a.ekind == 3) hi = sat_add(r, a.eoff_i);
  } else if (a.unit == 1) {
    if (a.skind == 1 || a.skind == 3 || a.ekind == 1 || a.ekind == 3) {
      if (a.key_f64) range_bounds<double>(a, r, ss, se, lo, hi);
      else range_bounds<int64_t>(a, r, ss, se, lo, hi);
    }
  } else {
    const int64_t g = a.gnum[r], g0 = a.gnum[ss], g1 = a.gnum[se];
    auto gstart = [&](int64_t gg) { return a.gpos[gg]; };
    auto gend = [&](int64_t gg) { return gg + 1 < a.ngroups ? a.gpos[gg + 1] - 1 : a.n - 1; };
    if (a.skind == 1) {
      int64_t gg = g - a.soff_i;
      lo = gg < g0 ? ss : gstart(gg);
    } else if (a.skind == 3) {
      int64_t gg = sat_add(g, a.soff_i);
      lo = gg > g1 ? se + 1 : gstart(gg);
    }
    if (a.ekind == 1) {
      int64_t gg = g - a.eoff_i;
      hi = gg < g0 ? ss - 1 : gend(gg);
    } else if (a.ekind == 3) {
      int64_t gg = sat_add(g, a.eoff_i);
      hi = gg > g1 ? se : gend(gg);
    }
  }
  if (lo < ss) lo = ss;
  if (hi > se) hi = se;
  lo_out[r] = lo;
  hi_out[r] = hi;
}

// ---------------------------------------------------------- framed aggregates
__global__ __launch_bounds__(kBlock) void win_frame_sum_kernel(const int64_t* psum, bool f64, const int64_t* pcnt,
                                                               const int64_t* lo, const int64_t* hi, int64_t n,
                                                               int64_t* sum_out, int64_t* cnt_out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  const int64_t l = lo[r], h = hi[r];
  const bool empty = h < l;
  if (sum_out != nullptr) {
    if (f64) {
      double s = empty ? 0.0
                       : __builtin_bit_cast(double, psum[h]) - (l > 0 ? __builtin_bit_cast(double, psum[l - 1]) : 0.0);
      sum_out[r] = __builtin_bit_cast(int64_t, s);
    } else {
      uint64_t s = empty ? 0 : (uint64_t)psum[h] - (l > 0 ? (uint64_t)psum[l - 1] : 0);
      sum_out[r] = (int64_t)s;
    }
  }
  if (cnt_out != nullptr) cnt_out[r] = empty ? 0 : pcnt[h] - (l > 0 ? pcnt[l - 1] : 0);
}

template <bool F64, bool MAX>
__global__ __launch_bounds__(kBlock) void win_frame_minmax_kernel(const int64_t* vals, const uint8_t* valid,
                                                                  const int64_t* lo, const int64_t* hi, int64_t n,
                                                                  int64_t* out, uint8_t* out_valid) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  bool any = false;
  int64_t bi = 0;
  double bf = 0;
  for (int64_t j = lo[r]; j <= hi[r]; ++j) {
    if (valid != nullptr && !valid[j]) continue;
    if (F64) {
      double x = __builtin_bit_cast(double, vals[j]);
      if (!any || (MAX ? x > bf : x < bf)) bf = x;
    } else {
      int64_t x = vals[j];
      if (!any || (MAX ? x > bi : x < bi)) bi = x;
    }
    any = true;
  }
  out[r] = F64 ? __builtin_bit_cast(int64_t, bf) : bi;
  out_valid[r] = any;
}

// Sliding min / max of any width in O(1) per row: a sparse table
// (level k holds the op over [i, i + 2^k)) built level by level, each level
// one pass over the previous one; a frame [lo, hi] is covered by two
// overlapping power-of-two blocks. NULLs enter as the op's identity; the
// frame's NULL-free flag comes from the caller's prefix count (or hi >= lo).
// Floats travel as order-preserving int64 images.
__device__ inline int64_t f64_ord(int64_t bits) { return bits >= 0 ? bits : (bits ^ INT64_MAX); }

__global__ __launch_bounds__(kBlock) void win_sparse_init_kernel(const int64_t* __restrict__ vals, bool f64,
                                                                 const uint8_t* __restrict__ valid, int64_t n,
                                                                 bool is_max, int64_t* __restrict__ t0) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool ok = !valid || valid[i];
    const int64_t v = f64 ? f64_ord(vals[i]) : vals[i];
    t0[i] = ok ? v : (is_max ? INT64_MIN : INT64_MAX);
  }
}

__global__ __launch_bounds__(kBlock) void win_sparse_level_kernel(const int64_t* __restrict__ prev,
                                                                  int64_t* __restrict__ next, int64_t n, int64_t half,
                                                                  bool is_max) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = prev[i];
    if (i + half < n) {
      const int64_t b = prev[i + half];
      next[i] = is_max ? (a > b ? a : b) : (a < b ? a : b);
    } else {
      next[i] = a;
    }
  }
}

__global__ __launch_bounds__(kBlock) void win_sparse_query_kernel(const int64_t* __restrict__ table, int levels,
                                                                  int64_t n, const int64_t* __restrict__ lo,
                                                                  const int64_t* __restrict__ hi,
                                                                  const int64_t* __restrict__ pcnt, bool is_max,
                                                                  bool f64, int64_t* __restrict__ out,
                                                                  uint8_t* __restrict__ out_valid) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = lo[r], h = hi[r];
    if (h < l || l < 0 || h >= n) {
      out[r] = 0;
      out_valid[r] = 0;
      continue;
    }
    const int64_t w = h - l + 1;
    int k = 63 - __builtin_clzll((unsigned long long)w);
    if (k >= levels) k = levels - 1;   // defensive: the host sized levels for the widest frame
    const int64_t* t = table + (int64_t)k * n;
    const int64_t a = t[l], b = t[h - ((int64_t)1 << k) + 1];
    int64_t m = is_max ? (a > b ? a : b) : (a < b ? a : b);
    const bool any = pcnt ? (pcnt[h] - (l > 0 ? pcnt[l - 1] : 0)) > 0 : true;
    if (f64) m = f64_ord(m);           // the map is its own inverse
    out[r] = any ? m : 0;
    out_valid[r] = any;
  }
}

// ------------------------------------------------------------------- ranking
__global__ __launch_bounds__(kBlock) void win_rank_kernel(int fn, int64_t arg, int64_t n, const int64_t* seg_start,
                                                          const int64_t* seg_end, const int64_t* peer_start,
                                                          const int64_t* peer_end, const int64_t* dense,
                                                          int64_t* out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  const int64_t ss = seg_start ? seg_start[r] : 0;
  const int64_t se = seg_end ? seg_end[r] : n - 1;
  const int64_t size = se - ss + 1;
  int64_t v = 0;
  switch (fn) {
    case kWinRowNumber: v = r - ss + 1; break;
    case kWinRank: v = (peer_start ? peer_start[r] : ss) - ss + 1; break;
    case kWinDenseRank: v = dense[r]; break;
    case kWinPercentRank: {
      const int64_t rk = (peer_start ? peer_start[r] : ss) - ss;
      double d = size > 1 ? (double)rk / (double)(size - 1) : 0.0;
      v = __builtin_bit_cast(int64_t, d);
      break;
    }
    case kWinCumeDist: {
      const int64_t pe = peer_end ? peer_end[r] : se;
      double d = (double)(pe - ss + 1) / (double)size;
      v = __builtin_bit_cast(int64_t, d);
      break;
    }
    case kWinNtile: {
      const int64_t j = r - ss;
      const int64_t q = size / arg, rem = size % arg;
      if (q == 0) v = j + 1;
      else if (j < rem * (q + 1)) v = j / (q + 1) + 1;
      else v = (j - rem * (q + 1)) / q + rem + 1;
      break;
    }
    default: break;
  }
  out[r] = v;
}

__global__ __launch_bounds__(kBlock) void win_index_kernel(int fn, int64_t arg, int64_t n, const int64_t* seg_start,
                                                           const int64_t* seg_end, const int64_t* lo,
                                                           const int64_t* hi, int64_t* out) {
  const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (r >= n) return;
  int64_t idx = -1;
  switch (fn) {
    case kWinLag: {
      const int64_t ss = seg_start ? seg_start[r] : 0;
      const int64_t j = r - arg;
      const int64_t se = seg_end ? seg_end[r] : n - 1;
      idx = (j >= ss && j <= se) ? j : -1;
      break;
    }
    case kWinFirst: idx = lo[r] <= hi[r] ? lo[r] : -1; break;
    case kWinLast: idx = lo[r] <= hi[r] ? hi[r] : -1; break;
    case kWinNth: {
      const int64_t j = lo[r] + arg - 1;
      idx = (lo[r] <= hi[r] && j <= hi[r]) ? j : -1;
      break;
    }
    default: break;
  }
  out[r] = idx;
}

}  // namespace

int64_t win_scan_tiles(int64_t n) { return (n + kWTile - 1) / kWTile; }

void win_seg_scan(const void* ids, bool ids64, const void* ids2, bool ids2_64, const void* vals, int vkind,
                  const uint8_t* valid, int64_t n, int op, bool reverse, int* tflag, int64_t* tval, int64_t* out,
                  int* err, hipStream_t s) {
  ScanArgs a{ids, ids64, ids2, ids2_64, vals, vkind, valid, n, reverse};
  switch (op) {
    case 0: seg_scan_impl<0>(a, tflag, tval, out, err, s); break;
    case 1: seg_scan_impl<1>(a, tflag, tval, out, err, s); break;
    case 2: seg_scan_impl<2>(a, tflag, tval, out, err, s); break;
    case 3: seg_scan_impl<3>(a, tflag, tval, out, err, s); break;
    case 4: seg_scan_impl<4>(a, tflag, tval, out, err, s); break;
    case 5: seg_scan_impl<5>(a, tflag, tval, out, err, s); break;
    default: throw std::runtime_error("win_seg_scan: bad op");
  }
}

void win_bounds(int64_t n, const int64_t* seg_start, const int64_t* seg_end, const int64_t* peer_start,
                const int64_t* peer_end, int unit, int skind, int64_t soff_i, double soff_f, int ekind,
                int64_t eoff_i, double eoff_f, const void* key, bool key_f64, const uint8_t* key_valid, bool desc,
                const int64_t* gnum, const int64_t* gpos, int64_t ngroups, int64_t* lo, int64_t* hi,
                hipStream_t s) {
  if (n == 0) return;
  BoundArgs a{n, seg_start, seg_end, peer_start, peer_end, unit, skind, ekind, soff_i, eoff_i, soff_f, eoff_f,
              key, key_f64, key_valid, desc, gnum, gpos, ngroups};
  hipLaunchKernelGGL(win_bounds_kernel, dim3(grid_for(n, kBlock, INT32_MAX)), dim3(kBlock), 0, s, a, lo, hi);
  check_launch("win.bounds", s);
}

void win_frame_sum(const int64_t* psum, bool f64, const int64_t* pcnt, const int64_t* lo, const int64_t* hi,
                   int64_t n, int64_t* sum_out, int64_t* cnt_out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(win_frame_sum_kernel, dim3(grid_for(n, kBlock, INT32_MAX)), dim3(kBlock), 0, s, psum, f64, pcnt,
                     lo, hi, n, sum_out, cnt_out);
  check_launch("win.frame_sum", s);
}

void win_sparse_build(const int64_t* vals, bool f64, const uint8_t* valid, int64_t n, bool is_max, int levels,
                      int64_t* table, hipStream_t s) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 1 << 16)), b(kBlock);
  hipLaunchKernelGGL(win_sparse_init_kernel, g, b, 0, s, vals, f64, valid, n, is_max, table);
  for (int k = 1; k < levels; ++k)
    hipLaunchKernelGGL(win_sparse_level_kernel, g, b, 0, s, table + (int64_t)(k - 1) * n, table + (int64_t)k * n, n,
                       (int64_t)1 << (k - 1), is_max);
  check_launch("win_sparse_build", s);
}

void win_sparse_query(const int64_t* table, int levels, int64_t n, const int64_t* lo, const int64_t* hi,
                      const int64_t* pcnt, bool is_max, bool f64, int64_t* out, uint8_t* out_valid, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(win_sparse_query_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, s, table, levels,
                     n, lo, hi, pcnt, is_max, f64, out, out_valid);
  check_launch("win_sparse_query", s);
}

void win_frame_minmax(const int64_t* vals, bool f64, bool is_max, const uint8_t* valid, const int64_t* lo,
                      const int64_t* hi, int64_t n, int64_t* out, uint8_t* out_valid, hipStream_t s) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, INT32_MAX)), b(kBlock);
  if (f64) {
    if (is_max) hipLaunchKernelGGL((win_frame_minmax_kernel<true, true>), g, b, 0, s, vals, valid, lo, hi, n, out, out_valid);
    else hipLaunchKernelGGL((win_frame_minmax_kernel<true, false>), g, b, 0, s, vals, valid, lo, hi, n, out, out_valid);
  } else {
    if (is_max) hipLaunchKernelGGL((win_frame_minmax_kernel<false, true>), g, b, 0, s, vals, valid, lo, hi, n, out, out_valid);
    else hipLaunchKernelGGL((win_frame_minmax_kernel<false, false>), g, b, 0, s, vals, valid, lo, hi, n, out, out_valid);
  }
  check_launch("win.frame_minmax", s);
}

void win_rank(int fn, int64_t arg, int64_t n, const int64_t* seg_start, const int64_t* seg_end,
              const int64_t* peer_start, const int64_t* peer_end, const int64_t* dense, int64_t* out,
              hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(win_rank_kernel, dim3(grid_for(n, kBlock, INT32_MAX)), dim3(kBlock), 0, s, fn, arg, n, seg_start,
                     seg_end, peer_start, peer_end, dense, out);
  check_launch("win.rank", s);
}

void win_index(int fn, int64_t arg, int64_t n, const int64_t* seg_start, const int64_t* seg_end, const int64_t* lo,
               const int64_t* hi, int64_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(win_index_kernel, dim3(grid_for(n, kBlock, INT32_MAX)), dim3(kBlock), 0, s, fn, arg, n,
                     seg_start, seg_end, lo, hi, out);
  check_launch("win.index", s);
}

}  // namespace kern
}  // namespace igloo
