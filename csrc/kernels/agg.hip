// Fused hash-aggregate update: one pass over the group ids updates up to
// kMaxAggs aggregate states (SUM/COUNT/MIN/MAX over int64, int32, f64).
//
// Replaces DataFusion's AggregateExec (partial and final modes) that the
// reference reaches through QueryEngine::execute (reference
// crates/engine/src/lib.rs:54-57). Integer SUMs are exact: they accumulate
// into 128-bit (lo, hi) pairs so SF100 decimal sums cannot overflow.
//
// Three regimes, chosen on the host by group count:
//   * ngroups == 1: per-lane register accumulation, one atomic per wave;
//   * small ngroups (state fits LDS): per-workgroup LDS privatisation, one
//     global atomic per (workgroup, group, aggregate) at the end
//     (TPC-H Q1 has 4 groups);
//   * non-decreasing group ids (clustered keys): run-by-run register folding,
//     atomics only at chunk edges;
//   * otherwise: direct global atomics (high-cardinality GROUP BY).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

struct AggParams {
  int nagg;
  AggDesc d[kMaxAggs];
};

__device__ inline bool row_valid(const AggDesc& a, int64_t i) { return !a.valid || a.valid[i]; }

__device__ inline int64_t load_int(const AggDesc& a, int64_t i) {
  return a.src64 ? ((const int64_t*)a.src)[i] : (int64_t)((const int32_t*)a.src)[i];
}

// ---- state update primitives (work on LDS or global pointers alike) -------
__device__ inline void upd(const AggDesc& a, int64_t i, unsigned long long* lo, long long* hi) {
  switch (a.op) {
    case AGG_SUM_INT: {
      int64_t v = load_int(a, i);
      atomic_add_i128(lo, hi, v);
      break;
    }
    case AGG_SUM_F64:
      atomicAdd((double*)lo, ((const double*)a.src)[i]);
      break;
    case AGG_COUNT:
      atomicAdd(lo, 1ULL);
      break;
    case AGG_MIN_INT:
      atomicMin((long long*)lo, (long long)load_int(a, i));
      break;
    case AGG_MAX_INT:
      atomicMax((long long*)lo, (long long)load_int(a, i));
      break;
    case AGG_MIN_F64:
      atomicMin((long long*)lo, (long long)f64_to_ordered(((const double*)a.src)[i]));
      break;
    case AGG_MAX_F64:
      atomicMax((long long*)lo, (long long)f64_to_ordered(((const double*)a.src)[i]));
      break;
    case AGG_BIT_AND:
      atomicAnd(lo, (unsigned long long)load_int(a, i));
      break;
    case AGG_BIT_OR:
      atomicOr(lo, (unsigned long long)load_int(a, i));
      break;
    case AGG_BIT_XOR:
      atomicXor(lo, (unsigned long long)load_int(a, i));
      break;
  }
}

__device__ inline void init_state(int op, unsigned long long* lo, long long* hi) {
  switch (op) {
    case AGG_MIN_INT:
    case AGG_MIN_F64:
      *(long long*)lo = INT64_MAX;
      break;
    case AGG_MAX_INT:
    case AGG_MAX_F64:
      *(long long*)lo = INT64_MIN;
      break;
    case AGG_BIT_AND:
      *lo = ~0ULL;
      break;
    default:
      *lo = 0;
  }
  *hi = 0;
}

// merge an LDS/register state into the global output (a group id past the
// state arrays -- a replayed group count below the real one -- is dropped;
// the end-of-query check re-executes the query)
__device__ inline void merge_global(const AggDesc& a, int64_t g, unsigned long long lo, long long hi) {
  if (a.groups && (uint64_t)g >= (uint64_t)a.groups) return;
  unsigned long long* dlo = (unsigned long long*)a.dst + g;
  switch (a.op) {
    case AGG_SUM_INT:
      if (lo != 0 || hi != 0) atomic_add_i128_parts(dlo, a.dst2 ? (long long*)a.dst2 + g : nullptr, lo, hi);
      break;
    case AGG_SUM_F64: {
      double d;
      __builtin_memcpy(&d, &lo, 8);
      if (d != 0.0) atomicAdd((double*)dlo, d);
      break;
    }
    case AGG_COUNT:
      if (lo) atomicAdd(dlo, lo);
      break;
    case AGG_MIN_INT:
    case AGG_MIN_F64:
      if ((long long)lo != INT64_MAX) atomicMin((long long*)dlo, (long long)lo);
      break;
    case AGG_MAX_INT:
    case AGG_MAX_F64:
      if ((long long)lo != INT64_MIN) atomicMax((long long*)dlo, (long long)lo);
      break;
    case AGG_BIT_AND:
      if (lo != ~0ULL) atomicAnd(dlo, lo);
      break;
    case AGG_BIT_OR:
      if (lo) atomicOr(dlo, lo);
      break;
    case AGG_BIT_XOR:
      if (lo) atomicXor(dlo, lo);
      break;
  }
}

// ---------------------------------------------------------------- regimes
__global__ __launch_bounds__(kBlock) void agg_global_kernel(const int32_t* __restrict__ gid, int64_t n, AggParams p) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t g = gid[i];
    for (int k = 0; k < p.nagg; ++k) {
      const AggDesc& a = p.d[k];
      if (!row_valid(a, i) || (uint64_t)g >= (uint64_t)a.groups) continue;
      upd(a, i, (unsigned long long*)a.dst + g, a.dst2 ? (long long*)a.dst2 + g : nullptr);
    }
  }
}

// LDS layout: [nagg][ngroups] x {lo u64, hi i64}
__global__ __launch_bounds__(kBlock) void agg_lds_kernel(const int32_t* __restrict__ gid, int64_t n, int ngroups,
                                                        AggParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
  unsigned long long* slo = lds;
  long long* shi = (long long*)(lds + (size_t)p.nagg * ngroups);
  for (int idx = threadIdx.x; idx < p.nagg * ngroups; idx += blockDim.x) init_state(p.d[idx / ngroups].op, &slo[idx], &shi[idx]);
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int g = gid ? gid[i] : 0;
    if ((unsigned)g >= (unsigned)ngroups) continue;
    for (int k = 0; k < p.nagg; ++k) {
      const AggDesc& a = p.d[k];
      if (!row_valid(a, i)) continue;
      int idx = k * ngroups + g;
      upd(a, i, &slo[idx], &shi[idx]);
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < p.nagg * ngroups; idx += blockDim.x) {
    int k = idx / ngroups, g = idx % ngroups;
    merge_global(p.d[k], g, slo[idx], shi[idx]);
  }
}

// Non-decreasing group ids (clustered input, e.g. lineitem by l_orderkey):
// each wave takes 64 consecutive rows (coalesced loads), runs a segmented
// inclusive scan across lanes (segments = equal gids, so no head flags are
// needed), and the last lane of every segment writes the total. A segment
// that touches either edge of the 64-row tile may continue in a neighbouring
// tile and merges atomically; interior segments belong to this wave alone and
// are stored without atomics.
__device__ inline void seg_combine(int op, unsigned long long* lo, long long* hi, unsigned long long olo, long long ohi) {
  switch (op) {
    case AGG_SUM_INT: {
      unsigned long long s = *lo + olo;
      *hi = *hi + ohi + (s < *lo ? 1 : 0);
      *lo = s;
      break;
    }
    case AGG_SUM_F64: {
      double x, y;
      __builtin_memcpy(&x, lo, 8);
      __builtin_memcpy(&y, &olo, 8);
      x += y;
      __builtin_memcpy(lo, &x, 8);
      break;
    }
    case AGG_COUNT:
      *lo += olo;
      break;
    case AGG_MIN_INT:
    case AGG_MIN_F64:
      if ((long long)olo < (long long)*lo) *lo = olo;
      break;
    case AGG_BIT_AND:
      *lo &= olo;
      break;
    case AGG_BIT_OR:
      *lo |= olo;
      break;
    case AGG_BIT_XOR:
      *lo ^= olo;
      break;
    default:
      if ((long long)olo > (long long)*lo) *lo = olo;
      break;
  }
}

__device__ inline void row_state(const AggDesc& a, int64_t i, bool live, unsigned long long* lo, long long* hi) {
  init_state(a.op, lo, hi);
  if (!live || !row_valid(a, i)) return;
  switch (a.op) {
    case AGG_SUM_INT: {
      const int64_t v = load_int(a, i);
      *lo = (unsigned long long)v;
      *hi = v < 0 ? -1 : 0;
      break;
    }
    case AGG_SUM_F64:
      __builtin_memcpy(lo, &((const double*)a.src)[i], 8);
      break;
    case AGG_COUNT:
      *lo = 1;
      break;
    case AGG_MIN_INT:
    case AGG_MAX_INT:
    case AGG_BIT_AND:
    case AGG_BIT_OR:
    case AGG_BIT_XOR:
      *lo = (unsigned long long)load_int(a, i);
      break;
    default:
      *lo = (unsigned long long)f64_to_ordered(((const double*)a.src)[i]);
      break;
  }
}

__device__ inline void store_exclusive(const AggDesc& a, int64_t g, unsigned long long lo, long long hi) {
  if (a.groups && (uint64_t)g >= (uint64_t)a.groups) return;   // see merge_global
  ((unsigned long long*)a.dst)[g] = lo;
  if (a.op == AGG_SUM_INT && a.dst2) ((long long*)a.dst2)[g] = hi;
}

// Non-decreasing group ids, chunked: each lane folds kSortedRows consecutive
// rows in registers first (segments closed inside the chunk are stored
// directly), so the cross-lane segmented scan runs once per kSortedRows rows
// instead of once per row. Per lane: head = first segment of the chunk (gid
// gH, may continue from earlier lanes), tail = last segment (gid gT, may
// continue into later lanes); a one-segment chunk only has a tail. The scan
// chains tails with equal gids (non-decreasing gids: equal => contiguous).
// A segment that may cross the wave's tile (its chain starts at a one-segment
// lane 0, or it is lane 0's head, or lane 63's tail) merges atomically.
constexpr int kSortedRows = 8;

// A lane's 8 consecutive rows in as few loads as possible (full, aligned
// chunks: 2x16 B of gids, 4x16 B of int64/f64 values, one 8 B validity word).
// With one scalar load per row, 16 resident waves' 6 KB tiles overflow the
// 32 KB vector L1 and every line is refetched up to 8 times.
__device__ inline void load_gids8(const int32_t* gid, int64_t r0, int64_t n, int g[kSortedRows]) {
  if (r0 + kSortedRows <= n && ((uintptr_t)(gid + r0) & 15) == 0) {
    const int4 a = *(const int4*)(gid + r0), b = *(const int4*)(gid + r0 + 4);
    g[0] = a.x; g[1] = a.y; g[2] = a.z; g[3] = a.w;
    g[4] = b.x; g[5] = b.y; g[6] = b.z; g[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) g[j] = r0 + j < n ? gid[r0 + j] : -1;
  }
}

// raw 64-bit row payloads (int sign-extended / f64 bits / 1 for COUNT) and validity bits
__device__ inline unsigned load_vals8(const AggDesc& a, int64_t r0, int64_t n, unsigned long long v[kSortedRows]) {
  const bool full = r0 + kSortedRows <= n;
  unsigned ok = 0;
  if (a.valid) {
    if (full && ((uintptr_t)(a.valid + r0) & 7) == 0) {
      const unsigned long long w = *(const unsigned long long*)(a.valid + r0);
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) ok |= ((w >> (8 * j)) & 0xff) ? (1u << j) : 0u;
    } else {
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) ok |= (r0 + j < n && a.valid[r0 + j]) ? (1u << j) : 0u;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) ok |= r0 + j < n ? (1u << j) : 0u;
  }
  if (a.op == AGG_COUNT) {
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) v[j] = 1;
    return ok;
  }
  const bool wide = a.op == AGG_SUM_F64 || a.op == AGG_MIN_F64 || a.op == AGG_MAX_F64 || a.src64;
  if (wide) {
    const unsigned long long* src = (const unsigned long long*)a.src + r0;
    if (full && ((uintptr_t)src & 15) == 0) {
#pragma unroll
      for (int j = 0; j < kSortedRows; j += 2) {
        const ulonglong2 x = *(const ulonglong2*)(src + j);
        v[j] = x.x;
        v[j + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) v[j] = r0 + j < n ? src[j] : 0;
    }
    if (a.op == AGG_MIN_F64 || a.op == AGG_MAX_F64) {
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) {
        double d;
        __builtin_memcpy(&d, &v[j], 8);
        v[j] = (unsigned long long)f64_to_ordered(d);
      }
    }
  } else {
    const int32_t* src = (const int32_t*)a.src + r0;
    if (full && ((uintptr_t)src & 15) == 0) {
      const int4 x = *(const int4*)src, y = *(const int4*)(src + 4);
      v[0] = (long long)x.x; v[1] = (long long)x.y; v[2] = (long long)x.z; v[3] = (long long)x.w;
      v[4] = (long long)y.x; v[5] = (long long)y.y; v[6] = (long long)y.z; v[7] = (long long)y.w;
    } else {
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) v[j] = r0 + j < n ? (unsigned long long)(long long)src[j] : 0;
    }
  }
  return ok;
}

__global__ __launch_bounds__(kBlock) void agg_sorted_chunk_kernel(const int32_t* __restrict__ gid, int64_t n,
                                                                 AggParams p) {
  const int lane = lane_id();
  const int64_t wave_id = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  constexpr int64_t kTileRows = (int64_t)kWave * kSortedRows;
  for (int64_t base = wave_id * kTileRows; base < n; base += nwaves * kTileRows) {
    const int64_t r0 = base + (int64_t)lane * kSortedRows;
    int g[kSortedRows];
    load_gids8(gid, r0, n, g);
    const bool valid = g[0] >= 0;
    int gT = g[0];
    bool multi = false;
#pragma unroll
    for (int j = 1; j < kSortedRows; ++j) {
      if (g[j] >= 0) {
        multi |= g[j] != gT;
        gT = g[j];
      }
    }
    const int gH = g[0];
    // chain start lane over equal tails
    int og[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) og[s] = __shfl_up(gT, 1 << s, kWave);
    int start = lane;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
      const int o = __shfl_up(start, 1 << s, kWave);
      if (lane >= (1 << s) && og[s] == gT && o < start) start = o;
    }
    const bool multi0 = __shfl(multi ? 1 : 0, 0, kWave) != 0;
    const int prev_gT = og[0];
    const int prev_start = __shfl_up(start, 1, kWave);
    const int next_gH = __shfl_down(gH, 1, kWave);
    const bool has_carry = lane > 0 && prev_gT == gH;
    const bool head_atomic = lane == 0 || (has_carry && prev_start == 0 && !multi0);
    const bool tail_end = valid && (lane == kWave - 1 || next_gH != gT);
    const bool tail_atomic = lane == kWave - 1 || (start == 0 && !multi0);
    for (int k = 0; k < p.nagg; ++k) {
      const AggDesc& a = p.d[k];
      unsigned long long lo, hlo = 0;
      long long hi, hhi = 0;
      init_state(a.op, &lo, &hi);
      unsigned long long v[kSortedRows];
      const unsigned ok = load_vals8(a, r0, n, v);
      bool in_head = true;
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) {
        if (g[j] < 0) break;
        if (j > 0 && g[j] != g[j - 1]) {
          if (in_head) {
            hlo = lo;
            hhi = hi;
            in_head = false;
          } else {
            store_exclusive(a, g[j - 1], lo, hi);
          }
          init_state(a.op, &lo, &hi);
        }
        if (ok & (1u << j))
          seg_combine(a.op, &lo, &hi, v[j], a.op == AGG_SUM_INT && (long long)v[j] < 0 ? -1LL : 0LL);
      }
      // segmented inclusive scan of the tails across lanes
#pragma unroll
      for (int s = 0; s < 6; ++s) {
        const unsigned long long olo = __shfl_up(lo, 1 << s, kWave);
        const long long ohi = __shfl_up(hi, 1 << s, kWave);
        if (lane >= (1 << s) && og[s] == gT) seg_combine(a.op, &lo, &hi, olo, ohi);
      }
      const unsigned long long clo = __shfl_up(lo, 1, kWave);
      const long long chi = __shfl_up(hi, 1, kWave);
      if (valid && multi) {
        if (has_carry) seg_combine(a.op, &hlo, &hhi, clo, chi);
        if (head_atomic) merge_global(a, gH, hlo, hhi);
        else store_exclusive(a, gH, hlo, hhi);
      }
      if (tail_end) {
        if (tail_atomic) merge_global(a, gT, lo, hi);
        else store_exclusive(a, gT, lo, hi);
      }
    }
  }
}

// Single group: registers -> wave reduction (every lane ends with the total)
// -> workgroup combine in LDS -> one global atomic per workgroup and aggregate.
// (One atomic per WAVE put 16K same-address atomics on one word per launch:
// they serialise at the memory side, ~140 us for 15 MB of input.)
__device__ inline void wave_fold(const AggDesc& a, unsigned long long& lo, long long& hi) {
  for (int off = kWave / 2; off > 0; off >>= 1) {
    unsigned long long olo = __shfl_xor(lo, off, kWave);
    long long ohi = __shfl_xor(hi, off, kWave);
    switch (a.op) {
      case AGG_SUM_INT: {
        unsigned long long s = lo + olo;
        hi = hi + ohi + (s < lo ? 1 : 0);
        lo = s;
        break;
      }
      case AGG_SUM_F64: {
        double x, y;
        __builtin_memcpy(&x, &lo, 8);
        __builtin_memcpy(&y, &olo, 8);
        x += y;
        __builtin_memcpy(&lo, &x, 8);
        break;
      }
      case AGG_COUNT:
        lo += olo;
        break;
      case AGG_MIN_INT:
      case AGG_MIN_F64:
        lo = (long long)olo < (long long)lo ? olo : lo;
        break;
      case AGG_MAX_INT:
      case AGG_MAX_F64:
        lo = (long long)olo > (long long)lo ? olo : lo;
        break;
      case AGG_BIT_AND:
        lo &= olo;
        break;
      case AGG_BIT_OR:
        lo |= olo;
        break;
      case AGG_BIT_XOR:
        lo ^= olo;
        break;
    }
  }
}

__global__ __launch_bounds__(kBlock) void agg_single_kernel(int64_t n, AggParams p) {
  unsigned long long lo[kMaxAggs];
  long long hi[kMaxAggs];
#pragma unroll
  for (int k = 0; k < kMaxAggs; ++k)
    if (k < p.nagg) init_state(p.d[k].op, &lo[k], &hi[k]);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int k = 0; k < kMaxAggs; ++k) {
      if (k >= p.nagg) break;
      const AggDesc& a = p.d[k];
      if (!row_valid(a, i)) continue;
      switch (a.op) {
        case AGG_SUM_INT: {
          int64_t v = load_int(a, i);
          unsigned long long s = lo[k] + (unsigned long long)v;
          hi[k] += (v < 0 ? -1 : 0) + (s < lo[k] ? 1 : 0);
          lo[k] = s;
          break;
        }
        case AGG_SUM_F64: {
          double x;
          __builtin_memcpy(&x, &lo[k], 8);
          x += ((const double*)a.src)[i];
          __builtin_memcpy(&lo[k], &x, 8);
          break;
        }
        case AGG_COUNT:
          lo[k] += 1;
          break;
        case AGG_MIN_INT: {
          long long v = load_int(a, i);
          if (v < (long long)lo[k]) lo[k] = (unsigned long long)v;
          break;
        }
        case AGG_MAX_INT: {
          long long v = load_int(a, i);
          if (v > (long long)lo[k]) lo[k] = (unsigned long long)v;
          break;
        }
        case AGG_MIN_F64: {
          long long v = f64_to_ordered(((const double*)a.src)[i]);
          if (v < (long long)lo[k]) lo[k] = (unsigned long long)v;
          break;
        }
        case AGG_MAX_F64: {
          long long v = f64_to_ordered(((const double*)a.src)[i]);
          if (v > (long long)lo[k]) lo[k] = (unsigned long long)v;
          break;
        }
        case AGG_BIT_AND:
          lo[k] &= (unsigned long long)load_int(a, i);
          break;
        case AGG_BIT_OR:
          lo[k] |= (unsigned long long)load_int(a, i);
          break;
        case AGG_BIT_XOR:
          lo[k] ^= (unsigned long long)load_int(a, i);
          break;
      }
    }
  }
  __shared__ unsigned long long blo[kMaxAggs][kWavesPerBlock];
  __shared__ long long bhi[kMaxAggs][kWavesPerBlock];
  const int w = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < kMaxAggs; ++k)
    if (k < p.nagg) {
      wave_fold(p.d[k], lo[k], hi[k]);
      if (lane_id() == 0) {
        blo[k][w] = lo[k];
        bhi[k][w] = hi[k];
      }
    }
  __syncthreads();
  if (threadIdx.x < p.nagg) {
    const int k = threadIdx.x;
    unsigned long long l = blo[k][0];
    long long h = bhi[k][0];
    for (int v = 1; v < kWavesPerBlock; ++v) seg_combine(p.d[k].op, &l, &h, blo[k][v], bhi[k][v]);
    merge_global(p.d[k], 0, l, h);
  }
}


// ---- sorted GROUP BY key HAVING <aggregate> <cmp> <constant>, fused --------
// TPC-H Q18's "l_orderkey IN (SELECT l_orderkey FROM lineitem GROUP BY
// l_orderkey HAVING sum(l_quantity) > 300)": lineitem is clustered by
// l_orderkey, 600M rows form 150M runs of which ~6.5K pass. The general path
// materialises run ids, 150M 128-bit partial states, and compacts them; here
// each lane owns the runs that START among its 8 rows (vector loads), folds
// them in registers, follows its last run past its chunk with cache-hot
// scalar loads (at most kHavingMaxRun rows, else the overflow flag sends the
// host to the general path), and only the passing runs are written: a lane
// counts its passing runs, the wave takes one atomic for all of them, and a
// second walk over the same registers writes them. Output order depends on
// the atomics; the host sorts the (small) result by run start row.
constexpr int kHavingMaxAggs = 4;
constexpr int64_t kHavingMaxRun = 256;

struct HavingParams {
  int nagg;
  AggDesc d[kHavingMaxAggs];
  int hagg, hop;   // compared aggregate; 0 '=', 1 '<>', 2 '<', 3 '<=', 4 '>', 5 '>='
  long long hlo, hhi;  // integer constant as int128 (units of the aggregate's state)
  double hf;           // constant for f64 aggregates
};

__device__ inline bool having_ok(const HavingParams& p, unsigned long long lo, long long hi) {
  const int op = p.d[p.hagg].op;
  int c;
  if (op == AGG_SUM_F64 || op == AGG_MIN_F64 || op == AGG_MAX_F64) {
    double x;
    if (op == AGG_SUM_F64) __builtin_memcpy(&x, &lo, 8);
    else x = ordered_to_f64((long long)lo);
    if (x != x) return false;   // NaN compares false
    c = x < p.hf ? -1 : (x > p.hf ? 1 : 0);
  } else {
    const long long h = op == AGG_SUM_INT ? hi : ((long long)lo < 0 ? -1LL : 0LL);
    if (h != p.hhi) c = h < p.hhi ? -1 : 1;
    else c = lo < (unsigned long long)p.hlo ? -1 : (lo > (unsigned long long)p.hlo ? 1 : 0);
  }
  switch (p.hop) {
    case 0: return c == 0;
    case 1: return c != 0;
    case 2: return c < 0;
    case 3: return c <= 0;
    case 4: return c > 0;
    default: return c >= 0;
  }
}

// one row of aggregate a from global memory (overhang rows)
__device__ inline bool row_value(const AggDesc& a, int64_t i, unsigned long long* v) {
  if (a.valid && !a.valid[i]) return false;
  if (a.op == AGG_COUNT) {
    *v = 1;
  } else if (a.op == AGG_SUM_F64 || a.op == AGG_MIN_F64 || a.op == AGG_MAX_F64) {
    const double d = ((const double*)a.src)[i];
    if (a.op == AGG_SUM_F64) __builtin_memcpy(v, &d, 8);
    else *v = (unsigned long long)f64_to_ordered(d);
  } else {
    *v = a.src64 ? (unsigned long long)((const int64_t*)a.src)[i]
                 : (unsigned long long)(long long)((const int32_t*)a.src)[i];
  }
  return true;
}

__device__ inline void fold(int op, unsigned long long* lo, long long* hi, unsigned long long x) {
  seg_combine(op, lo, hi, x, op == AGG_SUM_INT && (long long)x < 0 ? -1LL : 0LL);
}

// The runs starting among a lane's 8 rows, folded for ONE aggregate: emit(j,
// lo, hi) for the run starting at row r0 + j. The last run is followed past
// the chunk (4 rows per round trip) while the key repeats, for at most
// kHavingMaxRun rows (*overflow set beyond).
template <typename K, typename Emit>
__device__ inline void fold_runs(const AggDesc& a, const K* __restrict__ keys, int64_t n, int64_t r0,
                                 const K (&k)[kSortedRows], unsigned starts, bool* overflow, bool wave_converged,
                                 Emit emit) {
  unsigned long long v[kSortedRows];
  const unsigned ok = load_vals8(a, r0, n, v);
  // the next lane's rows (shuffled in while the whole wave is converged): a
  // run that spills past this lane's chunk usually ends inside them
  unsigned long long nv[kSortedRows];
  unsigned nok = 0, nst = 0;
  if (wave_converged) {
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) nv[j] = __shfl_down(v[j], 1, kWave);
    nok = __shfl_down(ok, 1, kWave);
    nst = __shfl_down(starts, 1, kWave);
  }
  unsigned long long lo = 0;
  long long hi = 0;
  int open = -1;
#pragma unroll
  for (int j = 0; j < kSortedRows; ++j) {
    if ((starts >> j) & 1u) {
      if (open >= 0) emit(open, lo, hi);
      open = j;
      init_state(a.op, &lo, &hi);
    }
    if (open >= 0 && ((ok >> j) & 1u)) fold(a.op, &lo, &hi, v[j]);
  }
  if (open < 0) return;
  const K key = k[open];
  int64_t r = r0 + kSortedRows;
  bool more = r < n;
  if (more && wave_converged && lane_id() < kWave - 1) {
    // rows of the next lane up to its first run start
    const int64_t live = n - r < kSortedRows ? n - r : kSortedRows;
    const int c = nst ? __builtin_ctz(nst) : kSortedRows;
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j)
      if (j < c && j < live && ((nok >> j) & 1u)) fold(a.op, &lo, &hi, nv[j]);
    more = c == kSortedRows && live == kSortedRows;
    r += kSortedRows;
    more = more && r < n;
  }
  while (more) {
    K kk[4];
    unsigned long long x[4];
    bool xv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool in = r + q < n;
      kk[q] = in ? keys[r + q] : key;
      xv[q] = in && row_value(a, r + q, &x[q]);
      if (!in) kk[q] = (K)(key + 1);   // past the end: the run stops there
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (!more) break;
      if (kk[q] != key) {
        more = false;
        break;
      }
      if (xv[q]) fold(a.op, &lo, &hi, x[q]);
    }
    r += 4;
    if (more && r - (r0 + open) >= kHavingMaxRun) {
      *overflow = true;
      more = false;
    }
  }
  emit(open, lo, hi);
}

template <typename K>
__global__ __launch_bounds__(kBlock) void sorted_having_kernel(const K* __restrict__ keys, int64_t n, HavingParams p,
                                                              int64_t* __restrict__ rep, int64_t cap,
                                                              unsigned long long* __restrict__ counter) {
  const int lane = lane_id();
  const int64_t wave_id = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  constexpr int64_t kTileRows = (int64_t)kWave * kSortedRows;
  bool overflow = false;
  for (int64_t base = wave_id * kTileRows; base < n; base += nwaves * kTileRows) {
    const int64_t r0 = base + (int64_t)lane * kSortedRows;
    K k[kSortedRows];
    if (r0 + kSortedRows <= n && sizeof(K) == 4 && ((uintptr_t)(keys + r0) & 15) == 0) {
      const int4 a = *(const int4*)(keys + r0), b = *(const int4*)(keys + r0 + 4);
      k[0] = (K)a.x; k[1] = (K)a.y; k[2] = (K)a.z; k[3] = (K)a.w;
      k[4] = (K)b.x; k[5] = (K)b.y; k[6] = (K)b.z; k[7] = (K)b.w;
    } else {
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) k[j] = r0 + j < n ? keys[r0 + j] : (K)0;
    }
    const K kprev = (r0 < n && r0 > 0) ? keys[r0 - 1] : (K)0;
    unsigned starts = 0;
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) {
      const bool st = r0 + j < n && (r0 + j == 0 || k[j] != (j ? k[j - 1] : kprev));
      starts |= st ? (1u << j) : 0u;
    }
    // pass 0: the HAVING aggregate alone decides which runs pass
    unsigned passmask = 0;
    fold_runs(p.d[p.hagg], keys, n, r0, k, starts, &overflow, true, [&](int j, unsigned long long lo, long long hi) {
      if (having_ok(p, lo, hi)) passmask |= 1u << j;
    });
    const int npass = __popc(passmask);
    const int64_t inc = wave_inclusive_scan((int64_t)npass);
    const int64_t total = __shfl(inc, kWave - 1, kWave);
    if (total == 0) continue;
    // one atomic per wave for its passing runs; pass 1 writes them
    unsigned long long wbase = 0;
    if (lane == kWave - 1) wbase = atomicAdd(&counter[0], (unsigned long long)total);
    wbase = __shfl(wbase, kWave - 1, kWave);
    const int64_t slot0 = (int64_t)wbase + inc - npass;
    if (!passmask) continue;
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j)
      if ((passmask >> j) & 1u) {
        const int64_t o = slot0 + __popc(passmask & ((1u << j) - 1u));
        if (o < cap) rep[o] = r0 + j;
      }
    for (int a = 0; a < p.nagg; ++a) {
      const AggDesc& d = p.d[a];
      bool ovf2 = false;
      fold_runs(d, keys, n, r0, k, starts, &ovf2, false, [&](int j, unsigned long long lo, long long hi) {
        if (!((passmask >> j) & 1u)) return;
        const int64_t o = slot0 + __popc(passmask & ((1u << j) - 1u));
        if (o < cap) {
          ((unsigned long long*)d.dst)[o] = lo;
          if (d.dst2) ((long long*)d.dst2)[o] = hi;
        }
      });
    }
  }
  if (__any(overflow) && lane == 0) atomicOr(&counter[1], 1ULL);
}

// Streaming variant for the common shape (TPC-H Q18: HAVING sum(int32) with
// COUNT(*) alongside): every aggregate is either THE valued one -- a SUM over
// an int32 column without NULLs, summed in int64 (2^32 rows of int32 cannot
// overflow it) -- or a COUNT without a validity mask, which is the run's
// length. Each wave owns a contiguous span of rows and walks it in 512-row
// tiles (8 rows per lane, 16 B loads, the next tile prefetched into
// registers), so a run crossing lanes or tiles costs no extra memory round
// trip: the open run's value is carried from tile to tile, and across lanes
// it comes from one plain wave prefix sum of the lanes' totals -- the value
// of a run closing in lane l is (prefix at its end) - (prefix at its start),
// its start lane found from a ballot of the lanes holding run starts. A run
// is owned by the wave holding its first row; the one still open at the span
// end is followed past it 64 rows per step. No run-length limit.
constexpr int kScanTile = kWave * kSortedRows;

template <typename K>
__device__ inline void load_keys8(const K* __restrict__ keys, int64_t r0, int live, K k[kSortedRows]) {
  if (live == kSortedRows && ((uintptr_t)(keys + r0) & 15) == 0) {
    if (sizeof(K) == 4) {
      const int4 a = *(const int4*)(keys + r0), b = *(const int4*)(keys + r0 + 4);
      k[0] = (K)a.x; k[1] = (K)a.y; k[2] = (K)a.z; k[3] = (K)a.w;
      k[4] = (K)b.x; k[5] = (K)b.y; k[6] = (K)b.z; k[7] = (K)b.w;
    } else {
#pragma unroll
      for (int j = 0; j < kSortedRows; j += 2) {
        const longlong2 x = *(const longlong2*)(keys + r0 + j);
        k[j] = (K)x.x;
        k[j + 1] = (K)x.y;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) k[j] = j < live ? keys[r0 + j] : (K)0;
  }
}

// 8 values of VB bytes (4, 2, 1: int32 / int16 / int8, sign-extended) in one
// or two vector loads
template <int VB>
__device__ inline void load_v8(const void* __restrict__ src, int64_t r0, int live, int x[kSortedRows]) {
  if (VB == 4) {
    const int32_t* v = (const int32_t*)src;
    if (live == kSortedRows && ((uintptr_t)(v + r0) & 15) == 0) {
      const int4 a = *(const int4*)(v + r0), b = *(const int4*)(v + r0 + 4);
      x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
      x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
      return;
    }
  } else if (VB == 2) {
    const int16_t* v = (const int16_t*)src;
    if (live == kSortedRows && ((uintptr_t)(v + r0) & 15) == 0) {
      const uint4 a = *(const uint4*)(v + r0);
      const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[2 * j] = (int)(int16_t)(w[j] & 0xffff);
        x[2 * j + 1] = (int)(int16_t)(w[j] >> 16);
      }
      return;
    }
  } else {
    const int8_t* v = (const int8_t*)src;
    if (live == kSortedRows && ((uintptr_t)(v + r0) & 7) == 0) {
      const uint2 a = *(const uint2*)(v + r0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = (int)(int8_t)((a.x >> (8 * j)) & 0xff);
        x[4 + j] = (int)(int8_t)((a.y >> (8 * j)) & 0xff);
      }
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < kSortedRows; ++j)
    x[j] = j >= live ? 0 : VB == 4 ? ((const int32_t*)src)[r0 + j] : VB == 2 ? (int)((const int16_t*)src)[r0 + j]
                                                                          : (int)((const int8_t*)src)[r0 + j];
}

__device__ inline int load_v1(const void* src, int vb, int64_t i) {
  return vb == 4 ? ((const int32_t*)src)[i] : vb == 2 ? (int)((const int16_t*)src)[i] : (int)((const int8_t*)src)[i];
}

// the value of the compared aggregate for a run of `cnt` rows summing to `sum`
__device__ inline bool scan_run_passes(const HavingParams& p, int vagg, long long sum, long long cnt) {
  const long long x = p.hagg == vagg ? sum : cnt;
  return having_ok(p, (unsigned long long)x, x < 0 ? -1LL : 0LL);
}

__device__ inline void scan_run_write(const HavingParams& p, int vagg, int64_t o, long long sum, long long cnt) {
  for (int a = 0; a < p.nagg; ++a) {
    const long long x = a == vagg ? sum : cnt;
    ((long long*)p.d[a].dst)[o] = x;
    if (p.d[a].dst2) ((long long*)p.d[a].dst2)[o] = x < 0 ? -1LL : 0LL;
  }
}

template <typename K, int VB>
__global__ __launch_bounds__(kBlock) void sorted_having_scan_kernel(const K* __restrict__ keys, int64_t n, int64_t span,
                                                                   HavingParams p, int vagg, int64_t* __restrict__ rep,
                                                                   int64_t cap,
                                                                   unsigned long long* __restrict__ counter) {
  const int lane = lane_id();
  const int64_t wave_id = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t s = wave_id * span;
  if (s >= n) return;
  const int64_t e = s + span < n ? s + span : n;
  constexpr bool HAS_V = VB > 0;
  const void* __restrict__ vals = HAS_V ? p.d[vagg].src : nullptr;
  const uint64_t below = lane ? (~0ULL >> (kWave - lane)) : 0ULL;   // lanes < this one
  // the open run entering the tile: start row (-1: it began in an earlier
  // wave's span, which owns it) and its value up to the tile
  int64_t c_row = -1;
  long long c_v = 0;
  K last = s > 0 ? keys[s - 1] : (K)0;
  K k[kSortedRows], nk[kSortedRows];
  int v[kSortedRows] = {}, nvl[kSortedRows] = {};
  {
    const int64_t r0 = s + (int64_t)lane * kSortedRows;
    const int live = (int)(e - r0 < 0 ? 0 : (e - r0 < kSortedRows ? e - r0 : kSortedRows));
    load_keys8(keys, r0, live, nk);
    if (HAS_V) load_v8<VB>(vals, r0, live, nvl);
  }
  for (int64_t base = s; base < e; base += kScanTile) {
    const int64_t r0 = base + (int64_t)lane * kSortedRows;
    const int live = (int)(e - r0 < 0 ? 0 : (e - r0 < kSortedRows ? e - r0 : kSortedRows));
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) {
      k[j] = nk[j];
      if (HAS_V) v[j] = nvl[j];
    }
    if (base + kScanTile < e) {     // prefetch the next tile while this one is folded
      const int64_t q0 = r0 + kScanTile;
      const int ql = (int)(e - q0 < 0 ? 0 : (e - q0 < kSortedRows ? e - q0 : kSortedRows));
      load_keys8(keys, q0, ql, nk);
      if (HAS_V) load_v8<VB>(vals, q0, ql, nvl);
    }
    K kp = __shfl_up(k[kSortedRows - 1], 1, kWave);
    if (lane == 0) kp = last;
    unsigned starts = 0;
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) {
      const bool st = j < live && ((r0 + j == 0) || k[j] != (j ? k[j - 1] : kp));
      starts |= st ? (1u << j) : 0u;
    }
    // lane totals, the sum before the first start (head) and before the last one
    long long tot = 0, head = 0, pre_last = 0;
    const int fs = starts ? __builtin_ctz(starts) : kSortedRows;
    const int ls = starts ? 31 - __builtin_clz(starts) : -1;
#pragma unroll
    for (int j = 0; j < kSortedRows; ++j) {
      const long long x = HAS_V ? (long long)v[j] : 0LL;
      if (j == fs) head = tot;
      if (j == ls) pre_last = tot;
      tot += x;
    }
    if (!starts) head = tot;
    const long long incl = wave_inclusive_scan(tot);
    const long long excl = incl - tot;
    const uint64_t smask = __ballot(starts != 0);
    // prefix value at (and row of) this lane's last start
    const long long q_last = excl + pre_last;
    const int row_last = ls;   // within the lane
    // run closing at this lane's first start: its start is the last start of
    // the nearest lane below holding one, else the carried run
    const uint64_t lower = smask & below;
    const int m = lower ? 63 - __builtin_clzll(lower) : lane;
    const long long q_m = __shfl(q_last, m, kWave);
    const int rl_m = __shfl(row_last, m, kWave);
    long long close_v;
    int64_t close_row;
    if (lower) {
      close_v = excl + head - q_m;
      close_row = base + (int64_t)m * kSortedRows + rl_m;
    } else {
      close_v = c_v + excl + head;
      close_row = c_row;
    }
    // count passing runs: the closing one, then those between this lane's starts
    auto runs = [&](auto&& emit) {
      if (!starts) return;
      if (close_row >= 0) emit(close_row, close_v, r0 + fs - close_row);
      long long acc = 0;
      int open = fs;
#pragma unroll
      for (int j = 0; j < kSortedRows; ++j) {
        if (j > fs && ((starts >> j) & 1u)) {
          emit(r0 + open, acc, (long long)(j - open));
          acc = 0;
          open = j;
        }
        if (j >= fs && HAS_V) acc += (long long)v[j];
      }
    };
    int npass = 0;
    runs([&](int64_t, long long sum, long long cnt) { npass += scan_run_passes(p, vagg, sum, cnt) ? 1 : 0; });
    const int64_t pinc = wave_inclusive_scan((int64_t)npass);
    const int64_t ptotal = __shfl(pinc, kWave - 1, kWave);
    if (ptotal) {
      unsigned long long wbase = 0;
      if (lane == kWave - 1) wbase = atomicAdd(&counter[0], (unsigned long long)ptotal);
      wbase = __shfl(wbase, kWave - 1, kWave);
      int64_t o = (int64_t)wbase + pinc - npass;
      runs([&](int64_t row, long long sum, long long cnt) {
        if (!scan_run_passes(p, vagg, sum, cnt)) return;
        if (o < cap) {
          rep[o] = row;
          scan_run_write(p, vagg, o, sum, cnt);
        }
        ++o;
      });
    }
    // carry the run open at the tile's end
    const long long tile_tot = __shfl(incl, kWave - 1, kWave);
    if (smask) {
      const int mt = 63 - __builtin_clzll(smask);
      c_v = tile_tot - __shfl(q_last, mt, kWave);
      c_row = base + (int64_t)mt * kSortedRows + __shfl(row_last, mt, kWave);
    } else {
      c_v += tile_tot;
    }
    last = __shfl(k[kSortedRows - 1], kWave - 1, kWave);
  }
  if (c_row < 0) return;
  // follow the open run past the span, 64 rows per step
  const K rk = keys[e - 1];
  int64_t r = e;
  while (r < n) {
    const int64_t row = r + lane;
    const bool in = row < n;
    const bool same = in && keys[row] == rk;
    const uint64_t ms = __ballot(same);
    const int stop = ~ms ? __builtin_ctzll(~ms) : kWave;   // first lane off the run
    long long x = (HAS_V && lane < stop) ? (long long)load_v1(vals, VB, row) : 0LL;
    c_v += wave_reduce_sum(x);
    r += stop;
    if (stop < kWave) break;
  }
  if (lane == 0 && scan_run_passes(p, vagg, c_v, r - c_row)) {
    const unsigned long long o = atomicAdd(&counter[0], 1ULL);
    if ((int64_t)o < cap) {
      rep[o] = c_row;
      scan_run_write(p, vagg, (int64_t)o, c_v, r - c_row);
    }
  }
}
}  // namespace

int agg_lds_max_groups(int nagg) {
  // keep the LDS state at <= 64 KiB so several workgroups stay resident per CU
  const int bytes = 64 * 1024;
  return nagg > 0 ? bytes / (16 * nagg) : 0;
}

void sorted_having(const void* keys, bool key64, int64_t n, const AggDesc* descs, int nagg, int hagg, int hop,
                   long long hlo, long long hhi, double hf, int64_t* rep, int64_t cap, unsigned long long* counter,
                   hipStream_t stream) {
  if (n <= 0) return;
  if (nagg < 1 || nagg > kHavingMaxAggs || hagg < 0 || hagg >= nagg)
    throw std::runtime_error("sorted_having: 1..4 aggregates, compared one among them");
  HavingParams p{};
  p.nagg = nagg;
  for (int k = 0; k < nagg; ++k) p.d[k] = descs[k];
  p.hagg = hagg;
  p.hop = hop;
  p.hlo = hlo;
  p.hhi = hhi;
  p.hf = hf;
  // streaming shape: COUNTs without NULLs plus at most one NULL-free SUM over
  // int32 / int16 / int8 values (src64 codes 0 / 2 / 3; 2 and 3 only here)
  int vagg = -1;
  bool streaming = !debug_flag("having_general");
  for (int k = 0; k < nagg && streaming; ++k) {
    const AggDesc& d = descs[k];
    if (d.valid) streaming = false;
    else if (d.op == AGG_SUM_INT && d.src64 != 1 && d.src && vagg < 0) vagg = k;
    else if (d.op != AGG_COUNT) streaming = false;
  }
  for (int k = 0; k < nagg; ++k)
    if (descs[k].src64 > 1 && !(streaming && k == vagg))
      throw std::runtime_error("sorted_having: int16 / int8 values need the streaming kernel");
  if (streaming) {
    const int vb = vagg < 0 ? 0 : descs[vagg].src64 == 0 ? 4 : descs[vagg].src64 == 2 ? 2 : 1;
    const void* fns[2][4] = {{(const void*)sorted_having_scan_kernel<int32_t, 0>,
                              (const void*)sorted_having_scan_kernel<int32_t, 1>,
                              (const void*)sorted_having_scan_kernel<int32_t, 2>,
                              (const void*)sorted_having_scan_kernel<int32_t, 4>},
                             {(const void*)sorted_having_scan_kernel<int64_t, 0>,
                              (const void*)sorted_having_scan_kernel<int64_t, 1>,
                              (const void*)sorted_having_scan_kernel<int64_t, 2>,
                              (const void*)sorted_having_scan_kernel<int64_t, 4>}};
    const int vi = vb == 0 ? 0 : vb == 1 ? 1 : vb == 2 ? 2 : 3;
    const void* fn = fns[key64 ? 1 : 0][vi];
    // one resident round of waves (each owns one span): a second, partial
    // round would double the kernel's time
    static int resident[2][4] = {};
    int& res = resident[key64 ? 1 : 0][vi];
    if (!res) {
      int dev = 0, cus = 0, per_cu = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, 0);
      res = std::max(1, cus * std::max(1, per_cu));
    }
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    const int64_t blocks = std::min<int64_t>((tiles + kWavesPerBlock - 1) / kWavesPerBlock, res);
    const int64_t waves = blocks * kWavesPerBlock;
    const int64_t span = (tiles + waves - 1) / waves * kScanTile;
    const dim3 g((unsigned)((((n + span - 1) / span) + kWavesPerBlock - 1) / kWavesPerBlock)), b(kBlock);
    int64_t nn = n, sp = span, cp = cap;
    int va = vagg;
    void* args[] = {(void*)&keys, &nn, &sp, &p, &va, &rep, &cp, &counter};
    (void)hipLaunchKernel(fn, g, b, args, 0, stream);
    check_launch("sorted_having_scan", stream);
    return;
  }
  const dim3 g(grid_for(n, kBlock * kSortedRows, 32768)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(sorted_having_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, n, p, rep, cap, counter);
  else
    hipLaunchKernelGGL(sorted_having_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, n, p, rep, cap, counter);
  check_launch("sorted_having", stream);
}

void agg_update(const int32_t* gid, int64_t n, int ngroups, const AggDesc* descs, int nagg, hipStream_t stream,
                bool sorted_gids) {
  if (n == 0 || nagg == 0) return;
  if (nagg > kMaxAggs) throw std::runtime_error("agg_update: too many aggregates in one launch");
  AggParams p;
  p.nagg = nagg;
  for (int k = 0; k < nagg; ++k) {
    p.d[k] = descs[k];
    p.d[k].groups = ngroups > 1 ? ngroups : 1;
  }
  if (ngroups <= 1 || gid == nullptr) {
    // 1024 workgroups: 4 per CU stream the input, 1024 atomics per aggregate
    hipLaunchKernelGGL(agg_single_kernel, dim3(grid_for(n, kBlock * 4, 1024)), dim3(kBlock), 0, stream, n, p);
    check_launch("agg_single", stream);
  } else if (ngroups <= agg_lds_max_groups(nagg)) {
    size_t lds = (size_t)nagg * ngroups * 16;
    // fewer workgroups when the per-workgroup flush is large
    int64_t maxg = ngroups <= 64 ? 8192 : 2048;
    hipLaunchKernelGGL(agg_lds_kernel, dim3(grid_for(n, kBlock * 8, maxg)), dim3(kBlock), lds, stream, gid, n, ngroups, p);
    check_launch("agg_lds", stream);
  } else if (sorted_gids) {
    hipLaunchKernelGGL(agg_sorted_chunk_kernel, dim3(grid_for(n, kBlock * kSortedRows, 32768)), dim3(kBlock), 0, stream,
                       gid, n, p);
    check_launch("agg_sorted_chunk", stream);
  } else {
    hipLaunchKernelGGL(agg_global_kernel, dim3(grid_for(n, kBlock, 32768)), dim3(kBlock), 0, stream, gid, n, p);
    check_launch("agg_global", stream);
  }
}

}  // namespace kern
}  // namespace igloo

// ---- key histogram -----------------------------------------------------------
// counts[k - kmin] += 1 for every valid key in [kmin, kmin + span): COUNT per
// key over a dense domain (Q13's orders per customer) with 32-bit atomics
// straight from the key column (no shifted copy, no int64 counters).
namespace igloo {
namespace kern {
namespace {
template <typename K>
__global__ __launch_bounds__(kBlock) void key_histogram_kernel(const K* __restrict__ keys,
                                                              const uint8_t* __restrict__ valid, int64_t n,
                                                              int64_t kmin, int64_t span, int32_t* __restrict__ counts) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) continue;
    const int64_t s = (int64_t)keys[i] - kmin;
    if (s >= 0 && s < span) atomicAdd(&counts[s], 1);
  }
}
// Large domains (Q13: 150M orders over 15M customers) — device-scope atomics
// on a 60 MB table resolve past the per-XCD L2s (5.5 ms). Radix-partitioned
// instead: rows are bucketed by the high key bits (16384 keys per bucket: half the fan-out of 8192, so the scatter's partial-line writes combine in cache)
// into 16-bit low-bit codes, then each bucket is counted in LDS by one block.
//   pass 1: per (bucket, block) row counts      pass 2: stable-by-block scatter
//   pass 3: one block per bucket, LDS histogram of 16384 counters (64 KB).
constexpr int kHistBits = 14;
constexpr int kHistBucket = 1 << kHistBits;
constexpr int kHistBlocks = 2048;  // 8 per CU: the count and scatter passes are latency-bound (512 measured 1.0 + 3.3 ms for Q13)

template <typename K>
__device__ inline bool hist_key(const K* keys, const uint8_t* valid, int64_t i, int64_t kmin, int64_t span,
                                int64_t* s) {
  if (valid && !valid[i]) return false;
  *s = (int64_t)keys[i] - kmin;
  return *s >= 0 && *s < span;
}

template <typename K>
__global__ __launch_bounds__(kBlock) void hist_count_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t n, int64_t kmin, int64_t span, int nbk,
                                                           int32_t* __restrict__ cnt) {
  extern __shared__ int32_t lc[];
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) lc[b] = 0;
  __syncthreads();
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = blockIdx.x * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    int64_t s;
    if (hist_key(keys, valid, i, kmin, span, &s)) atomicAdd(&lc[s >> kHistBits], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) cnt[(int64_t)b * gridDim.x + blockIdx.x] = lc[b];
}

template <typename K>
__global__ __launch_bounds__(kBlock) void hist_scatter_kernel(const K* __restrict__ keys,
                                                             const uint8_t* __restrict__ valid, int64_t n, int64_t kmin,
                                                             int64_t span, int nbk, const int64_t* __restrict__ off,
                                                             uint16_t* __restrict__ part) {
  extern __shared__ int32_t cur[];
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) cur[b] = (int32_t)off[(int64_t)b * gridDim.x + blockIdx.x];
  __syncthreads();
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = blockIdx.x * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    int64_t s;
    if (hist_key(keys, valid, i, kmin, span, &s)) {
      const int32_t pos = atomicAdd(&cur[s >> kHistBits], 1);
      part[pos] = (uint16_t)(s & (kHistBucket - 1));
    }
  }
}

__global__ __launch_bounds__(kBlock) void hist_bucket_kernel(const uint16_t* __restrict__ part,
                                                            const int64_t* __restrict__ off, int64_t total,
                                                            int nblk, int64_t span, int32_t* __restrict__ counts) {
  __shared__ int32_t h[kHistBucket];
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < kHistBucket; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t lo = off[(int64_t)b * nblk];
  const int64_t hi = (int64_t)(b + 1) * nblk < (int64_t)gridDim.x * nblk ? off[(int64_t)(b + 1) * nblk] : total;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) atomicAdd(&h[part[i]], 1);
  __syncthreads();
  const int64_t base = (int64_t)b * kHistBucket;
  for (int i = threadIdx.x; i < kHistBucket && base + i < span; i += blockDim.x) counts[base + i] = h[i];
}
}  // namespace

int key_histogram_buckets(int64_t span) { return (int)((span + kHistBucket - 1) / kHistBucket); }

void key_histogram_partitioned(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin,
                               int64_t span, int phase, int32_t* cnt, const int64_t* off, int64_t total,
                               uint16_t* part, int32_t* counts, hipStream_t stream) {
  const int nbk = key_histogram_buckets(span);
  const size_t lds = (size_t)nbk * sizeof(int32_t);
  if (phase == 0) {
    if (key64)
      hipLaunchKernelGGL(hist_count_kernel<int64_t>, dim3(kHistBlocks), dim3(kBlock), lds, stream,
                         (const int64_t*)keys, valid, n, kmin, span, nbk, cnt);
    else
      hipLaunchKernelGGL(hist_count_kernel<int32_t>, dim3(kHistBlocks), dim3(kBlock), lds, stream,
                         (const int32_t*)keys, valid, n, kmin, span, nbk, cnt);
  } else if (phase == 1) {
    if (key64)
      hipLaunchKernelGGL(hist_scatter_kernel<int64_t>, dim3(kHistBlocks), dim3(kBlock), lds, stream,
                         (const int64_t*)keys, valid, n, kmin, span, nbk, off, part);
    else
      hipLaunchKernelGGL(hist_scatter_kernel<int32_t>, dim3(kHistBlocks), dim3(kBlock), lds, stream,
                         (const int32_t*)keys, valid, n, kmin, span, nbk, off, part);
  } else {
    hipLaunchKernelGGL(hist_bucket_kernel, dim3(nbk), dim3(kBlock), 0, stream, part, off, total, kHistBlocks, span,
                       counts);
  }
  check_launch("key_histogram_partitioned", stream);
}

int key_histogram_blocks() { return kHistBlocks; }

// ---- radix-partitioned aggregate ---------------------------------------------
// High-cardinality GROUP BY over unclustered group ids (TPC-H Q15: 22.7M
// lineitem rows over 1M suppliers). agg_global_kernel's direct atomics are one
// memory-side request per row and aggregate (scattered 8-byte atomics run at a
// fraction of the chip's store rate, and the 128-bit SUM's returning atomic
// waits for each). Partitioned like the key histogram above: rows are bucketed
// by the high group-id bits, their aggregate inputs scattered bucket by
// bucket, then one workgroup per bucket aggregates it in LDS and adds the
// result to the states with plain stores (a bucket owns its groups).
//   phase 0: per (bucket, block) row counts         (caller: exclusive scan)
//   phase 1: scatter of the low group-id bits and one 8-byte input per
//            aggregate (COUNT(*) needs none)
//   phase 2: one 1024-lane workgroup per bucket: LDS states, then the merge
// Integer SUMs accumulate in LDS as two no-return 64-bit halves (low 32 bits
// unsigned, the rest signed) and recombine exactly into the 128-bit state.
namespace {
constexpr int kPartBlocks = 512;
constexpr int kPartLds = 64 * 1024;
constexpr int kPartBlock2 = 1024;

struct PartParams {
  int nagg;
  AggDesc d[kMaxAggs];
  int64_t* vals[kMaxAggs];  // scattered inputs per aggregate (null: COUNT(*), 1 per row)
};

__device__ inline int64_t part_value(const AggDesc& a, int64_t i) {
  const bool ok = row_valid(a, i);
  switch (a.op) {
    case AGG_SUM_INT:
      return ok ? load_int(a, i) : 0;
    case AGG_SUM_F64: {
      const double d = ok ? ((const double*)a.src)[i] : 0.0;
      int64_t r;
      __builtin_memcpy(&r, &d, 8);
      return r;
    }
    case AGG_COUNT:
      return ok ? 1 : 0;
    case AGG_MIN_INT:
      return ok ? load_int(a, i) : INT64_MAX;
    case AGG_MAX_INT:
      return ok ? load_int(a, i) : INT64_MIN;
    case AGG_MIN_F64:
      return ok ? f64_to_ordered(((const double*)a.src)[i]) : INT64_MAX;
    case AGG_MAX_F64:
      return ok ? f64_to_ordered(((const double*)a.src)[i]) : INT64_MIN;
    case AGG_BIT_AND:
      return ok ? load_int(a, i) : -1;
    default:  // OR, XOR
      return ok ? load_int(a, i) : 0;
  }
}

__global__ __launch_bounds__(kBlock) void aggp_count_kernel(const int32_t* __restrict__ gid, int64_t n, int64_t groups,
                                                           int bits, int nbk, int32_t* __restrict__ cnt) {
  extern __shared__ int32_t lc[];
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) lc[b] = 0;
  __syncthreads();
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = blockIdx.x * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    const uint32_t g = (uint32_t)gid[i];
    if (g < (uint64_t)groups) atomicAdd(&lc[g >> bits], 1);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) cnt[(int64_t)b * gridDim.x + blockIdx.x] = lc[b];
}

__global__ __launch_bounds__(kBlock) void aggp_scatter_kernel(const int32_t* __restrict__ gid, int64_t n,
                                                             int64_t groups, int bits, int nbk,
                                                             const int64_t* __restrict__ off,
                                                             uint16_t* __restrict__ pg, PartParams p) {
  extern __shared__ int32_t cur[];
  for (int b = threadIdx.x; b < nbk; b += blockDim.x) cur[b] = (int32_t)off[(int64_t)b * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint32_t low = (1u << bits) - 1;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = blockIdx.x * chunk, r1 = r0 + chunk < n ? r0 + chunk : n;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += blockDim.x) {
    const uint32_t g = (uint32_t)gid[i];
    if (g >= (uint64_t)groups) continue;
    const int32_t pos = atomicAdd(&cur[g >> bits], 1);
    pg[pos] = (uint16_t)(g & low);
    for (int k = 0; k < p.nagg; ++k)
      if (p.vals[k]) p.vals[k][pos] = part_value(p.d[k], i);
  }
}

__device__ inline void part_init(int op, unsigned long long* lo, long long* hi) { init_state(op, lo, hi); }

__global__ __launch_bounds__(kPartBlock2) void aggp_bucket_kernel(const uint16_t* __restrict__ pg,
                                                                 const int64_t* __restrict__ off,
                                                                 const int64_t* __restrict__ total, int nblk,
                                                                 int64_t groups, int bits, int slices, PartParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long st[];
  const int B = 1 << bits;
  unsigned long long* slo = st;
  long long* shi = (long long*)(st + (size_t)p.nagg * B);
  for (int idx = threadIdx.x; idx < p.nagg * B; idx += blockDim.x) part_init(p.d[idx >> bits].op, &slo[idx], &shi[idx]);
  __syncthreads();
  // `slices` workgroups share a bucket when the buckets are few (each takes
  // a contiguous slice of its rows and merges with atomics)
  const int b = blockIdx.x / slices, sl = blockIdx.x % slices;
  const int nbk = (int)gridDim.x / slices;
  const int64_t blo = off[(int64_t)b * nblk];
  const int64_t bhi = b + 1 < nbk ? off[(int64_t)(b + 1) * nblk] : *total;
  const int64_t lo = blo + (bhi - blo) * sl / slices;
  const int64_t hi = blo + (bhi - blo) * (sl + 1) / slices;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const int g = pg[i];
    for (int k = 0; k < p.nagg; ++k) {
      const AggDesc& a = p.d[k];
      const int idx = (k << bits) + g;
      const int64_t v = p.vals[k] ? p.vals[k][i] : 1;
      switch (a.op) {
        case AGG_SUM_INT:
          if (a.dst2) {
            atomicAdd(&slo[idx], (unsigned long long)(uint32_t)v);
            atomicAdd((unsigned long long*)&shi[idx], (unsigned long long)(v >> 32));
          } else {
            atomicAdd(&slo[idx], (unsigned long long)v);
          }
          break;
        case AGG_SUM_F64: {
          double d;
          __builtin_memcpy(&d, &v, 8);
          atomicAdd((double*)&slo[idx], d);
          break;
        }
        case AGG_COUNT:
          atomicAdd(&slo[idx], (unsigned long long)v);
          break;
        case AGG_MIN_INT:
        case AGG_MIN_F64:
          atomicMin((long long*)&slo[idx], (long long)v);
          break;
        case AGG_MAX_INT:
        case AGG_MAX_F64:
          atomicMax((long long*)&slo[idx], (long long)v);
          break;
        case AGG_BIT_AND:
          atomicAnd(&slo[idx], (unsigned long long)v);
          break;
        case AGG_BIT_OR:
          atomicOr(&slo[idx], (unsigned long long)v);
          break;
        case AGG_BIT_XOR:
          atomicXor(&slo[idx], (unsigned long long)v);
          break;
      }
    }
  }
  __syncthreads();
  // merge: this bucket's groups belong to this workgroup alone (plain stores)
  const int64_t g0 = (int64_t)b << bits;
  if (slices > 1) {
    for (int idx = threadIdx.x; idx < p.nagg * B; idx += blockDim.x) {
      const int k = idx >> bits;
      const int64_t g = g0 + (idx & (B - 1));
      if (g >= groups) continue;
      const AggDesc& a = p.d[k];
      unsigned long long x = slo[idx];
      long long h = 0;
      if (a.op == AGG_SUM_INT && a.dst2) {
        const __int128 t = ((__int128)shi[idx] << 32) + (__int128)x;
        x = (unsigned long long)t;
        h = (long long)(t >> 64);
      }
      merge_global(a, g, x, h);   // (identity states are skipped)
    }
    return;
  }
  for (int idx = threadIdx.x; idx < p.nagg * B; idx += blockDim.x) {
    const int k = idx >> bits;
    const int64_t g = g0 + (idx & (B - 1));
    if (g >= groups) continue;
    const AggDesc& a = p.d[k];
    unsigned long long* d = (unsigned long long*)a.dst + g;
    const unsigned long long x = slo[idx];
    switch (a.op) {
      case AGG_SUM_INT:
        if (a.dst2) {
          long long* d2 = (long long*)a.dst2 + g;
          // total = shi * 2^32 + slo (slo < 2^63, |shi| < 2^62): exact in 128 bits
          const __int128 t = ((__int128)shi[idx] << 32) + (__int128)x;
          const __int128 c = (((__int128)*d2) << 64) + (__int128)*d;
          const __int128 r = c + t;
          *d = (unsigned long long)r;
          *d2 = (long long)(r >> 64);
        } else {
          *d += x;
        }
        break;
      case AGG_SUM_F64: {
        double u, w;
        __builtin_memcpy(&u, d, 8);
        __builtin_memcpy(&w, &x, 8);
        u += w;
        __builtin_memcpy(d, &u, 8);
        break;
      }
      case AGG_COUNT:
        *d += x;
        break;
      case AGG_MIN_INT:
      case AGG_MIN_F64:
        if ((long long)x < (long long)*d) *d = x;
        break;
      case AGG_MAX_INT:
      case AGG_MAX_F64:
        if ((long long)x > (long long)*d) *d = x;
        break;
      case AGG_BIT_AND:
        *d &= x;
        break;
      case AGG_BIT_OR:
        *d |= x;
        break;
      case AGG_BIT_XOR:
        *d ^= x;
        break;
    }
  }
}
}  // namespace

int agg_part_bits(int nagg) {
  int b = 12;
  while (b > 6 && (int64_t)nagg * (int64_t(1) << b) * 16 > kPartLds) --b;
  return b;
}

int agg_part_buckets(int64_t ngroups, int nagg) {
  const int64_t B = int64_t(1) << agg_part_bits(nagg);
  return (int)((ngroups + B - 1) / B);
}

int agg_part_blocks() { return kPartBlocks; }

void agg_partitioned(const int32_t* gid, int64_t n, int64_t ngroups, const AggDesc* descs, int nagg, int phase,
                     int32_t* cnt, const int64_t* off, const int64_t* total, uint16_t* pg, int64_t* const* vals,
                     hipStream_t stream) {
  if (n <= 0) return;
  if (nagg <= 0 || nagg > kMaxAggs) throw std::runtime_error("agg_partitioned: 1..8 aggregates per launch");
  const int bits = agg_part_bits(nagg);
  const int nbk = agg_part_buckets(ngroups, nagg);
  PartParams p;
  p.nagg = nagg;
  for (int k = 0; k < nagg; ++k) {
    p.d[k] = descs[k];
    p.d[k].groups = ngroups;
    p.vals[k] = vals ? vals[k] : nullptr;
  }
  const size_t lds = (size_t)nbk * sizeof(int32_t);
  if (phase == 0) {
    hipLaunchKernelGGL(aggp_count_kernel, dim3(kPartBlocks), dim3(kBlock), lds, stream, gid, n, ngroups, bits, nbk, cnt);
  } else if (phase == 1) {
    hipLaunchKernelGGL(aggp_scatter_kernel, dim3(kPartBlocks), dim3(kBlock), lds, stream, gid, n, ngroups, bits, nbk,
                       off, pg, p);
  } else {
    const size_t st = (size_t)nagg * ((size_t)1 << bits) * 16;
    // few buckets: enough workgroups to fill the chip (256 CUs), slices merged atomically
    const int slices = nbk >= 128 ? 1 : std::min(64, (256 + nbk - 1) / nbk);
    hipLaunchKernelGGL(aggp_bucket_kernel, dim3(nbk * slices), dim3(kPartBlock2), st, stream, pg, off, total,
                       kPartBlocks, ngroups, bits, slices, p);
  }
  check_launch("agg_partitioned", stream);
}

void key_histogram(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin, int64_t span,
                   int32_t* counts, hipStream_t stream) {
  if (n <= 0) return;
  const dim3 g(grid_for(n, kBlock, 1 << 16)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(key_histogram_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, valid, n, kmin, span,
                       counts);
  else
    hipLaunchKernelGGL(key_histogram_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, valid, n, kmin, span,
                       counts);
  check_launch("key_histogram", stream);
}
}  // namespace kern
}  // namespace igloo
