// Fused scan kernels: conjunctive range filters and filter + small-domain
// GROUP BY + sums of products of affine terms, in one pass over the columns.
//
// The reference evaluates FilterExec -> ProjectionExec -> AggregateExec as a
// chain of Arrow compute kernels over materialised batches (DataFusion via
// reference crates/engine/src/lib.rs:55-56; filter.rs:47, projection.rs:60-64),
// i.e. one HBM round trip per expression node. The analytic scan shapes that
// dominate TPC-H have a fixed structure, so instead of interpreting arbitrary
// expressions these kernels take a small declarative description:
//   * filter  = AND of terms over int32/int64 columns: lo <= v <= hi (optionally
//     negated) or "v in set" for dictionary codes < 64, plus an optional
//     precomputed mask for anything else (LIKE, OR trees);
//   * group   = up to 2 small-domain keys (dictionary codes / small ints),
//     gid = sum((k_i - lo_i) * mul_i) < 16;
//   * aggregate = SUM / MIN / MAX of prod_{f<=3} (a_f + b_f * col_f) in exact
//     int64 fixed point (optionally overflow-checked), or COUNT.
//
// Code shape (what made these kernels VALU/SALU-bound before, and the fix):
//   * descriptor loops are OUTER and the lane's kFfRows rows INNER (unrolled),
//     so each term / factor / aggregate descriptor is fetched and branched on
//     once per 4 rows instead of once per row;
//   * a lane's rows live in one 8 x int64 register vector per row and a column
//     is picked with a VGPR-indexed move (uniform index), not a select chain;
//   * column addresses are a wave-uniform 64-bit base (SGPR) plus a 32-bit lane
//     offset, so loads use the saddr form with no 64-bit multiply per load.
//
// Aggregation: every (aggregate, group) cell owns int64 slots in LDS indexed by
// lane (shared by the block's waves; ds_add/ds_min/ds_max atomics), so a row
// costs two LDS adds per SUM and no cross-lane traffic. SUMs stay exact: the
// unsigned low and signed high 32-bit halves of each value go to separate slots
// and the block merge recombines them in int128. Cells x lanes are sized to
// the LDS budget (lanes share slots when there are many cells).
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kFfRows = 4;  // rows per lane per iteration (consecutive: base + 4 lane + j)
static_assert(kFfMaxCols == 8 && kFfRows == 4, "row vectors are written for 8 columns x 4 rows");
// row vector of VW >= NC int64 lanes (power of two, so a column index is masked, never out of range)
template <int NC>
constexpr int ff_vw() { return NC <= 1 ? 1 : NC <= 2 ? 2 : NC <= 4 ? 4 : 8; }
template <int VW>
using ff_vec = long long __attribute__((ext_vector_type(VW)));

// Branch-free column load (1/2/4/8-byte integer columns): two dword loads at
// the aligned dword holding the value and the next one for 8-byte columns (the
// same dword twice otherwise); p is the wave-uniform address of the
// iteration's first row. Keeping every load unconditional lets all of a row's
// loads be in flight at once (a width switch per load made the compiler wait
// after each one). Narrow columns (resident decimals whose values fit 8/16/32
// bits: l_discount, l_quantity, ...) cut the bytes a scan streams; a sub-dword
// value is shifted down and sign-extended. The aligned dword never leaves the
// allocation (PyTorch blocks are 512-byte multiples).
__device__ __forceinline__ int64_t ff_load(const FfColumn& c, int64_t base, uint32_t idx) {
  const int64_t w = c.width;
  const char* p = (const char*)c.ptr + base * w;
  const uint32_t off = idx * (uint32_t)w;
  const uint32_t mis = ((uint32_t)(uintptr_t)(p + off)) & 3u;
  const uint32_t a = off - mis;
  const uint32_t lo = *(const uint32_t*)(p + a);
  const uint32_t hi = *(const uint32_t*)(p + (a + (w == 8 ? 4u : 0u)));
  // both dwords are always consumed (a select let the compiler sink the second
  // load into a branch and wait on it). (A variant extracting sub-dword fields
  // with 32-bit shifts and selects was 50% slower on Q1/Q6: keep the 64-bit
  // funnel + sign-extending shift pair.)
  const uint64_t v = (((uint64_t)hi << 32) | lo) >> (mis * 8);
  const int sh = 64 - 8 * (int)w;
  return (int64_t)(v << sh) >> sh;
}

// Four consecutive rows of one column for a lane (rows base + 4 lane + j):
// one load of 4 w bytes per lane (dword / dwordx2 / dwordx4 / 2 x dwordx4, a
// wave reads one contiguous 256 w-byte span) and one bit-field extract per
// value — against two dword loads, a 64-bit funnel shift and a sign-extending
// shift pair per value for the row-strided form (ff_load). The width branch is
// wave-uniform (kernel argument). Full iterations only: the tail keeps ff_load.
struct FfQuad {
  int64_t v0, v1, v2, v3;
};
struct FfRaw {
  uint4 a, b;
};
// Load phase, branch-free: one dwordx4 per column at the lane's first row
// (a 1/2-byte column uses its first 4/8 bytes; the iteration is "full" only
// when those 16 bytes stay inside the column), plus a second dwordx4 for
// 8-byte columns. Loads in per-width branches made the compiler wait for each
// at the branch join; here every column's loads are in flight before the
// first wait and the values are extracted afterwards (ff_extract4).
__device__ __forceinline__ FfRaw ff_fetch4(const FfColumn& c, int64_t base, int lane) {
  const int64_t w = c.width;
  const char* p = (const char*)c.ptr + base * w;
  const uint32_t off = (uint32_t)lane * 4u * (uint32_t)w;
  FfRaw r;
  r.a = *(const uint4*)(p + off);
  if (w == 8) r.b = *(const uint4*)(p + off + 16);
  return r;
}
__device__ __forceinline__ FfQuad ff_extract4(const FfColumn& c, const FfRaw& r) {
  const int64_t w = c.width;
  FfQuad q;
  if (w == 1) {
    const int x = (int)r.a.x;
    q.v0 = (int8_t)x;
    q.v1 = (int8_t)(x >> 8);
    q.v2 = (int8_t)(x >> 16);
    q.v3 = x >> 24;
  } else if (w == 2) {
    q.v0 = (int16_t)r.a.x;
    q.v1 = (int)r.a.x >> 16;
    q.v2 = (int16_t)r.a.y;
    q.v3 = (int)r.a.y >> 16;
  } else if (w == 4) {
    q.v0 = (int)r.a.x;
    q.v1 = (int)r.a.y;
    q.v2 = (int)r.a.z;
    q.v3 = (int)r.a.w;
  } else {
    q.v0 = (int64_t)(((uint64_t)r.a.y << 32) | r.a.x);
    q.v1 = (int64_t)(((uint64_t)r.a.w << 32) | r.a.z);
    q.v2 = (int64_t)(((uint64_t)r.b.y << 32) | r.b.x);
    q.v3 = (int64_t)(((uint64_t)r.b.w << 32) | r.b.z);
  }
  return q;
}

// The row vectors are kernel locals (r0..r3) handed to helpers BY VALUE: an
// element read through a reference/struct lvalue is canonicalised into a
// dynamic GEP, which pins the vectors in scratch. NC (the number of input
// columns) is a compile-time bound, so the load block has no per-lane
// branches and every column's loads are issued before the first wait.
// A lane owns rows base + 4 lane + j (j < 4).
#define FF_LOAD_ROWS(NC, S, base, it)                                \
  ff_vec<ff_vw<NC>()> r0 = {}, r1 = r0, r2 = r0, r3 = r0;            \
  if ((it).full) {                                                   \
    FfRaw raw_[NC];                                                  \
    _Pragma("unroll") for (int c_ = 0; c_ < NC; ++c_)               \
      raw_[c_] = ff_fetch4(S.cols[c_], base, lane);                  \
    _Pragma("unroll") for (int c_ = 0; c_ < NC; ++c_) {             \
      const FfQuad q_ = ff_extract4(S.cols[c_], raw_[c_]);           \
      r0[c_] = q_.v0;                                                \
      r1[c_] = q_.v1;                                                \
      r2[c_] = q_.v2;                                                \
      r3[c_] = q_.v3;                                                \
    }                                                                \
  } else {                                                           \
    _Pragma("unroll") for (int c_ = 0; c_ < NC; ++c_) {             \
      r0[c_] = ff_load(S.cols[c_], base, (it).idx[0]);               \
      r1[c_] = ff_load(S.cols[c_], base, (it).idx[1]);               \
      r2[c_] = ff_load(S.cols[c_], base, (it).idx[2]);               \
      r3[c_] = ff_load(S.cols[c_], base, (it).idx[3]);               \
    }                                                                \
  }
#define FF_ROW(j) ((j) == 0 ? r0 : (j) == 1 ? r1 : (j) == 2 ? r2 : r3)

template <int VW>
__device__ __forceinline__ int64_t col_of(const ff_vec<VW> rv, int c) {
  return rv[c & (VW - 1)];
}

// Iteration setup: wave-uniform first row, per-lane row offsets (clamped into
// range for the tail; `live` marks real rows).
struct FfIter {
  int64_t base;
  uint32_t idx[kFfRows];
  bool live[kFfRows];
  bool full;  // all kWave * kFfRows rows in range (wave-uniform)
};
__device__ __forceinline__ FfIter ff_iter(int64_t base, int lane, int64_t n) {
  FfIter it;
  it.base = base;
  const int64_t rem = n - base;  // > 0
  it.full = rem >= (int64_t)kWave * kFfRows + 12;  // + 12: the last lane's 16-byte load of a 1-byte column
#pragma unroll
  for (int j = 0; j < kFfRows; ++j) {
    const int64_t r = kFfRows * lane + j;
    it.live[j] = r < rem;
    it.idx[j] = (uint32_t)(r < rem ? r : rem - 1);
  }
  return it;
}

// filter: all terms, descriptor-outer
template <int VW>
__device__ __forceinline__ void ff_pass4(const FfSpec& S, const ff_vec<VW> r0, const ff_vec<VW> r1,
                                         const ff_vec<VW> r2, const ff_vec<VW> r3, const FfIter& it, bool* pass) {
  // terms with an OR-group (kind >> 8 = g > 0) form one disjunction: the row
  // passes it when every term of at least one group holds (gok bit g)
  uint32_t gok[kFfRows];
  uint32_t used = 0;
#pragma unroll
  for (int j = 0; j < kFfRows; ++j) {
    pass[j] = it.live[j];
    gok[j] = 0xffffffffu;
  }
  for (int t = 0; t < S.nterms; ++t) {
    const FfTerm& T = S.terms[t];
    const int c = __builtin_amdgcn_readfirstlane(T.col);
    const int kind = T.kind & 0xff;
    const int grp = T.kind >> 8;
    const int64_t lo = T.lo, hi = T.hi;
    const uint64_t set = T.set;
    const int c2 = __builtin_amdgcn_readfirstlane((int)(set & 0xff));  // kind 3: second column
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) {
      const int64_t v = col_of<VW>(FF_ROW(j), c);
      bool hit;
      if (kind == 2) hit = v >= 0 && v < 64 && ((set >> (v & 63)) & 1ULL);
      else if (kind == 3) {
        const int64_t d = v - col_of<VW>(FF_ROW(j), c2);
        hit = d >= lo && d <= hi;
      } else {
        hit = v >= lo && v <= hi;
      }
      const bool ok = (kind == 1) ? !hit : hit;
      if (grp == 0) pass[j] &= ok;
      else if (!ok) gok[j] &= ~(1u << grp);
    }
    if (grp) used |= 1u << grp;
  }
  if (used) {
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) pass[j] &= (gok[j] & used) != 0;
  }
  if (S.mask) {
    const uint8_t* m = S.mask + it.base;
    if (it.full) {  // the lane's 4 mask bytes in one dword (mask buffers are 4-byte aligned)
      const uint32_t mw = *(const uint32_t*)(m + it.idx[0]);  // idx[0] = 4 lane
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) pass[j] &= ((mw >> (8 * j)) & 0xffu) != 0;
    } else {
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) pass[j] &= m[it.idx[j]] != 0;
    }
  }
}

// group ids: keys descriptor-outer
template <int VW>
__device__ __forceinline__ void ff_gid4(const FfSpec& S, const ff_vec<VW> r0, const ff_vec<VW> r1,
                                        const ff_vec<VW> r2, const ff_vec<VW> r3, int* gid) {
#pragma unroll
  for (int j = 0; j < kFfRows; ++j) gid[j] = 0;
  for (int k = 0; k < S.nkeys; ++k) {
    const int c = __builtin_amdgcn_readfirstlane(S.key_col[k]);
    const int lo = (int)S.key_lo[k], mul = (int)S.key_mul[k];  // small domains: codes and offsets fit in 32 bits
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) gid[j] += ((int)col_of<VW>(FF_ROW(j), c) - lo) * mul;
  }
}

// aggregate argument: product of affine factors, factor-outer. `val` holds
// the previous aggregate's values on entry (reused when A.shared > 0).
// Checked products take a 32 x 32 -> 64-bit multiply when both operands fit in
// 32 bits (the common case: fixed-point prices times small factors) and the
// overflow-checked 64-bit path otherwise.
template <int VW>
__device__ __forceinline__ void ff_value4(const FfAgg& A, const ff_vec<VW> r0, const ff_vec<VW> r1,
                                          const ff_vec<VW> r2, const ff_vec<VW> r3, int64_t* val, int* ovf) {
  const int shared = A.shared;
  if (shared == 0) {
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) val[j] = 1;
  }
  const bool checked = A.checked;
  for (int f = shared; f < A.nfac; ++f) {
    const FfFactor& F = A.f[f];
    const int c = __builtin_amdgcn_readfirstlane((int)F.col);
    const int64_t a = F.a, b = F.b;
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) {
      int64_t term;
      if (c < 0) term = a;
      else if (b == 1) term = (int64_t)((uint64_t)a + (uint64_t)col_of<VW>(FF_ROW(j), c));
      else if (b == -1) term = (int64_t)((uint64_t)a - (uint64_t)col_of<VW>(FF_ROW(j), c));
      else term = (int64_t)((uint64_t)a + (uint64_t)b * (uint64_t)col_of<VW>(FF_ROW(j), c));
      const int64_t x = val[j];
      if ((int64_t)(int32_t)x == x && (int64_t)(int32_t)term == term) {
        val[j] = (int64_t)(int32_t)x * (int64_t)(int32_t)term;
      } else if (checked) {
        int64_t r;
        if (__builtin_mul_overflow(x, term, &r)) *ovf = 1;
        val[j] = r;
      } else {
        val[j] = (int64_t)((uint64_t)x * (uint64_t)term);
      }
    }
  }
}

__device__ __forceinline__ int ff_wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

template <int NC>
__global__ __launch_bounds__(kBlock) void ff_mask_kernel(const FfSpec S, int64_t n, uint8_t* __restrict__ out) {
  const int wave = ff_wave_uniform(threadIdx.x / kWave), lane = lane_id();
  const int64_t per_iter = (int64_t)kWave * kFfRows;
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * per_iter;
  for (int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * per_iter; base < n; base += stride) {
    const FfIter it = ff_iter(base, lane, n);
    FF_LOAD_ROWS(NC, S, base, it)
    bool pass[kFfRows];
    ff_pass4<ff_vw<NC>()>(S, r0, r1, r2, r3, it, pass);
    uint8_t* o = out + base;
    if (it.full) {
      uint32_t w = 0;
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) w |= (uint32_t)pass[j] << (8 * j);
      *(uint32_t*)(o + kFfRows * lane) = w;
    } else {
#pragma unroll
      for (int j = 0; j < kFfRows; ++j)
        if (it.live[j]) o[it.idx[j]] = pass[j];
    }
  }
}

// LDS slot of (cell, half, lane): lanes fold onto `lanes` slots (a power of
// two <= 64 chosen on the host so cells * 2 * lanes int64 fit the LDS budget)
__device__ __forceinline__ int ff_slot(int cell, int half, int lane, int lanes) {
  return (cell * 2 + half) * lanes + (lane & (lanes - 1));
}

// LDS layout: cell = a * G + g for aggregates, NA * G + g for the row counts.
// 512-thread blocks (A/B at SF100: 256 -> 9.7 ms, 512 -> 9.2 ms, 1024 ->
// 10.5 ms for Q1): the LDS table is per block, so larger blocks put more
// waves behind the same LDS bytes (Q1: 54 cells x 2 halves x
// 64 lanes = 55 KB; at 256 threads only 2 blocks = 8 waves fit a CU and the
// streaming loads are latency-bound).
constexpr int kFfAggBlock = 512;

template <int NC>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void ff_agg_kernel(const FfSpec S, int64_t n, int lanes) {
  extern __shared__ int64_t acc[];
  const int wave = ff_wave_uniform(threadIdx.x / kWave), lane = lane_id();
  const int waves = blockDim.x / kWave;
  const int G = S.ngroups, NA = S.naggs;
  const int cells = (NA + 1) * G;
  for (int s = threadIdx.x; s < cells * 2 * lanes; s += blockDim.x) {
    const int cell = s / (2 * lanes), a = cell / G;
    int64_t init = 0;
    if (a < NA && S.aggs[a].op == 2) init = INT64_MAX;
    if (a < NA && S.aggs[a].op == 3) init = INT64_MIN;
    acc[s] = init;
  }
  __syncthreads();
  int ovf = 0;
  const int64_t per_iter = (int64_t)kWave * kFfRows;
  const int64_t stride = (int64_t)gridDim.x * waves * per_iter;
  for (int64_t base = ((int64_t)blockIdx.x * waves + wave) * per_iter; base < n; base += stride) {
    const FfIter it = ff_iter(base, lane, n);
    FF_LOAD_ROWS(NC, S, base, it)
    bool pass[kFfRows];
    ff_pass4<ff_vw<NC>()>(S, r0, r1, r2, r3, it, pass);
    int gid[kFfRows];
    ff_gid4<ff_vw<NC>()>(S, r0, r1, r2, r3, gid);
    // a key outside the (possibly replayed) domain never indexes past the cells
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) pass[j] = pass[j] && (unsigned)gid[j] < (unsigned)G;
    // per-row slot base (group g, this lane); aggregate a adds a * G cells
    int64_t* rowslot[kFfRows];
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) rowslot[j] = acc + ff_slot(gid[j], 0, lane, lanes);
    const int cell_stride = 2 * lanes;  // int64 per cell
#pragma unroll
    for (int j = 0; j < kFfRows; ++j)
      if (pass[j])
        __hip_atomic_fetch_add(rowslot[j] + NA * G * cell_stride, (int64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    int64_t val[kFfRows];
    for (int a = 0; a < NA; ++a) {
      const FfAgg& A = S.aggs[a];
      const int op = A.op;
      if (op == 1) continue;  // COUNT: the group row count (never a chain link: it has no factors)
      ff_value4<ff_vw<NC>()>(A, r0, r1, r2, r3, val, &ovf);
      const int aoff = a * G * cell_stride;
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) {
        if (!pass[j]) continue;
        int64_t* slot = rowslot[j] + aoff;
        if (op == 0) {
          __hip_atomic_fetch_add(slot, (int64_t)(uint32_t)(uint64_t)val[j], __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
          __hip_atomic_fetch_add(slot + lanes, val[j] >> 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (op == 2) {
          __hip_atomic_fetch_min(slot, val[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          __hip_atomic_fetch_max(slot, val[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
    }
  }
  __syncthreads();
  for (int s = threadIdx.x; s < G * (NA + 1); s += blockDim.x) {
    const int g = s / (NA + 1), a = s % (NA + 1);
    const int ccell = NA * G + g;
    if (a == NA || S.aggs[a].op == 1) {
      int64_t c = 0;
      for (int l = 0; l < lanes; ++l) c += acc[ff_slot(ccell, 0, l, lanes)];
      if (c) atomicAdd((unsigned long long*)(a == NA ? &S.counts[g] : &S.aggs[a].dst[g]), (unsigned long long)c);
      continue;
    }
    const FfAgg& A = S.aggs[a];
    const int cell = a * G + g;
    if (A.op == 0) {
      __int128 t = 0;
      for (int l = 0; l < lanes; ++l)
        t += ((__int128)acc[ff_slot(cell, 1, l, lanes)] << 32) + (__int128)(uint64_t)acc[ff_slot(cell, 0, l, lanes)];
      if (t != 0)
        atomic_add_i128_parts((unsigned long long*)&A.dst[g], (long long*)&A.dst2[g], (unsigned long long)(uint64_t)t,
                              (long long)(int64_t)(t >> 64));
    } else if (A.op == 2) {
      int64_t r = INT64_MAX;
      for (int l = 0; l < lanes; ++l) {
        const int64_t x = acc[ff_slot(cell, 0, l, lanes)];
        r = x < r ? x : r;
      }
      atomicMin((long long*)&A.dst[g], (long long)r);
    } else {
      int64_t r = INT64_MIN;
      for (int l = 0; l < lanes; ++l) {
        const int64_t x = acc[ff_slot(cell, 0, l, lanes)];
        r = x > r ? x : r;
      }
      atomicMax((long long*)&A.dst[g], (long long)r);
    }
  }
  if (__any(ovf) && lane == 0 && S.overflow) atomicOr(S.overflow, 1);
}

// ---------------------------------------------------------------------------
// One-hot MFMA aggregation (SUM / COUNT over <= 16 groups).
//
// A group-by SUM is a matrix product: D[g][c] += sum_k onehot[g][k] * x[k][c]
// over rows k. A wave takes 256 rows per iteration (4 per lane) and builds
//   A = one-hot of the rows' group ids (16 groups x 64 rows per MFMA, int8), and
//   B = the rows' aggregate values split into byte limbs (64 rows x 16 limb
//       columns per tile, int8),
// then v_mfma_i32_16x16x64_i8 accumulates D (16 x 16 int32) — exact integer
// sums with no atomics and no per-(row, aggregate) LDS traffic.
//
// Limbs: a value of w bits (bound from the factor column widths) takes
// ceil(w / 8) bytes of its two's-complement form. The top byte is signed; a
// lower byte u in [0, 255] is stored as u - 128 (= u ^ 0x80 read as int8) and
// the block merge adds back 128 x (rows of the group), taken from a column of
// 1s (the COUNT column). Filtered-out rows get group byte 0xff, so their
// one-hot row is zero and their limbs need no masking.
//
// LDS staging (per wave, column-major): column c holds 256 bytes, byte
// 4 * lane + j = row j of that lane, so a lane packs its 4 rows' limb l into
// ONE dword (two v_perm_b32 per limb) and a column is one conflict-free
// ds_write_b32. Fragment maps (gfx950, v_mfma_i32_16x16x64_i8): lane l holds
// A[m = l & 15][k = 16 (l >> 4) + j] and B[k = 16 (l >> 4) + j][n = l & 15]
// (j = 0..15, one byte each) and D[m = 4 (l >> 4) + i][n = l & 15] (i < 4);
// K-step s covers column bytes [64 s, 64 s + 64). The 272-byte column stride
// spreads the 16 columns one ds_read_b128 touches over all 64 banks.
// int32 accumulators gain at most 64 * 128 per MFMA, so they are folded into
// int64 every 2^12 iterations; a block merges its waves and adds each (group,
// aggregate) as int128 with two 64-bit atomics.
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int kMfmaCol = 272;                  // LDS bytes per limb column (256 rows + pad)
constexpr int kMfmaMaxTiles = 4;               // <= 64 limb columns
constexpr int kMfmaBlock = 256;

struct FfMfmaLayout {
  int32_t col0[kFfMaxAggs], nlimb[kFfMaxAggs];  // first limb column / limb count per aggregate (0 for COUNT)
  int32_t count_col, ncols;
};

__device__ __forceinline__ uint32_t bytes_eq(uint32_t x, uint32_t g4) {
  // 0x01 in each byte of x equal to the matching byte of g4, exactly
  const uint32_t d = x ^ g4;
  const uint32_t y = ~(((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d | 0x7f7f7f7fu);
  return y >> 7;
}

// byte b (0..3) of each of x0..x3 packed into one dword: two pair-perms + one merge
__device__ __forceinline__ uint32_t limb_dword(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t b) {
  // v_perm_b32(s0, s1, sel): selector byte values 0..3 pick s1's bytes, 4..7 s0's
  const uint32_t sel = b | ((b + 4) << 8);                      // (x_lo.b, x_hi.b) in bytes 0, 1
  const uint32_t p01 = __builtin_amdgcn_perm(x1, x0, sel);
  const uint32_t p23 = __builtin_amdgcn_perm(x3, x2, sel);
  return __builtin_amdgcn_perm(p23, p01, 0x05040100u);
}

template <int NC, int NT>
__global__ __launch_bounds__(kMfmaBlock) void ff_mfma_agg_kernel(const FfSpec S, const FfMfmaLayout Lay, int64_t n) {
  constexpr int kCols = NT * 16 + 1;   // limb columns + the group-id column
  // the waves' staging tiles, reused for the block merge once every wave is done
  static_assert(NT * 16 * 16 * sizeof(long long) <= kCols * kMfmaCol, "merge buffer fits the tiles");
  __shared__ __attribute__((aligned(16))) uint8_t tile[kMfmaBlock / kWave][kCols * kMfmaCol];
  auto red = reinterpret_cast<long long (*)[NT * 16][16]>(&tile[0][0]);
  const int wave = ff_wave_uniform(threadIdx.x / kWave), lane = lane_id();
  const int waves = kMfmaBlock / kWave;
  uint8_t* T = tile[wave];
  uint8_t* gidb = T + NT * 16 * kMfmaCol;
  // unused limb columns stay 0, the count column holds 1s
  for (int c = 0; c < NT * 16; ++c)
    *reinterpret_cast<uint32_t*>(T + c * kMfmaCol + 4 * lane) = c == Lay.count_col ? 0x01010101u : 0u;
  v4i acc[NT];
  long long acc64[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    acc[t] = v4i{0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) acc64[t][i] = 0;
  }
  int ovf = 0, steps = 0;
  const int NA = S.naggs;
  const uint32_t g4 = (uint32_t)(lane & 15) * 0x01010101u;
  const int q16 = 16 * (lane >> 4);
  const int64_t per_iter = (int64_t)kWave * kFfRows;
  const int64_t stride = (int64_t)gridDim.x * waves * per_iter;
  for (int64_t base = ((int64_t)blockIdx.x * waves + wave) * per_iter; base < n; base += stride) {
    const FfIter it = ff_iter(base, lane, n);
    FF_LOAD_ROWS(NC, S, base, it)
    bool pass[kFfRows];
    ff_pass4<ff_vw<NC>()>(S, r0, r1, r2, r3, it, pass);
    int gid[kFfRows];
    ff_gid4<ff_vw<NC>()>(S, r0, r1, r2, r3, gid);
    uint32_t gw = 0;
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) gw |= (uint32_t)(pass[j] ? gid[j] & 0xff : 0xff) << (8 * j);
    *reinterpret_cast<uint32_t*>(gidb + 4 * lane) = gw;
    // each aggregate's values for this lane's 4 rows, straight into limb
    // columns (product chains reuse the previous aggregate's value)
    int64_t val[kFfRows];
    for (int a = 0; a < NA; ++a) {
      const FfAgg& A = S.aggs[a];
      if (A.op == 1) continue;
      ff_value4<ff_vw<NC>()>(A, r0, r1, r2, r3, val, &ovf);
      const int c0 = Lay.col0[a], nl = Lay.nlimb[a];
      const uint32_t l0 = (uint32_t)val[0], l1 = (uint32_t)val[1], l2 = (uint32_t)val[2], l3 = (uint32_t)val[3];
      const uint32_t h0 = (uint32_t)(val[0] >> 32), h1 = (uint32_t)(val[1] >> 32), h2 = (uint32_t)(val[2] >> 32),
                     h3 = (uint32_t)(val[3] >> 32);
      for (int l = 0; l < nl; ++l) {
        uint32_t d = l < 4 ? limb_dword(l0, l1, l2, l3, l) : limb_dword(h0, h1, h2, h3, l - 4);
        if (l != nl - 1) d ^= 0x80808080u;   // lower limbs: u - 128 as int8
        *reinterpret_cast<uint32_t*>(T + (c0 + l) * kMfmaCol + 4 * lane) = d;
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint4 gv = *reinterpret_cast<const uint4*>(gidb + 64 * s + q16);
      v4i af;
      af[0] = (int)bytes_eq(gv.x, g4);
      af[1] = (int)bytes_eq(gv.y, g4);
      af[2] = (int)bytes_eq(gv.z, g4);
      af[3] = (int)bytes_eq(gv.w, g4);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const uint4 bw = *reinterpret_cast<const uint4*>(T + (16 * t + (lane & 15)) * kMfmaCol + 64 * s + q16);
        const v4i bf = v4i{(int)bw.x, (int)bw.y, (int)bw.z, (int)bw.w};
        acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, acc[t], 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (++steps == (1 << 12)) {
      steps = 0;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        for (int i = 0; i < 4; ++i) acc64[t][i] += acc[t][i];
        acc[t] = v4i{0, 0, 0, 0};
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
    for (int i = 0; i < 4; ++i) acc64[t][i] += acc[t][i];
  __syncthreads();
  // D[m = 4 (lane >> 4) + i][n = lane & 15] of tile t -> red[wave][16 t + n][m]
#pragma unroll
  for (int t = 0; t < NT; ++t)
    for (int i = 0; i < 4; ++i) red[wave][16 * t + (lane & 15)][4 * (lane >> 4) + i] = acc64[t][i];
  __syncthreads();
  const int G = S.ngroups;
  for (int s = threadIdx.x; s < G * (NA + 1); s += kMfmaBlock) {
    const int g = s / (NA + 1), a = s % (NA + 1);
    auto limb_sum = [&](int col) {
      long long x = 0;
      for (int w = 0; w < waves; ++w) x += red[w][col][g];
      return x;
    };
    const long long cnt = limb_sum(Lay.count_col);
    if (a == NA || S.aggs[a].op == 1) {
      if (cnt) atomicAdd((unsigned long long*)(a == NA ? &S.counts[g] : &S.aggs[a].dst[g]), (unsigned long long)cnt);
      continue;
    }
    const int nl = Lay.nlimb[a];
    __int128 tot = 0;
    for (int l = 0; l < nl; ++l) {
      const long long x = limb_sum(Lay.col0[a] + l) + (l == nl - 1 ? 0 : 128 * cnt);
      tot += (__int128)x << (8 * l);
    }
    if (tot != 0)
      atomic_add_i128_parts((unsigned long long*)&S.aggs[a].dst[g], (long long*)&S.aggs[a].dst2[g],
                            (unsigned long long)(uint64_t)tot, (long long)(int64_t)(tot >> 64));
  }
  if (__any(ovf) && lane == 0 && S.overflow) atomicOr(S.overflow, 1);
}

}  // namespace

template <int NC>
void launch_mask(const FfSpec& spec, int64_t n, uint8_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(ff_mask_kernel<NC>, dim3(grid_for(n, kBlock * kFfRows * 2, 256 * 16)), dim3(kBlock), 0, stream,
                     spec, n, out);
}

constexpr int kFfLdsMax = 64 * 1024;

template <int NC>
void launch_agg(const FfSpec& spec, int64_t n, hipStream_t stream) {
  // per-lane slots while they fit the LDS budget, fewer (shared) lanes beyond
  const size_t cells = (size_t)(spec.naggs + 1) * spec.ngroups;
  int lanes = kWave;
  while (lanes > 1 && cells * 2 * lanes * sizeof(int64_t) > (size_t)kFfLdsMax) lanes >>= 1;
  const size_t lds = cells * 2 * lanes * sizeof(int64_t);
  constexpr int block = kFfAggBlock;
  // persistent-style grid: about as many blocks as stay resident (LDS-limited,
  // 160 KB per CU; at most 2048 threads), each streaming many rows, so the
  // per-block init/merge is amortised
  int per_cu = (int)((160 * 1024) / (lds ? lds : 1));
  per_cu = per_cu < 1 ? 1 : per_cu;
  per_cu = per_cu > 2048 / block ? 2048 / block : per_cu;
  hipLaunchKernelGGL(ff_agg_kernel<NC>, dim3(grid_for(n, block * kFfRows * 4, 256 * per_cu)), dim3(block), lds,
                     stream, spec, n, lanes);
}

void ff_mask(const FfSpec& spec, int64_t n, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  switch (spec.ncols) {
    case 1: launch_mask<1>(spec, n, out, stream); break;
    case 2: launch_mask<2>(spec, n, out, stream); break;
    case 3: launch_mask<3>(spec, n, out, stream); break;
    case 4: launch_mask<4>(spec, n, out, stream); break;
    case 5: launch_mask<5>(spec, n, out, stream); break;
    case 6: launch_mask<6>(spec, n, out, stream); break;
    case 7: launch_mask<7>(spec, n, out, stream); break;
    default: launch_mask<8>(spec, n, out, stream); break;
  }
  check_launch("ff_mask", stream);
}

// Off by default: kernel-level A/B at SF100 (scripts/ff_ab.sh, rocprofv3)
// measured the interpreted one-hot MFMA path at 9.2 ms for Q1 against 6.6 ms
// for the LDS-atomic kernel (the per-row value/limb interpretation dominates
// either way); the generated scan kernels (exec/fused_jit.py) replace both
// on warm queries.
static bool g_ff_mfma = debug_flag("ff_mfma");

bool ff_set_mfma(bool on) {
  const bool prev = g_ff_mfma;
  g_ff_mfma = on;
  return prev;
}

template <int NC>
static void launch_mfma(const FfSpec& spec, const FfMfmaLayout& lay, int nt, int64_t n, hipStream_t stream) {
  // persistent-style: about as many blocks as stay resident (LDS-limited)
  const int lds = (kMfmaBlock / kWave) * (nt * 16 + 1) * kMfmaCol;
  int per_cu = (160 * 1024) / lds;
  per_cu = per_cu < 1 ? 1 : per_cu > 8 ? 8 : per_cu;
  const unsigned grid = grid_for(n, kMfmaBlock * kFfRows * 8, 256 * per_cu);
  switch (nt) {
    case 1: hipLaunchKernelGGL((ff_mfma_agg_kernel<NC, 1>), dim3(grid), dim3(kMfmaBlock), 0, stream, spec, lay, n); break;
    case 2: hipLaunchKernelGGL((ff_mfma_agg_kernel<NC, 2>), dim3(grid), dim3(kMfmaBlock), 0, stream, spec, lay, n); break;
    case 3: hipLaunchKernelGGL((ff_mfma_agg_kernel<NC, 3>), dim3(grid), dim3(kMfmaBlock), 0, stream, spec, lay, n); break;
    default: hipLaunchKernelGGL((ff_mfma_agg_kernel<NC, 4>), dim3(grid), dim3(kMfmaBlock), 0, stream, spec, lay, n); break;
  }
}

// SUM / COUNT only, <= 16 groups, <= 64 limb columns: the one-hot MFMA path
static bool try_mfma(const FfSpec& spec, int64_t n, hipStream_t stream) {
  if (!g_ff_mfma || spec.ngroups > 16) return false;
  FfMfmaLayout lay{};
  int col = 0;
  for (int a = 0; a < spec.naggs; ++a) {
    const FfAgg& A = spec.aggs[a];
    if (A.op != 0 && A.op != 1) return false;
    if (A.op == 1) continue;
    const int w = A.vbits > 0 && A.vbits <= 64 ? A.vbits : 64;
    const int nl = (w + 7) / 8;
    lay.col0[a] = col;
    lay.nlimb[a] = nl;
    col += nl;
  }
  lay.count_col = col++;
  lay.ncols = col;
  const int nt = (col + 15) / 16;
  if (nt > kMfmaMaxTiles) return false;
  switch (spec.ncols) {
    case 1: launch_mfma<1>(spec, lay, nt, n, stream); break;
    case 2: launch_mfma<2>(spec, lay, nt, n, stream); break;
    case 3: launch_mfma<3>(spec, lay, nt, n, stream); break;
    case 4: launch_mfma<4>(spec, lay, nt, n, stream); break;
    case 5: launch_mfma<5>(spec, lay, nt, n, stream); break;
    case 6: launch_mfma<6>(spec, lay, nt, n, stream); break;
    case 7: launch_mfma<7>(spec, lay, nt, n, stream); break;
    default: launch_mfma<8>(spec, lay, nt, n, stream); break;
  }
  check_launch("ff_aggregate_mfma", stream);
  return true;
}

void ff_aggregate(const FfSpec& spec, int64_t n, hipStream_t stream) {
  if (n == 0) return;
  if (try_mfma(spec, n, stream)) return;
  switch (spec.ncols) {
    case 1: launch_agg<1>(spec, n, stream); break;
    case 2: launch_agg<2>(spec, n, stream); break;
    case 3: launch_agg<3>(spec, n, stream); break;
    case 4: launch_agg<4>(spec, n, stream); break;
    case 5: launch_agg<5>(spec, n, stream); break;
    case 6: launch_agg<6>(spec, n, stream); break;
    case 7: launch_agg<7>(spec, n, stream); break;
    default: launch_agg<8>(spec, n, stream); break;
  }
  check_launch("ff_aggregate", stream);
}

}  // namespace kern
}  // namespace igloo
