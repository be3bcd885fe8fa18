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
// Every descriptor loop has a wave-uniform trip count, so the per-row code is
// straight-line loads + compares + multiply-adds.
//
// Aggregation: each lane pre-reduces its kFfRows rows, the wave reduces each
// (group, aggregate) with cross-lane shuffles (int128 sums exact through
// 32-bit halves), lane 0 accumulates into wave-private LDS slots, and the
// block merges its slots into global memory with one atomic per slot.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kFfRows = 4;  // rows per lane per iteration (coalesced: base + j*64 + lane)

// Branch-free column load (int32 / int64 columns): two dword loads at
// p + row*w and p + row*w + (w-4) (the same dword twice for int32 columns).
// Keeping every load unconditional lets all of a row's loads be in flight at
// once (a width switch per load made the compiler wait after each one).
__device__ __forceinline__ int64_t ff_load(const FfColumn& c, int64_t row) {
  const char* p = (const char*)c.ptr + row * c.width;
  const uint32_t lo = *(const uint32_t*)p;
  const uint32_t hi = *(const uint32_t*)(p + (c.width - 4));
  // both dwords are always consumed (a select let the compiler sink the second
  // load into a branch and wait on it): int32 columns sign-extend via shifts
  const int64_t v = (int64_t)(((uint64_t)hi << 32) | lo);
  const int sh = c.width == 8 ? 0 : 32;
  return (int64_t)((uint64_t)v << sh) >> sh;
}

// Column values of one lane's rows as 32 named scalars (no array at all:
// any dynamically indexed local array ended up in scratch). The wave-uniform
// column number is resolved by a select chain over the static slots.
#define FF_COLS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
static_assert(kFfMaxCols == 8 && kFfRows == 4, "FfRowVals is written for 8 columns x 4 rows");
struct FfRowVals {
#define FF_DECL(c) int64_t c##_0, c##_1, c##_2, c##_3;
#define FF_DECL2(c) FF_DECL(v##c)
  FF_COLS(FF_DECL2)
#undef FF_DECL2
#undef FF_DECL
};

// NC (the number of input columns) is a template parameter: the load block
// has no branches, so every column's loads are issued before the first wait.
template <int NC>
__device__ __forceinline__ void ff_load_rows(const FfSpec& S, const int64_t* rows, FfRowVals& R) {
#define FF_LD(c)                                   \
  if constexpr (c < NC) {                         \
    R.v##c##_0 = ff_load(S.cols[c], rows[0]);     \
    R.v##c##_1 = ff_load(S.cols[c], rows[1]);     \
    R.v##c##_2 = ff_load(S.cols[c], rows[2]);     \
    R.v##c##_3 = ff_load(S.cols[c], rows[3]);     \
  }
  FF_COLS(FF_LD)
#undef FF_LD
}

template <int NC>
__device__ __forceinline__ int64_t col_of(const FfRowVals& R, int c, int j) {
  c = __builtin_amdgcn_readfirstlane(c);
  int64_t out = 0;
#define FF_SEL(k)                                                                                      \
  if constexpr (k < NC)                                                                               \
    out = (c == k) ? (j == 0 ? R.v##k##_0 : j == 1 ? R.v##k##_1 : j == 2 ? R.v##k##_2 : R.v##k##_3) : out;
  FF_COLS(FF_SEL)
#undef FF_SEL
  return out;
}

template <int NC>
__device__ __forceinline__ bool ff_pass(const FfSpec& S, const FfRowVals& R, int j, int64_t row) {
  bool ok = true;
  for (int t = 0; t < S.nterms; ++t) {
    const FfTerm& T = S.terms[t];
    const int64_t v = col_of<NC>(R, T.col, j);
    const bool in_range = v >= T.lo && v <= T.hi;
    const bool in_set = v >= 0 && v < 64 && ((T.set >> (v & 63)) & 1ULL);
    const bool hit = T.kind == 2 ? in_set : in_range;
    ok &= (T.kind == 1) ? !hit : hit;
  }
  if (S.mask) ok &= S.mask[row] != 0;
  return ok;
}

template <int NC>
__device__ __forceinline__ int64_t ff_value(const FfAgg& A, const FfRowVals& R, int j, int* ovf) {
  int64_t acc = 1;
  for (int f = 0; f < A.nfac; ++f) {
    const FfFactor& F = A.f[f];
    const int64_t term =
        F.col < 0 ? F.a : (int64_t)((uint64_t)F.a + (uint64_t)F.b * (uint64_t)col_of<NC>(R, (int)F.col, j));
    if (A.checked) {
      int64_t r;
      if (__builtin_mul_overflow(acc, term, &r)) *ovf = 1;
      acc = r;
    } else {
      acc = (int64_t)((uint64_t)acc * (uint64_t)term);
    }
  }
  return acc;
}

__device__ __forceinline__ void ff_rows(int64_t base, int lane, int64_t n, int64_t* rows, bool* live) {
#pragma unroll
  for (int j = 0; j < kFfRows; ++j) {
    const int64_t r = base + j * kWave + lane;
    live[j] = r < n;
    rows[j] = r < n ? r : n - 1;
  }
}

template <int NC>
__global__ __launch_bounds__(kBlock) void ff_mask_kernel(const FfSpec S, int64_t n, uint8_t* __restrict__ out) {
  const int wave = threadIdx.x / kWave, lane = lane_id();
  const int64_t per_iter = (int64_t)kWave * kFfRows;
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * per_iter;
  for (int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * per_iter; base < n; base += stride) {
    int64_t rows[kFfRows];
    bool live[kFfRows];
    ff_rows(base, lane, n, rows, live);
    FfRowVals R;
    ff_load_rows<NC>(S, rows, R);
#pragma unroll
    for (int j = 0; j < kFfRows; ++j)
      if (live[j]) out[rows[j]] = ff_pass<NC>(S, R, j, rows[j]);
  }
}

__device__ inline int64_t wsum(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}
__device__ inline int64_t wmin(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(v, off, kWave);
    v = o < v ? o : v;
  }
  return v;
}
__device__ inline int64_t wmax(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(v, off, kWave);
    v = o > v ? o : v;
  }
  return v;
}

template <int NC>
__global__ __launch_bounds__(kBlock) void ff_agg_kernel(const FfSpec S, int64_t n) {
  // [wave][group][agg or count][lo, hi]
  __shared__ int64_t slots[kWavesPerBlock][kFfMaxGroups][kFfMaxAggs + 1][2];
  const int wave = threadIdx.x / kWave, lane = lane_id();
  const int G = S.ngroups, NA = S.naggs;
  for (int s = threadIdx.x; s < kWavesPerBlock * kFfMaxGroups * (kFfMaxAggs + 1); s += kBlock) {
    const int w = s / (kFfMaxGroups * (kFfMaxAggs + 1));
    const int rem = s % (kFfMaxGroups * (kFfMaxAggs + 1));
    const int g = rem / (kFfMaxAggs + 1), a = rem % (kFfMaxAggs + 1);
    int64_t init = 0;
    if (a < NA && S.aggs[a].op == 2) init = INT64_MAX;
    if (a < NA && S.aggs[a].op == 3) init = INT64_MIN;
    slots[w][g][a][0] = init;
    slots[w][g][a][1] = 0;
  }
  __syncthreads();
  int ovf = 0;
  const int64_t per_iter = (int64_t)kWave * kFfRows;
  const int64_t stride = (int64_t)gridDim.x * kWavesPerBlock * per_iter;
  for (int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wave) * per_iter; base < n; base += stride) {
    int64_t rows[kFfRows];
    bool live[kFfRows];
    ff_rows(base, lane, n, rows, live);
    FfRowVals R;
    ff_load_rows<NC>(S, rows, R);
    bool pass[kFfRows];
    int gid[kFfRows];
    bool any = false;
#pragma unroll
    for (int j = 0; j < kFfRows; ++j) {
      pass[j] = live[j] && ff_pass<NC>(S, R, j, rows[j]);
      int g = 0;
      for (int k = 0; k < S.nkeys; ++k) g += (int)((col_of<NC>(R, S.key_col[k], j) - S.key_lo[k]) * S.key_mul[k]);
      gid[j] = g;
      any |= pass[j];
    }
    if (!__ballot(any)) continue;
    // row counts per group
    for (int g = 0; g < G; ++g) {
      int cnt = 0;
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) cnt += pass[j] && gid[j] == g;
      if (!__ballot(cnt != 0)) continue;
      const int64_t wc = wsum(cnt);
      if (lane == 0) slots[wave][g][kFfMaxAggs][0] += wc;
    }
    // aggregates: argument values once per row, then one reduction per group
#pragma unroll
    for (int a = 0; a < kFfMaxAggs; ++a) {
      if (a >= NA) continue;
      const FfAgg& A = S.aggs[a];
      int64_t val[kFfRows];
#pragma unroll
      for (int j = 0; j < kFfRows; ++j) val[j] = (pass[j] && A.op != 1) ? ff_value<NC>(A, R, j, &ovf) : 0;
      for (int g = 0; g < G; ++g) {
        bool m[kFfRows];
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < kFfRows; ++j) {
          m[j] = pass[j] && gid[j] == g;
          cnt += m[j];
        }
        if (!__ballot(cnt != 0)) continue;
        if (A.op == 0) {  // exact sum: per-lane partial in 32-bit halves
          int64_t lo = 0, hi = 0;
#pragma unroll
          for (int j = 0; j < kFfRows; ++j)
            if (m[j]) {
              lo += (int64_t)(uint32_t)(uint64_t)val[j];
              hi += val[j] >> 32;
            }
          const int64_t slo = wsum(lo), shi = wsum(hi);
          if (lane == 0) {
            __int128 acc = ((__int128)slots[wave][g][a][1] << 64) | (unsigned __int128)(uint64_t)slots[wave][g][a][0];
            acc += ((__int128)shi << 32) + (__int128)slo;
            slots[wave][g][a][0] = (int64_t)(uint64_t)acc;
            slots[wave][g][a][1] = (int64_t)(acc >> 64);
          }
        } else if (A.op == 1) {
          const int64_t wc = wsum(cnt);
          if (lane == 0) slots[wave][g][a][0] += wc;
        } else if (A.op == 2) {
          int64_t r = INT64_MAX;
#pragma unroll
          for (int j = 0; j < kFfRows; ++j)
            if (m[j]) r = val[j] < r ? val[j] : r;
          r = wmin(r);
          if (lane == 0 && r < slots[wave][g][a][0]) slots[wave][g][a][0] = r;
        } else {
          int64_t r = INT64_MIN;
#pragma unroll
          for (int j = 0; j < kFfRows; ++j)
            if (m[j]) r = val[j] > r ? val[j] : r;
          r = wmax(r);
          if (lane == 0 && r > slots[wave][g][a][0]) slots[wave][g][a][0] = r;
        }
      }
    }
  }
  __syncthreads();
  for (int s = threadIdx.x; s < G * (NA + 1); s += kBlock) {
    const int g = s / (NA + 1), a = s % (NA + 1);
    if (a == NA) {
      int64_t c = 0;
      for (int w = 0; w < kWavesPerBlock; ++w) c += slots[w][g][kFfMaxAggs][0];
      if (c) atomicAdd((unsigned long long*)&S.counts[g], (unsigned long long)c);
      continue;
    }
    const FfAgg& A = S.aggs[a];
    if (A.op == 0) {
      __int128 acc = 0;
      for (int w = 0; w < kWavesPerBlock; ++w)
        acc += ((__int128)slots[w][g][a][1] << 64) | (unsigned __int128)(uint64_t)slots[w][g][a][0];
      if (acc != 0)
        atomic_add_i128_parts((unsigned long long*)&A.dst[g], (long long*)&A.dst2[g], (unsigned long long)(uint64_t)acc,
                              (long long)(int64_t)(acc >> 64));
    } else if (A.op == 1) {
      int64_t c = 0;
      for (int w = 0; w < kWavesPerBlock; ++w) c += slots[w][g][a][0];
      if (c) atomicAdd((unsigned long long*)&A.dst[g], (unsigned long long)c);
    } else if (A.op == 2) {
      int64_t r = INT64_MAX;
      for (int w = 0; w < kWavesPerBlock; ++w) r = slots[w][g][a][0] < r ? slots[w][g][a][0] : r;
      atomicMin((long long*)&A.dst[g], (long long)r);
    } else {
      int64_t r = INT64_MIN;
      for (int w = 0; w < kWavesPerBlock; ++w) r = slots[w][g][a][0] > r ? slots[w][g][a][0] : r;
      atomicMax((long long*)&A.dst[g], (long long)r);
    }
  }
  if (__any(ovf) && lane == 0 && S.overflow) atomicOr(S.overflow, 1);
}

}  // namespace

template <int NC>
void launch_mask(const FfSpec& spec, int64_t n, uint8_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(ff_mask_kernel<NC>, dim3(grid_for(n, kBlock * kFfRows * 2, 256 * 16)), dim3(kBlock), 0, stream,
                     spec, n, out);
}

template <int NC>
void launch_agg(const FfSpec& spec, int64_t n, hipStream_t stream) {
  hipLaunchKernelGGL(ff_agg_kernel<NC>, dim3(grid_for(n, kBlock * kFfRows * 4, 256 * 8)), dim3(kBlock), 0, stream, spec,
                     n);
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

void ff_aggregate(const FfSpec& spec, int64_t n, hipStream_t stream) {
  if (n == 0) return;
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
