// GPU hash tables for equi-joins and GROUP BY.
//
// Replaces the reference's HashJoinExec build/probe, which keys a
// HashMap<Vec<u8>, Vec<RecordBatch>> on Debug-formatted key bytes and probes
// row by row (reference crates/engine/src/operators/hash_join.rs:101-128,
// :141-203), and DataFusion's AggregateExec group table.
//
// Layout (struct-of-arrays, one HBM line per probe in the common case):
//   hashed mode: tkeys[cap] int64 (kEmptyKey = empty) + thead[cap] int32,
//                open addressing with linear probing, cap = pow2 >= 2n;
//   direct mode: when the key domain [kmin, kmin+cap) is dense enough the
//                key itself is the slot (a perfect hash): no key array, no
//                probing, one random read per probe row. TPC-H keys are
//                dense integers, so most joins take this path.
// Duplicate build keys are chained through next[row] (atomicExch on the
// slot head), so the same table serves unique (PK) and multi-match joins.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kMaxGrid = 256 * 8 * 16;  // 32768 blocks: every CU gets many waves of random loads

template <typename K>
__device__ inline bool load_key(const K* keys, const uint8_t* valid, int64_t i, int64_t* out) {
  if (valid && !valid[i]) return false;
  *out = (int64_t)keys[i];
  return true;
}

// Find the slot holding `k` (hashed mode); -1 when absent.
__device__ inline int64_t find_slot(const int64_t* __restrict__ tkeys, int64_t mask, int64_t k) {
  int64_t slot = (int64_t)(mix64((uint64_t)k) & (uint64_t)mask);
  for (;;) {
    int64_t tk = tkeys[slot];
    if (tk == k) return slot;
    if (tk == kEmptyKey) return -1;
    slot = (slot + 1) & mask;
  }
}

// Insert-or-find `k` (hashed mode); returns the slot and whether the key
// already existed.
__device__ inline int64_t insert_slot(int64_t* __restrict__ tkeys, int64_t mask, int64_t k, bool* existed) {
  int64_t slot = (int64_t)(mix64((uint64_t)k) & (uint64_t)mask);
  for (;;) {
    unsigned long long prev = atomicCAS((unsigned long long*)&tkeys[slot], (unsigned long long)kEmptyKey,
                                        (unsigned long long)k);
    if ((int64_t)prev == kEmptyKey) { *existed = false; return slot; }
    if ((int64_t)prev == k) { *existed = true; return slot; }
    slot = (slot + 1) & mask;
  }
}

// Optional 1-hash Bloom filter over the build keys (<= 4 MB, so it stays in a
// XCD's L2): a selective probe (most probe keys absent) answers from L2 and
// never touches the HBM-sized table.
// Bloom bit of key k. With kExactBits set in bmask (direct-mapped tables whose
// key span fits the bitmap, ops/hashing.py JoinTable) the "filter" is an exact
// membership bitmap indexed by k - kmin: no false positives, so a probe reads
// the table only for keys that are present. Callers range-check k first.
constexpr uint64_t kExactBits = 1ull << 63;
__device__ inline uint64_t bloom_bit(int64_t k, uint64_t bmask, int64_t kmin) {
  return (bmask & kExactBits) ? (uint64_t)(k - kmin) : ((mix64((uint64_t)k) >> 7) & bmask);
}

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void join_build_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t n, int64_t* __restrict__ tkeys,
                                                           int32_t* __restrict__ thead, int32_t* __restrict__ next,
                                                           int64_t cap, int64_t kmin, unsigned long long* dups,
                                                           uint32_t* __restrict__ bits, uint64_t bmask) {
  const int64_t mask = cap - 1;
  unsigned long long local_dups = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k;
    if (!load_key(keys, valid, i, &k)) { next[i] = -1; continue; }
    int64_t slot;
    if (DIRECT) {
      slot = k - kmin;
      // a key outside the span only occurs under a replayed key range that the
      // end-of-query check will reject (ops/_lib.py Speculation): stay in bounds
      if ((uint64_t)slot >= (uint64_t)cap) continue;
    } else {
      bool existed;
      slot = insert_slot(tkeys, mask, k, &existed);
    }
    int32_t old = atomicExch(&thead[slot], (int32_t)i);
    next[i] = old;
    local_dups += old != -1;
    if (bits) {
      const uint64_t bb = bloom_bit(k, bmask, kmin);
      atomicOr(&bits[bb >> 5], 1u << (bb & 31));
    }
  }
  // one atomic per wave for the duplicate counter
  for (int off = kWave / 2; off > 0; off >>= 1) local_dups += __shfl_xor(local_dups, off, kWave);
  if (lane_id() == 0 && local_dups) atomicAdd(dups, local_dups);
}

template <typename K, bool DIRECT>
__device__ inline int32_t probe_head(const K* keys, const uint8_t* valid, int64_t j, const int64_t* tkeys,
                                     const int32_t* thead, int64_t cap, int64_t kmin, const uint32_t* bits,
                                     uint64_t bmask) {
  int64_t k;
  if (!load_key(keys, valid, j, &k)) return -1;
  if (DIRECT && (k - kmin < 0 || k - kmin >= cap)) return -1;
  if (bits) {
    const uint64_t b = bloom_bit(k, bmask, kmin);
    if (!((bits[b >> 5] >> (b & 31)) & 1u)) return -1;
  }
  if (DIRECT) return thead[k - kmin];
  int64_t s = find_slot(tkeys, cap - 1, k);
  return s < 0 ? -1 : thead[s];
}

// counts[j] = number of build matches of probe row j; first[j] = one match or -1.
template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void join_probe_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t m, const int64_t* __restrict__ tkeys,
                                                           const int32_t* __restrict__ thead,
                                                           const int32_t* __restrict__ next, int64_t cap, int64_t kmin,
                                                           int32_t* __restrict__ counts, int32_t* __restrict__ first,
                                                           uint8_t* __restrict__ build_matched,
                                                           const uint32_t* __restrict__ bits, uint64_t bmask) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    int32_t h = probe_head<K, DIRECT>(keys, valid, j, tkeys, thead, cap, kmin, bits, bmask);
    if (first) first[j] = h;
    if (counts) {
      int32_t c = 0;
      for (int32_t r = h; r != -1; r = next[r]) {
        ++c;
        if (build_matched) build_matched[r] = 1;
      }
      counts[j] = c;
    } else if (build_matched) {
      for (int32_t r = h; r != -1; r = next[r]) build_matched[r] = 1;
    }
  }
}

// first-match probe, direct-mapped table, 4 rows per lane: all key loads,
// then all filter-bit loads, then all head loads are issued before their
// results are needed, so a lane keeps 4 misses in flight instead of one
// dependent chain (600M-row lineitem probes were latency-bound).
constexpr int kProbeRows = 4;

template <typename K>
__global__ __launch_bounds__(kBlock) void join_probe_first_direct_kernel(
    const K* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t m, const int32_t* __restrict__ thead,
    int64_t cap, int64_t kmin, int32_t* __restrict__ first, const uint32_t* __restrict__ bits, uint64_t bmask) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j0 < m; j0 += stride * kProbeRows) {
    int64_t s[kProbeRows];
    bool ok[kProbeRows];
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) {
      const int64_t j = j0 + r * stride;
      ok[r] = j < m && (!valid || valid[j]);
      s[r] = ok[r] ? (int64_t)keys[j] - kmin : -1;
      ok[r] = ok[r] && s[r] >= 0 && s[r] < cap;
    }
    if (bits) {
      uint32_t w[kProbeRows];
#pragma unroll
      for (int r = 0; r < kProbeRows; ++r) {
        const uint64_t b = ok[r] ? bloom_bit(s[r] + kmin, bmask, kmin) : 0;
        w[r] = ok[r] ? (bits[b >> 5] >> (b & 31)) & 1u : 0u;
      }
#pragma unroll
      for (int r = 0; r < kProbeRows; ++r) ok[r] = ok[r] && w[r];
    }
    int32_t h[kProbeRows];
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) h[r] = ok[r] ? thead[s[r]] : -1;
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) {
      const int64_t j = j0 + r * stride;
      if (j < m) first[j] = h[r];
    }
  }
}

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void join_expand_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                            int64_t m, const int64_t* __restrict__ tkeys,
                                                            const int32_t* __restrict__ thead,
                                                            const int32_t* __restrict__ next, int64_t cap, int64_t kmin,
                                                            const int64_t* __restrict__ offsets,
                                                            int32_t* __restrict__ out_probe,
                                                            int32_t* __restrict__ out_build,
                                                            const uint32_t* __restrict__ bits, uint64_t bmask) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    int32_t h = probe_head<K, DIRECT>(keys, valid, j, tkeys, thead, cap, kmin, bits, bmask);
    int64_t o = offsets[j];
    for (int32_t r = h; r != -1; r = next[r]) {
      out_probe[o] = (int32_t)j;
      out_build[o] = r;
      ++o;
    }
  }
}

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void groupby_build_kernel(const K* __restrict__ keys, int64_t n,
                                                              int64_t* __restrict__ tkeys, int32_t* __restrict__ trow,
                                                              int64_t cap, int64_t kmin) {
  const int64_t mask = cap - 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = (int64_t)keys[i];
    int64_t slot;
    if (DIRECT) {
      slot = k - kmin;
      // a key outside the span only occurs under a replayed key range that the
      // end-of-query check will reject (ops/_lib.py Speculation): stay in bounds
      if ((uint64_t)slot >= (uint64_t)cap) continue;
    } else {
      bool existed;
      slot = insert_slot(tkeys, mask, k, &existed);
    }
    // first occurrence row: plain read first avoids most atomics on hot groups
    if (trow[slot] > (int32_t)i) atomicMin(&trow[slot], (int32_t)i);
  }
}

// Direct-mapped GROUP BY over a small key span (Q5's 5 nations, Q7/Q9's
// (nation, year) pairs over millions of rows): the first-row table lives in
// LDS per workgroup, so the atomics that would serialise on a handful of
// global words stay on-chip; one global atomicMin per touched slot per
// workgroup at the end.
constexpr int64_t kGroupLdsSlots = 16384;

template <typename K>
__global__ __launch_bounds__(kBlock) void groupby_build_lds_kernel(const K* __restrict__ keys, int64_t n,
                                                                  int32_t* __restrict__ trow, int64_t cap,
                                                                  int64_t kmin) {
  __shared__ int32_t srow[kGroupLdsSlots];
  for (int64_t s = threadIdx.x; s < cap; s += blockDim.x) srow[s] = INT32_MAX;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t slot = (int64_t)keys[i] - kmin;
    if ((uint64_t)slot >= (uint64_t)cap) continue;   // see groupby_build_kernel
    if (srow[slot] > (int32_t)i) atomicMin(&srow[slot], (int32_t)i);
  }
  __syncthreads();
  for (int64_t s = threadIdx.x; s < cap; s += blockDim.x) {
    const int32_t r = srow[s];
    if (r != INT32_MAX && trow[s] > r) atomicMin(&trow[s], r);
  }
}

// also zeroes gid_of_slot: a slot the (replayed) group count leaves unassigned
// then maps to group 0 instead of an uninitialised id (see groupby_build_kernel)
__global__ __launch_bounds__(kBlock) void occupied_kernel(const int32_t* __restrict__ trow, int64_t cap,
                                                         uint8_t* __restrict__ occ, int32_t* __restrict__ gid_of_slot) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cap; i += (int64_t)gridDim.x * blockDim.x) {
    occ[i] = trow[i] != INT32_MAX;
    gid_of_slot[i] = 0;
  }
}

// gid_of_slot[slots[g]] = g ; rep_row[g] = trow[slots[g]]
template <typename S>
__global__ __launch_bounds__(kBlock) void assign_gid_kernel(const S* __restrict__ slots, int64_t g,
                                                           const int32_t* __restrict__ trow,
                                                           int32_t* __restrict__ gid_of_slot,
                                                           int32_t* __restrict__ rep_row) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = (int64_t)slots[i];
    gid_of_slot[s] = (int32_t)i;
    rep_row[i] = trow[s];
  }
}

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void groupby_lookup_kernel(const K* __restrict__ keys, int64_t n,
                                                               const int64_t* __restrict__ tkeys,
                                                               const int32_t* __restrict__ gid_of_slot, int64_t cap,
                                                               int64_t kmin, int32_t* __restrict__ gid) {
  const int64_t mask = cap - 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k = (int64_t)keys[i];
    int64_t slot = DIRECT ? k - kmin : find_slot(tkeys, mask, k);
    if (DIRECT && (uint64_t)slot >= (uint64_t)cap) slot = 0;   // see groupby_build_kernel
    gid[i] = gid_of_slot[slot];
  }
}

#define DISPATCH_KEY(key64, direct, KERNEL, ...)                                      \
  do {                                                                                \
    if (key64) {                                                                      \
      if (direct) hipLaunchKernelGGL((KERNEL<int64_t, true>), __VA_ARGS__);           \
      else hipLaunchKernelGGL((KERNEL<int64_t, false>), __VA_ARGS__);                 \
    } else {                                                                          \
      if (direct) hipLaunchKernelGGL((KERNEL<int32_t, true>), __VA_ARGS__);           \
      else hipLaunchKernelGGL((KERNEL<int32_t, false>), __VA_ARGS__);                 \
    }                                                                                 \
  } while (0)

template <typename I>
__global__ __launch_bounds__(kBlock) void fill_runs_kernel(const I* __restrict__ starts, int64_t nruns, int64_t n,
                                                          int32_t* __restrict__ gid) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nruns; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = starts[r], e = r + 1 < nruns ? (int64_t)starts[r + 1] : n;
    for (int64_t i = b; i < e; ++i) gid[i] = (int32_t)r;
  }
}

}  // namespace

void fill_runs(const void* starts, bool starts64, int64_t nruns, int64_t n, int32_t* gid, hipStream_t stream) {
  if (nruns == 0) return;
  dim3 g(grid_for(nruns, kBlock, kMaxGrid)), b(kBlock);
  if (starts64) hipLaunchKernelGGL(fill_runs_kernel<int64_t>, g, b, 0, stream, (const int64_t*)starts, nruns, n, gid);
  else hipLaunchKernelGGL(fill_runs_kernel<int32_t>, g, b, 0, stream, (const int32_t*)starts, nruns, n, gid);
  check_launch("fill_runs", stream);
}

void join_build(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t* tkeys, int32_t* thead,
                int32_t* next, int64_t cap, int64_t kmin, bool direct, unsigned long long* dups, uint32_t* bits,
                uint64_t bmask, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (key64) {
    if (direct) hipLaunchKernelGGL((join_build_kernel<int64_t, true>), g, b, 0, stream, (const int64_t*)keys, valid, n, tkeys, thead, next, cap, kmin, dups, bits, bmask);
    else hipLaunchKernelGGL((join_build_kernel<int64_t, false>), g, b, 0, stream, (const int64_t*)keys, valid, n, tkeys, thead, next, cap, kmin, dups, bits, bmask);
  } else {
    if (direct) hipLaunchKernelGGL((join_build_kernel<int32_t, true>), g, b, 0, stream, (const int32_t*)keys, valid, n, tkeys, thead, next, cap, kmin, dups, bits, bmask);
    else hipLaunchKernelGGL((join_build_kernel<int32_t, false>), g, b, 0, stream, (const int32_t*)keys, valid, n, tkeys, thead, next, cap, kmin, dups, bits, bmask);
  }
  check_launch("join_build", stream);
}

void join_probe(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const int32_t* thead, const int32_t* next, int64_t cap, int64_t kmin, bool direct, int32_t* counts,
                int32_t* first, uint8_t* build_matched, const uint32_t* bits, uint64_t bmask, hipStream_t stream) {
  if (m == 0) return;
  dim3 g(grid_for(m, kBlock, kMaxGrid)), b(kBlock);
  if (direct && first && !counts && !build_matched) {
    const dim3 g4(grid_for((m + kProbeRows - 1) / kProbeRows, kBlock, kMaxGrid));
    if (key64)
      hipLaunchKernelGGL(join_probe_first_direct_kernel<int64_t>, g4, b, 0, stream, (const int64_t*)keys, valid, m,
                         thead, cap, kmin, first, bits, bmask);
    else
      hipLaunchKernelGGL(join_probe_first_direct_kernel<int32_t>, g4, b, 0, stream, (const int32_t*)keys, valid, m,
                         thead, cap, kmin, first, bits, bmask);
    check_launch("join_probe_first_direct", stream);
    return;
  }
  if (key64) {
    if (direct) hipLaunchKernelGGL((join_probe_kernel<int64_t, true>), g, b, 0, stream, (const int64_t*)keys, valid, m, tkeys, thead, next, cap, kmin, counts, first, build_matched, bits, bmask);
    else hipLaunchKernelGGL((join_probe_kernel<int64_t, false>), g, b, 0, stream, (const int64_t*)keys, valid, m, tkeys, thead, next, cap, kmin, counts, first, build_matched, bits, bmask);
  } else {
    if (direct) hipLaunchKernelGGL((join_probe_kernel<int32_t, true>), g, b, 0, stream, (const int32_t*)keys, valid, m, tkeys, thead, next, cap, kmin, counts, first, build_matched, bits, bmask);
    else hipLaunchKernelGGL((join_probe_kernel<int32_t, false>), g, b, 0, stream, (const int32_t*)keys, valid, m, tkeys, thead, next, cap, kmin, counts, first, build_matched, bits, bmask);
  }
  check_launch("join_probe", stream);
}

void join_expand(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const int32_t* thead, const int32_t* next, int64_t cap, int64_t kmin, bool direct,
                 const int64_t* offsets, int32_t* out_probe, int32_t* out_build, const uint32_t* bits, uint64_t bmask,
                 hipStream_t stream) {
  if (m == 0) return;
  dim3 g(grid_for(m, kBlock, kMaxGrid)), b(kBlock);
  if (key64) {
    if (direct) hipLaunchKernelGGL((join_expand_kernel<int64_t, true>), g, b, 0, stream, (const int64_t*)keys, valid, m, tkeys, thead, next, cap, kmin, offsets, out_probe, out_build, bits, bmask);
    else hipLaunchKernelGGL((join_expand_kernel<int64_t, false>), g, b, 0, stream, (const int64_t*)keys, valid, m, tkeys, thead, next, cap, kmin, offsets, out_probe, out_build, bits, bmask);
  } else {
    if (direct) hipLaunchKernelGGL((join_expand_kernel<int32_t, true>), g, b, 0, stream, (const int32_t*)keys, valid, m, tkeys, thead, next, cap, kmin, offsets, out_probe, out_build, bits, bmask);
    else hipLaunchKernelGGL((join_expand_kernel<int32_t, false>), g, b, 0, stream, (const int32_t*)keys, valid, m, tkeys, thead, next, cap, kmin, offsets, out_probe, out_build, bits, bmask);
  }
  check_launch("join_expand", stream);
}

void groupby_build(const void* keys, bool key64, int64_t n, int64_t* tkeys, int32_t* trow, int64_t cap, int64_t kmin,
                   bool direct, hipStream_t stream) {
  if (n == 0) return;
  if (direct && cap <= kGroupLdsSlots) {
    // a few hundred workgroups: enough to fill the CUs, few end-of-block merges
    const dim3 g(grid_for(n, kBlock * 16, 1024)), b(kBlock);
    if (key64)
      hipLaunchKernelGGL(groupby_build_lds_kernel<int64_t>, g, b, 0, stream, (const int64_t*)keys, n, trow, cap, kmin);
    else
      hipLaunchKernelGGL(groupby_build_lds_kernel<int32_t>, g, b, 0, stream, (const int32_t*)keys, n, trow, cap, kmin);
    check_launch("groupby_build_lds", stream);
    return;
  }
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (key64) {
    if (direct) hipLaunchKernelGGL((groupby_build_kernel<int64_t, true>), g, b, 0, stream, (const int64_t*)keys, n, tkeys, trow, cap, kmin);
    else hipLaunchKernelGGL((groupby_build_kernel<int64_t, false>), g, b, 0, stream, (const int64_t*)keys, n, tkeys, trow, cap, kmin);
  } else {
    if (direct) hipLaunchKernelGGL((groupby_build_kernel<int32_t, true>), g, b, 0, stream, (const int32_t*)keys, n, tkeys, trow, cap, kmin);
    else hipLaunchKernelGGL((groupby_build_kernel<int32_t, false>), g, b, 0, stream, (const int32_t*)keys, n, tkeys, trow, cap, kmin);
  }
  check_launch("groupby_build", stream);
}

void groupby_occupied(const int32_t* trow, int64_t cap, uint8_t* occ, int32_t* gid_of_slot, hipStream_t stream) {
  hipLaunchKernelGGL(occupied_kernel, dim3(grid_for(cap, kBlock, kMaxGrid)), dim3(kBlock), 0, stream, trow, cap, occ, gid_of_slot);
  check_launch("groupby_occupied", stream);
}

void groupby_assign(const void* slots, bool slots64, int64_t g, const int32_t* trow, int32_t* gid_of_slot,
                    int32_t* rep_row, hipStream_t stream) {
  if (g == 0) return;
  dim3 gr(grid_for(g, kBlock, kMaxGrid)), b(kBlock);
  if (slots64)
    hipLaunchKernelGGL(assign_gid_kernel<int64_t>, gr, b, 0, stream, (const int64_t*)slots, g, trow, gid_of_slot, rep_row);
  else
    hipLaunchKernelGGL(assign_gid_kernel<int32_t>, gr, b, 0, stream, (const int32_t*)slots, g, trow, gid_of_slot, rep_row);
  check_launch("groupby_assign", stream);
}

void groupby_lookup(const void* keys, bool key64, int64_t n, const int64_t* tkeys, const int32_t* gid_of_slot,
                    int64_t cap, int64_t kmin, bool direct, int32_t* gid, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (key64) {
    if (direct) hipLaunchKernelGGL((groupby_lookup_kernel<int64_t, true>), g, b, 0, stream, (const int64_t*)keys, n, tkeys, gid_of_slot, cap, kmin, gid);
    else hipLaunchKernelGGL((groupby_lookup_kernel<int64_t, false>), g, b, 0, stream, (const int64_t*)keys, n, tkeys, gid_of_slot, cap, kmin, gid);
  } else {
    if (direct) hipLaunchKernelGGL((groupby_lookup_kernel<int32_t, true>), g, b, 0, stream, (const int32_t*)keys, n, tkeys, gid_of_slot, cap, kmin, gid);
    else hipLaunchKernelGGL((groupby_lookup_kernel<int32_t, false>), g, b, 0, stream, (const int32_t*)keys, n, tkeys, gid_of_slot, cap, kmin, gid);
  }
  check_launch("groupby_lookup", stream);
}

}  // namespace kern
}  // namespace igloo

// ---- probe + compaction in two passes --------------------------------------
// First-match probes whose result is a row selection (inner join on a unique
// build side, semi / anti joins): instead of writing first[] for every probe
// row and compacting it (first: 4 B/row written, compared, flag-compacted:
// ~15 B of traffic per probe row for a 600M-row lineitem probe), pass 1
// writes one hit bit per row and a count per 8192-row tile; pass 2 (after an
// exclusive scan of the tile counts) re-probes only the hit rows and writes
// (probe row, build row) at their final positions, in row order.
namespace igloo {
namespace kern {
namespace {
constexpr int kHitTile = 8192;                 // rows per tile
constexpr int kHitWords = kHitTile / kWave;    // 64-bit hit words per tile (128)

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void probe_hits_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t m, const int64_t* __restrict__ tkeys,
                                                           const int32_t* __restrict__ thead, int64_t cap,
                                                           int64_t kmin, const uint32_t* __restrict__ bits,
                                                           uint64_t bmask, bool negate,
                                                           unsigned long long* __restrict__ words,
                                                           int64_t* __restrict__ tile_counts) {
  __shared__ int64_t red[kWavesPerBlock];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    int64_t cnt = 0;
#pragma unroll 4
    for (int it = 0; it < kHitTile / kBlock; ++it) {
      const int64_t row = t * kHitTile + (int64_t)it * kBlock + threadIdx.x;
      bool hit = false;
      if (row < m) {
        const int32_t h = probe_head<K, DIRECT>(keys, valid, row, tkeys, thead, cap, kmin, bits, bmask);
        hit = (h >= 0) != negate;
      }
      const unsigned long long b = __ballot(hit);
      if (lane == 0 && t * kHitTile + (int64_t)it * kBlock + wave * kWave < m)
        words[t * kHitWords + it * kWavesPerBlock + wave] = b;
      cnt += __popcll(b);
    }
    if (lane == 0) red[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t s = 0;
      for (int w = 0; w < kWavesPerBlock; ++w) s += red[w];
      tile_counts[t] = s;
    }
    __syncthreads();
  }
}

template <typename K, bool DIRECT, typename O>
__global__ __launch_bounds__(kBlock) void probe_write_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                            int64_t m, const int64_t* __restrict__ tkeys,
                                                            const int32_t* __restrict__ thead, int64_t cap,
                                                            int64_t kmin, const unsigned long long* __restrict__ words,
                                                            const int64_t* __restrict__ tile_off,
                                                            O* __restrict__ out_probe, int32_t* __restrict__ out_build) {
  __shared__ int64_t woff[kHitWords];
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t nrows = m - t * kHitTile < kHitTile ? m - t * kHitTile : kHitTile;
    const int nwords = (int)((nrows + kWave - 1) / kWave);
    const unsigned long long w0 = threadIdx.x < nwords ? words[t * kHitWords + threadIdx.x] : 0ULL;
    int64_t total;
    const int64_t ex = block_exclusive_scan((int64_t)__popcll(w0), scratch, &total);
    if (threadIdx.x < kHitWords) woff[threadIdx.x] = ex;
    __syncthreads();
    if (total) {
      const int64_t base = tile_off[t];
      for (int w = wave; w < nwords; w += kWavesPerBlock) {
        const unsigned long long b = words[t * kHitWords + w];
        if (!((b >> lane) & 1ULL)) continue;
        const int64_t row = t * kHitTile + (int64_t)w * kWave + lane;
        const int64_t pos = base + woff[w] + __popcll(b & ((1ULL << lane) - 1ULL));
        out_probe[pos] = (O)row;
        if (out_build) out_build[pos] = probe_head<K, DIRECT>(keys, valid, row, tkeys, thead, cap, kmin, nullptr, 0);
      }
    }
    __syncthreads();
  }
}
}  // namespace

int64_t probe_hit_tiles(int64_t m) { return (m + kHitTile - 1) / kHitTile; }

void probe_hits(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const int32_t* thead, int64_t cap, int64_t kmin, bool direct, const uint32_t* bits, uint64_t bmask,
                bool negate, unsigned long long* words, int64_t* tile_counts, hipStream_t stream) {
  if (m == 0) return;
  const dim3 g(grid_for(probe_hit_tiles(m), 1, 1 << 16)), b(kBlock);
#define IG_PH(KT, D)                                                                                              \
  hipLaunchKernelGGL((probe_hits_kernel<KT, D>), g, b, 0, stream, (const KT*)keys, valid, m, tkeys, thead, cap, kmin, \
                     bits, bmask, negate, words, tile_counts)
  if (key64) {
    if (direct) IG_PH(int64_t, true);
    else IG_PH(int64_t, false);
  } else {
    if (direct) IG_PH(int32_t, true);
    else IG_PH(int32_t, false);
  }
#undef IG_PH
  check_launch("probe_hits", stream);
}

void probe_write(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const int32_t* thead, int64_t cap, int64_t kmin, bool direct, const unsigned long long* words,
                 const int64_t* tile_off, void* out_probe, bool out64, int32_t* out_build, hipStream_t stream) {
  if (m == 0) return;
  const dim3 g(grid_for(probe_hit_tiles(m), 1, 1 << 16)), b(kBlock);
#define IG_PW(KT, D, OT)                                                                                           \
  hipLaunchKernelGGL((probe_write_kernel<KT, D, OT>), g, b, 0, stream, (const KT*)keys, valid, m, tkeys, thead, cap, \
                     kmin, words, tile_off, (OT*)out_probe, out_build)
#define IG_PW2(KT, D) \
  if (out64) IG_PW(KT, D, int64_t); else IG_PW(KT, D, int32_t)
  if (key64) {
    if (direct) { IG_PW2(int64_t, true); }
    else { IG_PW2(int64_t, false); }
  } else {
    if (direct) { IG_PW2(int32_t, true); }
    else { IG_PW2(int32_t, false); }
  }
#undef IG_PW2
#undef IG_PW
  check_launch("probe_write", stream);
}
}  // namespace kern
}  // namespace igloo
