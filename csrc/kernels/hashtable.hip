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
// Every slot's head row (thead, one atomicExch per build row) serves unique
// (PK) builds. A build with duplicate keys adds a CSR layout: per-slot counts,
// an exclusive scan into cstart[cap+1] and a scatter of the row ids into
// crows[n], so a multi-match probe reads one contiguous run instead of
// pointer-chasing a next[] chain through HBM. Row ids (thead, crows, cstart,
// probe outputs) are int32 below 2^31 build rows and int64 above (R).
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
// A slot's key is read before it is claimed: a key already in the table (every
// row of a low-cardinality GROUP BY -- Q22's 7 country codes over 4M rows,
// which serialised on 7 words as one CAS per row) costs one load, and only an
// empty slot takes the CAS. Keys are never removed or changed once set, so a
// stale read can only show EMPTY, which the CAS then settles -- the read may
// therefore be a plain (L1-cached) load: hot slots are served per CU instead
// of queueing on one L2 line.
__device__ inline int64_t insert_slot(int64_t* __restrict__ tkeys, int64_t mask, int64_t k, bool* existed) {
  int64_t slot = (int64_t)(mix64((uint64_t)k) & (uint64_t)mask);
  for (;;) {
    const int64_t cur = tkeys[slot];
    if (cur == k) { *existed = true; return slot; }
    if (cur == kEmptyKey) {
      unsigned long long prev = atomicCAS((unsigned long long*)&tkeys[slot], (unsigned long long)kEmptyKey,
                                          (unsigned long long)k);
      if ((int64_t)prev == kEmptyKey) { *existed = false; return slot; }
      if ((int64_t)prev == k) { *existed = true; return slot; }
    }
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

__device__ inline int32_t atomic_add(int32_t* p, int32_t v) { return atomicAdd(p, v); }
__device__ inline int64_t atomic_add(int64_t* p, int64_t v) {
  return (int64_t)atomicAdd(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
}
__device__ inline int32_t atomic_exch(int32_t* p, int32_t v) { return atomicExch(p, v); }
__device__ inline int64_t atomic_exch(int64_t* p, int64_t v) {
  return (int64_t)atomicExch(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v);
}

template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void join_build_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t n, int64_t* __restrict__ tkeys,
                                                           R* __restrict__ thead, int64_t cap, int64_t kmin,
                                                           unsigned long long* dups, uint32_t* __restrict__ bits,
                                                           uint64_t bmask) {
  const int64_t mask = cap - 1;
  unsigned long long local_dups = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t k;
    if (!load_key(keys, valid, i, &k)) continue;
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
    const R old = atomic_exch(&thead[slot], (R)i);
    local_dups += old != (R)-1;
    if (bits) {
      const uint64_t bb = bloom_bit(k, bmask, kmin);
      atomicOr(&bits[bb >> 5], 1u << (bb & 31));
    }
  }
  // one atomic per wave for the duplicate counter
  for (int off = kWave / 2; off > 0; off >>= 1) local_dups += __shfl_xor(local_dups, off, kWave);
  if (lane_id() == 0 && local_dups) atomicAdd(dups, local_dups);
}

// slot of build row i (its key is in the table), -1 for a NULL key
template <typename K, bool DIRECT>
__device__ inline int64_t build_slot(const K* keys, const uint8_t* valid, int64_t i, const int64_t* tkeys,
                                     int64_t cap, int64_t kmin) {
  int64_t k;
  if (!load_key(keys, valid, i, &k)) return -1;
  if (DIRECT) {
    const int64_t s = k - kmin;
    return (uint64_t)s < (uint64_t)cap ? s : -1;
  }
  return find_slot(tkeys, cap - 1, k);
}

// CSR pass 1: rows per slot (cnt zeroed by the caller)
template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void join_csr_count_kernel(const K* __restrict__ keys,
                                                               const uint8_t* __restrict__ valid, int64_t n,
                                                               const int64_t* __restrict__ tkeys, R* __restrict__ cnt,
                                                               int64_t cap, int64_t kmin) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = build_slot<K, DIRECT>(keys, valid, i, tkeys, cap, kmin);
    if (s >= 0) atomic_add(&cnt[s], (R)1);
  }
}

// CSR pass 2 (cstart = exclusive scan of cnt): every row claims a position of
// its slot's run by counting cnt back down
template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void join_csr_scatter_kernel(const K* __restrict__ keys,
                                                                 const uint8_t* __restrict__ valid, int64_t n,
                                                                 const int64_t* __restrict__ tkeys,
                                                                 R* __restrict__ cnt, const R* __restrict__ cstart,
                                                                 R* __restrict__ crows, int64_t cap, int64_t kmin) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = build_slot<K, DIRECT>(keys, valid, i, tkeys, cap, kmin);
    if (s < 0) continue;
    const R pos = atomic_add(&cnt[s], (R)-1) - 1;
    crows[(int64_t)cstart[s] + pos] = (R)i;
  }
}

// slot holding probe row j's key, -1 when the key is NULL, outside the span,
// filtered out by the bitmap or (hashed) absent; a direct slot may be empty
template <typename K, bool DIRECT>
__device__ inline int64_t probe_slot(const K* keys, const uint8_t* valid, int64_t j, const int64_t* tkeys,
                                     int64_t cap, int64_t kmin, const uint32_t* bits, uint64_t bmask) {
  int64_t k;
  if (!load_key(keys, valid, j, &k)) return -1;
  if (DIRECT && (k - kmin < 0 || k - kmin >= cap)) return -1;
  if (bits) {
    const uint64_t b = bloom_bit(k, bmask, kmin);
    if (!((bits[b >> 5] >> (b & 31)) & 1u)) return -1;
  }
  if (DIRECT) return k - kmin;
  return find_slot(tkeys, cap - 1, k);
}

// counts[j] = number of build matches of probe row j; first[j] = one match or
// -1; build_matched[r] = 1 for every matched build row. cstart/crows: the CSR
// runs of a duplicate-key build (null: unique build, thead only).
template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void join_probe_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t m, const int64_t* __restrict__ tkeys,
                                                           const R* __restrict__ thead, const R* __restrict__ cstart,
                                                           const R* __restrict__ crows, int64_t cap, int64_t kmin,
                                                           int32_t* __restrict__ counts, R* __restrict__ first,
                                                           uint8_t* __restrict__ build_matched,
                                                           const uint32_t* __restrict__ bits, uint64_t bmask) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = probe_slot<K, DIRECT>(keys, valid, j, tkeys, cap, kmin, bits, bmask);
    R h = (R)-1;
    int64_t a = 0, e = 0;
    if (s >= 0) {
      if (cstart) {
        a = cstart[s];
        e = cstart[s + 1];
        if (a < e) h = crows[a];
      } else {
        h = thead[s];
        e = h >= 0;
      }
    }
    if (first) first[j] = h;
    if (counts) counts[j] = (int32_t)(e - a);
    if (build_matched) {
      if (cstart) {
        for (int64_t r = a; r < e; ++r) build_matched[crows[r]] = 1;
      } else if (h >= 0) {
        build_matched[h] = 1;
      }
    }
  }
}

// first-match probe, direct-mapped table, 4 rows per lane: all key loads,
// then all filter-bit loads, then all head loads are issued before their
// results are needed, so a lane keeps 4 misses in flight instead of one
// dependent chain (600M-row lineitem probes were latency-bound).
constexpr int kProbeRows = 4;

template <typename K, typename R>
__global__ __launch_bounds__(kBlock) void join_probe_first_direct_kernel(
    const K* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t m, const R* __restrict__ thead,
    int64_t cap, int64_t kmin, R* __restrict__ first, const uint32_t* __restrict__ bits, uint64_t bmask) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j0 < m; j0 += stride * kProbeRows) {
    // unconditional (clamped) loads, results selected afterwards: a load under
    // a per-lane condition becomes a branch whose merge waits for it
    int64_t s[kProbeRows];
    bool ok[kProbeRows];
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) {
      const int64_t j = j0 + r * stride;
      const int64_t jc = j < m ? j : m - 1;
      const bool v = !valid || valid[jc];
      s[r] = (int64_t)keys[jc] - kmin;
      ok[r] = j < m && v && s[r] >= 0 && s[r] < cap;
    }
    if (bits) {
      uint32_t w[kProbeRows];
#pragma unroll
      for (int r = 0; r < kProbeRows; ++r) {
        const uint64_t b = ok[r] || !(bmask & kExactBits) ? bloom_bit(s[r] + kmin, bmask, kmin) : 0;
        w[r] = bits[b >> 5] >> (b & 31);
      }
#pragma unroll
      for (int r = 0; r < kProbeRows; ++r) ok[r] = ok[r] && (w[r] & 1u);
    }
    R h[kProbeRows];
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) h[r] = thead[ok[r] ? s[r] : 0];
#pragma unroll
    for (int r = 0; r < kProbeRows; ++r) {
      const int64_t j = j0 + r * stride;
      if (j < m) first[j] = ok[r] ? h[r] : (R)-1;
    }
  }
}

// every (probe row, build row) match at offsets[j] (exclusive scan of counts)
template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void join_expand_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                            int64_t m, const int64_t* __restrict__ tkeys,
                                                            const R* __restrict__ thead, const R* __restrict__ cstart,
                                                            const R* __restrict__ crows, int64_t cap, int64_t kmin,
                                                            const int64_t* __restrict__ offsets,
                                                            int32_t* __restrict__ out_probe, R* __restrict__ out_build,
                                                            const uint32_t* __restrict__ bits, uint64_t bmask,
                                                            int64_t out_cap) {
  // out_cap: pairs the outputs hold (sized by a possibly replayed total):
  // writes past it are dropped; the end-of-query check rejects the run
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < m; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = probe_slot<K, DIRECT>(keys, valid, j, tkeys, cap, kmin, bits, bmask);
    if (s < 0) continue;
    int64_t o = offsets[j];
    if (cstart) {
      const int64_t e = cstart[s + 1];
      for (int64_t r = cstart[s]; r < e && o < out_cap; ++r, ++o) {
        out_probe[o] = (int32_t)j;
        out_build[o] = crows[r];
      }
    } else {
      const R h = thead[s];
      if (h >= 0 && o < out_cap) {
        out_probe[o] = (int32_t)j;
        out_build[o] = h;
      }
    }
  }
}

// First-row table of a GROUP BY. Hashed keys (!DIRECT) go through a small
// per-workgroup LDS cache of (slot -> smallest row): rows of a hot group take
// an LDS atomic, and each workgroup sends one global atomicMin per cached slot
// at the end. Without it a low-cardinality GROUP BY (Q22's 7 country codes
// over 636K rows) had every wave's atomics -- and reads -- queue on the same
// few L2 lines: 262 us for 636K rows. Slots the cache cannot hold (a
// high-cardinality GROUP BY) take the global path directly.
constexpr int kRowCache = 256;

template <typename K, bool DIRECT>
__global__ __launch_bounds__(kBlock) void groupby_build_kernel(const K* __restrict__ keys, int64_t n,
                                                              int64_t* __restrict__ tkeys, int32_t* __restrict__ trow,
                                                              int64_t cap, int64_t kmin) {
  __shared__ int32_t cslot[DIRECT ? 1 : kRowCache];
  __shared__ int32_t crow[DIRECT ? 1 : kRowCache];
  if (!DIRECT) {
    for (int h = threadIdx.x; h < kRowCache; h += blockDim.x) {
      cslot[h] = -1;
      crow[h] = INT32_MAX;
    }
    __syncthreads();
  }
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
      const int h = (int)(slot & (kRowCache - 1));
      int cur = cap <= ((int64_t)1 << 31) ? cslot[h] : -2;    // (slots must fit the int32 cache)
      if (cur == -1) {
        cur = atomicCAS(&cslot[h], -1, (int32_t)slot);
        if (cur == -1) cur = (int32_t)slot;
      }
      if (cur == (int32_t)slot) {
        atomicMin(&crow[h], (int32_t)i);
        continue;
      }
    }
    // first occurrence row: plain read first avoids most atomics on hot groups
    if (trow[slot] > (int32_t)i) atomicMin(&trow[slot], (int32_t)i);
  }
  if (!DIRECT) {
    __syncthreads();
    for (int h = threadIdx.x; h < kRowCache; h += blockDim.x)
      if (cslot[h] >= 0 && trow[cslot[h]] > crow[h]) atomicMin(&trow[cslot[h]], crow[h]);
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
__global__ __launch_bounds__(kBlock) void assign_gid_kernel(const S* __restrict__ slots, int64_t g, int64_t cap,
                                                           const int32_t* __restrict__ trow,
                                                           int32_t* __restrict__ gid_of_slot,
                                                           int32_t* __restrict__ rep_row) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < g; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t s = (int64_t)slots[i];
    if ((uint64_t)s >= (uint64_t)cap) {   // a replayed group count past the real one: unwritten slot ids
      rep_row[i] = 0;
      continue;
    }
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


template <typename I>
__global__ __launch_bounds__(kBlock) void fill_runs_kernel(const I* __restrict__ starts, int64_t nruns, int64_t n,
                                                          int32_t* __restrict__ gid) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nruns; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t b = starts[r], e = r + 1 < nruns ? (int64_t)starts[r + 1] : n;
    // a replayed run count can leave the starts' tail unwritten: stay in [0, n)
    b = b < 0 ? 0 : (b > n ? n : b);
    e = e < b ? b : (e > n ? n : e);
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

// launch KERNEL<K, DIRECT, R> with keys cast to the key type
#define DISPATCH_KEY3(key64, direct, R, KERNEL, g, b, shm, st, keys, ...)                                  \
  do {                                                                                                    \
    if (key64) {                                                                                          \
      if (direct) hipLaunchKernelGGL((KERNEL<int64_t, true, R>), g, b, shm, st, (const int64_t*)(keys), __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<int64_t, false, R>), g, b, shm, st, (const int64_t*)(keys), __VA_ARGS__);       \
    } else {                                                                                              \
      if (direct) hipLaunchKernelGGL((KERNEL<int32_t, true, R>), g, b, shm, st, (const int32_t*)(keys), __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<int32_t, false, R>), g, b, shm, st, (const int32_t*)(keys), __VA_ARGS__);       \
    }                                                                                                     \
  } while (0)

void join_build(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t* tkeys, void* thead, bool rid64,
                int64_t cap, int64_t kmin, bool direct, unsigned long long* dups, uint32_t* bits, uint64_t bmask,
                hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (rid64)
    DISPATCH_KEY3(key64, direct, int64_t, join_build_kernel, g, b, 0, stream, keys, valid, n, tkeys, (int64_t*)thead,
                  cap, kmin, dups, bits, bmask);
  else
    DISPATCH_KEY3(key64, direct, int32_t, join_build_kernel, g, b, 0, stream, keys, valid, n, tkeys, (int32_t*)thead,
                  cap, kmin, dups, bits, bmask);
  check_launch("join_build", stream);
}

void join_csr_count(const void* keys, bool key64, const uint8_t* valid, int64_t n, const int64_t* tkeys, void* cnt,
                    bool rid64, int64_t cap, int64_t kmin, bool direct, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (rid64)
    DISPATCH_KEY3(key64, direct, int64_t, join_csr_count_kernel, g, b, 0, stream, keys, valid, n, tkeys, (int64_t*)cnt,
                  cap, kmin);
  else
    DISPATCH_KEY3(key64, direct, int32_t, join_csr_count_kernel, g, b, 0, stream, keys, valid, n, tkeys, (int32_t*)cnt,
                  cap, kmin);
  check_launch("join_csr_count", stream);
}

void join_csr_scatter(const void* keys, bool key64, const uint8_t* valid, int64_t n, const int64_t* tkeys, void* cnt,
                      const void* cstart, void* crows, bool rid64, int64_t cap, int64_t kmin, bool direct,
                      hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, kMaxGrid)), b(kBlock);
  if (rid64)
    DISPATCH_KEY3(key64, direct, int64_t, join_csr_scatter_kernel, g, b, 0, stream, keys, valid, n, tkeys,
                  (int64_t*)cnt, (const int64_t*)cstart, (int64_t*)crows, cap, kmin);
  else
    DISPATCH_KEY3(key64, direct, int32_t, join_csr_scatter_kernel, g, b, 0, stream, keys, valid, n, tkeys,
                  (int32_t*)cnt, (const int32_t*)cstart, (int32_t*)crows, cap, kmin);
  check_launch("join_csr_scatter", stream);
}

template <typename R>
static void join_probe_t(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                         const R* thead, const R* cstart, const R* crows, int64_t cap, int64_t kmin, bool direct,
                         int32_t* counts, R* first, uint8_t* build_matched, const uint32_t* bits, uint64_t bmask,
                         hipStream_t stream) {
  const dim3 b(kBlock);
  if (direct && first && !counts && !build_matched && !cstart) {
    const dim3 g4(grid_for((m + kProbeRows - 1) / kProbeRows, kBlock, kMaxGrid));
    if (key64)
      hipLaunchKernelGGL((join_probe_first_direct_kernel<int64_t, R>), g4, b, 0, stream, (const int64_t*)keys, valid,
                         m, thead, cap, kmin, first, bits, bmask);
    else
      hipLaunchKernelGGL((join_probe_first_direct_kernel<int32_t, R>), g4, b, 0, stream, (const int32_t*)keys, valid,
                         m, thead, cap, kmin, first, bits, bmask);
    check_launch("join_probe_first_direct", stream);
    return;
  }
  const dim3 g(grid_for(m, kBlock, kMaxGrid));
  DISPATCH_KEY3(key64, direct, R, join_probe_kernel, g, b, 0, stream, keys, valid, m, tkeys, thead, cstart, crows, cap,
                kmin, counts, first, build_matched, bits, bmask);
  check_launch("join_probe", stream);
}

void join_probe(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const void* thead, const void* cstart, const void* crows, bool rid64, int64_t cap, int64_t kmin,
                bool direct, int32_t* counts, void* first, uint8_t* build_matched, const uint32_t* bits,
                uint64_t bmask, hipStream_t stream) {
  if (m == 0) return;
  if (rid64)
    join_probe_t<int64_t>(keys, key64, valid, m, tkeys, (const int64_t*)thead, (const int64_t*)cstart,
                          (const int64_t*)crows, cap, kmin, direct, counts, (int64_t*)first, build_matched, bits,
                          bmask, stream);
  else
    join_probe_t<int32_t>(keys, key64, valid, m, tkeys, (const int32_t*)thead, (const int32_t*)cstart,
                          (const int32_t*)crows, cap, kmin, direct, counts, (int32_t*)first, build_matched, bits,
                          bmask, stream);
}

void join_expand(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const void* thead, const void* cstart, const void* crows, bool rid64, int64_t cap, int64_t kmin,
                 bool direct, const int64_t* offsets, int32_t* out_probe, void* out_build, const uint32_t* bits,
                 uint64_t bmask, int64_t out_cap, hipStream_t stream) {
  if (m == 0) return;
  dim3 g(grid_for(m, kBlock, kMaxGrid)), b(kBlock);
  if (rid64)
    DISPATCH_KEY3(key64, direct, int64_t, join_expand_kernel, g, b, 0, stream, keys, valid, m, tkeys,
                  (const int64_t*)thead, (const int64_t*)cstart, (const int64_t*)crows, cap, kmin, offsets, out_probe,
                  (int64_t*)out_build, bits, bmask, out_cap);
  else
    DISPATCH_KEY3(key64, direct, int32_t, join_expand_kernel, g, b, 0, stream, keys, valid, m, tkeys,
                  (const int32_t*)thead, (const int32_t*)cstart, (const int32_t*)crows, cap, kmin, offsets, out_probe,
                  (int32_t*)out_build, bits, bmask, out_cap);
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
  // (hashed: several rows per lane, so each workgroup's row cache covers many rows)
  dim3 g(grid_for(n, direct ? kBlock : kBlock * 8, kMaxGrid)), b(kBlock);
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

void groupby_assign(const void* slots, bool slots64, int64_t g, int64_t cap, const int32_t* trow,
                    int32_t* gid_of_slot, int32_t* rep_row, hipStream_t stream) {
  if (g == 0) return;
  dim3 gr(grid_for(g, kBlock, kMaxGrid)), b(kBlock);
  if (slots64)
    hipLaunchKernelGGL(assign_gid_kernel<int64_t>, gr, b, 0, stream, (const int64_t*)slots, g, cap, trow, gid_of_slot,
                       rep_row);
  else
    hipLaunchKernelGGL(assign_gid_kernel<int32_t>, gr, b, 0, stream, (const int32_t*)slots, g, cap, trow, gid_of_slot,
                       rep_row);
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

// Batched head lookup of kHitBatch probe rows per lane: every key load, then
// every filter-bit load, then every table load is issued before any result is
// used, so a lane keeps kHitBatch misses in flight (a row-at-a-time dependent
// chain left the 600M-row lineitem probes at ~10% of HBM bandwidth,
// profiles/r3_sf100_pmc_roofline.txt). With an exact membership bitmap the bit
// IS the answer and the table is not read at all (need_head false).
constexpr int kHitBatch = 8;
// probe_write: tiles with at most this many hits list them in LDS and give
// every lane whole hits (denser tiles walk their hit words)
constexpr int kSparseHits = 2048;
//
// All loads are unconditional (indices clamped into range, results selected
// afterwards): a load under a per-lane condition compiles to a branch whose
// merge waits for it, which would serialise the batch again.
template <typename K, bool DIRECT, typename R>
__device__ inline void probe_heads(const K* __restrict__ keys, const uint8_t* __restrict__ valid, int64_t m,
                                   const int64_t (&row)[kHitBatch], const int64_t* __restrict__ tkeys,
                                   const R* __restrict__ thead, int64_t cap, int64_t kmin,
                                   const uint32_t* __restrict__ bits, uint64_t bmask, bool need_head,
                                   int64_t (&h)[kHitBatch]) {
  int64_t k[kHitBatch], rc[kHitBatch];
  bool ok[kHitBatch];
#pragma unroll
  for (int r = 0; r < kHitBatch; ++r) {
    rc[r] = row[r] < m ? row[r] : m - 1;
    k[r] = (int64_t)keys[rc[r]];
  }
  uint8_t vb[kHitBatch];
#pragma unroll
  for (int r = 0; r < kHitBatch; ++r) vb[r] = 1;
  if (valid) {
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) vb[r] = valid[rc[r]];
  }
#pragma unroll
  for (int r = 0; r < kHitBatch; ++r) {
    ok[r] = row[r] < m && vb[r];
    if (DIRECT) ok[r] = ok[r] && k[r] - kmin >= 0 && k[r] - kmin < cap;
  }
  if (bits) {
    uint32_t w[kHitBatch];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) {
      // exact bitmaps index by k - kmin: out-of-span keys (ok false) read bit 0
      const uint64_t b = ok[r] || !(bmask & kExactBits) ? bloom_bit(k[r], bmask, kmin) : 0;
      w[r] = bits[b >> 5] >> (b & 31);
    }
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) ok[r] = ok[r] && (w[r] & 1u);
  }
  if (!need_head) {
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) h[r] = ok[r] ? 0 : -1;
    return;
  }
  if (DIRECT) {
    R x[kHitBatch];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) x[r] = thead[ok[r] ? k[r] - kmin : 0];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) h[r] = ok[r] ? x[r] : -1;
  } else {
    // first slot of every row in flight together; collisions walk on serially
    const int64_t mask = cap - 1;
    int64_t slot[kHitBatch], tk[kHitBatch];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) {
      slot[r] = (int64_t)(mix64((uint64_t)k[r]) & (uint64_t)mask);
      tk[r] = tkeys[slot[r]];
    }
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) {
      while (ok[r] && tk[r] != k[r] && tk[r] != kEmptyKey) {
        slot[r] = (slot[r] + 1) & mask;
        tk[r] = tkeys[slot[r]];
      }
      ok[r] = ok[r] && tk[r] == k[r];
    }
    R x[kHitBatch];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) x[r] = thead[ok[r] ? slot[r] : 0];
#pragma unroll
    for (int r = 0; r < kHitBatch; ++r) h[r] = ok[r] ? x[r] : -1;
  }
}

template <typename K, bool DIRECT, typename R>
__global__ __launch_bounds__(kBlock) void probe_hits_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                           int64_t m, const int64_t* __restrict__ tkeys,
                                                           const R* __restrict__ thead, int64_t cap,
                                                           int64_t kmin, const uint32_t* __restrict__ bits,
                                                           uint64_t bmask, bool negate,
                                                           unsigned long long* __restrict__ words,
                                                           int64_t* __restrict__ tile_counts) {
  __shared__ int64_t red[kWavesPerBlock];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  // a direct table with an exact bitmap: bit set <=> key present
  const bool need_head = !(DIRECT && bits && (bmask & kExactBits));
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    int64_t cnt = 0;
    for (int it0 = 0; it0 < kHitTile / kBlock; it0 += kHitBatch) {
      int64_t row[kHitBatch];
      int64_t h[kHitBatch];
#pragma unroll
      for (int r = 0; r < kHitBatch; ++r) row[r] = t * kHitTile + (int64_t)(it0 + r) * kBlock + threadIdx.x;
      probe_heads<K, DIRECT, R>(keys, valid, m, row, tkeys, thead, cap, kmin, bits, bmask, need_head, h);
#pragma unroll
      for (int r = 0; r < kHitBatch; ++r) {
        const bool hit = row[r] < m && ((h[r] >= 0) != negate);
        const unsigned long long b = __ballot(hit);
        if (lane == 0 && t * kHitTile + (int64_t)(it0 + r) * kBlock + wave * kWave < m)
          words[t * kHitWords + (it0 + r) * kWavesPerBlock + wave] = b;
        cnt += __popcll(b);
      }
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

template <typename K, bool DIRECT, typename R, typename O>
__global__ __launch_bounds__(kBlock) void probe_write_kernel(const K* __restrict__ keys, const uint8_t* __restrict__ valid,
                                                            int64_t m, const int64_t* __restrict__ tkeys,
                                                            const R* __restrict__ thead, int64_t cap,
                                                            int64_t kmin, const unsigned long long* __restrict__ words,
                                                            const int64_t* __restrict__ tile_off,
                                                            O* __restrict__ out_probe, R* __restrict__ out_build,
                                                            int64_t out_cap) {
  __shared__ int64_t woff[kHitWords];
  __shared__ int64_t scratch[kWavesPerBlock + 1];
  __shared__ uint16_t hits[kSparseHits];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    // a tile without hits (its offset equals the next one's): nothing to
    // load, scan or write (selective probes: most tiles)
    if ((t + 1 < tiles ? tile_off[t + 1] : out_cap) <= tile_off[t]) continue;
    const int64_t nrows = m - t * kHitTile < kHitTile ? m - t * kHitTile : kHitTile;
    const int nwords = (int)((nrows + kWave - 1) / kWave);
    const unsigned long long w0 = threadIdx.x < nwords ? words[t * kHitWords + threadIdx.x] : 0ULL;
    int64_t total;
    const int64_t ex = block_exclusive_scan((int64_t)__popcll(w0), scratch, &total);
    if (threadIdx.x < kHitWords) woff[threadIdx.x] = ex;
    __syncthreads();
    if (total && total <= kSparseHits) {
      // a sparse tile: its hit rows listed in LDS first (in row order: the
      // list index IS the output offset inside the tile), then every lane
      // takes whole hits -- the work follows the hits, not the 8192 rows
      const int64_t base = tile_off[t];
      if (threadIdx.x < nwords) {
        unsigned long long w = w0;
        int o = (int)ex;
        while (w) {
          const int b = __ffsll((long long)w) - 1;
          hits[o++] = (uint16_t)(threadIdx.x * kWave + b);
          w &= w - 1ULL;
        }
      }
      __syncthreads();
      for (int64_t i0 = 0; i0 < total; i0 += (int64_t)kBlock * kHitBatch) {
        int64_t row[kHitBatch];
#pragma unroll
        for (int r = 0; r < kHitBatch; ++r) {
          const int64_t i = i0 + (int64_t)r * kBlock + threadIdx.x;
          row[r] = i < total ? t * kHitTile + hits[i] : m;
        }
        int64_t h[kHitBatch];
        if (out_build) probe_heads<K, DIRECT, R>(keys, valid, m, row, tkeys, thead, cap, kmin, nullptr, 0, true, h);
#pragma unroll
        for (int r = 0; r < kHitBatch; ++r) {
          if (row[r] >= m) continue;
          const int64_t pos = base + i0 + (int64_t)r * kBlock + threadIdx.x;
          if (pos >= out_cap) continue;   // a replayed (undersized) total: see join_expand_kernel
          out_probe[pos] = (O)row[r];
          if (out_build) out_build[pos] = (R)h[r];
        }
      }
    } else if (total) {
      const int64_t base = tile_off[t];
      // kHitBatch hit words per wave at a time (waves own words wave, wave+4, ...)
      for (int w0 = wave; w0 < nwords; w0 += kWavesPerBlock * kHitBatch) {
        unsigned long long b[kHitBatch];
        int64_t row[kHitBatch];
#pragma unroll
        for (int r = 0; r < kHitBatch; ++r) {
          const int w = w0 + r * kWavesPerBlock;
          b[r] = w < nwords ? words[t * kHitWords + w] : 0ULL;
          // rows that are not hits are pushed past m: probe_heads skips them
          row[r] = ((b[r] >> lane) & 1ULL) ? t * kHitTile + (int64_t)w * kWave + lane : m;
        }
        int64_t h[kHitBatch];
        if (out_build) probe_heads<K, DIRECT, R>(keys, valid, m, row, tkeys, thead, cap, kmin, nullptr, 0, true, h);
#pragma unroll
        for (int r = 0; r < kHitBatch; ++r) {
          if (row[r] >= m) continue;
          const int w = w0 + r * kWavesPerBlock;
          const int64_t pos = base + woff[w] + __popcll(b[r] & ((1ULL << lane) - 1ULL));
          if (pos >= out_cap) continue;   // a replayed (undersized) total: see join_expand_kernel
          out_probe[pos] = (O)row[r];
          if (out_build) out_build[pos] = (R)h[r];
        }
      }
    }
    __syncthreads();
  }
}
}  // namespace

namespace {

// probe_hits for int32 keys against a direct table with an exact membership
// bitmap (no head read at all: the bit decides): every lane takes 4
// consecutive rows per step -- one 16-byte key load and one 4-byte validity
// load instead of 4 + 4 scalar loads -- and the 64-bit hit words are put
// together from each 16-lane group's nibbles. Same tiles, words and counts
// as probe_hits_kernel (probe_write reads them unchanged).
constexpr int kBitsRows = 4;
constexpr int kBitsSteps = kHitTile / (kBlock * kBitsRows);   // 8

// 4 consecutive keys (16-byte aligned) in one or two 16-byte loads
__device__ inline void load4(const int32_t* p, int32_t (&k)[4]) {
  const int4 v = *reinterpret_cast<const int4*>(p);
  k[0] = v.x;
  k[1] = v.y;
  k[2] = v.z;
  k[3] = v.w;
}
__device__ inline void load4(const int64_t* p, int64_t (&k)[4]) {
  const longlong2 a = *reinterpret_cast<const longlong2*>(p);
  const longlong2 b = *reinterpret_cast<const longlong2*>(p + 2);
  k[0] = a.x;
  k[1] = a.y;
  k[2] = b.x;
  k[3] = b.y;
}

template <typename K>
__global__ __launch_bounds__(kBlock) void probe_bits_kernel(const K* __restrict__ keys,
                                                           const uint8_t* __restrict__ valid, int64_t m,
                                                           int64_t cap, int64_t kmin,
                                                           const uint32_t* __restrict__ bits, bool negate,
                                                           unsigned long long* __restrict__ words,
                                                           int64_t* __restrict__ tile_counts) {
  __shared__ int64_t red[kWavesPerBlock];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    int64_t cnt = 0;
#pragma unroll 2
    for (int g = 0; g < kBitsSteps; ++g) {
      const int64_t r0 = t * kHitTile + (int64_t)g * (kBlock * kBitsRows) + (int64_t)threadIdx.x * kBitsRows;
      K k[kBitsRows];
      uint32_t vb = 0x01010101u;
      if (r0 + kBitsRows <= m) {
        load4(keys + r0, k);
        if (valid) vb = *reinterpret_cast<const uint32_t*>(valid + r0);
      } else {
        vb = 0;
#pragma unroll
        for (int j = 0; j < kBitsRows; ++j) {
          const bool in = r0 + j < m;
          k[j] = in ? keys[r0 + j] : K(0);
          if (in && (!valid || valid[r0 + j])) vb |= 1u << (8 * j);
        }
      }
      uint32_t nib = 0;
#pragma unroll
      for (int j = 0; j < kBitsRows; ++j) {
        const int64_t d = (int64_t)k[j] - kmin;
        bool ok = ((vb >> (8 * j)) & 0xffu) != 0 && d >= 0 && d < cap;
        if (ok) ok = (bits[(uint64_t)d >> 5] >> (d & 31)) & 1u;
        const bool hit = r0 + j < m && (ok != negate);
        nib |= (hit ? 1u : 0u) << j;
      }
      cnt += __popc(nib);
      // rows 4*lane .. 4*lane+3 of this wave's 256 are bits 4*(lane%16) .. +3
      // of word lane/16: OR the 16 nibbles of each lane group together
      unsigned long long w = (unsigned long long)nib << (4 * (lane & 15));
      w |= __shfl_xor(w, 1, kWave);
      w |= __shfl_xor(w, 2, kWave);
      w |= __shfl_xor(w, 4, kWave);
      w |= __shfl_xor(w, 8, kWave);
      const int64_t wrow = t * kHitTile + (int64_t)g * (kBlock * kBitsRows) + (int64_t)wave * (kWave * kBitsRows) +
                           (int64_t)(lane >> 4) * kWave;
      if ((lane & 15) == 0 && wrow < m)
        words[t * kHitWords + g * (kHitWords / kBitsSteps) + wave * kBitsRows + (lane >> 4)] = w;
    }
    cnt = wave_reduce_sum(cnt);
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

// The same probe for large probe sides: the membership bitmap, folded
// modulo 64 KiB (word i = OR of the bitmap's words i, i + 16K, ...), sits in
// LDS, read by every workgroup once; a probe key whose folded bit is clear
// is out without touching L2 (each global bitmap read moves a whole cache
// line for 4 useful bytes), and only folded hits consult the exact bitmap
// (none when the bitmap fits the fold: then the fold is exact). Workgroups of
// 1024 lanes, two per CU, loop over the tiles.
constexpr int kFoldWords = 16384;
constexpr int kFoldBlock = 1024;
constexpr int kFoldWaves = kFoldBlock / kWave;
constexpr int kFoldSteps = kHitTile / (kFoldBlock * kBitsRows);   // 2

template <typename K>
__global__ __launch_bounds__(kFoldBlock) void probe_fold_kernel(const K* __restrict__ keys,
                                                               const uint8_t* __restrict__ valid, int64_t m,
                                                               int64_t cap, int64_t kmin,
                                                               const uint32_t* __restrict__ bits, bool negate,
                                                               unsigned long long* __restrict__ words,
                                                               int64_t* __restrict__ tile_counts) {
  __shared__ uint32_t fold[kFoldWords];
  __shared__ int64_t red[kFoldWaves];
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  const int64_t nbw = (cap + 31) >> 5;
  for (int i = threadIdx.x; i < kFoldWords; i += kFoldBlock) {
    uint32_t v = 0;
    for (int64_t j = i; j < nbw; j += kFoldWords) v |= bits[j];
    fold[i] = v;
  }
  __syncthreads();
  const bool exact = nbw <= kFoldWords;
  const int64_t tiles = (m + kHitTile - 1) / kHitTile;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    int64_t cnt = 0;
#pragma unroll
    for (int g = 0; g < kFoldSteps; ++g) {
      const int64_t r0 = t * kHitTile + (int64_t)g * (kFoldBlock * kBitsRows) + (int64_t)threadIdx.x * kBitsRows;
      K k[kBitsRows];
      uint32_t vb = 0x01010101u;
      if (r0 + kBitsRows <= m) {
        load4(keys + r0, k);
        if (valid) vb = *reinterpret_cast<const uint32_t*>(valid + r0);
      } else {
        vb = 0;
#pragma unroll
        for (int j = 0; j < kBitsRows; ++j) {
          const bool in = r0 + j < m;
          k[j] = in ? keys[r0 + j] : K(0);
          if (in && (!valid || valid[r0 + j])) vb |= 1u << (8 * j);
        }
      }
      uint32_t nib = 0;
#pragma unroll
      for (int j = 0; j < kBitsRows; ++j) {
        const int64_t d = (int64_t)k[j] - kmin;
        bool ok = ((vb >> (8 * j)) & 0xffu) != 0 && d >= 0 && d < cap;
        if (ok) ok = (fold[(d >> 5) & (kFoldWords - 1)] >> (d & 31)) & 1u;
        if (ok && !exact) ok = (bits[(uint64_t)d >> 5] >> (d & 31)) & 1u;
        const bool hit = r0 + j < m && (ok != negate);
        nib |= (hit ? 1u : 0u) << j;
      }
      cnt += __popc(nib);
      unsigned long long w = (unsigned long long)nib << (4 * (lane & 15));
      w |= __shfl_xor(w, 1, kWave);
      w |= __shfl_xor(w, 2, kWave);
      w |= __shfl_xor(w, 4, kWave);
      w |= __shfl_xor(w, 8, kWave);
      const int64_t wrow = t * kHitTile + (int64_t)g * (kFoldBlock * kBitsRows) +
                           (int64_t)wave * (kWave * kBitsRows) + (int64_t)(lane >> 4) * kWave;
      if ((lane & 15) == 0 && wrow < m)
        words[t * kHitWords + g * (kHitWords / kFoldSteps) + wave * kBitsRows + (lane >> 4)] = w;
    }
    cnt = wave_reduce_sum(cnt);
    if (lane == 0) red[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t s = 0;
      for (int w = 0; w < kFoldWaves; ++w) s += red[w];
      tile_counts[t] = s;
    }
    __syncthreads();
  }
}

}  // namespace

int64_t probe_hit_tiles(int64_t m) { return (m + kHitTile - 1) / kHitTile; }

// workgroups of a probe_hits / probe_write launch at most (both loop over
// their tiles): tunable for the A/B in scripts/bench_probe.py
static int g_probe_grid_cap = 1 << 16;
void set_probe_grid_cap(int cap) { g_probe_grid_cap = cap > 0 ? cap : (1 << 16); }
// 0: scalar probe_hits_kernel only, 1: + the vector bitmap probe, 2: + the LDS-folded
// bitmap for large probe sides (scripts/bench_probe.py A/B)
static int g_probe_bits = 2;
void set_probe_bits(int mode) { g_probe_bits = mode; }
constexpr int64_t kFoldMinRows = 1 << 22;   // below: the fold's build per workgroup does not pay
constexpr int64_t kFoldGrid = 512;          // two 1024-lane workgroups (64 KiB LDS each) per CU

void probe_hits(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const void* thead, bool rid64, int64_t cap, int64_t kmin, bool direct, const uint32_t* bits,
                uint64_t bmask, bool negate, unsigned long long* words, int64_t* tile_counts, hipStream_t stream) {
  if (m == 0) return;
  const dim3 g(grid_for(probe_hit_tiles(m), 1, g_probe_grid_cap)), b(kBlock);
  const bool vec = direct && bits && (bmask & kExactBits) && ((uintptr_t)keys & 15) == 0 &&
                   ((uintptr_t)valid & 3) == 0;
  if (vec && g_probe_bits >= 2 && m >= kFoldMinRows) {
    const int64_t tiles = probe_hit_tiles(m);
    const dim3 gf((unsigned)(tiles < kFoldGrid ? tiles : kFoldGrid)), bf(kFoldBlock);
    if (key64)
      hipLaunchKernelGGL(probe_fold_kernel<int64_t>, gf, bf, 0, stream, static_cast<const int64_t*>(keys), valid, m,
                         cap, kmin, bits, negate, words, tile_counts);
    else
      hipLaunchKernelGGL(probe_fold_kernel<int32_t>, gf, bf, 0, stream, static_cast<const int32_t*>(keys), valid, m,
                         cap, kmin, bits, negate, words, tile_counts);
  } else if (vec && g_probe_bits >= 1) {
    if (key64)
      hipLaunchKernelGGL(probe_bits_kernel<int64_t>, g, b, 0, stream, static_cast<const int64_t*>(keys), valid, m, cap,
                         kmin, bits, negate, words, tile_counts);
    else
      hipLaunchKernelGGL(probe_bits_kernel<int32_t>, g, b, 0, stream, static_cast<const int32_t*>(keys), valid, m, cap,
                         kmin, bits, negate, words, tile_counts);
  } else if (rid64)
    DISPATCH_KEY3(key64, direct, int64_t, probe_hits_kernel, g, b, 0, stream, keys, valid, m, tkeys,
                  (const int64_t*)thead, cap, kmin, bits, bmask, negate, words, tile_counts);
  else
    DISPATCH_KEY3(key64, direct, int32_t, probe_hits_kernel, g, b, 0, stream, keys, valid, m, tkeys,
                  (const int32_t*)thead, cap, kmin, bits, bmask, negate, words, tile_counts);
  check_launch("probe_hits", stream);
}

template <typename R, typename O>
static void probe_write_t(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                          const R* thead, int64_t cap, int64_t kmin, bool direct, const unsigned long long* words,
                          const int64_t* tile_off, O* out_probe, R* out_build, int64_t out_cap, hipStream_t stream) {
  const dim3 g(grid_for(probe_hit_tiles(m), 1, g_probe_grid_cap)), b(kBlock);
  if (key64) {
    if (direct)
      hipLaunchKernelGGL((probe_write_kernel<int64_t, true, R, O>), g, b, 0, stream, (const int64_t*)keys, valid, m,
                         tkeys, thead, cap, kmin, words, tile_off, out_probe, out_build, out_cap);
    else
      hipLaunchKernelGGL((probe_write_kernel<int64_t, false, R, O>), g, b, 0, stream, (const int64_t*)keys, valid, m,
                         tkeys, thead, cap, kmin, words, tile_off, out_probe, out_build, out_cap);
  } else {
    if (direct)
      hipLaunchKernelGGL((probe_write_kernel<int32_t, true, R, O>), g, b, 0, stream, (const int32_t*)keys, valid, m,
                         tkeys, thead, cap, kmin, words, tile_off, out_probe, out_build, out_cap);
    else
      hipLaunchKernelGGL((probe_write_kernel<int32_t, false, R, O>), g, b, 0, stream, (const int32_t*)keys, valid, m,
                         tkeys, thead, cap, kmin, words, tile_off, out_probe, out_build, out_cap);
  }
  check_launch("probe_write", stream);
}

void probe_write(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const void* thead, bool rid64, int64_t cap, int64_t kmin, bool direct, const unsigned long long* words,
                 const int64_t* tile_off, void* out_probe, bool out64, void* out_build, int64_t out_cap,
                 hipStream_t stream) {
  if (m == 0) return;
  if (rid64) {
    if (out64)
      probe_write_t<int64_t, int64_t>(keys, key64, valid, m, tkeys, (const int64_t*)thead, cap, kmin, direct, words,
                                      tile_off, (int64_t*)out_probe, (int64_t*)out_build, out_cap, stream);
    else
      probe_write_t<int64_t, int32_t>(keys, key64, valid, m, tkeys, (const int64_t*)thead, cap, kmin, direct, words,
                                      tile_off, (int32_t*)out_probe, (int64_t*)out_build, out_cap, stream);
  } else {
    if (out64)
      probe_write_t<int32_t, int64_t>(keys, key64, valid, m, tkeys, (const int32_t*)thead, cap, kmin, direct, words,
                                      tile_off, (int64_t*)out_probe, (int32_t*)out_build, out_cap, stream);
    else
      probe_write_t<int32_t, int32_t>(keys, key64, valid, m, tkeys, (const int32_t*)thead, cap, kmin, direct, words,
                                      tile_off, (int32_t*)out_probe, (int32_t*)out_build, out_cap, stream);
  }
}
}  // namespace kern
}  // namespace igloo
