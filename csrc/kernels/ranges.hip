// Sorted-key join primitives for clustered inputs (lineitem by l_orderkey,
// orders by o_orderkey, and every join output that preserved that order).
//
//   sorted_ranges: for each probe key, the range [lo, lo+cnt) of equal keys in
//     a non-decreasing build column — one lower-bound binary search, then a
//     short forward scan (TPC-H keys repeat <= 7 times) that falls back to a
//     second binary search for long runs. Replaces two torch.searchsorted
//     passes.
//   expand_ranges: the (probe row, build row) pairs of those ranges, output
//     parallel and load balanced: a workgroup owns 2048 consecutive outputs,
//     finds the probe rows overlapping them with two binary searches over the
//     exclusive offsets, stages those offsets in LDS and lets every lane
//     binary-search its outputs there; stores are coalesced. Replaces
//     torch.repeat_interleave + cumsum + index_select (one thread per probe
//     row writing its run: 17 ms for one 60M-pair expansion at SF100).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kExpItems = 8;
constexpr int kExpTile = kBlock * kExpItems;
constexpr int kScanRun = 16;

template <typename K>
__global__ __launch_bounds__(kBlock) void sorted_ranges_kernel(const K* __restrict__ big, int64_t nb,
                                                              const K* __restrict__ q,
                                                              const uint8_t* __restrict__ qvalid, int64_t nq,
                                                              int64_t* __restrict__ lo_out,
                                                              int64_t* __restrict__ cnt_out,
                                                              const K* __restrict__ fence, int64_t nf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
    if (qvalid && !qvalid[i]) {
      lo_out[i] = 0;
      cnt_out[i] = 0;
      continue;
    }
    const K key = q[i];
    int64_t a = 0, b = nb;
    if (fence) {
      // fence[j] = big[j * kFence] (a 1/kFence sample small enough to stay in
      // L2 / MALL): its lower bound j brackets the answer to one kFence-row
      // window, so the search touches ~3 HBM lines instead of ~20
      int64_t fa = 0, fb = nf;
      while (fa < fb) {
        const int64_t m = (fa + fb) >> 1;
        if (fence[m] < key) fa = m + 1;
        else fb = m;
      }
      a = fa > 0 ? (fa - 1) * kFence : 0;
      b = fa * kFence < nb ? fa * kFence : nb;
    }
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (big[m] < key) a = m + 1;
      else b = m;
    }
    int64_t e = a;
    int k = 0;
    while (e < nb && k < kScanRun && big[e] == key) {
      ++e;
      ++k;
    }
    if (k == kScanRun && e < nb && big[e] == key) {
      int64_t a2 = e, b2 = nb;
      while (a2 < b2) {
        const int64_t m = (a2 + b2) >> 1;
        if (big[m] <= key) a2 = m + 1;
        else b2 = m;
      }
      e = a2;
    }
    lo_out[i] = a;
    cnt_out[i] = e - a;
  }
}

// largest r in [0, n) with off[r] <= t (off non-decreasing, off[0] <= t)
__device__ inline int64_t row_of(const int64_t* off, int64_t n, int64_t t) {
  int64_t a = 0, b = n - 1;
  while (a < b) {
    const int64_t m = (a + b + 1) >> 1;
    if (off[m] <= t) a = m;
    else b = m - 1;
  }
  return a;
}

template <typename O>
__global__ __launch_bounds__(kBlock) void expand_ranges_kernel(const int64_t* __restrict__ off,
                                                              const int64_t* __restrict__ lo, int64_t ns,
                                                              int64_t total, O* __restrict__ sidx,
                                                              O* __restrict__ bidx) {
  __shared__ int64_t soff[kExpTile + 1];
  __shared__ int64_t rr[2];
  const int64_t t0 = (int64_t)blockIdx.x * kExpTile;
  if (t0 >= total) return;
  const int64_t t1 = t0 + kExpTile < total ? t0 + kExpTile : total;
  if (threadIdx.x == 0) {
    rr[0] = row_of(off, ns, t0);
    rr[1] = row_of(off, ns, t1 - 1);
  }
  __syncthreads();
  const int64_t r0 = rr[0], nr = rr[1] - rr[0] + 1;
  if (nr <= kExpTile) {
    for (int64_t k = threadIdx.x; k < nr; k += blockDim.x) soff[k] = off[r0 + k];
    __syncthreads();
    // each lane expands kExpItems CONSECUTIVE outputs: one search for the
    // first, then a forward walk over the (LDS) range starts, and the lane's
    // outputs leave as whole vectors (a strided layout searched per output)
    const int64_t ta = t0 + (int64_t)threadIdx.x * kExpItems;
    if (ta < t1) {
      int64_t j = row_of(soff, nr, ta);
      int64_t base = lo[r0 + j] - soff[j];
      O sv[kExpItems], bv[kExpItems];
#pragma unroll
      for (int k = 0; k < kExpItems; ++k) {
        const int64_t t = ta + k;
        while (j + 1 < nr && soff[j + 1] <= t) {
          ++j;
          base = lo[r0 + j] - soff[j];
        }
        sv[k] = (O)(r0 + j);
        bv[k] = (O)(base + t);
      }
      if (ta + kExpItems <= t1 && (((uintptr_t)(sidx + ta) | (uintptr_t)(bidx + ta)) & 15) == 0) {
        constexpr int kV = 16 / (int)sizeof(O);   // elements per 16-byte store
        typedef O OV __attribute__((ext_vector_type(kV)));
#pragma unroll
        for (int k = 0; k < kExpItems; k += kV) {
          OV a, b;
#pragma unroll
          for (int q = 0; q < kV; ++q) {
            a[q] = sv[k + q];
            b[q] = bv[k + q];
          }
          *(OV*)(sidx + ta + k) = a;
          *(OV*)(bidx + ta + k) = b;
        }
      } else {
#pragma unroll
        for (int k = 0; k < kExpItems; ++k)
          if (ta + k < t1) {
            sidx[ta + k] = sv[k];
            bidx[ta + k] = bv[k];
          }
      }
    }
  } else {  // many empty ranges inside the tile: search the global offsets
    for (int k = 0; k < kExpItems; ++k) {
      const int64_t t = t0 + threadIdx.x + (int64_t)k * kBlock;
      if (t >= t1) break;
      const int64_t r = row_of(off, ns, t);
      sidx[t] = (O)r;
      bidx[t] = (O)(lo[r] + (t - off[r]));
    }
  }
}

}  // namespace

void sorted_ranges(const void* big, bool key64, int64_t nb, const void* q, const uint8_t* qvalid, int64_t nq,
                   int64_t* lo, int64_t* cnt, const void* fence, int64_t nf, hipStream_t stream) {
  if (nq <= 0) return;
  const unsigned grid = grid_for(nq, kBlock, 1 << 16);
  if (key64)
    hipLaunchKernelGGL(sorted_ranges_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const int64_t*>(big), nb, static_cast<const int64_t*>(q), qvalid, nq, lo, cnt,
                       static_cast<const int64_t*>(fence), nf);
  else
    hipLaunchKernelGGL(sorted_ranges_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const int32_t*>(big), nb, static_cast<const int32_t*>(q), qvalid, nq, lo, cnt,
                       static_cast<const int32_t*>(fence), nf);
  check_launch("sorted_ranges", stream);
}

void expand_ranges(const int64_t* off, const int64_t* lo, int64_t ns, int64_t total, void* sidx, void* bidx,
                   bool out64, hipStream_t stream) {
  if (total <= 0 || ns <= 0) return;
  const unsigned grid = (unsigned)((total + kExpTile - 1) / kExpTile);
  if (out64)
    hipLaunchKernelGGL(expand_ranges_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, stream, off, lo, ns, total,
                       static_cast<int64_t*>(sidx), static_cast<int64_t*>(bidx));
  else
    hipLaunchKernelGGL(expand_ranges_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, stream, off, lo, ns, total,
                       static_cast<int32_t*>(sidx), static_cast<int32_t*>(bidx));
  check_launch("expand_ranges", stream);
}

}  // namespace kern
}  // namespace igloo

// ---- sorted ranges + a second equality key ---------------------------------
// Two-column equi-join whose big side is sorted on the first key (partsupp by
// ps_partkey joined on (partkey, suppkey): TPC-H Q9): after sorted_ranges on
// the first key, each probe row scans its (short) range for the second key.
// Pass 0 counts matches per probe row; pass 1 writes the (probe, build) pairs
// at the exclusive offsets of those counts.
namespace igloo {
namespace kern {
namespace {

// MASKED: big2 is a byte mask over the big side (a filter the big column was
// not compacted by: the join probes the table's own sorted key column) and a
// range row matches where it is set; small2 is unused.
template <typename K2, typename O, bool WRITE, bool MASKED = false>
__global__ __launch_bounds__(kBlock) void sorted_match_kernel(const K2* __restrict__ big2,
                                                             const K2* __restrict__ small2,
                                                             const int64_t* __restrict__ lo,
                                                             const int64_t* __restrict__ cnt, int64_t ns,
                                                             int32_t* __restrict__ counts,
                                                             const int64_t* __restrict__ offsets,
                                                             O* __restrict__ sidx, O* __restrict__ bidx,
                                                             int64_t out_cap, O* __restrict__ first) {
  const uint8_t* __restrict__ mask = reinterpret_cast<const uint8_t*>(big2);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ns; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = lo[i], c = cnt[i];
    const K2 key = MASKED ? K2{} : small2[i];
    int64_t o = WRITE ? offsets[i] : 0;
    int32_t m = 0;
    int64_t f = -1;
    for (int64_t k = 0; k < c; ++k) {
      if (MASKED ? mask[l + k] != 0 : big2[l + k] == key) {
        if (WRITE) {
          // (offsets from a device scan; the outputs sized by a possibly
          // replayed total: never written past it)
          if (o >= 0 && o < out_cap) {
            sidx[o] = (O)i;
            bidx[o] = (O)(l + k);
          }
          ++o;
        }
        if (m == 0) f = l + k;
        ++m;
      }
    }
    if (!WRITE) {
      counts[i] = m;
      // count pass: the first match too (a row with exactly one match -- every
      // row, for a foreign key into a primary key -- needs no write pass)
      if (first) first[i] = (O)f;
    }
  }
}

template <typename K2, bool MASKED>
void launch_match(const void* big2, const void* small2, const int64_t* lo, const int64_t* cnt, int64_t ns,
                  int32_t* counts, const int64_t* offsets, void* sidx, void* bidx, bool out64, int64_t out_cap,
                  int32_t* first, hipStream_t stream) {
  const dim3 g(grid_for(ns, kBlock, 1 << 16)), b(kBlock);
  const K2* B = static_cast<const K2*>(big2);
  const K2* S = static_cast<const K2*>(small2);
  if (!offsets)
    hipLaunchKernelGGL((sorted_match_kernel<K2, int32_t, false, MASKED>), g, b, 0, stream, B, S, lo, cnt, ns, counts,
                       nullptr, nullptr, nullptr, 0, first);
  else if (out64)
    hipLaunchKernelGGL((sorted_match_kernel<K2, int64_t, true, MASKED>), g, b, 0, stream, B, S, lo, cnt, ns, nullptr,
                       offsets, static_cast<int64_t*>(sidx), static_cast<int64_t*>(bidx), out_cap, nullptr);
  else
    hipLaunchKernelGGL((sorted_match_kernel<K2, int32_t, true, MASKED>), g, b, 0, stream, B, S, lo, cnt, ns, nullptr,
                       offsets, static_cast<int32_t*>(sidx), static_cast<int32_t*>(bidx), out_cap, nullptr);
}

}  // namespace

void sorted_match(const void* big2, const void* small2, bool key64, const int64_t* lo, const int64_t* cnt,
                  int64_t ns, int32_t* counts, const int64_t* offsets, void* sidx, void* bidx, bool out64,
                  int64_t out_cap, int32_t* first, hipStream_t stream) {
  if (ns <= 0) return;
  if (key64)
    launch_match<int64_t, false>(big2, small2, lo, cnt, ns, counts, offsets, sidx, bidx, out64, out_cap, first,
                                 stream);
  else
    launch_match<int32_t, false>(big2, small2, lo, cnt, ns, counts, offsets, sidx, bidx, out64, out_cap, first,
                                 stream);
  check_launch("sorted_match", stream);
}

void sorted_masked(const uint8_t* mask, const int64_t* lo, const int64_t* cnt, int64_t ns, int32_t* counts,
                   const int64_t* offsets, void* sidx, void* bidx, bool out64, int64_t out_cap, hipStream_t stream) {
  if (ns <= 0) return;
  launch_match<int32_t, true>(mask, nullptr, lo, cnt, ns, counts, offsets, sidx, bidx, out64, out_cap, nullptr,
                              stream);
  check_launch("sorted_masked", stream);
}

}  // namespace kern
}  // namespace igloo

// ---- dense range index over a sorted key column -----------------------------
// For a non-decreasing key column whose value span is close to its length
// (partsupp.ps_partkey: 4 rows per key; orders.o_orderkey: 1 of 4 values used)
// a lower-bound table first[k - kmin] = first row with key >= k turns each
// range lookup into two adjacent loads instead of a ~27-step binary search
// whose probes miss the cache when the queries arrive in random key order
// (Q9 probes partsupp in lineitem order: 11 ms searching vs ~1 ms indexed).
// Row i fills the entries between the previous row's key and its own.
namespace igloo {
namespace kern {
namespace {

// Gaps longer than kGapFill are not filled (one lane would serialise them):
// the key's own entry is still written and *long_gap is set, so the caller
// pre-fills the table with -1, rebuilds, and runs the fix-up pass
// (long_gap == null) that searches the entries left at -1.
constexpr int64_t kGapFill = 64;

template <typename K, typename I>
__global__ __launch_bounds__(kBlock) void dense_index_kernel(const K* __restrict__ big, int64_t nb, int64_t kmin,
                                                            int64_t kmax, I* __restrict__ first,
                                                            int32_t* __restrict__ long_gap) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= nb; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prev = i == 0 ? kmin - 1 : (int64_t)big[i - 1];
    const int64_t cur = i == nb ? kmax + 1 : (int64_t)big[i];
    if (cur == prev) continue;
    int64_t k = cur - prev > kGapFill ? cur : prev + 1;
    if (k != prev + 1) *long_gap = 1;
    // keys outside [kmin, kmax] (a replayed range narrower than the data)
    // never index past the table's kmax - kmin + 2 entries
    const int64_t hi = cur < kmax + 1 ? cur : kmax + 1;
    for (k = k < kmin ? kmin : k; k <= hi; ++k) first[k - kmin] = (I)i;
  }
}

// long-gap fix-up: entries still holding the sentinel get a lower-bound search
// (neighbouring lanes search neighbouring keys, so the probes share cache lines)
template <typename K, typename I>
__global__ __launch_bounds__(kBlock) void dense_fill_kernel(const K* __restrict__ big, int64_t nb, int64_t kmin,
                                                           int64_t span, I sentinel, I* __restrict__ first) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k <= span; k += (int64_t)gridDim.x * blockDim.x) {
    if (first[k] != sentinel) continue;
    const int64_t key = kmin + k;
    int64_t a = 0, b = nb;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if ((int64_t)big[m] < key) a = m + 1;
      else b = m;
    }
    first[k] = (I)a;
  }
}

template <typename K, typename I>
__global__ __launch_bounds__(kBlock) void dense_ranges_kernel(const I* __restrict__ first, int64_t kmin, int64_t kmax,
                                                             const K* __restrict__ q,
                                                             const uint8_t* __restrict__ qvalid, int64_t nq,
                                                             int64_t* __restrict__ lo_out,
                                                             int64_t* __restrict__ cnt_out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = (int64_t)q[i];
    int64_t lo = 0, c = 0;
    if ((!qvalid || qvalid[i]) && k >= kmin && k <= kmax) {
      lo = (int64_t)first[k - kmin];
      c = (int64_t)first[k - kmin + 1] - lo;
    }
    lo_out[i] = lo;
    cnt_out[i] = c;
  }
}

template <typename K>
void dense_launch(bool build, const void* big, int64_t nb, int64_t kmin, int64_t kmax, void* first, bool first64,
                  int32_t* long_gap, const void* q, const uint8_t* qvalid, int64_t nq, int64_t* lo, int64_t* cnt, hipStream_t stream) {
  const dim3 b(kBlock);
  if (build && !long_gap) {  // fix-up pass
    const int64_t span = kmax - kmin + 1;
    const dim3 g(grid_for(span + 1, kBlock, 1 << 16));
    if (first64)
      hipLaunchKernelGGL((dense_fill_kernel<K, int64_t>), g, b, 0, stream, static_cast<const K*>(big), nb, kmin, span,
                         (int64_t)-1, static_cast<int64_t*>(first));
    else
      hipLaunchKernelGGL((dense_fill_kernel<K, int32_t>), g, b, 0, stream, static_cast<const K*>(big), nb, kmin, span,
                         (int32_t)-1, static_cast<int32_t*>(first));
  } else if (build) {
    const dim3 g(grid_for(nb + 1, kBlock, 1 << 16));
    if (first64)
      hipLaunchKernelGGL((dense_index_kernel<K, int64_t>), g, b, 0, stream, static_cast<const K*>(big), nb, kmin, kmax,
                         static_cast<int64_t*>(first), long_gap);
    else
      hipLaunchKernelGGL((dense_index_kernel<K, int32_t>), g, b, 0, stream, static_cast<const K*>(big), nb, kmin, kmax,
                         static_cast<int32_t*>(first), long_gap);
  } else {
    const dim3 g(grid_for(nq, kBlock, 1 << 16));
    if (first64)
      hipLaunchKernelGGL((dense_ranges_kernel<K, int64_t>), g, b, 0, stream, static_cast<const int64_t*>(first), kmin,
                         kmax, static_cast<const K*>(q), qvalid, nq, lo, cnt);
    else
      hipLaunchKernelGGL((dense_ranges_kernel<K, int32_t>), g, b, 0, stream, static_cast<const int32_t*>(first), kmin,
                         kmax, static_cast<const K*>(q), qvalid, nq, lo, cnt);
  }
}

}  // namespace

void dense_index_build(const void* big, bool key64, int64_t nb, int64_t kmin, int64_t kmax, void* first, bool first64,
                       int32_t* long_gap, hipStream_t stream) {
  if (key64)
    dense_launch<int64_t>(true, big, nb, kmin, kmax, first, first64, long_gap, nullptr, nullptr, 0, nullptr, nullptr,
                          stream);
  else
    dense_launch<int32_t>(true, big, nb, kmin, kmax, first, first64, long_gap, nullptr, nullptr, 0, nullptr, nullptr,
                          stream);
  check_launch("dense_index_build", stream);
}

void dense_ranges(const void* first, bool first64, int64_t kmin, int64_t kmax, const void* q, bool key64,
                  const uint8_t* qvalid, int64_t nq, int64_t* lo, int64_t* cnt, hipStream_t stream) {
  if (nq <= 0) return;
  if (key64)
    dense_launch<int64_t>(false, nullptr, 0, kmin, kmax, const_cast<void*>(first), first64, nullptr, q, qvalid, nq, lo,
                          cnt, stream);
  else
    dense_launch<int32_t>(false, nullptr, 0, kmin, kmax, const_cast<void*>(first), first64, nullptr, q, qvalid, nq, lo,
                          cnt, stream);
  check_launch("dense_ranges", stream);
}

}  // namespace kern
}  // namespace igloo

// ---- EXISTS over a sorted range with a column comparison ----------------------
// Semi / anti join whose residual compares one column of each side
// (Q21: EXISTS (l2.l_orderkey = l1.l_orderkey AND l2.l_suppkey <> l1.l_suppkey)):
// hit[i] = any k in [lo[i], lo[i]+cnt[i]) with big2[k] OP small2[i], scanned
// in place instead of expanding every pair and gathering both columns.
namespace igloo {
namespace kern {
namespace {
// mask (optional): only the big rows set in it exist (a filtered big side
// searched in place, exec/joins.py _in_place_semi); op 6: any such row
template <typename K2>
__global__ __launch_bounds__(kBlock) void sorted_exists_kernel(const K2* __restrict__ big2,
                                                              const K2* __restrict__ small2,
                                                              const int64_t* __restrict__ lo,
                                                              const int64_t* __restrict__ cnt, int64_t ns, int op,
                                                              const uint8_t* __restrict__ mask,
                                                              uint8_t* __restrict__ hit) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < ns; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t l = lo[i], c = cnt[i];
    const K2 v = op == 6 ? K2{} : small2[i];
    bool any = false;
    for (int64_t k = 0; k < c && !any; ++k) {
      if (mask && !mask[l + k]) continue;
      const K2 b = op == 6 ? K2{} : big2[l + k];
      switch (op) {
        case 0: any = b == v; break;
        case 1: any = b != v; break;
        case 2: any = b < v; break;
        case 3: any = b <= v; break;
        case 4: any = b > v; break;
        case 5: any = b >= v; break;
        default: any = true; break;
      }
    }
    hit[i] = any;
  }
}
}  // namespace

void sorted_exists(const void* big2, const void* small2, bool key64, const int64_t* lo, const int64_t* cnt,
                   int64_t ns, int op, const uint8_t* mask, uint8_t* hit, hipStream_t stream) {
  if (ns <= 0) return;
  const dim3 g(grid_for(ns, kBlock, 1 << 16)), b(kBlock);
  if (key64)
    hipLaunchKernelGGL(sorted_exists_kernel<int64_t>, g, b, 0, stream, (const int64_t*)big2, (const int64_t*)small2,
                       lo, cnt, ns, op, mask, hit);
  else
    hipLaunchKernelGGL(sorted_exists_kernel<int32_t>, g, b, 0, stream, (const int32_t*)big2, (const int32_t*)small2,
                       lo, cnt, ns, op, mask, hit);
  check_launch("sorted_exists", stream);
}
}  // namespace kern
}  // namespace igloo

// ---- lookups into UNIQUE sorted keys ----------------------------------------
// A search into a key column known to hold distinct values (a primary key,
// ops/hashing.py key_unique) pairs every probe row with at most one row:
// hit[i] (0/1) and pos[i] (int32 row, 0 on a miss) replace the (lo, cnt)
// int64 pair -- 5 instead of 16 output bytes per probe row, and no compare /
// narrowing pass over them afterwards (exec/joins.py _unique_pairs).
namespace igloo {
namespace kern {
namespace {

template <typename K>
__global__ __launch_bounds__(kBlock) void unique_search_kernel(const K* __restrict__ big, int64_t nb,
                                                              const K* __restrict__ q,
                                                              const uint8_t* __restrict__ qvalid, int64_t nq,
                                                              uint8_t* __restrict__ hit, int32_t* __restrict__ pos,
                                                              const K* __restrict__ fence, int64_t nf) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
    if (qvalid && !qvalid[i]) {
      hit[i] = 0;
      pos[i] = 0;
      continue;
    }
    const K key = q[i];
    int64_t a = 0, b = nb;
    if (fence) {
      int64_t fa = 0, fb = nf;
      while (fa < fb) {
        const int64_t m = (fa + fb) >> 1;
        if (fence[m] < key) fa = m + 1;
        else fb = m;
      }
      a = fa > 0 ? (fa - 1) * kFence : 0;
      b = fa * kFence < nb ? fa * kFence : nb;
    }
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (big[m] < key) a = m + 1;
      else b = m;
    }
    const bool h = a < nb && big[a] == key;
    hit[i] = h ? 1 : 0;
    pos[i] = h ? (int32_t)a : 0;
  }
}

template <typename K, typename I>
__global__ __launch_bounds__(kBlock) void unique_dense_kernel(const I* __restrict__ first, int64_t kmin, int64_t kmax,
                                                             const K* __restrict__ q,
                                                             const uint8_t* __restrict__ qvalid, int64_t nq,
                                                             uint8_t* __restrict__ hit, int32_t* __restrict__ pos) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nq; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = (int64_t)q[i];
    int64_t lo = 0;
    bool h = false;
    if ((!qvalid || qvalid[i]) && k >= kmin && k <= kmax) {
      lo = (int64_t)first[k - kmin];
      h = (int64_t)first[k - kmin + 1] > lo;
    }
    hit[i] = h ? 1 : 0;
    pos[i] = h ? (int32_t)lo : 0;
  }
}

}  // namespace

void unique_lookup(const void* big, bool key64, int64_t nb, const void* first, bool first64, int64_t kmin,
                   int64_t kmax, const void* q, const uint8_t* qvalid, int64_t nq, uint8_t* hit, int32_t* pos,
                   const void* fence, int64_t nf, hipStream_t stream) {
  if (nq <= 0) return;
  const unsigned grid = grid_for(nq, kBlock, 1 << 16);
  if (first) {
    if (key64 && first64)
      hipLaunchKernelGGL((unique_dense_kernel<int64_t, int64_t>), dim3(grid), dim3(kBlock), 0, stream,
                         static_cast<const int64_t*>(first), kmin, kmax, static_cast<const int64_t*>(q), qvalid, nq,
                         hit, pos);
    else if (key64)
      hipLaunchKernelGGL((unique_dense_kernel<int64_t, int32_t>), dim3(grid), dim3(kBlock), 0, stream,
                         static_cast<const int32_t*>(first), kmin, kmax, static_cast<const int64_t*>(q), qvalid, nq,
                         hit, pos);
    else if (first64)
      hipLaunchKernelGGL((unique_dense_kernel<int32_t, int64_t>), dim3(grid), dim3(kBlock), 0, stream,
                         static_cast<const int64_t*>(first), kmin, kmax, static_cast<const int32_t*>(q), qvalid, nq,
                         hit, pos);
    else
      hipLaunchKernelGGL((unique_dense_kernel<int32_t, int32_t>), dim3(grid), dim3(kBlock), 0, stream,
                         static_cast<const int32_t*>(first), kmin, kmax, static_cast<const int32_t*>(q), qvalid, nq,
                         hit, pos);
  } else if (key64) {
    hipLaunchKernelGGL(unique_search_kernel<int64_t>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const int64_t*>(big), nb, static_cast<const int64_t*>(q), qvalid, nq, hit, pos,
                       static_cast<const int64_t*>(fence), nf);
  } else {
    hipLaunchKernelGGL(unique_search_kernel<int32_t>, dim3(grid), dim3(kBlock), 0, stream,
                       static_cast<const int32_t*>(big), nb, static_cast<const int32_t*>(q), qvalid, nq, hit, pos,
                       static_cast<const int32_t*>(fence), nf);
  }
  check_launch("unique_lookup", stream);
}

}  // namespace kern
}  // namespace igloo
