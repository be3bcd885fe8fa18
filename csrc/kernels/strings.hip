// UTF-8 string kernels over Arrow large-string layout (int64 offsets + bytes).
//
// * str_like: SQL LIKE/ILIKE with '%' and '_' (pattern pre-tokenised on the
//   host so escapes are already resolved). Greedy wildcard matching with a
//   single backtrack point: linear in the usual case.
// * str_case: upper/lower — the reference's `capitalize` UDF uppercases the
//   whole string (reference crates/engine/src/lib.rs:84-91). ASCII bytes are
//   mapped on the GPU; the kernel reports whether any non-ASCII byte was seen
//   so the host can fall back to full Unicode case mapping.
// * str_substr: SUBSTRING(s FROM a FOR b) in characters (UTF-8 aware).
// * str_hash64 / str_eq_rows / str_cmp_const: hashing and comparisons for
//   GROUP BY, join verification and predicates on plain string columns.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__device__ inline uint8_t fold(uint8_t c, bool ci) { return ci && c >= 'A' && c <= 'Z' ? c + 32 : c; }

__device__ bool like_match(const uint8_t* s, int64_t n, const uint8_t* pat, const uint8_t* kind, int m, bool ci) {
  int64_t si = 0, ss = 0;
  int pi = 0, star = -1;
  while (si < n) {
    if (pi < m && (kind[pi] == 1 || (kind[pi] == 0 && fold(pat[pi], ci) == fold(s[si], ci)))) {
      // '_' consumes one UTF-8 character
      if (kind[pi] == 1) {
        ++si;
        while (si < n && (s[si] & 0xC0) == 0x80) ++si;
      } else {
        ++si;
      }
      ++pi;
    } else if (pi < m && kind[pi] == 2) {
      star = pi++;
      ss = si;
    } else if (star != -1) {
      pi = star + 1;
      si = ++ss;
    } else {
      return false;
    }
  }
  while (pi < m && kind[pi] == 2) ++pi;
  return pi == m;
}

__global__ __launch_bounds__(kBlock) void like_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                     int64_t n, const uint8_t* __restrict__ pat,
                                                     const uint8_t* __restrict__ kind, int m, bool ci, bool negate,
                                                     uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = off[i];
    bool r = like_match(chars + a, off[i + 1] - a, pat, kind, m, ci);
    out[i] = r != negate;
  }
}

// LDS-staged LIKE: a block takes 256 consecutive strings, copies their byte
// range into LDS with 16-byte coalesced loads, then each lane matches its
// string out of LDS. The per-lane byte-serial scan of the simple kernel above
// touches a new 64-byte line every few bytes per lane; staging turns the HBM
// traffic into one streaming read of the character buffer.
constexpr int kLikeTileBytes = 24576;
constexpr int kLikeMaxPattern = 256;

__global__ __launch_bounds__(kBlock) void like_tile_kernel(const int64_t* __restrict__ off,
                                                          const uint8_t* __restrict__ chars, int64_t n,
                                                          const uint8_t* __restrict__ pat,
                                                          const uint8_t* __restrict__ kind, int m, bool ci,
                                                          bool negate, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kLikeTileBytes];
  __shared__ uint8_t spat[kLikeMaxPattern], skind[kLikeMaxPattern];
  for (int i = threadIdx.x; i < m; i += kBlock) {
    spat[i] = pat[i];
    skind[i] = kind[i];
  }
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t i0 = t * kBlock;
    const int64_t i1 = i0 + kBlock < n ? i0 + kBlock : n;
    const uintptr_t lo = (uintptr_t)(chars + off[i0]);
    const uintptr_t hi = (uintptr_t)(chars + off[i1]);
    const uintptr_t start = lo & ~(uintptr_t)15;       // never below the allocation (>= 256 B aligned)
    const uintptr_t full_end = hi & ~(uintptr_t)15;    // vector loads stop here; the tail goes bytewise
    const bool staged = hi - start <= (uintptr_t)kLikeTileBytes;
    __syncthreads();  // previous tile finished reading buf; pattern visible on the first pass
    if (staged) {
      const int64_t nvec = (int64_t)(full_end - start) / 16;
      for (int64_t v = threadIdx.x; v < nvec; v += kBlock)
        *(uint4*)(buf + v * 16) = *(const uint4*)(start + v * 16);
      for (uintptr_t a = full_end + threadIdx.x; a < hi; a += kBlock) buf[a - start] = *(const uint8_t*)a;
    }
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i < i1) {
      const int64_t a = off[i], len = off[i + 1] - a;
      bool r;
      if (staged)
        r = like_match(buf + ((uintptr_t)(chars + a) - start), len, spat, skind, m, ci);
      else
        r = like_match(chars + a, len, spat, skind, m, ci);
      out[i] = r != negate;
    }
  }
}

__global__ __launch_bounds__(kBlock) void case_kernel(const uint8_t* __restrict__ in, int64_t nbytes, bool to_upper,
                                                     uint8_t* __restrict__ out, int* __restrict__ non_ascii) {
  int found = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x) {
    uint8_t c = in[i];
    found |= c >= 0x80;
    if (to_upper) c = (c >= 'a' && c <= 'z') ? c - 32 : c;
    else c = (c >= 'A' && c <= 'Z') ? c + 32 : c;
    out[i] = c;
  }
  if (__any(found) && lane_id() == 0) atomicOr(non_ascii, 1);
}

// byte range [b, e) of characters [start, start+len) (1-based SQL semantics)
__device__ inline void substr_range(const uint8_t* s, int64_t n, int64_t start, int64_t len, bool has_len,
                                    int64_t* b, int64_t* e) {
  // SQL: characters from position start (1-based); start<1 shortens len
  int64_t first = start, last;  // character positions (1-based, inclusive/exclusive)
  if (has_len) {
    last = start + len;  // exclusive
    if (len < 0) last = start;
  } else {
    last = INT64_MAX;
  }
  if (first < 1) first = 1;
  int64_t pos = 1, byte = 0;
  int64_t bb = n, ee = n;
  while (byte < n) {
    if (pos == first) bb = byte;
    if (pos == last) { ee = byte; break; }
    // advance one UTF-8 character
    ++byte;
    while (byte < n && (s[byte] & 0xC0) == 0x80) ++byte;
    ++pos;
  }
  if (bb > ee) bb = ee;
  if (last <= first) bb = ee = (bb < n ? bb : n);
  *b = bb;
  *e = ee;
}

__global__ __launch_bounds__(kBlock) void substr_len_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                           int64_t n, int64_t start, int64_t len, bool has_len,
                                                           int64_t* __restrict__ out_len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = off[i], b, e;
    substr_range(chars + a, off[i + 1] - a, start, len, has_len, &b, &e);
    out_len[i] = e - b;
  }
}

__global__ __launch_bounds__(kBlock) void substr_copy_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                            int64_t n, int64_t start, int64_t len, bool has_len,
                                                            const int64_t* __restrict__ new_off, uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = off[i], b, e;
    substr_range(chars + a, off[i + 1] - a, start, len, has_len, &b, &e);
    int64_t d = new_off[i];
    for (int64_t k = b; k < e; ++k) out[d + k - b] = chars[a + k];
  }
}

__device__ inline uint64_t hash_bytes(const uint8_t* s, int64_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)n;
  int64_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) w |= (uint64_t)s[k + j] << (8 * j);
    h = mix64(h ^ w) + 0x632BE59BD9B4E019ULL;
  }
  uint64_t w = 0;
  for (int j = 0; k + j < n; ++j) w |= (uint64_t)s[k + j] << (8 * j);
  return mix64(h ^ w ^ 0xA0761D6478BD642FULL);
}

__global__ __launch_bounds__(kBlock) void hash_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                     int64_t n, const uint8_t* __restrict__ valid, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (valid && !valid[i]) { out[i] = 0x7fffffffffffff00LL; continue; }
    int64_t a = off[i];
    uint64_t h = hash_bytes(chars + a, off[i + 1] - a);
    if ((int64_t)h == kEmptyKey) h ^= 1;  // keep clear of the hash-table sentinel
    out[i] = (int64_t)h;
  }
}

__device__ inline int cmp_bytes(const uint8_t* a, int64_t na, const uint8_t* b, int64_t nb) {
  int64_t m = na < nb ? na : nb;
  for (int64_t k = 0; k < m; ++k) {
    if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
  }
  return na == nb ? 0 : (na < nb ? -1 : 1);
}

template <typename I>
__global__ __launch_bounds__(kBlock) void eq_rows_kernel(const int64_t* __restrict__ aoff, const uint8_t* __restrict__ achars,
                                                        const I* __restrict__ ai, const int64_t* __restrict__ boff,
                                                        const uint8_t* __restrict__ bchars, const I* __restrict__ bi,
                                                        int64_t n, int* __restrict__ mismatches) {
  int bad = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t x = ai ? (int64_t)ai[i] : i, y = bi ? (int64_t)bi[i] : i;
    int64_t a0 = aoff[x], b0 = boff[y];
    bad |= cmp_bytes(achars + a0, aoff[x + 1] - a0, bchars + b0, boff[y + 1] - b0) != 0;
  }
  if (__any(bad) && lane_id() == 0) atomicAdd(mismatches, 1);
}

// op: 0 '=', 1 '<>', 2 '<', 3 '<=', 4 '>', 5 '>='
__global__ __launch_bounds__(kBlock) void cmp_const_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                          int64_t n, const uint8_t* __restrict__ c, int64_t cn, int op,
                                                          uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = off[i];
    int r = cmp_bytes(chars + a, off[i + 1] - a, c, cn);
    bool v;
    switch (op) {
      case 0: v = r == 0; break;
      case 1: v = r != 0; break;
      case 2: v = r < 0; break;
      case 3: v = r <= 0; break;
      case 4: v = r > 0; break;
      default: v = r >= 0; break;
    }
    out[i] = v;
  }
}

// 8-byte big-endian prefix as an order-preserving uint64 (minus sign flip):
// first sort key for ORDER BY on strings.
__global__ __launch_bounds__(kBlock) void prefix_key_kernel(const int64_t* __restrict__ off, const uint8_t* __restrict__ chars,
                                                           int64_t n, int64_t skip, int64_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t a = off[i] + skip, e = off[i + 1];
    uint64_t k = 0;
    for (int j = 0; j < 8; ++j) k = (k << 8) | (a + j < e ? chars[a + j] : 0);
    out[i] = (int64_t)(k ^ 0x8000000000000000ULL);
  }
}

}  // namespace

void str_like(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* pat, const uint8_t* kind, int m,
              bool case_insensitive, bool negate, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  if (m <= kLikeMaxPattern)
    hipLaunchKernelGGL(like_tile_kernel, dim3(grid_for(n, kBlock, 256 * 8 * 4)), dim3(kBlock), 0, stream, off, chars, n,
                       pat, kind, m, case_insensitive, negate, out);
  else
    hipLaunchKernelGGL(like_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, pat, kind,
                       m, case_insensitive, negate, out);
  check_launch("str_like", stream);
}

void str_case(const uint8_t* in, int64_t nbytes, bool to_upper, uint8_t* out, int* non_ascii, hipStream_t stream) {
  if (nbytes == 0) return;
  hipLaunchKernelGGL(case_kernel, dim3(grid_for(nbytes, kBlock, 65536)), dim3(kBlock), 0, stream, in, nbytes, to_upper,
                     out, non_ascii);
  check_launch("str_case", stream);
}

void str_substr_lengths(const int64_t* off, const uint8_t* chars, int64_t n, int64_t start, int64_t len, bool has_len,
                        int64_t* out_len, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(substr_len_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, start,
                     len, has_len, out_len);
  check_launch("str_substr_lengths", stream);
}

void str_substr_copy(const int64_t* off, const uint8_t* chars, int64_t n, int64_t start, int64_t len, bool has_len,
                     const int64_t* new_off, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(substr_copy_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, start,
                     len, has_len, new_off, out);
  check_launch("str_substr_copy", stream);
}

void str_hash64(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* valid, int64_t* out,
                hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(hash_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, valid, out);
  check_launch("str_hash64", stream);
}

void str_eq_rows(const int64_t* aoff, const uint8_t* achars, const void* ai, const int64_t* boff, const uint8_t* bchars,
                 const void* bi, bool idx64, int64_t n, int* mismatches, hipStream_t stream) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 65536)), b(kBlock);
  if (idx64)
    hipLaunchKernelGGL(eq_rows_kernel<int64_t>, g, b, 0, stream, aoff, achars, (const int64_t*)ai, boff, bchars,
                       (const int64_t*)bi, n, mismatches);
  else
    hipLaunchKernelGGL(eq_rows_kernel<int32_t>, g, b, 0, stream, aoff, achars, (const int32_t*)ai, boff, bchars,
                       (const int32_t*)bi, n, mismatches);
  check_launch("str_eq_rows", stream);
}

void str_cmp_const(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* c, int64_t cn, int op,
                   uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(cmp_const_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, c, cn,
                     op, out);
  check_launch("str_cmp_const", stream);
}

void str_prefix_key(const int64_t* off, const uint8_t* chars, int64_t n, int64_t skip, int64_t* out,
                    hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(prefix_key_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, skip,
                     out);
  check_launch("str_prefix_key", stream);
}

}  // namespace kern
}  // namespace igloo
