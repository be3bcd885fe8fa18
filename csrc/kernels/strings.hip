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
constexpr int kLikeTileBytes = 16384;  // 256 rows of ~50-byte comments; 24.6 KB LDS per block -> 6 blocks per CU
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

// LIKE over '%'-separated literal segments (no '_', case-sensitive) — the
// shape of nearly every analytic LIKE: 'PROMO%', '%BRASS', '%green%',
// '%special%requests%'. Per tile of 256 strings staged in LDS:
//   1. every lane takes 16-byte chunks of the tile and marks, for every
//      segment, the positions where it starts: 4-byte windows built with
//      v_alignbyte from five dwords are compared against the segment prefix in
//      registers, the rare candidates are verified byte-wise, and the 16-bit
//      mask goes to an LDS bitmap (one LDS read per 16 positions);
//   2. each lane then walks its string greedily: the earliest hit of segment 0
//      at/after the cursor, then segment 1 after that, ... using bit scans.
// (A variant that prefetches the next tile into registers while matching the
// current one, with the chunk tail taken by a lane shuffle, measured 6.2 ms
// against this kernel's 5.0 ms for Q13 at SF100: the extra registers cost
// more occupancy than the overlap gained. Removing the LDS bank conflicts --
// the window's fifth dword from the neighbouring lane, mask pairs stored as
// one dword -- took them from 54M to 0.2M per suite but ran 3 % slower:
// profiles/r4_select_like_ab.txt.)
constexpr int kSegMax = 4;

__device__ inline int next_hit(const uint64_t* bits, int from, int last) {
  // smallest p in [from, last] with bit p set, or -1
  if (from > last) return -1;
  int w = from >> 6;
  uint64_t word = bits[w] & (~0ULL << (from & 63));
  const int lw = last >> 6;
  while (true) {
    if (word) {
      const int p = (w << 6) + __builtin_ctzll(word);
      return p <= last ? p : -1;
    }
    if (++w > lw) return -1;
    word = bits[w];
  }
}

// Greedy walk of one row [b0, b1) of a tile over the per-segment hit bitmaps:
// the earliest hit of segment 0 at/after the cursor, then segment 1 after it, ...
template <int SEGS, int WORDS>
__device__ inline bool seg_walk(const uint64_t (&bits)[SEGS][WORDS], const int32_t* soff, int nseg, bool anchor_start,
                                bool anchor_end, int b0, int b1) {
  int cur = b0;
  bool r = true;
  for (int sg = 0; sg < nseg && r; ++sg) {
    const int sl = soff[sg + 1] - soff[sg];
    const bool last = sg == nseg - 1;
    if (sg == 0 && anchor_start) {
      r = cur + sl <= b1 && ((bits[0][cur >> 6] >> (cur & 63)) & 1ULL);
      cur += sl;
    } else if (last && anchor_end) {
      const int p = b1 - sl;
      r = p >= cur && ((bits[sg][p >> 6] >> (p & 63)) & 1ULL);
      cur = b1;
    } else {
      const int p = next_hit(bits[sg], cur, b1 - sl);
      r = p >= 0;
      cur = p + sl;
    }
  }
  if (r && anchor_end && (nseg == 0 || (nseg == 1 && anchor_start))) r = cur == b1;
  return r;
}

// oversized tile: literal-by-literal search of one string in global memory
__device__ inline bool seg_search(const uint8_t* s, int64_t L, const uint8_t* sseg, const int32_t* soff, int nseg,
                                  bool anchor_start, bool anchor_end) {
  int64_t cur = 0;
  bool r = true;
  for (int sg = 0; sg < nseg && r; ++sg) {
    const int s0 = soff[sg], sl = soff[sg + 1] - s0;
    const bool last = sg == nseg - 1;
    auto eq = [&](int64_t p) {
      for (int k = 0; k < sl; ++k)
        if (s[p + k] != sseg[s0 + k]) return false;
      return true;
    };
    if (sg == 0 && anchor_start) {
      r = cur + sl <= L && eq(cur);
      cur += sl;
    } else if (last && anchor_end) {
      r = L - sl >= cur && eq(L - sl);
      cur = L;
    } else {
      int64_t p = cur;
      while (p + sl <= L && !eq(p)) ++p;
      r = p + sl <= L;
      cur = p + sl;
    }
  }
  if (r && anchor_end && (nseg == 0 || (nseg == 1 && anchor_start))) r = cur == L;
  return r;
}

// BLOCK threads take BLOCK consecutive strings per tile of at most TILE bytes.
// BLOCK = 64 makes every wave its own workgroup: the three tile barriers are
// single-wave barriers, and a wave waiting on its tile's loads never holds up
// the three others' matching (the 256-thread shape syncs all four per tile).
template <int BLOCK, int TILE, int SEGS = kSegMax>
__global__ __launch_bounds__(BLOCK) void like_seg_kernel(const int64_t* __restrict__ off,
                                                         const uint8_t* __restrict__ chars, int64_t n,
                                                         const uint8_t* __restrict__ seg, const int32_t* seg_off,
                                                         int nseg, bool anchor_start, bool anchor_end, bool negate,
                                                         uint8_t* __restrict__ out) {
  constexpr int kSegBits = TILE / 64;  // 64-bit words per segment bitmap
  __shared__ __attribute__((aligned(16))) uint8_t buf[TILE + 64];
  __shared__ uint64_t bits[SEGS][kSegBits];
  __shared__ uint8_t sseg[kLikeMaxPattern];
  __shared__ int32_t soff[SEGS + 1];
  const int total = seg_off[nseg];
  for (int i = threadIdx.x; i < total; i += BLOCK) sseg[i] = seg[i];
  if (threadIdx.x <= nseg) soff[threadIdx.x] = seg_off[threadIdx.x];
  const int64_t tiles = (n + BLOCK - 1) / BLOCK;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t i0 = t * BLOCK;
    const int64_t i1 = i0 + BLOCK < n ? i0 + BLOCK : n;
    const uintptr_t lo = (uintptr_t)(chars + off[i0]);
    const uintptr_t hi = (uintptr_t)(chars + off[i1]);
    const uintptr_t start = lo & ~(uintptr_t)15;
    const uintptr_t full_end = hi & ~(uintptr_t)15;
    const int len = (int)(hi - start);
    const bool staged = hi - start <= (uintptr_t)TILE;
    __syncthreads();  // previous tile done; pattern visible on the first pass
    if (staged) {
      const int64_t nvec = (int64_t)(full_end - start) / 16;
      for (int64_t v = threadIdx.x; v < nvec; v += BLOCK) *(uint4*)(buf + v * 16) = *(const uint4*)(start + v * 16);
      for (uintptr_t a = full_end + threadIdx.x; a < hi; a += BLOCK) buf[a - start] = *(const uint8_t*)a;
      if (threadIdx.x < 64) buf[len + threadIdx.x] = 0;  // pad: comparisons may read past the tile end
      __syncthreads();
      // each lane tests the 16 positions of one 16-byte chunk against every
      // segment's 4-byte prefix in registers (v_alignbyte windows), verifies
      // the rare candidates byte-wise, and stores a 16-bit hit mask
      const int nchunks = ((len + 63) >> 6) * 4;
      for (int j = threadIdx.x; j < nchunks; j += BLOCK) {
        const uint4 v = *(const uint4*)(buf + j * 16);
        const uint32_t d[5] = {v.x, v.y, v.z, v.w, *(const uint32_t*)(buf + j * 16 + 16)};
        for (int sg = 0; sg < nseg; ++sg) {
          const int s0 = soff[sg], sl = soff[sg + 1] - s0;
          const int pl = sl < 4 ? sl : 4;
          uint32_t pref = 0;
          for (int k = 0; k < pl; ++k) pref |= (uint32_t)sseg[s0 + k] << (8 * k);
          const uint32_t pmask = pl == 4 ? 0xffffffffu : ((1u << (8 * pl)) - 1);
          uint32_t m = 0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t w = __builtin_amdgcn_alignbyte(d[(q >> 2) + 1], d[q >> 2], q & 3);
            m |= (uint32_t)((w & pmask) == pref) << q;
          }
          const int base = j * 16;
          const int room = len - sl - base + 1;  // positions base+q with q < room fit in the tile
          m &= room >= 16 ? 0xffffu : room <= 0 ? 0u : ((1u << room) - 1);
          if (sl > 4) {
            for (uint32_t c = m; c; c &= c - 1) {
              const int q = __builtin_ctz(c);
              for (int k = 4; k < sl; ++k)
                if (buf[base + q + k] != sseg[s0 + k]) {
                  m &= ~(1u << q);
                  break;
                }
            }
          }
          ((uint16_t*)bits[sg])[j] = (uint16_t)m;
        }
      }
    }
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i < i1) {
      const int64_t a = off[i], e = off[i + 1];
      const bool r = staged ? seg_walk(bits, soff, nseg, anchor_start, anchor_end,
                                       (int)((uintptr_t)(chars + a) - start), (int)((uintptr_t)(chars + e) - start))
                            : seg_search(chars + a, e - a, sseg, soff, nseg, anchor_start, anchor_end);
      out[i] = r != negate;
    }
  }
}

// Segments of >= 7 bytes ('%special%requests%', '%Customer%Complaints%'):
// every occurrence at position p contains the aligned dword at a = p rounded
// up to 4, and that dword equals the segment's bytes a-p .. a-p+3 (a-p < 4,
// a-p+3 <= 6 < length). So the positions p of a 16-byte chunk can only hold a
// hit if one of the chunk's 5 aligned dwords equals one of the segment's 4
// leading dword windows: 16 plain compares per chunk and segment, no byte
// windows -- the byte-exact test (v_alignbyte windows + verification) runs
// only for the chunks that pass, gathered into a per-wave LDS list so the
// wave runs them densely instead of idling lanes on a divergent branch.
// Chunks come straight from global memory (16-byte loads, the fifth dword
// from the same lines); LDS holds only the hit bitmaps and the lists.
constexpr int kLikeDwordTile = 32768;

template <int SEGS, int TILE, int kU>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void like_dword_kernel(const int64_t* __restrict__ off,
                                                           const uint8_t* __restrict__ chars, int64_t n,
                                                           const uint8_t* __restrict__ seg, const int32_t* seg_off,
                                                           int nseg, bool anchor_start, bool anchor_end, bool negate,
                                                           uint8_t* __restrict__ out, int64_t nbytes) {
  constexpr int kWords = TILE / 64;
  constexpr int kChunks = TILE / 16;
  constexpr int kListLen = kChunks / kWavesPerBlock + kWave;
  __shared__ uint64_t bits[SEGS][kWords];
  __shared__ uint16_t cand[kWavesPerBlock][kListLen];
  constexpr int kDataCap = 64;   // listed chunks whose bytes are kept in LDS (later ones are reloaded)
  __shared__ uint32_t cdat[kWavesPerBlock][5][kDataCap];
  __shared__ uint8_t sseg[kLikeMaxPattern];
  __shared__ int32_t soff[SEGS + 1];
  const int total = seg_off[nseg];
  for (int i = threadIdx.x; i < total; i += kBlock) sseg[i] = seg[i];
  if (threadIdx.x <= nseg) soff[threadIdx.x] = seg_off[threadIdx.x];
  __syncthreads();
  uint32_t P[SEGS][4];
#pragma unroll
  for (int sg = 0; sg < SEGS; ++sg)
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      const int s0 = soff[sg < nseg ? sg : 0] + o;
      // wave-uniform: kept in scalar registers (compares take an SGPR operand)
      P[sg][o] = __builtin_amdgcn_readfirstlane((uint32_t)sseg[s0] | ((uint32_t)sseg[s0 + 1] << 8) |
                                                ((uint32_t)sseg[s0 + 2] << 16) | ((uint32_t)sseg[s0 + 3] << 24));
    }
  const int wave = threadIdx.x / kWave, lane = lane_id();
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  const uint8_t* const chars_end = chars + nbytes;
  // the tile's byte range is known one tile ahead (no offsets -> chars load chain)
  int64_t t_lo = 0, t_hi = 0;
  if ((int64_t)blockIdx.x < tiles) {
    const int64_t f0 = (int64_t)blockIdx.x * kBlock;
    t_lo = off[f0];
    t_hi = off[f0 + kBlock < n ? f0 + kBlock : n];
  }
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t i0 = t * kBlock;
    const int64_t i1 = i0 + kBlock < n ? i0 + kBlock : n;
    const int64_t i = i0 + threadIdx.x;
    // this row's bounds now: their loads overlap the tile's matching
    const int64_t ra = i < i1 ? off[i] : 0, re = i < i1 ? off[i + 1] : 0;
    const uintptr_t lo = (uintptr_t)(chars + t_lo);
    const uintptr_t hi = (uintptr_t)(chars + t_hi);
    {
      const int64_t tn = t + gridDim.x;
      if (tn < tiles) {
        const int64_t f0 = tn * kBlock;
        t_lo = off[f0];
        t_hi = off[f0 + kBlock < n ? f0 + kBlock : n];
      }
    }
    const uintptr_t start = lo & ~(uintptr_t)15;   // never below the allocation (>= 256 B aligned)
    const int len = (int)(hi - start);
    const bool fits = hi - start <= (uintptr_t)TILE;
    const uint8_t* base = (const uint8_t*)start;
    // 20 bytes from chunk j (16 B and the next dword). Bytes past the tile
    // are the next rows' (positions that would need them are masked by
    // `room`); only the buffer's last bytes are read one by one.
    const int64_t avail = chars_end - base;
    auto load = [&](int j, uint32_t d[5]) {
      const int b = j * 16;
      if (b + 20 <= avail) {
        const uint4 v = *(const uint4*)(base + b);
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        d[4] = *(const uint32_t*)(base + b + 16);
      } else {
#pragma unroll
        for (int w = 0; w < 5; ++w) {
          uint32_t x = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (b + 4 * w + k < avail) x |= (uint32_t)base[b + 4 * w + k] << (8 * k);
          d[w] = x;
        }
      }
    };
    __syncthreads();   // the previous tile's walk is done with the bitmaps
    if (fits) {
      const int nchunks = (len + 15) >> 4;
      int ncand = 0;
      // kU chunks per lane in flight: all loads issued before any compare
      for (int j0 = wave * kWave; j0 < nchunks; j0 += kU * kBlock) {
        uint32_t d[kU][5];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = j0 + u * kBlock + lane;
          if (j < nchunks) load(j, d[u]);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int j = j0 + u * kBlock + lane;
          if (j0 + u * kBlock >= nchunks) break;   // wave-uniform
          bool any = false;
          if (j < nchunks) {
#pragma unroll
            for (int sg = 0; sg < SEGS; ++sg) {
              if (sg >= nseg) break;
              bool f = d[u][0] == P[sg][0];
#pragma unroll
              for (int w = 1; w < 4; ++w)
                f |= (d[u][w] == P[sg][0]) | (d[u][w] == P[sg][1]) | (d[u][w] == P[sg][2]) | (d[u][w] == P[sg][3]);
              f |= (d[u][4] == P[sg][1]) | (d[u][4] == P[sg][2]) | (d[u][4] == P[sg][3]);
              any |= f;
              ((uint16_t*)bits[sg])[j] = 0;
            }
          }
          const uint64_t bal = __ballot(any);
          if (any) {
            const int c = ncand + lane_prefix(bal);
            cand[wave][c] = (uint16_t)j;
            if (c < kDataCap)
#pragma unroll
              for (int w = 0; w < 5; ++w) cdat[wave][w][c] = d[u][w];
          }
          ncand += __popcll(bal);
        }
      }
      // byte-exact masks for the listed chunks (same wave: ordered after the zeroing)
      for (int c = lane; c < ncand; c += kWave) {
        const int j = cand[wave][c];
        uint32_t d[5];
        if (c < kDataCap) {
#pragma unroll
          for (int w = 0; w < 5; ++w) d[w] = cdat[wave][w][c];
        } else {
          load(j, d);
        }
        const int b = j * 16;
#pragma unroll
        for (int sg = 0; sg < SEGS; ++sg) {
          if (sg >= nseg) break;
          const int s0 = soff[sg], sl = soff[sg + 1] - s0;
          uint32_t m = 0;
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const uint32_t w = __builtin_amdgcn_alignbyte(d[(q >> 2) + 1], d[q >> 2], q & 3);
            m |= (uint32_t)(w == P[sg][0]) << q;
          }
          const int room = len - sl - b + 1;
          m &= room >= 16 ? 0xffffu : room <= 0 ? 0u : ((1u << room) - 1);
          for (uint32_t c2 = m; c2; c2 &= c2 - 1) {
            const int q = __builtin_ctz(c2);
            for (int k = 4; k < sl; ++k)
              if (base[b + q + k] != sseg[s0 + k]) {
                m &= ~(1u << q);
                break;
              }
          }
          ((uint16_t*)bits[sg])[j] = (uint16_t)m;
        }
      }
    }
    __syncthreads();
    if (i < i1) {
      const bool r = fits ? seg_walk(bits, soff, nseg, anchor_start, anchor_end,
                                     (int)((uintptr_t)(chars + ra) - start), (int)((uintptr_t)(chars + re) - start))
                          : seg_search(chars + ra, re - ra, sseg, soff, nseg, anchor_start, anchor_end);
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

// String IN (constants) in one pass: row i is set when its bytes equal one of
// the nv constants vb[voff[v] .. voff[v+1]) -- or, with vmode[v] = 1, start
// with them (substr(x, 1, L) IN (...) for a constant of exactly L code points;
// UTF-8 is self-synchronising, so a byte prefix of L code points is the
// substring). Replaces one compare pass per constant plus the substring copy
// (TPC-H Q22's country codes: 7 passes over 15M phone numbers).
constexpr int kInSetWords = 256;   // constants staged in LDS as words

__global__ __launch_bounds__(kBlock) void in_set_kernel(const int64_t* __restrict__ off,
                                                       const uint8_t* __restrict__ chars, int64_t n,
                                                       const uint8_t* __restrict__ vb, const int32_t* __restrict__ voff,
                                                       const uint8_t* __restrict__ vmode, int nv,
                                                       uint8_t* __restrict__ out) {
  // constants of at most 8 bytes (the usual case: codes, flags, short names)
  // compare as masked words against the row's first bytes, loaded once; the
  // constants' words, lengths and modes are built once per workgroup in LDS
  // (not re-read byte by byte from global memory for every row)
  __shared__ uint64_t cword[kInSetWords];
  __shared__ int32_t clen[kInSetWords];
  int maxb = 0;
  for (int v = 0; v < nv; ++v) maxb = max(maxb, voff[v + 1] - voff[v]);
  const bool words = maxb <= 8;
  const bool staged = words && nv <= kInSetWords;
  if (staged) {
    for (int v = threadIdx.x; v < nv; v += blockDim.x) {
      const int32_t c0 = voff[v], vl = voff[v + 1] - c0;
      uint64_t cw = 0;
      for (int32_t j = 0; j < vl; ++j) cw |= (uint64_t)vb[c0 + j] << (8 * j);
      cword[v] = cw;
      clen[v] = vmode[v] ? -vl - 1 : vl;   // negative: prefix match of length -clen-1
    }
    __syncthreads();
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = off[i], len = off[i + 1] - a;
    bool hit = false;
    if (staged) {
      const int nb = len < maxb ? (int)len : maxb;
      uint64_t w = 0;
      for (int j = 0; j < nb; ++j) w |= (uint64_t)chars[a + j] << (8 * j);
      for (int v = 0; v < nv && !hit; ++v) {
        const int32_t cl = clen[v];
        const int32_t vl = cl < 0 ? -cl - 1 : cl;
        if (cl < 0 ? len < vl : len != vl) continue;
        const uint64_t m = vl >= 8 ? ~0ull : ((1ull << (8 * vl)) - 1);
        hit = (w & m) == cword[v];
      }
    } else if (words) {
      const int nb = len < maxb ? (int)len : maxb;
      uint64_t w = 0;
      for (int j = 0; j < nb; ++j) w |= (uint64_t)chars[a + j] << (8 * j);
      for (int v = 0; v < nv && !hit; ++v) {
        const int32_t c0 = voff[v], vl = voff[v + 1] - c0;
        if (vmode[v] ? len < vl : len != vl) continue;
        uint64_t cw = 0;
        for (int32_t j = 0; j < vl; ++j) cw |= (uint64_t)vb[c0 + j] << (8 * j);
        const uint64_t m = vl >= 8 ? ~0ull : ((1ull << (8 * vl)) - 1);
        hit = (w & m) == cw;
      }
    } else {
      for (int v = 0; v < nv && !hit; ++v) {
        const int32_t c0 = voff[v], vl = voff[v + 1] - c0;
        if (vmode[v] ? len < vl : len != vl) continue;
        bool eq = true;
        for (int32_t j = 0; j < vl && eq; ++j) eq = chars[a + j] == vb[c0 + j];
        hit = eq;
      }
    }
    out[i] = hit;
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

void str_like_segments(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* seg, const int32_t* seg_off,
                       int nseg, bool anchor_start, bool anchor_end, bool negate, uint8_t* out, int64_t nbytes,
                       int min_seg, hipStream_t stream) {
  if (n == 0) return;
  if (nseg > kSegMax) throw std::runtime_error("str_like_segments: too many segments");
  const bool dword_filter = !debug_flag("like_nodword");
  if (dword_filter && nseg >= 1 && nseg <= 2 && min_seg >= 7) {
    const dim3 g(grid_for(n, kBlock, 256 * 8 * 4)), b(kBlock);
    constexpr int u = 1;   // (2 and 4 rows per lane measured no faster: profiles/r5_ab_like_*.txt)
#define IGLOO_LIKE_DWORD(S, U)                                                                                  \
  hipLaunchKernelGGL((like_dword_kernel<S, kLikeDwordTile, U>), g, b, 0, stream, off, chars, n, seg, seg_off, nseg, \
                     anchor_start, anchor_end, negate, out, nbytes)
    if (nseg == 1) {
      if (u >= 4) IGLOO_LIKE_DWORD(1, 4);
      else if (u == 2) IGLOO_LIKE_DWORD(1, 2);
      else IGLOO_LIKE_DWORD(1, 1);
    } else {
      if (u >= 4) IGLOO_LIKE_DWORD(2, 4);
      else if (u == 2) IGLOO_LIKE_DWORD(2, 2);
      else IGLOO_LIKE_DWORD(2, 1);
    }
#undef IGLOO_LIKE_DWORD
    check_launch("str_like_segments", stream);
    return;
  }
  // (a one-wave-per-workgroup variant with 4 / 8 KB tiles measured slower for
  // Q13 at SF100, 14.6 vs 11.7 ms per query: profiles/r3_ab_like_wave.txt)
  // one or two segments (nearly every analytic LIKE): a bitmap sized for
  // them frees 4-6 KB of LDS per workgroup, one or two more resident
  // workgroups per CU (-9 % / -10 % for two / one segment,
  // profiles/r4_select_like_ab.txt)
  if (nseg <= 1)
    hipLaunchKernelGGL((like_seg_kernel<kBlock, kLikeTileBytes, 1>), dim3(grid_for(n, kBlock, 256 * 8 * 4)),
                       dim3(kBlock), 0, stream, off, chars, n, seg, seg_off, nseg, anchor_start, anchor_end, negate, out);
  else if (nseg <= 2)
    hipLaunchKernelGGL((like_seg_kernel<kBlock, kLikeTileBytes, 2>), dim3(grid_for(n, kBlock, 256 * 8 * 4)),
                       dim3(kBlock), 0, stream, off, chars, n, seg, seg_off, nseg, anchor_start, anchor_end, negate, out);
  else
    hipLaunchKernelGGL((like_seg_kernel<kBlock, kLikeTileBytes>), dim3(grid_for(n, kBlock, 256 * 8 * 4)), dim3(kBlock),
                       0, stream, off, chars, n, seg, seg_off, nseg, anchor_start, anchor_end, negate, out);
  check_launch("str_like_segments", stream);
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

// Order-preserving 8-byte chunks of each string: out[k * n + i] holds bytes
// [8k, 8k + 8) of string i big-endian, zero padded (a shorter string sorts
// first on a common prefix, as in byte-wise UTF-8 order), sign bit flipped so
// signed int64 order equals unsigned byte order. An LSD sort over the chunks
// (last chunk first) orders the strings: ops/strings.py sort_ranks.
__global__ __launch_bounds__(kBlock) void prefix_keys_kernel(const int64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ chars, int64_t n,
                                                             int chunks, int64_t* __restrict__ out) {
  const int64_t total = n * chunks;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / n, i = t - k * n;
    const int64_t a = off[i], len = off[i + 1] - a, b0 = 8 * k;
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t p = b0 + j;
      v = (v << 8) | (p < len ? (uint64_t)chars[a + p] : 0u);
    }
    out[t] = (int64_t)(v ^ 0x8000000000000000ull);
  }
}

void str_prefix_keys(const int64_t* off, const uint8_t* chars, int64_t n, int chunks, int64_t* out,
                     hipStream_t stream) {
  if (n == 0 || chunks <= 0) return;
  hipLaunchKernelGGL(prefix_keys_kernel, dim3(grid_for(n * chunks, kBlock, 65536)), dim3(kBlock), 0, stream, off,
                     chars, n, chunks, out);
  check_launch("str_prefix_keys", stream);
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

void str_in_set(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* vb, const int32_t* voff,
                const uint8_t* vmode, int nv, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(in_set_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, vb, voff,
                     vmode, nv, out);
  check_launch("str_in_set", stream);
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
