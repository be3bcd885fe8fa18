// MFMA hash / compare experiment: the two SQL shapes
// where a matrix instruction could replace VALU work, each as a VALU kernel
// and an MFMA kernel over the same data, so rocprofv3 counters
// (SQ_INSTS_MFMA, SQ_INSTS_VALU, FETCH_SIZE) and times compare them
// (scripts/mfma_hash_ab.py; decision in BASELINE.md).
//
// (a) composite-key hashing (multi-column GROUP BY / join keys, Q9 / Q18 /
//     Q21 shapes): 16 key bytes per row (four int32 columns).
//     VALU: two 64-bit mixes. MFMA: v_mfma_i32_16x16x64_i8 projects 16 rows'
//     key bytes onto 16 fixed random int8 directions (D = X . R), then every
//     lane mixes its 4 projections and the 16 lanes of a row XOR-reduce.
// (b) IN-list candidate compare (Q12 / Q16 / Q19 / Q22 shapes): a string's
//     first 16 bytes against up to 16 patterns of one length L.
//     VALU: masked 2 x 64-bit compares per pattern. MFMA: D = X . P
//     (16 rows x 16 patterns per instruction) and |x - p|^2 = x.x - 2 D + p.p
//     (x.x by v_dot4), zero <=> equal; a row's hit is a ballot over its
//     16 pattern lanes.
// Operand layout of v_mfma_i32_16x16x64_i8 (gfx950, as in fused.hip): lane l
// holds A[row l & 15][k = 16 (l >> 4) + j] and B[k = 16 (l >> 4) + j][col
// l & 15] (j < 16); D: col = l & 15, row = 4 (l >> 4) + i (i < 4). Only
// k < 16 carries data here (lanes 0..15); the other k are zero.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

// ---- (a) composite-key hash
__global__ __launch_bounds__(kBlock) void hash16_valu_kernel(const int32_t* __restrict__ k0,
                                                           const int32_t* __restrict__ k1,
                                                           const int32_t* __restrict__ k2,
                                                           const int32_t* __restrict__ k3, int64_t n,
                                                           uint32_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t a = (uint64_t)(uint32_t)k0[r] | ((uint64_t)(uint32_t)k1[r] << 32);
    const uint64_t b = (uint64_t)(uint32_t)k2[r] | ((uint64_t)(uint32_t)k3[r] << 32);
    out[r] = (uint32_t)(mix64(a) ^ (mix64(b) * 0x9e3779b97f4a7c15ull >> 7));
  }
}

// one wave = 64 rows per iteration: 4 MFMA steps of 16 rows each
__global__ __launch_bounds__(kBlock) void hash16_mfma_kernel(const int32_t* __restrict__ k0,
                                                           const int32_t* __restrict__ k1,
                                                           const int32_t* __restrict__ k2,
                                                           const int32_t* __restrict__ k3, int64_t n,
                                                           const int8_t* __restrict__ proj,   // [16 k][16 cols]
                                                           uint32_t* __restrict__ out) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) / kWave;
  // B fragment: lanes 0..15 hold R[k = 0..15][col = lane]; other k are zero
  v4i bf = {0, 0, 0, 0};
  if (lane < 16) {
    uint32_t w[4];
    for (int q = 0; q < 4; ++q) {
      uint32_t v = 0;
      for (int j = 0; j < 4; ++j) v |= (uint32_t)(uint8_t)proj[(4 * q + j) * 16 + lane] << (8 * j);
      w[q] = v;
    }
    bf = v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
  }
  for (int64_t base = wave * kWave; base < n; base += nw * kWave) {
    const int64_t r = base + lane;
    const bool ok = r < n;
    const int x0 = ok ? k0[r] : 0, x1 = ok ? k1[r] : 0, x2 = ok ? k2[r] : 0, x3 = ok ? k3[r] : 0;
    uint32_t h = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // rows 16 s .. 16 s + 15 of the tile into the A fragment of lanes 0..15
      const int src = 16 * s + (lane & 15);
      const int y0 = __shfl(x0, src, kWave), y1 = __shfl(x1, src, kWave), y2 = __shfl(x2, src, kWave),
                y3 = __shfl(x3, src, kWave);
      const v4i af = lane < 16 ? v4i{y0, y1, y2, y3} : v4i{0, 0, 0, 0};
      const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, v4i{0, 0, 0, 0}, 0, 0, 0);
      // lane holds D[row 4 (lane >> 4) + i][col lane & 15]: mix, XOR over the
      // row's 16 lanes (xor offsets < 16 stay in the group), then lane R of
      // the tile (row R = 16 s + 4 g + i) takes it from group g's first lane
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t v = fmix32((uint32_t)d[i] + 0x9e3779b9u * (uint32_t)(lane & 15));
        v ^= __shfl_xor(v, 1, kWave);
        v ^= __shfl_xor(v, 2, kWave);
        v ^= __shfl_xor(v, 4, kWave);
        v ^= __shfl_xor(v, 8, kWave);
        const uint32_t t = __shfl(v, 16 * ((lane & 15) >> 2), kWave);
        if ((lane >> 4) == s && (lane & 3) == i) h = t;
      }
    }
    if (ok) out[r] = h;
  }
}

// ---- (b) IN-list compare over the first 16 bytes
struct InList16 {
  uint64_t lo[16], hi[16];   // patterns (zero-padded)
  uint64_t mlo, mhi;         // byte mask of the first L bytes
  int npat, len;
  int pnorm[16];             // sum of the pattern's squared bytes (int8)
};

__device__ __forceinline__ void load16(const uint8_t* p, int64_t avail, uint64_t* lo, uint64_t* hi) {
  uint64_t a = 0, b = 0;
  for (int j = 0; j < 16; ++j) {
    const uint64_t v = j < avail ? p[j] : 0;
    if (j < 8) a |= v << (8 * j);
    else b |= v << (8 * (j - 8));
  }
  *lo = a;
  *hi = b;
}

__global__ __launch_bounds__(kBlock) void inlist16_valu_kernel(const int64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ chars, int64_t n, InList16 P,
                                                             uint8_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = off[r], len = off[r + 1] - o;
    uint64_t lo, hi;
    load16(chars + o, len < 16 ? len : 16, &lo, &hi);
    lo &= P.mlo;
    hi &= P.mhi;
    bool hit = false;
    for (int p = 0; p < P.npat; ++p) hit |= (lo == P.lo[p]) & (hi == P.hi[p]);
    out[r] = hit && len == P.len;
  }
}

__global__ __launch_bounds__(kBlock) void inlist16_mfma_kernel(const int64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ chars, int64_t n, InList16 P,
                                                             uint8_t* __restrict__ out) {
  const int lane = lane_id();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int col = lane & 15;
  v4i bf = {0, 0, 0, 0};
  if (lane < 16 && col < P.npat)
    bf = v4i{(int)(uint32_t)P.lo[col], (int)(uint32_t)(P.lo[col] >> 32), (int)(uint32_t)P.hi[col],
             (int)(uint32_t)(P.hi[col] >> 32)};
  const int pn = col < P.npat ? P.pnorm[col] : 0x7fffffff;
  for (int64_t base = wave * kWave; base < n; base += nw * kWave) {
    const int64_t r = base + lane;
    const bool ok = r < n;
    int64_t len = 0;
    uint64_t lo = 0, hi = 0;
    if (ok) {
      const int64_t o = off[r];
      len = off[r + 1] - o;
      load16(chars + o, len < 16 ? len : 16, &lo, &hi);
      lo &= P.mlo;
      hi &= P.mhi;
    }
    const int w0 = (int)(uint32_t)lo, w1 = (int)(uint32_t)(lo >> 32), w2 = (int)(uint32_t)hi,
              w3 = (int)(uint32_t)(hi >> 32);
    // |x|^2 over signed bytes: four v_dot4_i32_i8
    int xn = __builtin_amdgcn_sdot4(w0, w0, 0, false);
    xn = __builtin_amdgcn_sdot4(w1, w1, xn, false);
    xn = __builtin_amdgcn_sdot4(w2, w2, xn, false);
    xn = __builtin_amdgcn_sdot4(w3, w3, xn, false);
    const bool len_ok = ok && len == P.len;
    uint8_t mine = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int src = 16 * s + (lane & 15);
      const int y0 = __shfl(w0, src, kWave), y1 = __shfl(w1, src, kWave), y2 = __shfl(w2, src, kWave),
                y3 = __shfl(w3, src, kWave);
      const v4i af = lane < 16 ? v4i{y0, y1, y2, y3} : v4i{0, 0, 0, 0};
      const v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf, v4i{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // row 16 s + 4 (lane >> 4) + i of the tile: its |x|^2 from the lane that loaded it
        const int rxn = __shfl(xn, 16 * s + 4 * (lane >> 4) + i, kWave);
        const bool eq = col < P.npat && rxn - 2 * d[i] + pn == 0;
        const uint64_t bal = __ballot(eq);
        const int any = ((bal >> (16 * (lane >> 4))) & 0xFFFFull) != 0;
        const int t = __shfl(any, 16 * ((lane & 15) >> 2), kWave);
        if ((lane >> 4) == s && (lane & 3) == i) mine = (uint8_t)t;
      }
    }
    if (ok) out[r] = mine && len_ok;
  }
}

}  // namespace

void probe_hash16(bool mfma, const int32_t* k0, const int32_t* k1, const int32_t* k2, const int32_t* k3, int64_t n,
                  const int8_t* proj, uint32_t* out, hipStream_t s) {
  if (n == 0) return;
  const dim3 g(grid_for(n, kBlock, 1 << 14)), b(kBlock);
  if (mfma) hipLaunchKernelGGL(hash16_mfma_kernel, g, b, 0, s, k0, k1, k2, k3, n, proj, out);
  else hipLaunchKernelGGL(hash16_valu_kernel, g, b, 0, s, k0, k1, k2, k3, n, out);
  check_launch("probe_hash16", s);
}

void probe_inlist16(bool mfma, const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* pats, int npat,
                    int len, uint8_t* out, hipStream_t s) {
  if (npat < 1 || npat > 16 || len < 1 || len > 16) throw std::runtime_error("probe_inlist16: 1..16 patterns of 1..16 bytes");
  InList16 P{};
  P.npat = npat;
  P.len = len;
  P.mlo = len >= 8 ? ~0ull : ((1ull << (8 * len)) - 1);
  P.mhi = len <= 8 ? 0ull : (len >= 16 ? ~0ull : ((1ull << (8 * (len - 8))) - 1));
  for (int p = 0; p < npat; ++p) {
    uint64_t lo = 0, hi = 0;
    int nrm = 0;
    for (int j = 0; j < len; ++j) {
      const uint8_t c = pats[p * 16 + j];
      if (j < 8) lo |= (uint64_t)c << (8 * j);
      else hi |= (uint64_t)c << (8 * (j - 8));
      const int v = (int8_t)c;
      nrm += v * v;
    }
    P.lo[p] = lo;
    P.hi[p] = hi;
    P.pnorm[p] = nrm;
  }
  const dim3 g(grid_for(n, kBlock, 1 << 14)), b(kBlock);
  if (mfma) hipLaunchKernelGGL(inlist16_mfma_kernel, g, b, 0, s, off, chars, n, P, out);
  else hipLaunchKernelGGL(inlist16_valu_kernel, g, b, 0, s, off, chars, n, P, out);
  check_launch("probe_inlist16", s);
}

}  // namespace kern
}  // namespace igloo
