// Cryptographic digests of string columns: md5, sha224, sha256, sha384,
// sha512 (DataFusion's md5 / sha2 family / digest(), reference
// Cargo.lock:1062-1090 datafusion-functions with md-5 and sha2).
//
// One lane per row: the lane walks its string in 64-byte (md5, sha-256) or
// 128-byte (sha-512) blocks straight from HBM, applies the final padding
// block(s) in registers, and writes the lowercase hex digest at row * width
// of a fixed-width output (offsets are row * width). The message schedule is
// a rolling 16-word window (w[i & 15]) so SHA-512 keeps 16 x 64-bit words in
// VGPRs instead of 80. A dictionary-coded column is hashed once per
// dictionary entry and the codes gather the result (host side).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// byte k of the padded message (length len bytes): data, 0x80, zeros, then the
// bit length (little-endian for md5, big-endian for sha) in the last lenbytes
__device__ __forceinline__ uint8_t padded_byte(const uint8_t* s, int64_t len, int64_t total, int64_t k,
                                               bool little, int lenbytes) {
  if (k < len) return s[k];
  if (k == len) return 0x80;
  const int64_t tail = total - lenbytes;
  if (k < tail) return 0;
  const int j = (int)(k - tail);     // 0 .. lenbytes-1
  const uint64_t bits = (uint64_t)len * 8ull;
  int shift;
  if (little) shift = 8 * j;
  else shift = 8 * (lenbytes - 1 - j);
  return shift >= 64 ? 0 : (uint8_t)(bits >> shift);
}

// ---------------------------------------------------------------- md5
__constant__ uint32_t kMd5K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
__constant__ int kMd5S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

__device__ void md5(const uint8_t* s, int64_t len, uint32_t h[4]) {
  h[0] = 0x67452301;
  h[1] = 0xefcdab89;
  h[2] = 0x98badcfe;
  h[3] = 0x10325476;
  const int64_t total = ((len + 8) / 64 + 1) * 64;
  for (int64_t blk = 0; blk < total; blk += 64) {
    uint32_t m[16];
    const bool full = blk + 64 <= len;
    for (int i = 0; i < 16; ++i) {
      uint32_t w = 0;
      for (int b = 0; b < 4; ++b) {
        const int64_t k = blk + 4 * i + b;
        const uint8_t v = full ? s[k] : padded_byte(s, len, total, k, true, 8);
        w |= (uint32_t)v << (8 * b);
      }
      m[i] = w;
    }
    uint32_t a = h[0], bb = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
      uint32_t f;
      int g;
      if (i < 16) {
        f = (bb & c) | (~bb & d);
        g = i;
      } else if (i < 32) {
        f = (d & bb) | (~d & c);
        g = (5 * i + 1) & 15;
      } else if (i < 48) {
        f = bb ^ c ^ d;
        g = (3 * i + 5) & 15;
      } else {
        f = c ^ (bb | ~d);
        g = (7 * i) & 15;
      }
      const uint32_t tmp = d;
      d = c;
      c = bb;
      bb = bb + rotl32(a + f + kMd5K[i] + m[g], kMd5S[i]);
      a = tmp;
    }
    h[0] += a;
    h[1] += bb;
    h[2] += c;
    h[3] += d;
  }
}

// ---------------------------------------------------------------- sha-256
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ void sha256(const uint8_t* s, int64_t len, bool is224, uint32_t h[8]) {
  if (is224) {
    const uint32_t iv[8] = {0xc1059ed8, 0x367cd507, 0x3070dd17, 0xf70e5939,
                            0xffc00b31, 0x68581511, 0x64f98fa7, 0xbefa4fa4};
    for (int i = 0; i < 8; ++i) h[i] = iv[i];
  } else {
    const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                            0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    for (int i = 0; i < 8; ++i) h[i] = iv[i];
  }
  const int64_t total = ((len + 8) / 64 + 1) * 64;
  for (int64_t blk = 0; blk < total; blk += 64) {
    uint32_t w[16];
    const bool full = blk + 64 <= len;
    for (int i = 0; i < 16; ++i) {
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b) {
        const int64_t k = blk + 4 * i + b;
        const uint8_t v = full ? s[k] : padded_byte(s, len, total, k, false, 8);
        x = (x << 8) | v;
      }
      w[i] = x;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; ++i) {
      uint32_t wi;
      if (i < 16) {
        wi = w[i];
      } else {
        const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
        const uint32_t s0 = rotr32(w15, 7) ^ rotr32(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr32(w2, 17) ^ rotr32(w2, 19) ^ (w2 >> 10);
        wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      }
      const uint32_t S1 = rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + kSha256K[i] + wi;
      const uint32_t S0 = rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
}

// ---------------------------------------------------------------- sha-512
__constant__ uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};

__device__ void sha512(const uint8_t* s, int64_t len, bool is384, uint64_t h[8]) {
  if (is384) {
    const uint64_t iv[8] = {0xcbbb9d5dc1059ed8ull, 0x629a292a367cd507ull, 0x9159015a3070dd17ull,
                            0x152fecd8f70e5939ull, 0x67332667ffc00b31ull, 0x8eb44a8768581511ull,
                            0xdb0c2e0d64f98fa7ull, 0x47b5481dbefa4fa4ull};
    for (int i = 0; i < 8; ++i) h[i] = iv[i];
  } else {
    const uint64_t iv[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                            0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                            0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
    for (int i = 0; i < 8; ++i) h[i] = iv[i];
  }
  const int64_t total = ((len + 16) / 128 + 1) * 128;
  for (int64_t blk = 0; blk < total; blk += 128) {
    uint64_t w[16];
    const bool full = blk + 128 <= len;
    for (int i = 0; i < 16; ++i) {
      uint64_t x = 0;
      for (int b = 0; b < 8; ++b) {
        const int64_t k = blk + 8 * i + b;
        const uint8_t v = full ? s[k] : padded_byte(s, len, total, k, false, 16);
        x = (x << 8) | v;
      }
      w[i] = x;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 80; ++i) {
      uint64_t wi;
      if (i < 16) {
        wi = w[i];
      } else {
        const uint64_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
        const uint64_t s0 = rotr64(w15, 1) ^ rotr64(w15, 8) ^ (w15 >> 7);
        const uint64_t s1 = rotr64(w2, 19) ^ rotr64(w2, 61) ^ (w2 >> 6);
        wi = w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      }
      const uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
      const uint64_t ch = (e & f) ^ (~e & g);
      const uint64_t t1 = hh + S1 + ch + kSha512K[i] + wi;
      const uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
      const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint64_t t2 = S0 + mj;
      hh = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = b;
      b = a;
      a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
}

__device__ __forceinline__ void put_hex(uint8_t* o, uint8_t v) {
  const char* hx = "0123456789abcdef";
  o[0] = (uint8_t)hx[v >> 4];
  o[1] = (uint8_t)hx[v & 15];
}

__global__ __launch_bounds__(kBlock) void digest_hex_kernel(int algo, const int64_t* __restrict__ off,
                                                          const uint8_t* __restrict__ chars, int64_t n,
                                                          uint8_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = off[r], len = off[r + 1] - b;
    const uint8_t* s = chars + b;
    if (algo == kDigestMd5) {
      uint32_t h[4];
      md5(s, len, h);
      uint8_t* o = out + r * 32;
      for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k) put_hex(o + 8 * i + 2 * k, (uint8_t)(h[i] >> (8 * k)));   // little-endian
    } else if (algo == kDigestSha224 || algo == kDigestSha256) {
      uint32_t h[8];
      sha256(s, len, algo == kDigestSha224, h);
      const int words = algo == kDigestSha224 ? 7 : 8;
      uint8_t* o = out + r * (int64_t)(8 * words);
      for (int i = 0; i < words; ++i)
        for (int k = 0; k < 4; ++k) put_hex(o + 8 * i + 2 * k, (uint8_t)(h[i] >> (24 - 8 * k)));
    } else {
      uint64_t h[8];
      sha512(s, len, algo == kDigestSha384, h);
      const int words = algo == kDigestSha384 ? 6 : 8;
      uint8_t* o = out + r * (int64_t)(16 * words);
      for (int i = 0; i < words; ++i)
        for (int k = 0; k < 8; ++k) put_hex(o + 16 * i + 2 * k, (uint8_t)(h[i] >> (56 - 8 * k)));
    }
  }
}

// ---------------------------------------------------------------- uuid v4
// 128 random bits per row from a counter-based mixer (seed, row), version 4
// and RFC 4122 variant bits set, formatted 8-4-4-4-12.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void uuid_kernel(uint64_t seed, int64_t n, uint8_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    uint64_t hi = mix64(seed ^ mix64((uint64_t)r * 2 + 1));
    uint64_t lo = mix64(hi ^ seed ^ ((uint64_t)r << 1));
    hi = (hi & ~0xF000ull) | 0x4000ull;                      // version 4
    lo = (lo & 0x3FFFFFFFFFFFFFFFull) | 0x8000000000000000ull;  // variant 10
    uint8_t bytes[16];
    for (int k = 0; k < 8; ++k) {
      bytes[k] = (uint8_t)(hi >> (56 - 8 * k));
      bytes[8 + k] = (uint8_t)(lo >> (56 - 8 * k));
    }
    uint8_t* o = out + r * 36;
    int p = 0;
    for (int k = 0; k < 16; ++k) {
      if (k == 4 || k == 6 || k == 8 || k == 10) o[p++] = '-';
      put_hex(o + p, bytes[k]);
      p += 2;
    }
  }
}

}  // namespace

int digest_width(int algo) {
  switch (algo) {
    case kDigestMd5: return 32;
    case kDigestSha224: return 56;
    case kDigestSha256: return 64;
    case kDigestSha384: return 96;
    case kDigestSha512: return 128;
  }
  return -1;
}

void digest_hex(int algo, const int64_t* off, const uint8_t* chars, int64_t n, uint8_t* out, hipStream_t s) {
  if (digest_width(algo) < 0) throw std::runtime_error("digest: unknown algorithm");
  if (n == 0) return;
  hipLaunchKernelGGL(digest_hex_kernel, dim3(grid_for(n, kBlock, 1 << 14)), dim3(kBlock), 0, s, algo, off, chars, n,
                     out);
  check_launch("digest_hex", s);
}

void uuid_v4(uint64_t seed, int64_t n, uint8_t* out, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(uuid_kernel, dim3(grid_for(n, kBlock, 1 << 14)), dim3(kBlock), 0, s, seed, n, out);
  check_launch("uuid_v4", s);
}

}  // namespace kern
}  // namespace igloo
