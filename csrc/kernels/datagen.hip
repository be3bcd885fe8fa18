// Synthetic TPC-H-shaped text columns (comments, names, phones, addresses,
// part names), generated directly in HBM.
//
// The reference ships only a 176-byte placeholder instead of Parquet data
// (reference data/sample.parquet:1-3) and has no generator; SF100 needs
// ~10 GB of strings, so generation runs on the GPU. The per-row generator is
// __host__ __device__: the CPU build runs the identical code, so CPU tests and
// GPU runs see byte-identical data. Randomness is a counter-based hash of
// (seed, row, draw), so any row range can be generated independently — each
// rank generates only its own partition.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__host__ __device__ inline uint64_t rnd(uint64_t seed, int64_t row, int draw) {
  return mix64(seed ^ mix64((uint64_t)row * 0x9E3779B97F4A7C15ULL + (uint64_t)draw * 0xC2B2AE3D27D4EB4FULL));
}

__host__ __device__ inline void put(uint8_t* out, int64_t& len, uint8_t c) {
  if (out) out[len] = c;
  ++len;
}

__host__ __device__ inline void put_word(uint8_t* out, int64_t& len, const TextGenParams& p, int w) {
  int32_t a = p.vocab_off[w], b = p.vocab_off[w + 1];
  for (int32_t k = a; k < b; ++k) put(out, len, p.vocab[k]);
}

__host__ __device__ inline void put_int(uint8_t* out, int64_t& len, int64_t v, int width) {
  char buf[24];
  int n = 0;
  if (v < 0) v = -v;
  do {
    buf[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v > 0 && n < 20);
  for (int k = n; k < width; ++k) put(out, len, '0');
  while (n > 0) put(out, len, (uint8_t)buf[--n]);
}

__host__ __device__ int64_t gen_row(const TextGenParams& p, int64_t row, uint8_t* out) {
  int64_t len = 0;
  const int64_t r = p.row_ids ? p.row_ids[row] : row + p.row_base;  // global row id: rank-independent data
  switch (p.kind) {
    case TEXT_WORDS: {
      int span = p.max_len - p.min_len + 1;
      int nw = p.min_len + (int)(rnd(p.seed, r, 0) % (uint64_t)span);
      bool inject = p.inject_every > 0 && (rnd(p.seed, r, 99) % (uint64_t)p.inject_every) == 0;
      int inject_at = inject ? (int)(rnd(p.seed, r, 98) % (uint64_t)nw) : -1;
      for (int w = 0; w < nw; ++w) {
        if (w) put(out, len, ' ');
        if (w == inject_at) {
          for (int k = 0; k < p.inject_len; ++k) put(out, len, p.inject[k]);
          put(out, len, ' ');
        }
        put_word(out, len, p, (int)(rnd(p.seed, r, 1 + w) % (uint64_t)p.vocab_n));
      }
      if (p.suffix_char) put(out, len, (uint8_t)p.suffix_char);
      break;
    }
    case TEXT_DISTINCT_WORDS: {  // p_name: min_len distinct vocabulary words
      int chosen[8];
      int nw = p.min_len < 8 ? p.min_len : 8;
      int draw = 1;
      for (int w = 0; w < nw; ++w) {
        int c;
        bool dup;
        do {
          c = (int)(rnd(p.seed, r, draw++) % (uint64_t)p.vocab_n);
          dup = false;
          for (int k = 0; k < w; ++k) dup |= chosen[k] == c;
        } while (dup && draw < 64);
        chosen[w] = c;
        if (w) put(out, len, ' ');
        put_word(out, len, p, c);
      }
      break;
    }
    case TEXT_ALNUM: {  // v-string: random characters from a 64-symbol alphabet
      const char* al = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ,.";
      int span = p.max_len - p.min_len + 1;
      int n = p.min_len + (int)(rnd(p.seed, r, 0) % (uint64_t)span);
      for (int k = 0; k < n; ++k) {
        uint64_t x = rnd(p.seed, r, 1 + k);
        put(out, len, (uint8_t)al[x & 63]);
      }
      break;
    }
    case TEXT_PREFIX_INT: {  // e.g. Customer#000000042
      for (int k = 0; k < p.inject_len; ++k) put(out, len, p.inject[k]);
      put_int(out, len, r + 1, p.min_len);
      break;
    }
    case TEXT_PREFIX_RANDINT: {  // e.g. Clerk#000000951: prefix + random int in [1, max_len]
      for (int k = 0; k < p.inject_len; ++k) put(out, len, p.inject[k]);
      put_int(out, len, 1 + (int64_t)(rnd(p.seed, r, 0) % (uint64_t)p.max_len), p.min_len);
      break;
    }
    case TEXT_PHONE: {  // CC-ddd-ddd-dddd, CC = nationkey + 10
      int cc = (p.aux ? p.aux[row] : 0) + 10;
      put_int(out, len, cc, 2);
      put(out, len, '-');
      put_int(out, len, 100 + (int64_t)(rnd(p.seed, r, 1) % 900), 3);
      put(out, len, '-');
      put_int(out, len, 100 + (int64_t)(rnd(p.seed, r, 2) % 900), 3);
      put(out, len, '-');
      put_int(out, len, 1000 + (int64_t)(rnd(p.seed, r, 3) % 9000), 4);
      break;
    }
  }
  return len;
}

__global__ __launch_bounds__(kBlock) void textgen_len_kernel(TextGenParams p, int64_t n, int64_t* __restrict__ lens) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    lens[i] = gen_row(p, i, nullptr);
}

__global__ __launch_bounds__(kBlock) void textgen_write_kernel(TextGenParams p, int64_t n, const int64_t* __restrict__ off,
                                                              uint8_t* __restrict__ chars) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    gen_row(p, i, chars + off[i]);
}

}  // namespace

void textgen_lengths(const TextGenParams& p, int64_t n, int64_t* lens, bool device, hipStream_t stream) {
  if (n == 0) return;
  if (!device) {
    for (int64_t i = 0; i < n; ++i) lens[i] = gen_row(p, i, nullptr);
    return;
  }
  hipLaunchKernelGGL(textgen_len_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, p, n, lens);
  check_launch("textgen_lengths", stream);
}

void textgen_write(const TextGenParams& p, int64_t n, const int64_t* off, uint8_t* chars, bool device,
                   hipStream_t stream) {
  if (n == 0) return;
  if (!device) {
    for (int64_t i = 0; i < n; ++i) gen_row(p, i, chars + off[i]);
    return;
  }
  hipLaunchKernelGGL(textgen_write_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, p, n, off, chars);
  check_launch("textgen_write", stream);
}

}  // namespace kern
}  // namespace igloo
