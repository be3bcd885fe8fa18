// Shared device helpers for the igloo gfx950 relational kernels.
//
// Every kernel in csrc/kernels is written for CDNA4 (wave64): lane masks are
// 64-bit, block sizes are multiples of 64, and wave-level prefix sums use
// ballot + mbcnt instead of warp-32 idioms.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace igloo {
namespace kern {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int64_t kEmptyKey = INT64_MIN;  // hash-table empty-slot sentinel

#define IGLOO_HIP_CHECK(expr)                                                            \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +       \
                               " at " __FILE__ ":" + std::to_string(__LINE__));          \
  } while (0)

// Launch-error check after every kernel launch. With IGLOO_DEBUG=sync_check the
// stream is also synchronised so an asynchronous fault is attributed to the
// launch that caused it (SURVEY §5.2 debug mode).
void check_launch(const char* what, hipStream_t stream);

// IGLOO_DEBUG: comma list of debug / experimental tokens (``token`` or
// ``token=value``), shared with the Python side (igloo_amd/utils/switches.py)
inline bool debug_flag(const char* token) {
  const char* e = std::getenv("IGLOO_DEBUG");
  if (!e) return false;
  const std::string s(e), t(token);
  size_t p = 0;
  while (p <= s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    std::string tok = s.substr(p, q - p);
    const size_t eq = tok.find('=');
    if (eq != std::string::npos) tok = tok.substr(0, eq);
    while (!tok.empty() && tok.front() == ' ') tok.erase(tok.begin());
    while (!tok.empty() && tok.back() == ' ') tok.pop_back();
    if (tok == t) return true;
    p = q + 1;
  }
  return false;
}

inline unsigned grid_for(int64_t n, int per_block, int64_t max_blocks = 1 << 20) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (unsigned)g;
}

// 64-bit finaliser (murmur3 fmix64): good avalanche, cheap on the VALU.
__host__ __device__ inline uint64_t mix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

__host__ __device__ inline uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bU;
  h ^= h >> 13;
  h *= 0xc2b2ae35U;
  h ^= h >> 16;
  return h;
}

__device__ inline int lane_id() { return threadIdx.x & (kWave - 1); }

// Number of set bits in `mask` below this lane (v_mbcnt_lo/hi).
__device__ inline int lane_prefix(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// Inclusive wave64 scan of an int64 value via shfl_up.
__device__ inline int64_t wave_inclusive_scan(int64_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int64_t o = __shfl_up(v, off, kWave);
    if (lane >= off) v += o;
  }
  return v;
}

__device__ inline int64_t wave_reduce_sum(int64_t v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Exclusive block scan (kBlock threads). Returns this thread's exclusive
// prefix; *total receives the block total. `scratch` needs kWavesPerBlock+1
// int64 slots of LDS.
__device__ inline int64_t block_exclusive_scan(int64_t v, int64_t* scratch, int64_t* total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int64_t inc = wave_inclusive_scan(v);
  if (lane == kWave - 1) scratch[wave] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) {
      int64_t t = scratch[w];
      scratch[w] = run;
      run += t;
    }
    scratch[kWavesPerBlock] = run;
  }
  __syncthreads();
  int64_t res = inc - v + scratch[wave];
  *total = scratch[kWavesPerBlock];
  __syncthreads();
  return res;
}

// Order-preserving int64 encoding of an IEEE double (for atomic min/max).
__host__ __device__ inline int64_t f64_to_ordered(double d) {
  int64_t b;
  __builtin_memcpy(&b, &d, 8);
  return b ^ ((b >> 63) & 0x7fffffffffffffffLL);
}
__host__ __device__ inline double ordered_to_f64(int64_t b) {
  b ^= ((b >> 63) & 0x7fffffffffffffffLL);
  double d;
  __builtin_memcpy(&d, &b, 8);
  return d;
}

// 128-bit atomic accumulate from two 64-bit atomics. The low word's returned
// old value tells each adder whether IT produced a carry, so the final
// (hi, lo) pair is exact regardless of interleaving.
// hi == nullptr: a narrow (int64) sum whose exact total is known to fit
// (ops/agg.py checks max|v| * rows): one modular 64-bit add, no carry word.
__device__ inline void atomic_add_i128(unsigned long long* lo, long long* hi, int64_t v) {
  if (hi == nullptr) {
    atomicAdd(lo, (unsigned long long)v);
    return;
  }
  unsigned long long ulo = (unsigned long long)v;
  long long vhi = v < 0 ? -1 : 0;
  unsigned long long old = atomicAdd(lo, ulo);
  unsigned long long sum = old + ulo;
  long long carry = sum < old ? 1 : 0;
  long long add_hi = vhi + carry;
  if (add_hi != 0) atomicAdd((unsigned long long*)hi, (unsigned long long)add_hi);
}

__device__ inline void atomic_add_i128_parts(unsigned long long* lo, long long* hi,
                                             unsigned long long ulo, long long vhi) {
  if (hi == nullptr) {
    atomicAdd(lo, ulo);
    return;
  }
  unsigned long long old = atomicAdd(lo, ulo);
  unsigned long long sum = old + ulo;
  long long carry = sum < old ? 1 : 0;
  long long add_hi = vhi + carry;
  if (add_hi != 0) atomicAdd((unsigned long long*)hi, (unsigned long long)add_hi);
}

}  // namespace kern
}  // namespace igloo
