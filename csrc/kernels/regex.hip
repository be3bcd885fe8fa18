// Regular-expression match tests on the GPU: regexp_like, ~ / ~* / !~ / !~*
// and SIMILAR TO (DataFusion's regex-backed functions, reference
// Cargo.lock:1062-1090). The pattern arrives as a byte-class DFA compiled on
// the host (igloo_amd/ops/regex_dfa.py); the workgroup stages the transition
// table (uint16 [states][classes]), the 256-entry byte -> class map and the
// per-state flags (1 accepting, 2 dead) in LDS, then each lane walks one
// string: one LDS lookup per byte, leaving as soon as the state accepts (an
// unanchored-end search) or can no longer accept. Strings are read with
// per-lane byte loads; rows are interleaved across the wave so neighbouring
// lanes start on neighbouring strings.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__global__ __launch_bounds__(kBlock) void regex_dfa_kernel(const int64_t* __restrict__ off,
                                                         const uint8_t* __restrict__ chars, int64_t n,
                                                         const uint16_t* __restrict__ table,
                                                         const uint8_t* __restrict__ cls,
                                                         const uint8_t* __restrict__ flags, int nstates,
                                                         int nclasses, int start, int anchored_end, int negate,
                                                         uint8_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  uint16_t* t = reinterpret_cast<uint16_t*>(lds);
  const int entries = nstates * nclasses;
  uint8_t* c = lds + 2 * ((entries + 7) & ~7);
  uint8_t* f = c + 256;
  for (int i = threadIdx.x; i < entries; i += blockDim.x) t[i] = table[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) c[i] = cls[i];
  for (int i = threadIdx.x; i < nstates; i += blockDim.x) f[i] = flags[i];
  __syncthreads();
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = chars + off[r];
    const int64_t len = off[r + 1] - off[r];
    int st = start;
    uint8_t hit = 0;
    bool done = false;
    for (int64_t k = 0; k < len; ++k) {
      const uint8_t fl = f[st];
      if (fl == 2 || (!anchored_end && fl == 1)) {
        hit = fl == 1;
        done = true;
        break;
      }
      st = t[st * nclasses + c[s[k]]];
    }
    if (!done) hit = f[st] == 1;
    out[r] = hit ^ (uint8_t)negate;
  }
}

}  // namespace

size_t regex_lds_bytes(int nstates, int nclasses) {
  return 2 * (((size_t)nstates * nclasses + 7) & ~(size_t)7) + 256 + nstates;
}

void regex_dfa_match(const int64_t* off, const uint8_t* chars, int64_t n, const uint16_t* table, const uint8_t* cls,
                     const uint8_t* flags, int nstates, int nclasses, int start, bool anchored_end, bool negate,
                     uint8_t* out, hipStream_t s) {
  if (n == 0) return;
  const size_t lds = regex_lds_bytes(nstates, nclasses);
  if (lds > 64 * 1024) throw std::runtime_error("regex: automaton too large for LDS");
  hipLaunchKernelGGL(regex_dfa_kernel, dim3(grid_for(n, kBlock, 1 << 14)), dim3(kBlock), lds, s, off, chars, n,
                     table, cls, flags, nstates, nclasses, start, anchored_end ? 1 : 0, negate ? 1 : 0, out);
  check_launch("regex_dfa", s);
}

}  // namespace kern
}  // namespace igloo
