// igloo-jit-kernel: igloo_jit_scan_agg
#define ROWS 4

typedef signed char i8; typedef short i16; typedef int i32; typedef long long i64;
typedef unsigned char u8; typedef unsigned int u32; typedef unsigned long long u64;
typedef i8 i8xR __attribute__((ext_vector_type(ROWS)));
typedef i16 i16xR __attribute__((ext_vector_type(ROWS)));
typedef i32 i32xR __attribute__((ext_vector_type(ROWS)));
typedef i64 i64xR __attribute__((ext_vector_type(ROWS)));
typedef u8 u8xR __attribute__((ext_vector_type(ROWS)));
#define WG_ADD(p, v) __hip_atomic_fetch_add((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define WG_MIN(p, v) __hip_atomic_fetch_min((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
#define WG_MAX(p, v) __hip_atomic_fetch_max((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
__device__ __forceinline__ void add128(i64* lo, i64* hi, __int128 v) {
  if (v == 0) return;
  const u64 vl = (u64)v;
  const u64 vh = (u64)(i64)(v >> 64);
  const u64 old = atomicAdd((unsigned long long*)lo, (unsigned long long)vl);
  const u64 carry = (old + vl) < old ? 1ull : 0ull;
  if (vh + carry) atomicAdd((unsigned long long*)hi, (unsigned long long)(vh + carry));
}
__device__ __forceinline__ i64 wsum(i64 v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ i64 wmin(i64 v) {
  for (int o = 32; o > 0; o >>= 1) { const i64 u = __shfl_xor(v, o, 64); v = u < v ? u : v; }
  return v;
}
__device__ __forceinline__ i64 wmax(i64 v) {
  for (int o = 32; o > 0; o >>= 1) { const i64 u = __shfl_xor(v, o, 64); v = u > v ? u : v; }
  return v;
}

extern "C" __global__ __launch_bounds__(256) void igloo_jit_scan_agg(
    const i32* __restrict__ c0, const u8* __restrict__ mk, i64* __restrict__ counts, i64* __restrict__ d0, i64* __restrict__ e0, int* __restrict__ ovf, i64 n, i64 f0lo, i64 f0hi) {
  int of = 0;
  i64 cn = 0;
  i64 s0 = 0;
  const i64 step = (i64)gridDim.x * 1024;
  for (i64 r = ((i64)blockIdx.x * 256 + threadIdx.x) * 4; r < n; r += step) {
    i32 x0_0;
    i32 x0_1;
    i32 x0_2;
    i32 x0_3;
    bool lv0;
    bool mk0;
    bool lv1;
    bool mk1;
    bool lv2;
    bool mk2;
    bool lv3;
    bool mk3;
    if (r + 4 <= n) {
      const i32xR q0 = *(const i32xR*)(c0 + r);
      const u8xR mq = *(const u8xR*)(mk + r);
      x0_0 = q0[0];
      lv0 = true;
      mk0 = mq[0] != 0;
      x0_1 = q0[1];
      lv1 = true;
      mk1 = mq[1] != 0;
      x0_2 = q0[2];
      lv2 = true;
      mk2 = mq[2] != 0;
      x0_3 = q0[3];
      lv3 = true;
      mk3 = mq[3] != 0;
    } else {
      lv0 = r + 0 < n;
      x0_0 = lv0 ? (i32)c0[r + 0] : 0;
      mk0 = lv0 && mk[r + 0] != 0;
      lv1 = r + 1 < n;
      x0_1 = lv1 ? (i32)c0[r + 1] : 0;
      mk1 = lv1 && mk[r + 1] != 0;
      lv2 = r + 2 < n;
      x0_2 = lv2 ? (i32)c0[r + 2] : 0;
      mk2 = lv2 && mk[r + 2] != 0;
      lv3 = r + 3 < n;
      x0_3 = lv3 ? (i32)c0[r + 3] : 0;
      mk3 = lv3 && mk[r + 3] != 0;
    }
    const bool p0 = lv0 && (x0_0 >= f0lo) && mk0;
    if (p0) {
      const i64 v0_0 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x0_0);
      cn += 1;
      s0 += (i64)v0_0;
    }
    const bool p1 = lv1 && (x0_1 >= f0lo) && mk1;
    if (p1) {
      const i64 v0_1 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x0_1);
      cn += 1;
      s0 += (i64)v0_1;
    }
    const bool p2 = lv2 && (x0_2 >= f0lo) && mk2;
    if (p2) {
      const i64 v0_2 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x0_2);
      cn += 1;
      s0 += (i64)v0_2;
    }
    const bool p3 = lv3 && (x0_3 >= f0lo) && mk3;
    if (p3) {
      const i64 v0_3 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x0_3);
      cn += 1;
      s0 += (i64)v0_3;
    }
  }
  __shared__ i64 red[4][2];
  const int w_ = threadIdx.x >> 6;
  { const i64 t_ = wsum(cn); if ((threadIdx.x & 63) == 0) red[w_][0] = t_; }
  { const i64 t_ = wsum(s0); if ((threadIdx.x & 63) == 0) red[w_][1] = t_; }
  __syncthreads();
  if (threadIdx.x == 0) {
    i64 cn_b = red[0][0]; { i64 t_ = cn_b; for (int w = 1; w < 4; ++w) t_ += red[w][0]; cn_b = t_; }
    i64 s0_b = red[0][1]; { i64 t_ = s0_b; for (int w = 1; w < 4; ++w) t_ += red[w][1]; s0_b = t_; }
    if (cn_b) atomicAdd((unsigned long long*)counts, (unsigned long long)cn_b);
    add128(d0, e0, (__int128)s0_b);
  }
  if (of) atomicOr(ovf, 1);
}