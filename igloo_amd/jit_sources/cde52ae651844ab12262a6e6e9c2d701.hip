// igloo-jit-kernel: igloo_jit_scan_mask
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

extern "C" __global__ __launch_bounds__(256) void igloo_jit_scan_mask(
    const i8* __restrict__ c0, const i8* __restrict__ c1, const i8* __restrict__ c2, u8* __restrict__ out, i64 n, i64* __restrict__ tc, i64 f0lo, i64 f0hi, i64 f1lo, i64 f1hi, u64 f2bits, i64 f3lo, i64 f3hi, i64 f4lo, i64 f4hi, u64 f5bits, i64 f6lo, i64 f6hi, i64 f7lo, i64 f7hi, u64 f8bits, i64 f9lo, i64 f9hi) {
  __shared__ i32 red[4];
  const i64 ntiles = (n + 8191) / 8192;
  for (i64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
    i32 cnt = 0;
    for (int it = 0; it < 8; ++it) {
    const i64 r = t * 8192 + it * 1024 + threadIdx.x * 4;
    if (r >= n) break;
    i32 x0_0;
    i32 x0_1;
    i32 x0_2;
    i32 x0_3;
    i32 x1_0;
    i32 x1_1;
    i32 x1_2;
    i32 x1_3;
    i32 x2_0;
    i32 x2_1;
    i32 x2_2;
    i32 x2_3;
    bool lv0;
    bool lv1;
    bool lv2;
    bool lv3;
    if (r + 4 <= n) {
      const i8xR q0 = *(const i8xR*)(c0 + r);
      const i8xR q1 = *(const i8xR*)(c1 + r);
      const i8xR q2 = *(const i8xR*)(c2 + r);
      x0_0 = q0[0];
      x1_0 = q1[0];
      x2_0 = q2[0];
      lv0 = true;
      x0_1 = q0[1];
      x1_1 = q1[1];
      x2_1 = q2[1];
      lv1 = true;
      x0_2 = q0[2];
      x1_2 = q1[2];
      x2_2 = q2[2];
      lv2 = true;
      x0_3 = q0[3];
      x1_3 = q1[3];
      x2_3 = q2[3];
      lv3 = true;
    } else {
      lv0 = r + 0 < n;
      x0_0 = lv0 ? (i32)c0[r + 0] : 0;
      x1_0 = lv0 ? (i32)c1[r + 0] : 0;
      x2_0 = lv0 ? (i32)c2[r + 0] : 0;
      lv1 = r + 1 < n;
      x0_1 = lv1 ? (i32)c0[r + 1] : 0;
      x1_1 = lv1 ? (i32)c1[r + 1] : 0;
      x2_1 = lv1 ? (i32)c2[r + 1] : 0;
      lv2 = r + 2 < n;
      x0_2 = lv2 ? (i32)c0[r + 2] : 0;
      x1_2 = lv2 ? (i32)c1[r + 2] : 0;
      x2_2 = lv2 ? (i32)c2[r + 2] : 0;
      lv3 = r + 3 < n;
      x0_3 = lv3 ? (i32)c0[r + 3] : 0;
      x1_3 = lv3 ? (i32)c1[r + 3] : 0;
      x2_3 = lv3 ? (i32)c2[r + 3] : 0;
    }
    const bool p0 = lv0 && (x0_0 >= f0lo) && (((x1_0 >= f1lo && x1_0 <= f1hi) && ((u64)x2_0 < 64ull && ((f2bits >> (u32)x2_0) & 1ull)) && (x0_0 <= f3hi)) || ((x1_0 >= f4lo && x1_0 <= f4hi) && ((u64)x2_0 < 64ull && ((f5bits >> (u32)x2_0) & 1ull)) && (x0_0 <= f6hi)) || ((x1_0 >= f7lo && x1_0 <= f7hi) && ((u64)x2_0 < 64ull && ((f8bits >> (u32)x2_0) & 1ull)) && (x0_0 <= f9hi)));
    const bool p1 = lv1 && (x0_1 >= f0lo) && (((x1_1 >= f1lo && x1_1 <= f1hi) && ((u64)x2_1 < 64ull && ((f2bits >> (u32)x2_1) & 1ull)) && (x0_1 <= f3hi)) || ((x1_1 >= f4lo && x1_1 <= f4hi) && ((u64)x2_1 < 64ull && ((f5bits >> (u32)x2_1) & 1ull)) && (x0_1 <= f6hi)) || ((x1_1 >= f7lo && x1_1 <= f7hi) && ((u64)x2_1 < 64ull && ((f8bits >> (u32)x2_1) & 1ull)) && (x0_1 <= f9hi)));
    const bool p2 = lv2 && (x0_2 >= f0lo) && (((x1_2 >= f1lo && x1_2 <= f1hi) && ((u64)x2_2 < 64ull && ((f2bits >> (u32)x2_2) & 1ull)) && (x0_2 <= f3hi)) || ((x1_2 >= f4lo && x1_2 <= f4hi) && ((u64)x2_2 < 64ull && ((f5bits >> (u32)x2_2) & 1ull)) && (x0_2 <= f6hi)) || ((x1_2 >= f7lo && x1_2 <= f7hi) && ((u64)x2_2 < 64ull && ((f8bits >> (u32)x2_2) & 1ull)) && (x0_2 <= f9hi)));
    const bool p3 = lv3 && (x0_3 >= f0lo) && (((x1_3 >= f1lo && x1_3 <= f1hi) && ((u64)x2_3 < 64ull && ((f2bits >> (u32)x2_3) & 1ull)) && (x0_3 <= f3hi)) || ((x1_3 >= f4lo && x1_3 <= f4hi) && ((u64)x2_3 < 64ull && ((f5bits >> (u32)x2_3) & 1ull)) && (x0_3 <= f6hi)) || ((x1_3 >= f7lo && x1_3 <= f7hi) && ((u64)x2_3 < 64ull && ((f8bits >> (u32)x2_3) & 1ull)) && (x0_3 <= f9hi)));
    if (r + 4 <= n) *(u8xR*)(out + r) = u8xR{(u8)p0, (u8)p1, (u8)p2, (u8)p3};
    else { if (lv0) out[r + 0] = p0; if (lv1) out[r + 1] = p1; if (lv2) out[r + 2] = p2; if (lv3) out[r + 3] = p3; }
    cnt += (i32)p0 + (i32)p1 + (i32)p2 + (i32)p3;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) tc[t] = (i64)red[0] + (i64)red[1] + (i64)red[2] + (i64)red[3];
    __syncthreads();
  }
}