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
    const i8* __restrict__ c0, const i8* __restrict__ c1, const i16* __restrict__ c2, const i32* __restrict__ c3, const i8* __restrict__ c4, const i8* __restrict__ c5, const i16* __restrict__ c6, i64* __restrict__ counts, i64* __restrict__ d0, i64* __restrict__ e0, i64* __restrict__ d1, i64* __restrict__ e1, i64* __restrict__ d2, i64* __restrict__ e2, i64* __restrict__ d3, i64* __restrict__ e3, i64* __restrict__ d4, i64* __restrict__ e4, int* __restrict__ ovf, i64 n, i64 f0lo, i64 f0hi) {
  int of = 0;
  __shared__ i64 lds[2304];
  const int ln = threadIdx.x & 63;
  for (int s = threadIdx.x; s < 2304; s += 256) {
    const int k = s / 384;
    lds[s] = 0;
  }
  __syncthreads();
  const i64 step = (i64)gridDim.x * 1024;
  for (i64 r = ((i64)blockIdx.x * 256 + threadIdx.x) * 4; r < n; r += step) {
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
    i32 x3_0;
    i32 x3_1;
    i32 x3_2;
    i32 x3_3;
    i32 x4_0;
    i32 x4_1;
    i32 x4_2;
    i32 x4_3;
    i32 x5_0;
    i32 x5_1;
    i32 x5_2;
    i32 x5_3;
    i32 x6_0;
    i32 x6_1;
    i32 x6_2;
    i32 x6_3;
    bool lv0;
    bool lv1;
    bool lv2;
    bool lv3;
    if (r + 4 <= n) {
      const i8xR q0 = *(const i8xR*)(c0 + r);
      const i8xR q1 = *(const i8xR*)(c1 + r);
      const i16xR q2 = *(const i16xR*)(c2 + r);
      const i32xR q3 = *(const i32xR*)(c3 + r);
      const i8xR q4 = *(const i8xR*)(c4 + r);
      const i8xR q5 = *(const i8xR*)(c5 + r);
      const i16xR q6 = *(const i16xR*)(c6 + r);
      x0_0 = q0[0];
      x1_0 = q1[0];
      x2_0 = q2[0];
      x3_0 = q3[0];
      x4_0 = q4[0];
      x5_0 = q5[0];
      x6_0 = q6[0];
      lv0 = true;
      x0_1 = q0[1];
      x1_1 = q1[1];
      x2_1 = q2[1];
      x3_1 = q3[1];
      x4_1 = q4[1];
      x5_1 = q5[1];
      x6_1 = q6[1];
      lv1 = true;
      x0_2 = q0[2];
      x1_2 = q1[2];
      x2_2 = q2[2];
      x3_2 = q3[2];
      x4_2 = q4[2];
      x5_2 = q5[2];
      x6_2 = q6[2];
      lv2 = true;
      x0_3 = q0[3];
      x1_3 = q1[3];
      x2_3 = q2[3];
      x3_3 = q3[3];
      x4_3 = q4[3];
      x5_3 = q5[3];
      x6_3 = q6[3];
      lv3 = true;
    } else {
      lv0 = r + 0 < n;
      x0_0 = lv0 ? (i32)c0[r + 0] : 0;
      x1_0 = lv0 ? (i32)c1[r + 0] : 0;
      x2_0 = lv0 ? (i32)c2[r + 0] : 0;
      x3_0 = lv0 ? (i32)c3[r + 0] : 0;
      x4_0 = lv0 ? (i32)c4[r + 0] : 0;
      x5_0 = lv0 ? (i32)c5[r + 0] : 0;
      x6_0 = lv0 ? (i32)c6[r + 0] : 0;
      lv1 = r + 1 < n;
      x0_1 = lv1 ? (i32)c0[r + 1] : 0;
      x1_1 = lv1 ? (i32)c1[r + 1] : 0;
      x2_1 = lv1 ? (i32)c2[r + 1] : 0;
      x3_1 = lv1 ? (i32)c3[r + 1] : 0;
      x4_1 = lv1 ? (i32)c4[r + 1] : 0;
      x5_1 = lv1 ? (i32)c5[r + 1] : 0;
      x6_1 = lv1 ? (i32)c6[r + 1] : 0;
      lv2 = r + 2 < n;
      x0_2 = lv2 ? (i32)c0[r + 2] : 0;
      x1_2 = lv2 ? (i32)c1[r + 2] : 0;
      x2_2 = lv2 ? (i32)c2[r + 2] : 0;
      x3_2 = lv2 ? (i32)c3[r + 2] : 0;
      x4_2 = lv2 ? (i32)c4[r + 2] : 0;
      x5_2 = lv2 ? (i32)c5[r + 2] : 0;
      x6_2 = lv2 ? (i32)c6[r + 2] : 0;
      lv3 = r + 3 < n;
      x0_3 = lv3 ? (i32)c0[r + 3] : 0;
      x1_3 = lv3 ? (i32)c1[r + 3] : 0;
      x2_3 = lv3 ? (i32)c2[r + 3] : 0;
      x3_3 = lv3 ? (i32)c3[r + 3] : 0;
      x4_3 = lv3 ? (i32)c4[r + 3] : 0;
      x5_3 = lv3 ? (i32)c5[r + 3] : 0;
      x6_3 = lv3 ? (i32)c6[r + 3] : 0;
    }
    const bool p0 = lv0 && (x6_0 <= f0hi);
    if (p0) {
      const i32 v0_0 = x2_0;
      const i64 v1_0 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_0);
      const i64 v2_0 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_0);
      const i64 v3_0 = (i64)v2_0 * (i64)(100 - x4_0);
      const i64 v4_0 = (i64)v3_0 * (i64)(100 + x5_0);
      const i32 v5_0 = x4_0;
      const int b_ = ((i32)x1_0 * 1 + (i32)x0_0 * 2) * 64 + ln;
      WG_ADD(&lds[1920 + b_], (i64)1);
      WG_ADD(&lds[0 + b_], (i64)v0_0);
      WG_ADD(&lds[384 + b_], (i64)v1_0);
      WG_ADD(&lds[768 + b_], (i64)v3_0);
      WG_ADD(&lds[1152 + b_], (i64)v4_0);
      WG_ADD(&lds[1536 + b_], (i64)v5_0);
    }
    const bool p1 = lv1 && (x6_1 <= f0hi);
    if (p1) {
      const i32 v0_1 = x2_1;
      const i64 v1_1 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_1);
      const i64 v2_1 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_1);
      const i64 v3_1 = (i64)v2_1 * (i64)(100 - x4_1);
      const i64 v4_1 = (i64)v3_1 * (i64)(100 + x5_1);
      const i32 v5_1 = x4_1;
      const int b_ = ((i32)x1_1 * 1 + (i32)x0_1 * 2) * 64 + ln;
      WG_ADD(&lds[1920 + b_], (i64)1);
      WG_ADD(&lds[0 + b_], (i64)v0_1);
      WG_ADD(&lds[384 + b_], (i64)v1_1);
      WG_ADD(&lds[768 + b_], (i64)v3_1);
      WG_ADD(&lds[1152 + b_], (i64)v4_1);
      WG_ADD(&lds[1536 + b_], (i64)v5_1);
    }
    const bool p2 = lv2 && (x6_2 <= f0hi);
    if (p2) {
      const i32 v0_2 = x2_2;
      const i64 v1_2 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_2);
      const i64 v2_2 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_2);
      const i64 v3_2 = (i64)v2_2 * (i64)(100 - x4_2);
      const i64 v4_2 = (i64)v3_2 * (i64)(100 + x5_2);
      const i32 v5_2 = x4_2;
      const int b_ = ((i32)x1_2 * 1 + (i32)x0_2 * 2) * 64 + ln;
      WG_ADD(&lds[1920 + b_], (i64)1);
      WG_ADD(&lds[0 + b_], (i64)v0_2);
      WG_ADD(&lds[384 + b_], (i64)v1_2);
      WG_ADD(&lds[768 + b_], (i64)v3_2);
      WG_ADD(&lds[1152 + b_], (i64)v4_2);
      WG_ADD(&lds[1536 + b_], (i64)v5_2);
    }
    const bool p3 = lv3 && (x6_3 <= f0hi);
    if (p3) {
      const i32 v0_3 = x2_3;
      const i64 v1_3 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_3);
      const i64 v2_3 = (i64)((u64)0LL + (u64)1LL * (u64)(i64)x3_3);
      const i64 v3_3 = (i64)v2_3 * (i64)(100 - x4_3);
      const i64 v4_3 = (i64)v3_3 * (i64)(100 + x5_3);
      const i32 v5_3 = x4_3;
      const int b_ = ((i32)x1_3 * 1 + (i32)x0_3 * 2) * 64 + ln;
      WG_ADD(&lds[1920 + b_], (i64)1);
      WG_ADD(&lds[0 + b_], (i64)v0_3);
      WG_ADD(&lds[384 + b_], (i64)v1_3);
      WG_ADD(&lds[768 + b_], (i64)v3_3);
      WG_ADD(&lds[1152 + b_], (i64)v4_3);
      WG_ADD(&lds[1536 + b_], (i64)v5_3);
    }
  }
  __syncthreads();
  for (int s = threadIdx.x; s < 36; s += 256) {
    const int g = s / 6, o = s % 6;
    __int128 t = 0;
    if (o == 5) {
      for (int l = 0; l < 64; ++l) t += lds[1920 + g * 64 + l];
      if (t) atomicAdd((unsigned long long*)&counts[g], (unsigned long long)(i64)t);
      continue;
    }
    if (o == 0) {
      for (int l = 0; l < 64; ++l) t += lds[0 + g * 64 + l];
      add128(&d0[g], &e0[g], t);
    }
    if (o == 1) {
      for (int l = 0; l < 64; ++l) t += lds[384 + g * 64 + l];
      add128(&d1[g], &e1[g], t);
    }
    if (o == 2) {
      for (int l = 0; l < 64; ++l) t += lds[768 + g * 64 + l];
      add128(&d2[g], &e2[g], t);
    }
    if (o == 3) {
      for (int l = 0; l < 64; ++l) t += lds[1152 + g * 64 + l];
      add128(&d3[g], &e3[g], t);
    }
    if (o == 4) {
      for (int l = 0; l < 64; ++l) t += lds[1536 + g * 64 + l];
      add128(&d4[g], &e4[g], t);
    }
  }
  if (of) atomicOr(ovf, 1);
}