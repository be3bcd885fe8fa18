// igloo-jit-kernel: igloo_jit_expr

typedef signed char i8; typedef short i16; typedef int i32; typedef long long i64;
typedef unsigned char u8; typedef unsigned int u32; typedef unsigned long long u64;
__device__ __forceinline__ double i2d(i64 x) { union { i64 i; double d; } u; u.i = x; return u.d; }
__device__ __forceinline__ void civil(i32 z0, i32* y, i32* m, i32* d) {
  i64 z = (i64)z0 + 719468;
  i64 era = (z >= 0 ? z : z - 146096) / 146097;
  i64 doe = z - era * 146097;
  i64 yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  i64 doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  i64 mp = (5 * doy + 2) / 153;
  i64 mm = mp < 10 ? mp + 3 : mp - 9;
  *y = (i32)(yoe + era * 400 + (mm <= 2));
  *m = (i32)mm;
  *d = (i32)(doy - (153 * mp + 2) / 5 + 1);
}
__device__ __forceinline__ i64 days_from_civil(i64 y, i32 m, i32 d) {
  y -= m <= 2;
  i64 era = (y >= 0 ? y : y - 399) / 400;
  i64 yoe = y - era * 400;
  i64 doy = (153 * (m > 2 ? m - 3 : m + 9) + 2) / 5 + d - 1;
  i64 doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
__device__ __forceinline__ i32 date_part(i32 z, int f) {
  i32 y, m, d;
  civil(z, &y, &m, &d);
  switch (f) {
    case 0: return y;
    case 1: return m;
    case 2: return d;
    case 3: return (m - 1) / 3 + 1;
    case 4: return (i32)(((i64)z % 7 + 7 + 4) % 7);
    default: return (i32)((i64)z - days_from_civil(y, 1, 1) + 1);
  }
}
__device__ __forceinline__ i32 add_months(i32 z, i64 months, i64 days) {
  i32 y, m, d;
  civil(z, &y, &m, &d);
  i64 mi = (i64)y * 12 + (m - 1) + months;          // month index of the target month
  i64 ny = mi >= 0 ? mi / 12 : -((-mi + 11) / 12);
  i32 nm = (i32)(mi - ny * 12) + 1;
  i64 start = days_from_civil(ny, nm, 1);
  i64 ni = mi + 1;
  i64 ny2 = ni >= 0 ? ni / 12 : -((-ni + 11) / 12);
  i64 next = days_from_civil(ny2, (i32)(ni - ny2 * 12) + 1, 1);
  i64 r = start + (d - 1);
  if (r > next - 1) r = next - 1;
  return (i32)(r + days);
}

extern "C" __global__ __launch_bounds__(256) void igloo_jit_expr(const i64* __restrict__ c0, const i64* __restrict__ c1, const u8* __restrict__ v1, u8* __restrict__ out, u8* __restrict__ outv, int* __restrict__ errp, i64 n) {
  int err = 0;
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < n; i += (i64)gridDim.x * 256) {
    const i64 t1 = (i64)c0[i];
    const i64 t2 = (i64)((i64)((u64)(i64)(t1) * 100000ull));
    const i64 t3 = (i64)c1[i];
    const bool t4 = (t2) < (t3);
    out[i] = (u8)((t4) ? 1 : 0);
    outv[i] = (((v1[i] != 0))) ? 1 : 0;
  }
  if (err) atomicOr(errp, 1);
}