// String expression kernels (gfx950): the projection-side string work that
// used to round-trip through host Arrow compute.
//
// Parity: the reference evaluates projection expressions per batch with
// DataFusion's CPU kernels (reference crates/engine/src/operators/projection.rs:60-64)
// and its one UDF is a string transform (crates/engine/src/lib.rs:84-91).
//
//   str_char_length   characters (UTF-8 code points) per row
//   str_concat2       a || b over plain string columns (either side may be a
//                     one-row constant broadcast to every row); two passes:
//                     lengths, then an offset scan and the byte copy
//   fmt_*             CAST(int / decimal / date / bool AS VARCHAR): exact text
//                     (decimal point at the type's scale, ISO dates)
//   str_parse         CAST(varchar AS int / decimal / date / double / bool),
//                     exact for integers, fixed point and dates; a malformed
//                     value sets an error flag the host turns into the error
//
// All of them are one lane per row over the Arrow large-string layout (int64
// offsets + bytes): strings in these columns are short (names, codes,
// comments), so a lane-serial byte loop is bounded and the kernels are
// bandwidth-bound on the offsets / values they stream.
#include "common.h"
#include "kernels.h"
#include "textparse.h"

namespace igloo {
namespace kern {

namespace {

__global__ __launch_bounds__(kBlock) void char_length_kernel(const int64_t* __restrict__ off,
                                                             const uint8_t* __restrict__ chars, int64_t n,
                                                             int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = off[i], b = off[i + 1];
    int32_t c = 0;
    int64_t p = a;
    // 8 bytes at a time where aligned: count bytes that are not continuation bytes
    for (; p < b && (p & 7); ++p) c += (chars[p] & 0xC0) != 0x80;
    for (; p + 8 <= b; p += 8) {
      const uint64_t w = *reinterpret_cast<const uint64_t*>(chars + p);
      // continuation byte: top bits 10 -> bit7 set and bit6 clear
      const uint64_t cont = (w & 0x8080808080808080ULL) & ~((w << 1) & 0x8080808080808080ULL);
      c += 8 - __popcll(cont);
    }
    for (; p < b; ++p) c += (chars[p] & 0xC0) != 0x80;
    out[i] = c;
  }
}

__global__ __launch_bounds__(kBlock) void concat2_len_kernel(const int64_t* __restrict__ oa, bool ba,
                                                             const int64_t* __restrict__ ob, bool bb, int64_t n,
                                                             int64_t* __restrict__ len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ia = ba ? 0 : i, ib = bb ? 0 : i;
    len[i] = (oa[ia + 1] - oa[ia]) + (ob[ib + 1] - ob[ib]);
  }
}

__global__ __launch_bounds__(kBlock) void concat2_copy_kernel(const int64_t* __restrict__ oa,
                                                              const uint8_t* __restrict__ ca, bool ba,
                                                              const int64_t* __restrict__ ob,
                                                              const uint8_t* __restrict__ cb, bool bb, int64_t n,
                                                              const int64_t* __restrict__ off,
                                                              uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ia = ba ? 0 : i, ib = bb ? 0 : i;
    int64_t o = off[i];
    for (int64_t p = oa[ia]; p < oa[ia + 1]; ++p) out[o++] = ca[p];
    for (int64_t p = ob[ib]; p < ob[ib + 1]; ++p) out[o++] = cb[p];
  }
}

// kind: 0 int64 fixed point (scale), 1 int32, 2 date32, 3 bool (uint8)
__device__ inline int fmt_one(const void* vals, int kind, int64_t i, int scale, uint8_t* out) {
  switch (kind) {
    case 0:
      return format_fixed(static_cast<const int64_t*>(vals)[i], scale, out);
    case 1:
      return format_fixed(static_cast<const int32_t*>(vals)[i], 0, out);
    case 2:
      return format_date(static_cast<const int32_t*>(vals)[i], out);
    default: {
      const bool v = static_cast<const uint8_t*>(vals)[i] != 0;
      if (out) {
        const char* s = v ? "true" : "false";
        for (int k = 0; s[k]; ++k) out[k] = (uint8_t)s[k];
      }
      return v ? 4 : 5;
    }
  }
}

__global__ __launch_bounds__(kBlock) void fmt_len_kernel(const void* __restrict__ vals, int kind, int64_t n, int scale,
                                                         const uint8_t* __restrict__ valid,
                                                         int64_t* __restrict__ len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    len[i] = (valid && !valid[i]) ? 0 : fmt_one(vals, kind, i, scale, nullptr);
}

__global__ __launch_bounds__(kBlock) void fmt_write_kernel(const void* __restrict__ vals, int kind, int64_t n,
                                                           int scale, const uint8_t* __restrict__ valid,
                                                           const int64_t* __restrict__ off,
                                                           uint8_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (!(valid && !valid[i])) fmt_one(vals, kind, i, scale, out + off[i]);
}

__device__ inline void set_err_flag(int* err) { atomicCAS(err, 0, 1); }

// kind: 0 int64, 1 int32, 2 fixed point -> int64 at `scale`, 3 date32,
// 4 float64, 5 bool ("true"/"false"/"t"/"f"/"1"/"0", any case)
__global__ __launch_bounds__(kBlock) void parse_kernel(const int64_t* __restrict__ off,
                                                       const uint8_t* __restrict__ chars, int64_t n,
                                                       const uint8_t* __restrict__ valid, int kind, int scale,
                                                       void* __restrict__ out, int* __restrict__ err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool null = valid && !valid[i];
    const uint8_t* p = chars + off[i];
    const uint8_t* e = chars + off[i + 1];
    bool ok = true;
    switch (kind) {
      case 0:
      case 1: {
        int64_t v = 0;
        ok = null || parse_int(p, e, &v);
        if (kind == 1 && (v > INT32_MAX || v < INT32_MIN)) ok = false;
        if (kind == 0) static_cast<int64_t*>(out)[i] = null ? 0 : v;
        else static_cast<int32_t*>(out)[i] = null ? 0 : (int32_t)v;
        break;
      }
      case 2: {
        int64_t v = 0;
        ok = null || parse_decimal(p, e, scale, &v);
        static_cast<int64_t*>(out)[i] = null ? 0 : v;
        break;
      }
      case 3: {
        int32_t v = 0;
        ok = null || parse_date(p, e, &v);
        static_cast<int32_t*>(out)[i] = null ? 0 : v;
        break;
      }
      case 4: {
        double v = 0;
        ok = null || parse_f64(p, e, &v);
        static_cast<double*>(out)[i] = null ? 0.0 : v;
        break;
      }
      default: {
        uint8_t v = 0;
        if (!null) {
          if (ieq(p, e, "true") || ieq(p, e, "t") || ieq(p, e, "1")) v = 1;
          else if (!(ieq(p, e, "false") || ieq(p, e, "f") || ieq(p, e, "0"))) ok = false;
        }
        static_cast<uint8_t*>(out)[i] = v;
      }
    }
    if (!ok) set_err_flag(err);
  }
}

}  // namespace

void str_char_length(const int64_t* off, const uint8_t* chars, int64_t n, int32_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(char_length_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, out);
  check_launch("str_char_length", stream);
}

void str_concat2_lengths(const int64_t* oa, bool ba, const int64_t* ob, bool bb, int64_t n, int64_t* len,
                         hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(concat2_len_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, oa, ba, ob, bb, n,
                     len);
  check_launch("str_concat2_lengths", stream);
}

void str_concat2_copy(const int64_t* oa, const uint8_t* ca, bool ba, const int64_t* ob, const uint8_t* cb, bool bb,
                      int64_t n, const int64_t* off, uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(concat2_copy_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, oa, ca, ba, ob, cb,
                     bb, n, off, out);
  check_launch("str_concat2_copy", stream);
}

void fmt_lengths(const void* vals, int kind, int64_t n, int scale, const uint8_t* valid, int64_t* len,
                 hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(fmt_len_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, vals, kind, n, scale,
                     valid, len);
  check_launch("fmt_lengths", stream);
}

void fmt_write(const void* vals, int kind, int64_t n, int scale, const uint8_t* valid, const int64_t* off,
               uint8_t* out, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(fmt_write_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, vals, kind, n, scale,
                     valid, off, out);
  check_launch("fmt_write", stream);
}

void str_parse(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* valid, int kind, int scale,
               void* out, int* err, hipStream_t stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(parse_kernel, dim3(grid_for(n, kBlock, 65536)), dim3(kBlock), 0, stream, off, chars, n, valid,
                     kind, scale, out, err);
  check_launch("str_parse", stream);
}

}  // namespace kern
}  // namespace igloo
