// to_char / date_format: dates and timestamps formatted with a chrono-style
// pattern (DataFusion's to_char, reference Cargo.lock:1062
// datafusion-functions, which formats with chrono's strftime syntax).
//
// Two passes over one lane per row, like the other variable-length string
// producers: strfmt_len_kernel writes each row's output length (exclusive
// scan -> offsets on the host side), strfmt_write_kernel writes the bytes.
// Supported: %Y %C %y %m %d %e %j %H %k %I %l %M %S %p %P %f %.3f %.6f %.9f
// %a %A %b %h %B %u %w %F %T %D %R %s %% ; other characters are copied.
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

constexpr int kMaxFmt = 128;

struct Civil {
  int64_t y;
  int m, d, doy, dow;        // dow: 0 = Sunday
  int hh, mi, ss;
  int64_t us;                // microseconds within the second
  int64_t epoch_s;
};

__device__ inline Civil civil(int64_t t_us) {
  Civil c;
  int64_t days = t_us >= 0 ? t_us / 86400000000LL : -((-t_us + 86400000000LL - 1) / 86400000000LL);
  int64_t rem = t_us - days * 86400000000LL;
  c.epoch_s = t_us >= 0 ? t_us / 1000000 : -((-t_us + 999999) / 1000000);
  c.hh = (int)(rem / 3600000000LL);
  rem -= (int64_t)c.hh * 3600000000LL;
  c.mi = (int)(rem / 60000000LL);
  rem -= (int64_t)c.mi * 60000000LL;
  c.ss = (int)(rem / 1000000LL);
  c.us = rem - (int64_t)c.ss * 1000000LL;
  c.dow = (int)(((days % 7) + 11) % 7);   // 1970-01-01 was a Thursday (4)
  // civil_from_days
  int64_t z = days + 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int64_t y = yoe + era * 400;
  const int64_t doyp = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doyp + 2) / 153;
  const int d = (int)(doyp - (153 * mp + 2) / 5 + 1);
  const int m = (int)(mp < 10 ? mp + 3 : mp - 9);
  y += m <= 2;
  c.y = y;
  c.m = m;
  c.d = d;
  const bool leap = (y % 4 == 0 && y % 100 != 0) || y % 400 == 0;
  const int cum[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
  c.doy = cum[m - 1] + d + (leap && m > 2 ? 1 : 0);
  return c;
}

__constant__ char kDays[7][10] = {"Sunday", "Monday", "Tuesday", "Wednesday", "Thursday", "Friday", "Saturday"};
__constant__ char kMonths[12][10] = {"January", "February", "March",     "April",   "May",      "June",
                                     "July",    "August",   "September", "October", "November", "December"};

struct Out {
  uint8_t* p;      // null: count only
  int64_t n = 0;
  __device__ void ch(uint8_t c) {
    if (p) p[n] = c;
    ++n;
  }
  __device__ void num(int64_t v, int width, uint8_t pad = '0') {
    char buf[24];
    bool neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-v) : (uint64_t)v;
    int k = 0;
    do {
      buf[k++] = (char)('0' + u % 10);
      u /= 10;
    } while (u);
    if (neg) ch('-');
    for (int i = k; i < width; ++i) ch(pad);
    while (k) ch((uint8_t)buf[--k]);
  }
  __device__ void str(const char* s, int maxn) {
    for (int i = 0; i < maxn && s[i]; ++i) ch((uint8_t)s[i]);
  }
};

__device__ void format_one(const uint8_t* fmt, int flen, const Civil& c, Out& o) {
  for (int i = 0; i < flen; ++i) {
    const uint8_t f = fmt[i];
    if (f != '%' || i + 1 >= flen) {
      o.ch(f);
      continue;
    }
    uint8_t s = fmt[++i];
    int frac = 0;
    if (s == '.' && i + 1 < flen) {   // %.3f / %.6f / %.9f / %.f
      uint8_t dgt = fmt[i + 1];
      if (dgt == 'f') {
        frac = 9;
        ++i;
      } else if (i + 2 < flen && (dgt == '3' || dgt == '6' || dgt == '9') && fmt[i + 2] == 'f') {
        frac = dgt - '0';
        i += 2;
      }
      if (frac) {
        o.ch('.');
        const int64_t ns = c.us * 1000;
        int64_t v = frac == 3 ? ns / 1000000 : frac == 6 ? ns / 1000 : ns;
        o.num(v, frac);
        continue;
      }
      o.ch('%');
      o.ch('.');
      continue;
    }
    switch (s) {
      case 'Y': o.num(c.y, 4); break;
      case 'C': o.num(c.y / 100, 2); break;
      case 'y': o.num(((c.y % 100) + 100) % 100, 2); break;
      case 'm': o.num(c.m, 2); break;
      case 'd': o.num(c.d, 2); break;
      case 'e': o.num(c.d, 2, ' '); break;
      case 'j': o.num(c.doy, 3); break;
      case 'H': o.num(c.hh, 2); break;
      case 'k': o.num(c.hh, 2, ' '); break;
      case 'I': o.num(c.hh % 12 == 0 ? 12 : c.hh % 12, 2); break;
      case 'l': o.num(c.hh % 12 == 0 ? 12 : c.hh % 12, 2, ' '); break;
      case 'M': o.num(c.mi, 2); break;
      case 'S': o.num(c.ss, 2); break;
      case 'p': o.str(c.hh < 12 ? "AM" : "PM", 2); break;
      case 'P': o.str(c.hh < 12 ? "am" : "pm", 2); break;
      case 'f': o.num(c.us * 1000, 9); break;
      case 'a': o.str(kDays[c.dow], 3); break;
      case 'A': o.str(kDays[c.dow], 10); break;
      case 'b':
      case 'h': o.str(kMonths[c.m - 1], 3); break;
      case 'B': o.str(kMonths[c.m - 1], 10); break;
      case 'u': o.num(c.dow == 0 ? 7 : c.dow, 1); break;
      case 'w': o.num(c.dow, 1); break;
      case 'F': o.num(c.y, 4); o.ch('-'); o.num(c.m, 2); o.ch('-'); o.num(c.d, 2); break;
      case 'T': o.num(c.hh, 2); o.ch(':'); o.num(c.mi, 2); o.ch(':'); o.num(c.ss, 2); break;
      case 'R': o.num(c.hh, 2); o.ch(':'); o.num(c.mi, 2); break;
      case 'D': o.num(c.m, 2); o.ch('/'); o.num(c.d, 2); o.ch('/'); o.num(((c.y % 100) + 100) % 100, 2); break;
      case 's': o.num(c.epoch_s, 1); break;
      case '%': o.ch('%'); break;
      default: o.ch('%'); o.ch(s); break;
    }
  }
}

struct FmtArgs {
  uint8_t fmt[kMaxFmt];
  int flen;
  int is_date;     // values are int32 days (else int64 microseconds)
};

__device__ inline int64_t value_us(const FmtArgs& a, const void* v, int64_t r) {
  return a.is_date ? (int64_t)((const int32_t*)v)[r] * 86400000000LL : ((const int64_t*)v)[r];
}

__global__ __launch_bounds__(kBlock) void strfmt_len_kernel(FmtArgs a, const void* __restrict__ v, int64_t n,
                                                          int64_t* __restrict__ len) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    Out o{nullptr};
    format_one(a.fmt, a.flen, civil(value_us(a, v, r)), o);
    len[r] = o.n;
  }
}

__global__ __launch_bounds__(kBlock) void strfmt_write_kernel(FmtArgs a, const void* __restrict__ v, int64_t n,
                                                            const int64_t* __restrict__ off, int64_t out_cap,
                                                            uint8_t* __restrict__ out) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const Civil c = civil(value_us(a, v, r));
    Out probe{nullptr};
    format_one(a.fmt, a.flen, c, probe);
    const int64_t o0 = off[r];
    if (o0 < 0 || off[r + 1] - o0 != probe.n || off[r + 1] > out_cap) continue;   // bounded like strfn_copy
    Out o{out + o0};
    format_one(a.fmt, a.flen, c, o);
  }
}

}  // namespace

void strfmt_lengths(const uint8_t* fmt, int flen, bool is_date, const void* v, int64_t n, int64_t* len,
                    hipStream_t s) {
  if (flen > kMaxFmt) throw std::runtime_error("to_char: format longer than 128 bytes");
  if (n == 0) return;
  FmtArgs a;
  for (int i = 0; i < flen; ++i) a.fmt[i] = fmt[i];
  a.flen = flen;
  a.is_date = is_date;
  hipLaunchKernelGGL(strfmt_len_kernel, dim3(grid_for(n, kBlock, 1 << 14)), dim3(kBlock), 0, s, a, v, n, len);
  check_launch("strfmt_len", s);
}

void strfmt_write(const uint8_t* fmt, int flen, bool is_date, const void* v, int64_t n, const int64_t* off,
                  int64_t out_cap, uint8_t* out, hipStream_t s) {
  if (flen > kMaxFmt) throw std::runtime_error("to_char: format longer than 128 bytes");
  if (n == 0) return;
  FmtArgs a;
  for (int i = 0; i < flen; ++i) a.fmt[i] = fmt[i];
  a.flen = flen;
  a.is_date = is_date;
  hipLaunchKernelGGL(strfmt_write_kernel, dim3(grid_for(n, kBlock, 1 << 14)), dim3(kBlock), 0, s, a, v, n, off,
                     out_cap, out);
  check_launch("strfmt_write", s);
}

}  // namespace kern
}  // namespace igloo
