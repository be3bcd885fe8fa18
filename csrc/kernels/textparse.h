// Device text <-> value helpers shared by the CSV parser (csv.hip) and the
// string expression kernels (strexpr.hip): exact integer / fixed-point /
// date parsing, float parsing, and the inverse formatting used by
// CAST(... AS VARCHAR).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace igloo {
namespace kern {

__device__ inline int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

__device__ inline bool parse_int(const uint8_t* p, const uint8_t* e, int64_t* out) {
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
  if (p >= e) return false;
  uint64_t v = 0;
  for (; p < e; ++p) {
    const unsigned d = (unsigned)*p - '0';
    if (d > 9) return false;
    if (v > (uint64_t)922337203685477580ULL || (v == 922337203685477580ULL && d > 7 + (unsigned)neg)) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

// exact fixed point: digits[.digits] scaled to `scale` fractional digits
__device__ inline bool parse_decimal(const uint8_t* p, const uint8_t* e, int scale, int64_t* out) {
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
  if (p >= e) return false;
  __int128 v = 0;
  int frac = -1, digits = 0;
  for (; p < e; ++p) {
    if (*p == '.') {
      if (frac >= 0) return false;
      frac = 0;
      continue;
    }
    const unsigned d = (unsigned)*p - '0';
    if (d > 9) return false;
    if (frac >= 0) {
      if (frac == scale) {
        if (d != 0) return false;  // more fractional digits than the scale: not exact
        continue;
      }
      ++frac;
    }
    v = v * 10 + d;
    if (++digits > 36) return false;
  }
  for (int f = frac < 0 ? 0 : frac; f < scale; ++f) v *= 10;
  if (neg) v = -v;
  if (v > (__int128)INT64_MAX || v < (__int128)INT64_MIN) return false;
  *out = (int64_t)v;
  return true;
}

__device__ inline bool parse_f64(const uint8_t* p, const uint8_t* e, double* out) {
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
  if (p >= e) return false;
  uint64_t m = 0;
  int sig = 0, e10 = 0;
  bool any = false, dot = false;
  for (; p < e; ++p) {
    const uint8_t c = *p;
    if (c == '.') {
      if (dot) return false;
      dot = true;
      continue;
    }
    const unsigned d = (unsigned)c - '0';
    if (d > 9) break;
    any = true;
    if (sig < 19) {
      if (m || d) ++sig;
      m = m * 10 + d;
      if (dot) --e10;
    } else if (!dot) {
      ++e10;
    }
  }
  if (!any) return false;
  if (p < e) {
    if (*p != 'e' && *p != 'E') return false;
    ++p;
    int64_t x;
    if (!parse_int(p, e, &x) || x > 400 || x < -400) return false;
    e10 += (int)x;
  }
  double v = (double)m;
  // exact when m < 2^53 and |e10| <= 22 (both factors exactly representable)
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  if (e10 > 0) {
    while (e10 > 22) {
      v *= 1e22;
      e10 -= 22;
    }
    v *= p10[e10];
  } else if (e10 < 0) {
    while (e10 < -22) {
      v /= 1e22;
      e10 += 22;
    }
    v /= p10[-e10];
  }
  *out = neg ? -v : v;
  return true;
}

__device__ inline bool parse_date(const uint8_t* p, const uint8_t* e, int32_t* out) {
  if (e - p != 10 || p[4] != '-' || p[7] != '-') return false;
  int64_t y = 0, m = 0, d = 0;
  for (int k = 0; k < 4; ++k) {
    const unsigned c = (unsigned)p[k] - '0';
    if (c > 9) return false;
    y = y * 10 + c;
  }
  for (int k = 5; k < 7; ++k) {
    const unsigned c = (unsigned)p[k] - '0';
    if (c > 9) return false;
    m = m * 10 + c;
  }
  for (int k = 8; k < 10; ++k) {
    const unsigned c = (unsigned)p[k] - '0';
    if (c > 9) return false;
    d = d * 10 + c;
  }
  if (m < 1 || m > 12 || d < 1 || d > 31) return false;
  *out = (int32_t)days_from_civil(y, m, d);
  return true;
}

__device__ inline bool ieq(const uint8_t* p, const uint8_t* e, const char* lit) {
  int k = 0;
  for (; p + k < e; ++k) {
    if (!lit[k]) return false;
    uint8_t c = p[k];
    if (c >= 'A' && c <= 'Z') c += 32;
    if (c != (uint8_t)lit[k]) return false;
  }
  return lit[k] == 0;
}

// days since 1970-01-01 -> civil date (H. Hinnant's algorithm)
__device__ inline void civil_from_days(int64_t z, int64_t* y, int* m, int* d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  *d = (int)(doy - (153 * mp + 2) / 5 + 1);
  *m = (int)(mp < 10 ? mp + 3 : mp - 9);
  *y = yoe + era * 400 + (*m <= 2);
}

__device__ inline int u64_digits(uint64_t v) {
  int n = 1;
  while (v >= 10) {
    v /= 10;
    ++n;
  }
  return n;
}

// Text of a fixed-point value v * 10^-scale ("-12.05"; scale 0: an integer);
// returns the byte count, writes it when out != nullptr.
__device__ inline int format_fixed(int64_t v, int scale, uint8_t* out) {
  const bool neg = v < 0;
  const uint64_t u = neg ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  int digits = u64_digits(u);
  if (digits <= scale) digits = scale + 1;          // leading "0."
  const int len = (int)neg + digits + (scale > 0 ? 1 : 0);
  if (out) {
    uint64_t x = u;
    int pos = len - 1;
    for (int k = 0; k < scale; ++k) {
      out[pos--] = (uint8_t)('0' + x % 10);
      x /= 10;
    }
    if (scale > 0) out[pos--] = '.';
    do {
      out[pos--] = (uint8_t)('0' + x % 10);
      x /= 10;
    } while (x && pos >= (int)neg);
    while (pos >= (int)neg) out[pos--] = '0';
    if (neg) out[0] = '-';
  }
  return len;
}

// YYYY-MM-DD of a date32 (years 0000-9999; others as their decimal year)
__device__ inline int format_date(int32_t days, uint8_t* out) {
  int64_t y;
  int m, d;
  civil_from_days(days, &y, &m, &d);
  if (y < 0 || y > 9999) {
    const int n = format_fixed(y, 0, out);
    if (out) {
      out[n] = '-';
      out[n + 1] = (uint8_t)('0' + m / 10);
      out[n + 2] = (uint8_t)('0' + m % 10);
      out[n + 3] = '-';
      out[n + 4] = (uint8_t)('0' + d / 10);
      out[n + 5] = (uint8_t)('0' + d % 10);
    }
    return n + 6;
  }
  if (out) {
    out[0] = (uint8_t)('0' + y / 1000);
    out[1] = (uint8_t)('0' + y / 100 % 10);
    out[2] = (uint8_t)('0' + y / 10 % 10);
    out[3] = (uint8_t)('0' + y % 10);
    out[4] = '-';
    out[5] = (uint8_t)('0' + m / 10);
    out[6] = (uint8_t)('0' + m % 10);
    out[7] = '-';
    out[8] = (uint8_t)('0' + d / 10);
    out[9] = (uint8_t)('0' + d % 10);
  }
  return 10;
}

}  // namespace kern
}  // namespace igloo
