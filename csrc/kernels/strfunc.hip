// Scalar string functions over plain (offsets + bytes) UTF-8 columns:
// btrim / ltrim / rtrim, replace, lpad / rpad, reverse, repeat, left / right,
// initcap, translate, split_part (string -> string) and strpos / ascii /
// octet_length (string -> int32).
//
// String -> string functions run in two passes over the rows, one lane per
// row (grid-stride): pass 1 computes each output length with the SAME device
// routine that pass 2 uses to write (out == nullptr counts only), the host
// scans the lengths into offsets, pass 2 writes every row at its offset. Row
// strings are short (TPC-H comments <= 117 bytes), so a lane per row keeps the
// byte loops in registers; constant arguments (trim sets, search / replacement
// strings, fill) live in a small device buffer read through the L1/L2.
// Parity: DataFusion's string function library (datafusion-functions 48,
// reference Cargo.lock:1062), reached through SessionContext::sql
// (reference crates/engine/src/lib.rs:54-57).
#include "common.h"
#include "kernels.h"

namespace igloo {
namespace kern {

namespace {

__device__ __forceinline__ int utf8_len(uint8_t c) {
  return c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
}

// is the character at s[0..l) one of the characters of `set` (UTF-8)
__device__ bool in_set(const uint8_t* s, int l, const uint8_t* set, int64_t setlen) {
  for (int64_t k = 0; k < setlen;) {
    int m = utf8_len(set[k]);
    if (m == l) {
      bool eq = true;
      for (int q = 0; q < l; ++q) eq &= set[k + q] == s[q];
      if (eq) return true;
    }
    k += m;
  }
  return false;
}

// index (in characters) of the character s[0..l) in `set`, -1 when absent
__device__ int64_t set_index(const uint8_t* s, int l, const uint8_t* set, int64_t setlen) {
  int64_t idx = 0;
  for (int64_t k = 0; k < setlen; ++idx) {
    int m = utf8_len(set[k]);
    if (m == l) {
      bool eq = true;
      for (int q = 0; q < l; ++q) eq &= set[k + q] == s[q];
      if (eq) return idx;
    }
    k += m;
  }
  return -1;
}

// byte offset of the `k`-th character (0-based) of the `cnt`-th character of set
__device__ int64_t char_at(const uint8_t* set, int64_t setlen, int64_t k, int* l) {
  int64_t b = 0;
  for (int64_t i = 0; b < setlen; ++i) {
    int m = utf8_len(set[b]);
    if (i == k) {
      *l = m;
      return b;
    }
    b += m;
  }
  *l = 0;
  return setlen;
}

__device__ int64_t nchars(const uint8_t* s, int64_t n) {
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i) c += (s[i] & 0xC0) != 0x80;
  return c;
}

// byte offset of character index k (0-based; k >= chars -> n)
__device__ int64_t byte_of_char(const uint8_t* s, int64_t n, int64_t k) {
  if (k <= 0) return 0;
  int64_t c = 0;
  for (int64_t i = 0; i < n; ++i) {
    if ((s[i] & 0xC0) != 0x80) {
      if (c == k) return i;
      ++c;
    }
  }
  return n;
}

struct Emit {
  uint8_t* out;
  int64_t len = 0;
  __device__ void byte(uint8_t c) {
    if (out) out[len] = c;
    ++len;
  }
  __device__ void bytes(const uint8_t* p, int64_t m) {
    if (out)
      for (int64_t q = 0; q < m; ++q) out[len + q] = p[q];
    len += m;
  }
};

__device__ inline bool is_alnum(uint8_t c) {
  return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c >= 0x80;
}

__device__ int64_t apply(const StrFnArgs& a, const uint8_t* s, int64_t n, uint8_t* out) {
  Emit e{out};
  switch (a.fn) {
    case kSfTrim: {
      int64_t b = 0, t = n;
      if (a.n1 & 1) {
        while (b < t) {
          int l = utf8_len(s[b]);
          if (b + l > t || !in_set(s + b, l, a.a, a.alen)) break;
          b += l;
        }
      }
      if (a.n1 & 2) {
        while (t > b) {
          int64_t p = t - 1;
          while (p > b && (s[p] & 0xC0) == 0x80) --p;
          if (!in_set(s + p, (int)(t - p), a.a, a.alen)) break;
          t = p;
        }
      }
      e.bytes(s + b, t - b);
      break;
    }
    case kSfReplace: {
      if (a.alen == 0) {
        e.bytes(s, n);
        break;
      }
      for (int64_t i = 0; i < n;) {
        bool hit = i + a.alen <= n;
        for (int64_t q = 0; hit && q < a.alen; ++q) hit = s[i + q] == a.a[q];
        if (hit) {
          e.bytes(a.b, a.blen);
          i += a.alen;
        } else {
          e.byte(s[i++]);
        }
      }
      break;
    }
    case kSfLpad:
    case kSfRpad: {
      const int64_t want = a.n1 < 0 ? 0 : a.n1;
      const int64_t c = nchars(s, n);
      if (c >= want) {
        e.bytes(s, byte_of_char(s, n, want));
        break;
      }
      const int64_t fill_chars = nchars(a.a, a.alen);
      if (fill_chars == 0) {
        e.bytes(s, n);
        break;
      }
      if (a.fn == kSfRpad) e.bytes(s, n);
      for (int64_t k = 0; k < want - c; ++k) {
        int l;
        int64_t b = char_at(a.a, a.alen, k % fill_chars, &l);
        e.bytes(a.a + b, l);
      }
      if (a.fn == kSfLpad) e.bytes(s, n);
      break;
    }
    case kSfReverse: {
      for (int64_t t = n; t > 0;) {
        int64_t p = t - 1;
        while (p > 0 && (s[p] & 0xC0) == 0x80) --p;
        e.bytes(s + p, t - p);
        t = p;
      }
      break;
    }
    case kSfRepeat:
      for (int64_t k = 0; k < a.n1; ++k) e.bytes(s, n);
      break;
    case kSfLeft: {
      int64_t k = a.n1;
      if (k < 0) k = nchars(s, n) + k;
      e.bytes(s, byte_of_char(s, n, k < 0 ? 0 : k));
      break;
    }
    case kSfRight: {
      const int64_t c = nchars(s, n);
      int64_t skip = a.n1 >= 0 ? c - a.n1 : -a.n1;
      if (skip < 0) skip = 0;
      const int64_t b = byte_of_char(s, n, skip);
      e.bytes(s + b, n - b);
      break;
    }
    case kSfInitcap: {
      bool start = true;
      for (int64_t i = 0; i < n; ++i) {
        uint8_t ch = s[i];
        if (ch < 0x80 && ch >= 'A' && ch <= 'Z' && !start) ch += 32;
        else if (ch < 0x80 && ch >= 'a' && ch <= 'z' && start) ch -= 32;
        e.byte(ch);
        if ((ch & 0xC0) != 0x80) start = !is_alnum(ch);
      }
      break;
    }
    case kSfTranslate: {
      const int64_t to_chars = nchars(a.b, a.blen);
      for (int64_t i = 0; i < n;) {
        int l = utf8_len(s[i]);
        if (i + l > n) l = (int)(n - i);
        int64_t k = set_index(s + i, l, a.a, a.alen);
        if (k < 0) {
          e.bytes(s + i, l);
        } else if (k < to_chars) {
          int tl;
          int64_t b = char_at(a.b, a.blen, k, &tl);
          e.bytes(a.b + b, tl);
        }
        i += l;
      }
      break;
    }
    case kSfSplitPart: {
      // part n1 (1-based; negative counts from the end) of s split by a.a
      if (a.alen == 0) {
        if (a.n1 == 1 || a.n1 == -1) e.bytes(s, n);
        break;
      }
      int64_t parts = 1;
      for (int64_t i = 0; i + a.alen <= n;) {
        bool hit = true;
        for (int64_t q = 0; hit && q < a.alen; ++q) hit = s[i + q] == a.a[q];
        if (hit) {
          ++parts;
          i += a.alen;
        } else {
          ++i;
        }
      }
      int64_t want = a.n1 > 0 ? a.n1 : parts + a.n1 + 1;
      if (want < 1 || want > parts) break;
      int64_t cur = 1, b = 0;
      for (int64_t i = 0; i <= n;) {
        bool hit = i + a.alen <= n;
        for (int64_t q = 0; hit && q < a.alen; ++q) hit = s[i + q] == a.a[q];
        if (hit || i == n) {
          if (cur == want) {
            e.bytes(s + b, i - b);
            break;
          }
          ++cur;
          i += a.alen;
          b = i;
          if (!hit) break;
        } else {
          ++i;
        }
      }
      break;
    }
    default:
      break;
  }
  return e.len;
}

__global__ __launch_bounds__(kBlock) void strfn_len_kernel(StrFnArgs a, const int64_t* __restrict__ off,
                                                           const uint8_t* __restrict__ chars, int64_t n,
                                                           int64_t* __restrict__ out_len) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = off[i];
    out_len[i] = apply(a, chars + b, off[i + 1] - b, nullptr);
  }
}

__global__ __launch_bounds__(kBlock) void strfn_copy_kernel(StrFnArgs a, const int64_t* __restrict__ off,
                                                            const uint8_t* __restrict__ chars, int64_t n,
                                                            const int64_t* __restrict__ new_off,
                                                            uint8_t* __restrict__ out, int64_t out_cap) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = off[i];
    const int64_t o = new_off[i], e = new_off[i + 1];
    // the row's output range must lie in the buffer and match what the
    // length pass computes for it (a replayed total can disagree)
    if (o < 0 || e < o || e > out_cap) continue;
    if (apply(a, chars + b, off[i + 1] - b, nullptr) != e - o) continue;
    apply(a, chars + b, off[i + 1] - b, out + o);
  }
}

// one instantiation per function: a runtime switch over the three bodies in
// one kernel was mis-compiled (the octet-length branch stored stale data)
template <int FN>
__global__ __launch_bounds__(kBlock) void strfn_int_kernel(const uint8_t* __restrict__ pat, int64_t plen,
                                                           const int64_t* __restrict__ off,
                                                           const uint8_t* __restrict__ chars, int64_t n,
                                                           int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* s = chars + off[i];
    const int64_t m = off[i + 1] - off[i];
    int32_t v = 0;
    if constexpr (FN == kSfStrpos) {
      // 1-based character position of the first occurrence, 0 when absent
      int64_t c = 0;
      v = plen == 0 ? 1 : 0;
      for (int64_t j = 0; plen > 0 && j + plen <= m; ++j) {
        if ((s[j] & 0xC0) != 0x80) ++c;
        bool hit = true;
        for (int64_t q = 0; hit && q < plen; ++q) hit = s[j + q] == pat[q];
        if (hit) {
          v = (int32_t)c;
          break;
        }
      }
    } else if constexpr (FN == kSfAscii) {
      if (m > 0) {
        const uint8_t c0 = s[0];
        const int l = utf8_len(c0);
        uint32_t cp = l == 1 ? c0 : l == 2 ? (c0 & 0x1F) : l == 3 ? (c0 & 0x0F) : (c0 & 0x07);
        for (int q = 1; q < l && q < m; ++q) cp = (cp << 6) | (s[q] & 0x3F);
        v = (int32_t)cp;
      }
    } else {  // octet length
      v = (int32_t)m;
    }
    out[i] = v;
  }
}

}  // namespace

void str_fn_lengths(const StrFnArgs& a, const int64_t* off, const uint8_t* chars, int64_t n, int64_t* len,
                    hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(strfn_len_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, s, a, off, chars, n, len);
  check_launch("strfn.len", s);
}

void str_fn_copy(const StrFnArgs& a, const int64_t* off, const uint8_t* chars, int64_t n, const int64_t* new_off,
                 uint8_t* out, int64_t out_cap, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(strfn_copy_kernel, dim3(grid_for(n, kBlock, 1 << 16)), dim3(kBlock), 0, s, a, off, chars, n,
                     new_off, out, out_cap);
  check_launch("strfn.copy", s);
}

void str_fn_int(int fn, const uint8_t* pat, int64_t plen, const int64_t* off, const uint8_t* chars, int64_t n,
                int32_t* out, hipStream_t s) {
  if (n == 0) return;
  dim3 g(grid_for(n, kBlock, 1 << 16)), b(kBlock);
  if (fn == kSfStrpos)
    hipLaunchKernelGGL(strfn_int_kernel<kSfStrpos>, g, b, 0, s, pat, plen, off, chars, n, out);
  else if (fn == kSfAscii)
    hipLaunchKernelGGL(strfn_int_kernel<kSfAscii>, g, b, 0, s, pat, plen, off, chars, n, out);
  else if (fn == kSfOctetLength)
    hipLaunchKernelGGL(strfn_int_kernel<kSfOctetLength>, g, b, 0, s, pat, plen, off, chars, n, out);
  else
    throw std::runtime_error("str_fn_int: bad function");
  check_launch("strfn.int", s);
}

}  // namespace kern
}  // namespace igloo
