// ZSTD frame decoder (RFC 8878) written once for a wave of W lanes: the GPU
// instantiates it with one 64-lane wave per compressed Parquet page
// (csrc/kernels/zstd.hip pq_zstd_kernel), the host with a one-lane "wave"
// (the CPU reference the tests compare against pyarrow's libzstd).
//
// Execution model on the GPU (one wave, 64 lanes):
//   * every entropy decode (FSE tables, Huffman weights and literals,
//     sequences) runs UNIFORMLY: all lanes compute the same values, so table
//     builds, bit reads and state updates need no broadcasts; compressed
//     bytes are read from an LDS window the wave refills cooperatively
//     (coalesced 16 B per lane) instead of one dependent global load per byte;
//   * decoded literals are written 64 symbols at a time (lane k keeps symbol
//     k of each group) to a per-workgroup global literal buffer;
//   * sequences are decoded in batches of at most 64 (one per lane, at most
//     kRing / 2 output bytes) and executed like the snappy kernel: short
//     literals and matches whose source precedes the batch copy in parallel,
//     one lane each; matches reading this batch's output and long elements
//     are then copied in order by the whole wave. Recent output is mirrored
//     in a 16 KiB LDS ring; older bytes are re-read from the output after a
//     workgroup-scope fence.
// Dictionaries are not supported (Parquet writers never use them); the
// content checksum is skipped.
#pragma once

#include <cstdint>

namespace igloo {
namespace zstd {

enum : int {
  ZE_OK = 0,
  ZE_MAGIC = 20,    // not a zstd frame
  ZE_DICT = 21,     // frame needs a dictionary
  ZE_CORRUPT = 22,  // malformed block / section / bitstream
  ZE_SIZE = 23,     // output does not match the expected size
  ZE_TABLE = 24,    // malformed FSE / Huffman table
};

constexpr int kRing = 16384;        // LDS mirror of the most recent output
constexpr int kWin = 4096;          // LDS window of compressed bytes
constexpr int kMaxLit = 1 << 17;    // literals of one block (<= 128 KiB)
constexpr int kMaxHufLog = 11;

// sequence-symbol decoding entry: value base + extra bits of the symbol, FSE
// state transition (next = base + nb bits)
struct SeqEntry {
  uint32_t val;
  uint8_t xb;
  uint8_t nb;
  uint16_t base;
};

struct Scratch {
  uint8_t ring[kRing];
  uint8_t win[kWin];
  uint16_t huf[1 << kMaxHufLog];   // (symbol << 8) | bits
  SeqEntry ll[512], of[256], ml[512];
  SeqEntry wt[64];                 // Huffman weight table (accuracy log <= 6)
  int16_t norm[64];
  uint16_t next[64];
  uint8_t weights[256];
  int32_t hcnt[16], hstart[16];    // Huffman weight counts / table starts
};

// every decoder function is inlined into the kernel, so the decoder state and
// bit readers live in registers (a call boundary would put them in scratch)
#define ZINL __host__ __device__ __attribute__((always_inline)) inline

ZINL int hibit(uint32_t v) { return 31 - __builtin_clz(v); }

// baselines and extra bits of the literal-length / match-length codes
// (arithmetic + switch: no local arrays, which would live in scratch)
ZINL void ll_code(int c, uint32_t* base, int* xb) {
  if (c < 16) {
    *base = c;
    *xb = 0;
  } else if (c >= 25) {
    *xb = c - 19;
    *base = 1u << (c - 19);
  } else {
    switch (c) {
      case 16: *base = 16; *xb = 1; break;
      case 17: *base = 18; *xb = 1; break;
      case 18: *base = 20; *xb = 1; break;
      case 19: *base = 22; *xb = 1; break;
      case 20: *base = 24; *xb = 2; break;
      case 21: *base = 28; *xb = 2; break;
      case 22: *base = 32; *xb = 3; break;
      case 23: *base = 40; *xb = 3; break;
      default: *base = 48; *xb = 4; break;
    }
  }
}
ZINL void ml_code(int c, uint32_t* base, int* xb) {
  if (c < 32) {
    *base = c + 3;
    *xb = 0;
  } else if (c >= 43) {
    *xb = c - 36;
    *base = (1u << (c - 36)) + 3;
  } else {
    switch (c) {
      case 32: *base = 35; *xb = 1; break;
      case 33: *base = 37; *xb = 1; break;
      case 34: *base = 39; *xb = 1; break;
      case 35: *base = 41; *xb = 1; break;
      case 36: *base = 43; *xb = 2; break;
      case 37: *base = 47; *xb = 2; break;
      case 38: *base = 51; *xb = 3; break;
      case 39: *base = 59; *xb = 3; break;
      case 40: *base = 67; *xb = 4; break;
      case 41: *base = 83; *xb = 4; break;
      default: *base = 99; *xb = 5; break;
    }
  }
}

// predefined distributions (RFC 8878 3.1.1.3.2.2), at namespace scope so the
// device reads them from constant memory
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// Wv: W (lanes), lane(), sync() (barrier), fence() (prior global stores
// visible to the wave's later loads), any(bool), ballot(bool), scan(int64)
// (inclusive), bcast(int64, lane), ld(p) (load of bytes this wave wrote).
template <class Wv>
struct Decoder {
  Wv& wv;
  Scratch& s;
  const uint8_t* src;
  int64_t slen;
  uint8_t* dst;
  int64_t dcap;
  uint8_t* lit;          // literal buffer (kMaxLit bytes, global)
  int64_t wlo, whi;      // window [wlo, whi) of src in s.win
  int64_t op;            // output bytes written
  int64_t frame0;        // output position of the current frame
  int err;
  int64_t rep0, rep1, rep2;
  int huf_log;           // 0: no Huffman table yet
  int ll_log, of_log, ml_log;
  bool ll_ok, of_ok, ml_ok;

  ZINL Decoder(Wv& w, Scratch& sc, const uint8_t* s_, int64_t sl, uint8_t* d, int64_t dc, uint8_t* l)
      : wv(w), s(sc), src(s_), slen(sl), dst(d), dcap(dc), lit(l), wlo(0), whi(0), op(0), frame0(0), err(ZE_OK),
        rep0(1), rep1(4), rep2(8), huf_log(0), ll_log(0), of_log(0), ml_log(0), ll_ok(false), of_ok(false),
        ml_ok(false) {}

  ZINL void fail(int code) {
    if (err == ZE_OK) err = code;
  }

  // ---- compressed bytes through the LDS window ------------------------------
  ZINL void refill(int64_t lo) {
    if (lo < 0) lo = 0;
    lo -= (int64_t)(((uintptr_t)(src + lo)) & 15);   // 16-byte aligned window start (never before src)
    if (lo < 0) lo = 0;
    int64_t hi = lo + kWin;
    if (hi > slen) hi = slen;
    wv.sync();
    const int64_t n = hi - lo;
    const uint8_t* p = src + lo;
    if ((((uintptr_t)p) & 15) == 0) {
      for (int64_t k = (int64_t)wv.lane() * 16; k < n; k += (int64_t)Wv::W * 16) {
        if (k + 16 <= n) {
          *reinterpret_cast<uint4*>(s.win + k) = *reinterpret_cast<const uint4*>(p + k);
        } else {
          for (int64_t t = k; t < n; ++t) s.win[t] = p[t];
        }
      }
    } else {
      for (int64_t k = wv.lane(); k < n; k += Wv::W) s.win[k] = p[k];
    }
    wv.sync();
    wlo = lo;
    whi = hi;
  }
  // forward / backward reads: the window is refilled ahead of / behind i
  ZINL uint32_t fb(int64_t i) {
    if (i < 0 || i >= slen) {
      fail(ZE_CORRUPT);
      return 0;
    }
    if (i < wlo || i >= whi) refill(i);
    return wv.uni(s.win[i - wlo]);
  }
  ZINL uint32_t bb(int64_t i) {
    if (i < 0 || i >= slen) {
      fail(ZE_CORRUPT);
      return 0;
    }
    if (i < wlo || i >= whi) refill(i - kWin + 64);
    return wv.uni(s.win[i - wlo]);
  }
  // a table entry, made wave-uniform (scalar registers and scalar ALU on the GPU)
  ZINL SeqEntry ent(const SeqEntry* t, uint32_t st) {
    uint64_t raw;
    __builtin_memcpy(&raw, &t[st], 8);
    raw = wv.uni64(raw);
    SeqEntry e;
    __builtin_memcpy(&e, &raw, 8);
    return e;
  }
  ZINL uint64_t le(int64_t i, int n) {
    uint64_t v = 0;
    for (int k = 0; k < n; ++k) v |= (uint64_t)fb(i + k) << (8 * k);
    return v;
  }

  // ---- backward bitstream: bits [0, pos) of [base, base + len), read from
  // the top; c holds bits [low, low + k) ----------------------------------
  struct Back {
    int64_t base, pos, low;
    uint64_t c;
    int k;
  };
  ZINL bool back_init(Back& b, int64_t base, int64_t len) {
    if (len <= 0) {
      fail(ZE_CORRUPT);
      return false;
    }
    const uint32_t last = bb(base + len - 1);
    if (last == 0) {
      fail(ZE_CORRUPT);
      return false;
    }
    const int h = hibit(last);
    b.base = base;
    b.low = (len - 1) * 8;
    b.pos = b.low + h;
    b.c = last & ((1u << h) - 1u);
    b.k = h;
    return true;
  }
  ZINL void back_fill(Back& b) {
    while (b.k <= 56 && b.low > 0) {
      b.low -= 8;
      b.c = (b.c << 8) | bb(b.base + (b.low >> 3));
      b.k += 8;
    }
  }
  ZINL uint32_t peek(Back& b, int n) {  // n in [1, 32]
    if (b.k < n) back_fill(b);
    const uint64_t m = (1ull << n) - 1ull;
    if (b.k >= n) return (uint32_t)((b.c >> (b.k - n)) & m);
    return (uint32_t)((b.c << (n - b.k)) & m);   // past the stream start: zeros
  }
  ZINL void skip(Back& b, int n) {
    b.k -= n;
    b.pos -= n;
    if (b.k < 0) b.k = 0;
  }
  ZINL uint32_t read(Back& b, int n) {
    if (n <= 0) return 0;
    const uint32_t v = peek(b, n);
    skip(b, n);
    return v;
  }

  // ---- FSE tables -------------------------------------------------------------
  // Normalized counts at [p, limit): accuracy log (or -1), symbols, bytes used.
  ZINL int read_ncount(int64_t p, int64_t limit, int max_sym, int max_log, int* nsym, int* used) {
    int64_t bit = 0;
    auto get = [&](int n) -> uint32_t {
      const int64_t q = p + (bit >> 3);
      uint32_t x = 0;
      for (int j = 0; j < 4; ++j)
        if (q + j < limit) x |= fb(q + j) << (8 * j);
      return (x >> (bit & 7)) & ((1u << n) - 1u);
    };
    const int al = (int)get(4) + 5;
    bit += 4;
    if (al > max_log) return -1;
    int remaining = (1 << al) + 1, threshold = 1 << al, nb = al + 1, sym = 0;
    while (remaining > 1 && sym <= max_sym) {
      const int maxv = 2 * threshold - 1 - remaining;
      const uint32_t v = get(nb);
      int count;
      if ((int)(v & (uint32_t)(threshold - 1)) < maxv) {
        count = (int)(v & (uint32_t)(threshold - 1));
        bit += nb - 1;
      } else {
        count = (int)(v & (uint32_t)(2 * threshold - 1));
        if (count >= threshold) count -= maxv;
        bit += nb;
      }
      --count;
      remaining -= count < 0 ? -count : count;
      s.norm[sym++] = (int16_t)count;
      if (count == 0) {
        for (;;) {
          const int r = (int)get(2);
          bit += 2;
          for (int z = 0; z < r && sym <= max_sym; ++z) s.norm[sym++] = 0;
          if (r != 3) break;
        }
      }
      while (remaining < threshold) {
        --nb;
        threshold >>= 1;
      }
    }
    if (remaining != 1 || sym > max_sym + 1) return -1;
    *nsym = sym;
    *used = (int)((bit + 7) >> 3);
    if (p + *used > limit) return -1;
    return al;
  }

  // Decoding table from s.norm[0, nsym) (kind 0: plain symbols, 1: LL, 2: ML, 3: OF).
  ZINL bool build(int nsym, int al, SeqEntry* t, int kind) {
    const int size = 1 << al;
    int high = size - 1;
    for (int x = 0; x < nsym; ++x) {
      if (s.norm[x] == -1) {
        t[high--].val = (uint32_t)x;
        s.next[x] = 1;
      } else {
        s.next[x] = (uint16_t)(s.norm[x] < 0 ? 0 : s.norm[x]);
      }
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int x = 0; x < nsym; ++x)
      for (int i = 0; i < s.norm[x]; ++i) {
        t[pos].val = (uint32_t)x;
        do {
          pos = (pos + step) & mask;
        } while (pos > high);
      }
    if (pos != 0) return false;
    for (int u = 0; u < size; ++u) {
      const int x = (int)t[u].val;
      const int nx = s.next[x]++;
      const int nb = al - hibit((uint32_t)nx);
      SeqEntry e;
      e.nb = (uint8_t)nb;
      e.base = (uint16_t)((nx << nb) - size);
      if (kind == 1) {
        int xb;
        ll_code(x, &e.val, &xb);
        e.xb = (uint8_t)xb;
      } else if (kind == 2) {
        int xb;
        ml_code(x, &e.val, &xb);
        e.xb = (uint8_t)xb;
      } else if (kind == 3) {
        e.val = 1u << x;
        e.xb = (uint8_t)x;
      } else {
        e.val = (uint32_t)x;
        e.xb = 0;
      }
      t[u] = e;
    }
    wv.sync();
    return true;
  }

  ZINL void rle_table(SeqEntry* t, int x, int kind) {
    SeqEntry e;
    e.nb = 0;
    e.base = 0;
    int xb = 0;
    if (kind == 1) ll_code(x, &e.val, &xb);
    else if (kind == 2) ml_code(x, &e.val, &xb);
    else {
      e.val = 1u << x;
      xb = x;
    }
    e.xb = (uint8_t)xb;
    t[0] = e;
    wv.sync();
  }

  ZINL bool predefined(int kind) {
    const int16_t* d = kind == 1 ? kLLNorm : kind == 2 ? kMLNorm : kOFNorm;
    const int n = kind == 1 ? 36 : kind == 2 ? 53 : 29;
    for (int i = 0; i < n; ++i) s.norm[i] = d[i];
    return build(n, kind == 3 ? 5 : 6, kind == 1 ? s.ll : kind == 2 ? s.ml : s.of, kind);
  }

  // ---- Huffman --------------------------------------------------------------
  // Tree description at p: bytes used, or -1.
  ZINL int64_t read_huffman(int64_t p, int64_t limit) {
    const uint32_t hb = fb(p);
    int nw = 0;
    int64_t used;
    if (hb < 128) {
      const int64_t q = p + 1, qend = q + hb;
      if (hb == 0 || qend > limit) return -1;
      int nsym, u;
      const int al = read_ncount(q, qend, 255, 6, &nsym, &u);
      if (al < 0 || !build(nsym, al, s.wt, 0)) return -1;
      Back b;
      if (!back_init(b, q + u, hb - u)) return -1;
      uint32_t s1 = read(b, al), s2 = read(b, al);
      for (;;) {
        if (nw > 253) return -1;
        const SeqEntry e1 = ent(s.wt, s1);
        s.weights[nw++] = (uint8_t)e1.val;
        s1 = e1.base + read(b, e1.nb);
        if (b.pos < 0) {
          s.weights[nw++] = (uint8_t)ent(s.wt, s2).val;
          break;
        }
        const SeqEntry e2 = ent(s.wt, s2);
        s.weights[nw++] = (uint8_t)e2.val;
        s2 = e2.base + read(b, e2.nb);
        if (b.pos < 0) {
          s.weights[nw++] = (uint8_t)ent(s.wt, s1).val;
          break;
        }
      }
      used = 1 + hb;
    } else {
      nw = (int)hb - 127;
      const int nbytes = (nw + 1) / 2;
      if (p + 1 + nbytes > limit) return -1;
      for (int i = 0; i < nw; ++i) {
        const uint32_t v = fb(p + 1 + i / 2);
        s.weights[i] = (uint8_t)((i & 1) ? (v & 15) : (v >> 4));
      }
      used = 1 + nbytes;
    }
    if (err) return -1;
    uint32_t total = 0;
    for (int i = 0; i < nw; ++i) {
      if (s.weights[i] > kMaxHufLog) return -1;
      if (s.weights[i]) total += 1u << (s.weights[i] - 1);
    }
    if (total == 0 || nw >= 256) return -1;
    const int maxb = hibit(total) + 1;
    const uint32_t left = (1u << maxb) - total;
    if (left == 0 || (left & (left - 1)) || maxb > kMaxHufLog) return -1;
    s.weights[nw++] = (uint8_t)(hibit(left) + 1);
    // canonical table: lower weights (longer codes) first, by symbol within a weight
    int32_t* cnt = s.hcnt;
    int32_t* start = s.hstart;
    for (int w = 0; w < 16; ++w) cnt[w] = 0;
    for (int i = 0; i < nw; ++i) cnt[s.weights[i]]++;
    int nxt = 0;
    for (int w = 1; w <= maxb; ++w) {
      start[w] = nxt;
      nxt += cnt[w] << (w - 1);
    }
    if (nxt != (1 << maxb)) return -1;
    wv.sync();
    for (int x = 0; x < nw; ++x) {
      const int w = s.weights[x];
      if (!w) continue;
      const int len = 1 << (w - 1);
      const int st = start[w];
      const uint16_t e = (uint16_t)((x << 8) | (maxb + 1 - w));
      for (int k = wv.lane(); k < len; k += Wv::W) s.huf[st + k] = e;
      wv.sync();
      start[w] = st + len;
    }
    wv.sync();
    huf_log = maxb;
    return used;
  }

  // One Huffman stream [q, q + len) -> `count` literals at out.
  ZINL bool huf_stream(int64_t q, int64_t len, int64_t count, uint8_t* out) {
    Back b;
    if (!back_init(b, q, len)) return false;
    const int lane = wv.lane();
    uint32_t mine = 0;
    const int hl = huf_log;
    for (int64_t i = 0; i < count; ++i) {
      const uint32_t e = wv.uni(s.huf[peek(b, hl)]);
      skip(b, e & 0xff);
      if (lane == (int)(i & (Wv::W - 1))) mine = e >> 8;
      if ((i & (Wv::W - 1)) == Wv::W - 1) out[i - (Wv::W - 1) + lane] = (uint8_t)mine;
    }
    const int64_t r = count & (Wv::W - 1);
    if (r && lane < r) out[count - r + lane] = (uint8_t)mine;
    return b.pos == 0 && err == ZE_OK;
  }

  // ---- output -----------------------------------------------------------------
  ZINL void put(int64_t o, uint8_t v) {
    dst[o] = v;
    s.ring[o & (kRing - 1)] = v;
  }
  // output byte p while executing a batch ending at `end`
  ZINL uint8_t got(int64_t p, int64_t end) {
    return p >= end - kRing ? s.ring[p & (kRing - 1)] : wv.ld(dst + p);
  }

  // whole-wave copies (raw blocks, long literals, RLE)
  ZINL void copy_in(const uint8_t* from, int64_t n, bool written) {
    for (int64_t k = wv.lane(); k < n; k += Wv::W) put(op + k, written ? wv.ld(from + k) : from[k]);
    op += n;
  }
  ZINL void fill(uint8_t v, int64_t n) {
    for (int64_t k = wv.lane(); k < n; k += Wv::W) put(op + k, v);
    op += n;
  }

  // A batch of n <= W sequences (lane k holds sequence k).
  ZINL bool exec_batch(int n, int64_t ll, int64_t ml, int64_t off, const uint8_t* lsrc, bool lwritten,
                                      int64_t* lused, int64_t lsize) {
    const int lane = wv.lane();
    const bool act = lane < n;
    if (!act) ll = ml = 0;
    const int64_t li = wv.scan(ll), oi = wv.scan(ll + ml);
    const int64_t lpos = *lused + li - ll, opos = op + oi - ll - ml;
    const int64_t ltot = wv.bcast(li, n - 1), otot = wv.bcast(oi, n - 1);
    const int64_t bstart = op, bend = op + otot;
    const int64_t ms = opos + ll - off;
    const bool bad = act && ((ml > 0 && (off <= 0 || ms < frame0)));
    if (wv.any(bad) || *lused + ltot > lsize || bend > dcap) {
      fail(ZE_CORRUPT);
      return false;
    }
    const int64_t kLong = 2 * Wv::W;
    const bool dep = act && ml > 0 && ms + ml > bstart;
    const bool llong = act && ll > kLong, mlong = act && ml > kLong;
    const bool far = act && ml > 0 && ms < bend - kRing;
    if (wv.any(far)) wv.fence();
    // 1. short literals and matches whose source precedes the batch, one lane each
    if (act && !llong)
      for (int64_t b = 0; b < ll; ++b) put(opos + b, lwritten ? wv.ld(lsrc + lpos + b) : lsrc[lpos + b]);
    if (act && !dep && !mlong)
      for (int64_t b = 0; b < ml; ++b) put(opos + ll + b, got(ms + b, bend));
    // 2. in order: long literals and long matches by the whole wave, short
    //    dependent matches by their own lane (its ring reads see the earlier
    //    elements' writes: one wave's LDS operations complete in order)
    // (one lane copies a dependent match of at most kLane bytes; longer ones
    // take the whole wave, 64 bytes per step)
    constexpr int64_t kLane = 8;
    const uint64_t wl = wv.ballot(llong), wm = wv.ballot(mlong || (dep && ml > kLane)),
                   sd = wv.ballot(dep && ml <= kLane);
    for (uint64_t todo = wl | wm | sd; todo; todo &= todo - 1) {
      const int k = __builtin_ctzll(todo);
      if ((wl >> k) & 1) {
        const int64_t kl = wv.bcast(ll, k), ko = wv.bcast(opos, k), kp = wv.bcast(lpos, k);
        for (int64_t b = lane; b < kl; b += Wv::W) put(ko + b, lwritten ? wv.ld(lsrc + kp + b) : lsrc[kp + b]);
        wv.sync();
      }
      if ((wm >> k) & 1) {
        const int64_t kl = wv.bcast(ll, k), km = wv.bcast(ml, k), ko = wv.bcast(opos, k);
        const int64_t kof = wv.bcast(off, k), kms = ko + kl - kof;
        if (kms < bend - kRing) wv.fence();
        wv.sync();
        for (int64_t b = lane; b < km; b += Wv::W) {
          const int64_t j = kof >= km ? b : b % kof;
          put(ko + kl + b, got(kms + j, bend));
        }
        wv.sync();
      } else if (((sd >> k) & 1) && lane == k) {
        for (int64_t b = 0; b < ml; ++b) put(opos + ll + b, got(ms + (off >= ml ? b : b % off), bend));
      }
    }
    wv.sync();
    *lused += ltot;
    op = bend;
    return true;
  }

  // ---- blocks -----------------------------------------------------------------
  ZINL bool table(int mode, int kind, int64_t* p, int64_t end) {
    SeqEntry* t = kind == 1 ? s.ll : kind == 2 ? s.ml : s.of;
    int* lg = kind == 1 ? &ll_log : kind == 2 ? &ml_log : &of_log;
    bool* ok = kind == 1 ? &ll_ok : kind == 2 ? &ml_ok : &of_ok;
    const int max_sym = kind == 1 ? 35 : kind == 2 ? 52 : 31;
    if (mode == 0) {
      if (!predefined(kind)) return false;
      *lg = kind == 3 ? 5 : 6;
    } else if (mode == 1) {
      const int x = (int)fb(*p);
      *p += 1;
      if (x > max_sym) return false;
      rle_table(t, x, kind);
      *lg = 0;
    } else if (mode == 2) {
      int nsym, used;
      const int al = read_ncount(*p, end, max_sym, kind == 3 ? 8 : 9, &nsym, &used);
      if (al < 0 || !build(nsym, al, t, kind)) return false;
      *p += used;
      *lg = al;
    } else if (!*ok) {
      return false;
    }
    *ok = true;
    return true;
  }

  ZINL bool block(int64_t p, int64_t end) {
    // -- literals section
    const uint32_t b0 = fb(p);
    const int ltype = b0 & 3, sf = (b0 >> 2) & 3;
    const uint8_t* lsrc;
    bool lwritten;
    int64_t lsize;
    if (ltype <= 1) {
      int hdr;
      if (sf == 0 || sf == 2) {
        lsize = b0 >> 3;
        hdr = 1;
      } else if (sf == 1) {
        lsize = (b0 >> 4) | (fb(p + 1) << 4);
        hdr = 2;
      } else {
        lsize = (b0 >> 4) | (fb(p + 1) << 4) | (fb(p + 2) << 12);
        hdr = 3;
      }
      if (lsize > kMaxLit) return false;
      if (ltype == 0) {
        if (p + hdr + lsize > end) return false;
        lsrc = src + p + hdr;
        lwritten = false;
        p += hdr + lsize;
      } else {
        if (p + hdr >= end) return false;
        const uint8_t v = (uint8_t)fb(p + hdr);
        for (int64_t k = wv.lane(); k < lsize; k += Wv::W) lit[k] = v;
        wv.fence();
        lsrc = lit;
        lwritten = true;
        p += hdr + 1;
      }
    } else {
      const int hdr = sf <= 1 ? 3 : sf == 2 ? 4 : 5;
      const int bits = sf <= 1 ? 10 : sf == 2 ? 14 : 18;
      const int streams = sf == 0 ? 1 : 4;
      const uint64_t h = le(p, hdr);
      lsize = (int64_t)((h >> 4) & ((1u << bits) - 1u));
      const int64_t comp = (int64_t)((h >> (4 + bits)) & ((1u << bits) - 1u));
      int64_t q = p + hdr;
      const int64_t qend = q + comp;
      if (lsize > kMaxLit || qend > end) return false;
      if (ltype == 2) {
        const int64_t used = read_huffman(q, qend);
        if (used < 0) {
          fail(ZE_TABLE);
          return false;
        }
        q += used;
      } else if (!huf_log) {
        return false;
      }
      if (streams == 1) {
        if (!huf_stream(q, qend - q, lsize, lit)) return false;
      } else {
        if (q + 6 > qend) return false;
        const int64_t s1 = (int64_t)le(q, 2), s2 = (int64_t)le(q + 2, 2), s3 = (int64_t)le(q + 4, 2);
        q += 6;
        const int64_t s4 = qend - q - s1 - s2 - s3;
        const int64_t seg = (lsize + 3) / 4, last = lsize - 3 * seg;
        if (s4 < 0 || last < 0) return false;
        if (!huf_stream(q, s1, seg, lit) || !huf_stream(q + s1, s2, seg, lit + seg) ||
            !huf_stream(q + s1 + s2, s3, seg, lit + 2 * seg) || !huf_stream(q + s1 + s2 + s3, s4, last, lit + 3 * seg))
          return false;
      }
      wv.fence();
      lsrc = lit;
      lwritten = true;
      p = qend;
    }
    // -- sequences section
    if (p >= end) return false;
    const uint32_t c0 = fb(p);
    int64_t nseq;
    if (c0 < 128) {
      nseq = c0;
      p += 1;
    } else if (c0 < 255) {
      nseq = ((c0 - 128) << 8) + fb(p + 1);
      p += 2;
    } else {
      nseq = fb(p + 1) + (fb(p + 2) << 8) + 0x7F00;
      p += 3;
    }
    int64_t lused = 0;
    if (nseq > 0) {
      if (p >= end) return false;
      const uint32_t modes = fb(p++);
      if (modes & 3) return false;
      if (!table((modes >> 6) & 3, 1, &p, end) || !table((modes >> 4) & 3, 3, &p, end) ||
          !table((modes >> 2) & 3, 2, &p, end)) {
        fail(ZE_TABLE);
        return false;
      }
      Back b;
      if (!back_init(b, p, end - p)) return false;
      uint32_t sl = read(b, ll_log), so = read(b, of_log), sm = read(b, ml_log);
      const int lane = wv.lane();
      int64_t i = 0;
      while (i < nseq) {
        int n = 0;
        int64_t bout = 0, my_ll = 0, my_ml = 0, my_off = 0;
        while (i < nseq && n < Wv::W) {
          const SeqEntry eo = ent(s.of, so), em = ent(s.ml, sm), el = ent(s.ll, sl);
          const int64_t ofv = (int64_t)eo.val + read(b, eo.xb);
          const int64_t mlv = (int64_t)em.val + read(b, em.xb);
          const int64_t llv = (int64_t)el.val + read(b, el.xb);
          int64_t off;
          if (ofv > 3) {
            off = ofv - 3;
            rep2 = rep1;
            rep1 = rep0;
            rep0 = off;
          } else {
            const int idx = (int)ofv - 1 + (llv == 0 ? 1 : 0);
            if (idx == 0) {
              off = rep0;
            } else {
              off = idx == 3 ? rep0 - 1 : idx == 1 ? rep1 : rep2;
              if (off == 0) off = 1;
              if (idx != 1) rep2 = rep1;
              rep1 = rep0;
              rep0 = off;
            }
          }
          if (i + 1 < nseq) {
            sl = el.base + read(b, el.nb);
            sm = em.base + read(b, em.nb);
            so = eo.base + read(b, eo.nb);
          }
          // a batch stays within half the ring (one oversized sequence goes alone)
          if (n > 0 && bout + llv + mlv > kRing / 2) {
            // undo nothing: execute the batch first, then this sequence alone
            if (!exec_batch(n, my_ll, my_ml, my_off, lsrc, lwritten, &lused, lsize)) return false;
            n = 0;
            bout = 0;
          }
          if (lane == n) {
            my_ll = llv;
            my_ml = mlv;
            my_off = off;
          }
          ++n;
          bout += llv + mlv;
          ++i;
          if (err) return false;
        }
        if (n && !exec_batch(n, my_ll, my_ml, my_off, lsrc, lwritten, &lused, lsize)) return false;
      }
      if (b.pos != 0) return false;
    } else if (p != end) {
      return false;
    }
    // trailing literals
    const int64_t rest = lsize - lused;
    if (rest < 0 || op + rest > dcap) return false;
    copy_in(lsrc + lused, rest, lwritten);
    wv.sync();
    return err == ZE_OK;
  }

  // Whole input: frames (skippable ones skipped). Returns an error code.
  ZINL int run() {
    int64_t ip = 0;
    while (ip < slen && !err) {
      const uint32_t magic = (uint32_t)le(ip, 4);
      if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
        ip += 8 + (int64_t)le(ip + 4, 4);
        continue;
      }
      if (magic != 0xFD2FB528u) return ZE_MAGIC;
      ip += 4;
      const uint32_t fhd = fb(ip++);
      const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, csum = (fhd >> 2) & 1, did = fhd & 3;
      if (fhd & 8) return ZE_CORRUPT;
      if (!single) ip += 1;
      const int dbytes = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
      if (dbytes && le(ip, dbytes) != 0) return ZE_DICT;
      ip += dbytes;
      const int fbytes = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
      int64_t fcs = -1;
      if (fbytes) fcs = (int64_t)le(ip, fbytes) + (fbytes == 2 ? 256 : 0);
      ip += fbytes;
      frame0 = op;
      rep0 = 1;
      rep1 = 4;
      rep2 = 8;
      huf_log = 0;
      ll_ok = of_ok = ml_ok = false;
      for (;;) {
        const uint32_t bh = (uint32_t)le(ip, 3);
        ip += 3;
        const int last = bh & 1, type = (bh >> 1) & 3;
        const int64_t size = bh >> 3;
        if (err) return err;
        if (type == 0) {
          if (ip + size > slen || op + size > dcap) return ZE_CORRUPT;
          copy_in(src + ip, size, false);
          ip += size;
        } else if (type == 1) {
          if (op + size > dcap) return ZE_CORRUPT;
          fill((uint8_t)fb(ip), size);
          ip += 1;
        } else if (type == 2) {
          if (ip + size > slen || !block(ip, ip + size)) return err ? err : ZE_CORRUPT;
          ip += size;
        } else {
          return ZE_CORRUPT;
        }
        wv.sync();
        if (last) break;
      }
      if (csum) ip += 4;
      if (fcs >= 0 && op - frame0 != fcs) return ZE_SIZE;
    }
    if (err) return err;
    return op == dcap ? ZE_OK : ZE_SIZE;
  }
};

}  // namespace zstd
}  // namespace igloo
