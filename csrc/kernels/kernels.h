// Host-side API of the igloo gfx950 kernel library. Every entry point takes
// raw device pointers plus the HIP stream to launch on (the caller's current
// torch stream), never allocates, and never synchronises — so a caller may
// capture sequences of them into a hipGraph (cdna_hip_programming.md G9).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace igloo {
namespace kern {

constexpr int kMaxAggs = 8;
constexpr int kMaxGatherCols = 16;
constexpr int kMaxParts = 64;

// ---- select.hip / scan.hip ---------------------------------------------------
int64_t select_num_tiles(int64_t n);
void select_count(const uint8_t* mask, int64_t n, int64_t* tile_counts, int64_t* total, hipStream_t stream);
void select_write(const uint8_t* mask, int64_t n, const int64_t* tile_offsets, void* out, bool idx64, int64_t cap,
                  hipStream_t stream);
void scan_counts(int64_t* counts, int64_t n, int64_t* total, hipStream_t stream);
constexpr int kMaxCompactCols = 12;
struct CompactCol {
  const void* src;
  void* dst;
  int esz;              // 1, 2, 4, 8 or 16 bytes per row
  const uint8_t* sv;    // source validity (bytes) or null
  uint8_t* dv;          // destination validity
};
struct CompactArgs {
  CompactCol cols[kMaxCompactCols];
  int ncols;
  void* idx;            // optional: the surviving row indices too
  bool idx64;
};
// columns compacted by a mask whose tile offsets select_count produced (cap: rows the outputs hold)
void select_compact(const uint8_t* mask, int64_t n, const int64_t* tile_offsets, const CompactArgs& a, int64_t cap,
                    hipStream_t stream);
int64_t scan_workspace_tiles(int64_t n);
void exclusive_scan(const void* in, bool in64, int64_t n, int64_t* out, int64_t* tile_ws, int64_t* total,
                    hipStream_t stream);

// ---- sort.hip -------------------------------------------------------------------
constexpr int kMaxSortCols = 8;
// kind: 0 signed int (width 1/2/4/8), 1 float64, 2 uint8/bool, 3 float32.
// Field = ordered(value) - lo (DESC: span - that), `bits` wide; a nullable
// column adds a NULL flag bit above the field.
struct SortKeyCol {
  const void* ptr;
  const uint8_t* valid;
  uint64_t lo, span;
  int32_t kind, width, bits, desc, nulls_first, pad;
};
struct SortKeySpec {
  int32_t ncols, pad;
  SortKeyCol cols[kMaxSortCols];
};
int64_t radix_sort_ws_bytes(int64_t n);
// Stable LSD sort of (key, value) pairs on key bits [begin_bit, end_bit).
// Returns 0 when the result is in (k0, v0), 1 when in (k1, v1).
int radix_sort_pairs(void* k0, void* k1, bool key64, void* v0, void* v1, bool val64, int64_t n, int begin_bit,
                     int end_bit, void* ws, hipStream_t stream);
// out: uint32 keys when out32 (total field width <= 32), else uint64
void sort_key_pack(const SortKeySpec& spec, const void* perm, bool perm64, int64_t n, void* out, bool out32,
                   hipStream_t stream);
void radix_digit_hist(const void* keys, bool key64, int64_t n, int shift, uint64_t prefix, int pshift,
                      unsigned long long* hist, hipStream_t stream);
void radix_le_mask(const void* keys, bool key64, int64_t n, uint64_t bound, uint8_t* mask, hipStream_t stream);

// ---- pack.hip -------------------------------------------------------------------
constexpr int kMaxPackCols = 48;
struct PackCol {
  const void* src;  // pack: source column (row stride = width)
  void* dst;        // unpack: destination column
  int32_t width, offset;
};
struct PackSpec {
  int32_t ncols, row_bytes;
  PackCol cols[kMaxPackCols];
};
void pack_rows(const PackSpec& spec, const void* perm, bool perm64, int64_t n, uint8_t* out, hipStream_t stream);
void unpack_rows(const PackSpec& spec, const uint8_t* in, int64_t n, hipStream_t stream);

// ---- util.hip -------------------------------------------------------------------
void const_ints(int64_t* out, const int64_t* vals, int64_t n, hipStream_t stream);
constexpr int kMaxPackBits = 8;
void pack_bits(const void* const* cols, const bool* is64, const int64_t* lo, const int* shift, int ncols, int64_t n,
               int64_t* out, hipStream_t stream);
void differs_from_rep(const void* a, int elem_bytes, const void* rep, bool rep64, int64_t n, int* flag,
                      hipStream_t stream);
void mark_slot_rows(const int32_t* trow, int64_t cap, int64_t n, uint8_t* mark, hipStream_t stream);
void mark_keys(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin, int64_t dom,
               uint8_t* marks, hipStream_t stream);
void probe_marks(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t base, int64_t dom,
                 const uint8_t* marks, bool negate, uint8_t* out, hipStream_t stream);
void end_capture(hipStream_t stream);
// out: kStatsSlots int64 (min, max, unsorted flag, then per-block partials)
constexpr int kStatsMaxBlocks = 4096;
constexpr int kStatsSlots = 3 + 3 * kStatsMaxBlocks;
void column_stats(const void* keys, bool key64, const uint8_t* valid, int64_t n, long long* out, hipStream_t stream);
void run_bounds(const void* keys, bool key64, int64_t n, uint8_t* out, hipStream_t stream);

// ---- fused.hip ----------------------------------------------------------------
constexpr int kFfMaxCols = 8;
constexpr int kFfMaxTerms = 16;
constexpr int kFfMaxAggs = 8;
constexpr int kFfMaxGroups = 16;
constexpr int kFfMaxFactors = 3;
struct FfColumn {
  const void* ptr;
  int64_t width;  // bytes: 1, 2, 4, 8 (signed except 1 = uint8/bool)
};
// kind 0: lo <= v <= hi; 1: NOT (lo <= v <= hi); 2: v in bitmask `set` (0 <= v < 64);
// 3: lo <= v - col[set] <= hi (column-vs-column comparison, e.g. l_commitdate < l_receiptdate)
struct FfTerm {
  int32_t col, kind;
  int64_t lo, hi;
  uint64_t set;
};
// value factor: col < 0 -> a, else a + b * col
struct FfFactor {
  int64_t col, a, b;
};
// op: 0 sum (int128: dst = lo, dst2 = hi), 1 count, 2 min, 3 max (int64)
// shared > 0: the first `shared` factors equal the previous aggregate's whole
// product (its value is reused; the host orders aggregates to form such chains)
struct FfAgg {
  int32_t op, nfac;
  int32_t checked, shared;
  FfFactor f[kFfMaxFactors];
  int64_t* dst;
  int64_t* dst2;
  int32_t vbits, pad;   // bound on the value's two's-complement width (0 = 64)
};
struct FfSpec {
  int32_t ncols, nterms, nkeys, naggs, ngroups, pad;
  FfColumn cols[kFfMaxCols];
  FfTerm terms[kFfMaxTerms];
  int32_t key_col[2];
  int64_t key_lo[2];
  int64_t key_mul[2];
  FfAgg aggs[kFfMaxAggs];
  const uint8_t* mask;  // optional precomputed conjunct (nullptr = none)
  int64_t* counts;      // [ngroups] rows per group (aggregate only)
  int* overflow;        // set when a checked product overflows int64
};
void ff_mask(const FfSpec& spec, int64_t n, uint8_t* out, hipStream_t stream);
void ff_aggregate(const FfSpec& spec, int64_t n, hipStream_t stream);
// one-hot MFMA aggregation (SUM / COUNT, <= 16 groups) on / off; returns the previous setting
bool ff_set_mfma(bool on);

// ---- sketch.hip --------------------------------------------------------------
constexpr int kHllBits = 12;
constexpr int kHllRegisters = 1 << kHllBits;
constexpr int kHllMaxBlocks = 1024;
int hll_blocks(int64_t n);
// block_regs: [hll_blocks(n) x kHllRegisters] workspace; regs: [kHllRegisters] output
void hll_sketch(const void* keys, bool key64, const uint8_t* valid, int64_t n, uint8_t* block_regs, uint8_t* regs,
                hipStream_t stream);

// ---- hashtable.hip -----------------------------------------------------------
// bits/bmask: optional Bloom filter (bits: (bmask+1)/32 words, zeroed before
// join_build; nullptr disables it on build or probe)
// Row ids (thead, CSR cstart/crows, first / build-row outputs) are int32 when
// rid64 is false (build side < 2^31 rows) and int64 otherwise.
void join_build(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t* tkeys, void* thead, bool rid64,
                int64_t cap, int64_t kmin, bool direct, unsigned long long* dups, uint32_t* bits, uint64_t bmask,
                hipStream_t stream);
// CSR runs of a duplicate-key build: cnt[cap+1] zeroed -> per-slot counts;
// cstart = exclusive scan of cnt (cap+1 entries); scatter fills crows[n] and
// consumes cnt
void join_csr_count(const void* keys, bool key64, const uint8_t* valid, int64_t n, const int64_t* tkeys, void* cnt,
                    bool rid64, int64_t cap, int64_t kmin, bool direct, hipStream_t stream);
void join_csr_scatter(const void* keys, bool key64, const uint8_t* valid, int64_t n, const int64_t* tkeys, void* cnt,
                      const void* cstart, void* crows, bool rid64, int64_t cap, int64_t kmin, bool direct,
                      hipStream_t stream);
// cstart/crows null: unique build (thead only)
void join_probe(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const void* thead, const void* cstart, const void* crows, bool rid64, int64_t cap, int64_t kmin,
                bool direct, int32_t* counts, void* first, uint8_t* build_matched, const uint32_t* bits,
                uint64_t bmask, hipStream_t stream);
// first-match probe as a row selection: pass 1 hit bits (words[tiles*128]) + per-tile counts, pass 2
// (tile_off = exclusive scan of the counts) writes hit rows (+ their build rows) in row order
int64_t probe_hit_tiles(int64_t m);
void set_probe_grid_cap(int cap);
void set_probe_bits(int mode);
void probe_hits(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                const void* thead, bool rid64, int64_t cap, int64_t kmin, bool direct, const uint32_t* bits,
                uint64_t bmask, bool negate, unsigned long long* words, int64_t* tile_counts, hipStream_t stream);
void probe_write(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const void* thead, bool rid64, int64_t cap, int64_t kmin, bool direct, const unsigned long long* words,
                 const int64_t* tile_off, void* out_probe, bool out64, void* out_build, int64_t out_cap,
                 hipStream_t stream);
void join_expand(const void* keys, bool key64, const uint8_t* valid, int64_t m, const int64_t* tkeys,
                 const void* thead, const void* cstart, const void* crows, bool rid64, int64_t cap, int64_t kmin,
                 bool direct, const int64_t* offsets, int32_t* out_probe, void* out_build, const uint32_t* bits,
                 uint64_t bmask, int64_t out_cap, hipStream_t stream);
// run ids of a non-decreasing key column: gid[i] = r for rows in [starts[r], starts[r+1])
void fill_runs(const void* starts, bool starts64, int64_t nruns, int64_t n, int32_t* gid, hipStream_t stream);
void groupby_build(const void* keys, bool key64, int64_t n, int64_t* tkeys, int32_t* trow, int64_t cap, int64_t kmin,
                   bool direct, hipStream_t stream);
void groupby_occupied(const int32_t* trow, int64_t cap, uint8_t* occ, int32_t* gid_of_slot, hipStream_t stream);
void groupby_assign(const void* slots, bool slots64, int64_t g, int64_t cap, const int32_t* trow,
                    int32_t* gid_of_slot, int32_t* rep_row, hipStream_t stream);
void groupby_lookup(const void* keys, bool key64, int64_t n, const int64_t* tkeys, const int32_t* gid_of_slot,
                    int64_t cap, int64_t kmin, bool direct, int32_t* gid, hipStream_t stream);

// ---- agg.hip -------------------------------------------------------------------
enum AggOp : int {
  AGG_SUM_INT = 0,  // exact: dst = lo (u64), dst2 = hi (i64)
  AGG_SUM_F64 = 1,
  AGG_COUNT = 2,
  AGG_MIN_INT = 3,
  AGG_MAX_INT = 4,
  AGG_MIN_F64 = 5,  // state is the order-preserving int64 image of the double
  AGG_MAX_F64 = 6,
  AGG_BIT_AND = 7,  // integer bitwise folds (bit_and / bit_or / bit_xor)
  AGG_BIT_OR = 8,
  AGG_BIT_XOR = 9,
};

struct AggDesc {
  int op;
  int src64;             // integer sources: 1 = int64, 0 = int32
  const void* src;       // null for COUNT(*)
  const uint8_t* valid;  // null = all rows valid
  void* dst;             // [ngroups] 8-byte states
  void* dst2;            // [ngroups] high words for AGG_SUM_INT
  int64_t groups = 0;    // set by agg_update: states past it are never written (0: unchecked)
};

int agg_lds_max_groups(int nagg);
// sorted keys: GROUP BY key HAVING descs[hagg] <hop> constant, fused (agg.hip):
// passing runs -> rep[] (run start rows, unordered), descs[k].dst/dst2 [slot];
// counter[0] = runs written (may exceed cap), counter[1] = 1 when a run was
// longer than the kernel follows (caller falls back). hop: = <> < <= > >=
void sorted_having(const void* keys, bool key64, int64_t n, const AggDesc* descs, int nagg, int hagg, int hop,
                   long long hlo, long long hhi, double hf, int64_t* rep, int64_t cap, unsigned long long* counter,
                   hipStream_t stream);
// counts[k - kmin] += 1 per valid key in [kmin, kmin + span) (int32 counters, zeroed by the caller)
void key_histogram(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin, int64_t span,
                   int32_t* counts, hipStream_t stream);
// radix-partitioned variant for large domains (span <= 2^27, n < 2^31): phase 0 per-(bucket, block)
// counts -> cnt[buckets * blocks]; caller scans them into off; phase 1 scatters 16-bit low keys into
// part[total]; phase 2 counts each bucket in LDS into counts[span]
int key_histogram_buckets(int64_t span);
int key_histogram_blocks();
void key_histogram_partitioned(const void* keys, bool key64, const uint8_t* valid, int64_t n, int64_t kmin,
                               int64_t span, int phase, int32_t* cnt, const int64_t* off, int64_t total,
                               uint16_t* part, int32_t* counts, hipStream_t stream);
// radix-partitioned GROUP BY aggregate for many groups (agg.hip): phase 0 per-(bucket, block) row
// counts -> cnt[buckets * blocks] (caller scans them into off, total on the device); phase 1 scatters the
// low group-id bits into pg[n] and one int64 input per aggregate into vals[k][n] (vals[k] null: COUNT(*));
// phase 2 aggregates each bucket in LDS and adds it into the descs' zero / sentinel-initialised states.
int agg_part_bits(int nagg);
int agg_part_buckets(int64_t ngroups, int nagg);
int agg_part_blocks();
void agg_partitioned(const int32_t* gid, int64_t n, int64_t ngroups, const AggDesc* descs, int nagg, int phase,
                     int32_t* cnt, const int64_t* off, const int64_t* total, uint16_t* pg, int64_t* const* vals,
                     hipStream_t stream);
void agg_update(const int32_t* gid, int64_t n, int ngroups, const AggDesc* descs, int nagg, hipStream_t stream,
                bool sorted_gids = false);

// ---- gather.hip ----------------------------------------------------------------
struct GatherDesc {
  const void* src;
  void* dst;
  int elem_bytes;  // 1, 2, 4, 8, 16
  const uint8_t* src_valid;
  uint8_t* dst_valid;  // null = do not produce validity
  int64_t src_rows;    // indices outside [0, src_rows) gather NULL / zero (a replayed size can
                       // leave an index buffer's tail unwritten: never read past the source)
};
void gather_multi(const void* idx, bool idx64, int64_t n, const GatherDesc* descs, int ncols, hipStream_t stream);
// one field of a row-packed source (gather_packed): bytes [off, off + width) of
// each row, widened to out_bytes (sign-extended when flags & kPackedSigned);
// flags & kPackedInRange writes 1 for an index inside the source instead
constexpr int kMaxPackedFields = 16;
constexpr int kPackedSigned = 1;
constexpr int kPackedInRange = 2;
struct PackedField {
  void* dst;
  int32_t off;
  int32_t width;      // 1, 2, 4, 8 (naturally aligned inside the row)
  int32_t out_bytes;  // 1, 2, 4, 8
  int32_t flags;
};
// rows idx of a [src_rows, row_bytes] packed matrix (row_bytes 8/16/24/32)
// split into up to kMaxPackedFields output columns: one row load per index
// instead of one cache line per column (ops/packed_gather.py)
void gather_packed(const void* idx, bool idx64, int64_t n, const uint8_t* src, int64_t src_rows, int row_bytes,
                   const PackedField* fields, int nf, hipStream_t stream);
void str_gather_lengths(const int64_t* off, int64_t src_rows, const void* idx, bool idx64, int64_t n, int64_t* len,
                        hipStream_t stream);
void str_gather_copy(const int64_t* off, int64_t src_rows, const uint8_t* chars, const void* idx, bool idx64,
                     int64_t n, const int64_t* new_off, uint8_t* out, int64_t out_cap, hipStream_t stream);

// ---- strings.hip ---------------------------------------------------------------
void str_like(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* pat, const uint8_t* kind, int m,
              bool case_insensitive, bool negate, uint8_t* out, hipStream_t stream);
void str_case(const uint8_t* in, int64_t nbytes, bool to_upper, uint8_t* out, int* non_ascii, hipStream_t stream);
void str_substr_lengths(const int64_t* off, const uint8_t* chars, int64_t n, int64_t start, int64_t len, bool has_len,
                        int64_t* out_len, hipStream_t stream);
void str_substr_copy(const int64_t* off, const uint8_t* chars, int64_t n, int64_t start, int64_t len, bool has_len,
                     const int64_t* new_off, uint8_t* out, hipStream_t stream);
// string expressions (strexpr.hip)
void str_char_length(const int64_t* off, const uint8_t* chars, int64_t n, int32_t* out, hipStream_t stream);
void str_concat2_lengths(const int64_t* oa, bool ba, const int64_t* ob, bool bb, int64_t n, int64_t* len,
                         hipStream_t stream);
void str_concat2_copy(const int64_t* oa, const uint8_t* ca, bool ba, const int64_t* ob, const uint8_t* cb, bool bb,
                      int64_t n, const int64_t* off, uint8_t* out, hipStream_t stream);
void fmt_lengths(const void* vals, int kind, int64_t n, int scale, const uint8_t* valid, int64_t* len,
                 hipStream_t stream);
void fmt_write(const void* vals, int kind, int64_t n, int scale, const uint8_t* valid, const int64_t* off,
               uint8_t* out, hipStream_t stream);
void str_parse(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* valid, int kind, int scale,
               void* out, int* err, hipStream_t stream);
// LIKE made of '%'-separated literals (no '_'): segments concatenated in `seg`
// with offsets seg_off[nseg+1]; anchor_start/end = pattern does not begin/end with '%';
// min_seg = the shortest segment's length (host-known: picks the kernel)
void str_like_segments(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* seg, const int32_t* seg_off,
                       int nseg, bool anchor_start, bool anchor_end, bool negate, uint8_t* out, int64_t nbytes,
                       int min_seg, hipStream_t stream);
void wide_fits(const int64_t* lo, const int64_t* hi, int64_t n, int* flag, hipStream_t stream);
void avg_wide(const int64_t* sums, bool wide, const int64_t* cnt, int64_t n, int64_t up, int64_t* out,
              hipStream_t stream);
void str_prefix_keys(const int64_t* off, const uint8_t* chars, int64_t n, int chunks, int64_t* out,
                     hipStream_t stream);
void str_hash64(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* valid, int64_t* out,
                hipStream_t stream);
void str_eq_rows(const int64_t* aoff, const uint8_t* achars, const void* ai, const int64_t* boff, const uint8_t* bchars,
                 const void* bi, bool idx64, int64_t n, int* mismatches, hipStream_t stream);
void str_cmp_const(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* c, int64_t cn, int op,
                   uint8_t* out, hipStream_t stream);
// rows equal to (vmode 1: starting with) one of nv constants (bytes vb, offsets voff[nv + 1])
void str_in_set(const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* vb, const int32_t* voff,
                const uint8_t* vmode, int nv, uint8_t* out, hipStream_t stream);
void str_prefix_key(const int64_t* off, const uint8_t* chars, int64_t n, int64_t skip, int64_t* out,
                    hipStream_t stream);

// ---- partition.hip -------------------------------------------------------------
int64_t partition_run_blocks(int64_t n);
void partition_run(const void* keys, bool key64, int64_t n, int nparts, int64_t* counts_ws, int64_t* total,
                   void* perm, bool perm64, hipStream_t stream);
void partition_ids(const void* keys, bool key64, int64_t n, int nparts, int32_t* out, hipStream_t stream);
void date_part(const int32_t* days, int64_t n, int field, int32_t* out, hipStream_t stream);

// ---- datagen.hip ---------------------------------------------------------------
enum TextKind : int {
  TEXT_WORDS = 0,
  TEXT_DISTINCT_WORDS = 1,
  TEXT_ALNUM = 2,
  TEXT_PREFIX_INT = 3,
  TEXT_PREFIX_RANDINT = 4,
  TEXT_PHONE = 5,
};

struct TextGenParams {
  int kind;
  uint64_t seed;
  int64_t row_base;  // global row id of local row 0
  int min_len, max_len;
  const uint8_t* vocab;
  const int32_t* vocab_off;
  int vocab_n;
  const uint8_t* inject;  // injected phrase (WORDS) or prefix (PREFIX_*)
  int inject_len;
  int inject_every;
  int suffix_char;
  const int32_t* aux;  // per-row int input (PHONE: nation key)
  const int64_t* row_ids;  // optional per-row global ids (partitioned generation)
};
void textgen_lengths(const TextGenParams& p, int64_t n, int64_t* lens, bool device, hipStream_t stream);
void textgen_write(const TextGenParams& p, int64_t n, const int64_t* off, uint8_t* chars, bool device,
                   hipStream_t stream);

// ---- csv.hip -------------------------------------------------------------------
constexpr int64_t kCsvTile = 16 * 1024;  // bytes per wave in the row-splitting passes
enum CsvKind : int { CSV_SKIP = 0, CSV_INT32 = 1, CSV_INT64 = 2, CSV_DECIMAL = 3, CSV_FLOAT64 = 4, CSV_DATE = 5,
                     CSV_BOOL = 6, CSV_UTF8 = 7 };
struct CsvColumn {
  int32_t kind, scale;  // scale: CSV_DECIMAL fractional digits
  void* out;            // values [rows]; CSV_UTF8: int64 address of the field bytes
  int64_t* len;         // CSV_UTF8: byte length (bit 62 set: quoted field with "" escapes)
  uint8_t* valid;       // [rows] or null (then an empty numeric field is an error)
};
int64_t csv_num_tiles(int64_t n);
void csv_quote_parity(const uint8_t* buf, int64_t n, uint8_t quote, uint8_t* tile_par, hipStream_t stream);
// rows_end == null: count terminators per tile into tile_rows; else write them at tile_off[tile]
void csv_rows(const uint8_t* buf, int64_t n, int64_t start, uint8_t quote, const uint8_t* tile_state,
              int64_t* tile_rows, const int64_t* tile_off, int64_t* rows_end, hipStream_t stream);
void csv_parse(const uint8_t* buf, int64_t start, const int64_t* rows_end, int64_t nrows, const CsvColumn* cols,
               int ncols, uint8_t delim, uint8_t quote, int* err, hipStream_t stream);
void csv_str_lengths(const int64_t* len_flag, int64_t n, int64_t* len, hipStream_t stream);
void csv_str_copy(const int64_t* pos, const int64_t* len_flag, const int64_t* off, int64_t n, uint8_t quote,
                  uint8_t* out, hipStream_t stream);

// ---- digest.hip (md5 / sha2 hex digests of strings, uuid v4) --------------------
enum DigestAlgo : int { kDigestMd5 = 0, kDigestSha224 = 1, kDigestSha256 = 2, kDigestSha384 = 3, kDigestSha512 = 4 };
int digest_width(int algo);   // hex characters per digest
// out: n * digest_width(algo) bytes (row r at r * width)
void digest_hex(int algo, const int64_t* off, const uint8_t* chars, int64_t n, uint8_t* out, hipStream_t s);
void uuid_v4(uint64_t seed, int64_t n, uint8_t* out, hipStream_t s);   // out: n * 36 bytes

// ---- strfmt.hip (to_char / date_format with chrono-style patterns) --------------
// v: int32 days (is_date) or int64 microseconds; lengths pass, then writes at off (bounded by out_cap)
void strfmt_lengths(const uint8_t* fmt, int flen, bool is_date, const void* v, int64_t n, int64_t* len,
                    hipStream_t s);
void strfmt_write(const uint8_t* fmt, int flen, bool is_date, const void* v, int64_t n, const int64_t* off,
                  int64_t out_cap, uint8_t* out, hipStream_t s);

// ---- regex.hip (byte-class DFA match per string; table built by ops/regex_dfa.py) ---
size_t regex_lds_bytes(int nstates, int nclasses);
void regex_dfa_match(const int64_t* off, const uint8_t* chars, int64_t n, const uint16_t* table, const uint8_t* cls,
                     const uint8_t* flags, int nstates, int nclasses, int start, bool anchored_end, bool negate,
                     uint8_t* out, hipStream_t s);

// ---- mfma_probe.hip (MFMA vs VALU hash / compare experiment, scripts/mfma_hash_ab.py) ---
void probe_hash16(bool mfma, const int32_t* k0, const int32_t* k1, const int32_t* k2, const int32_t* k3, int64_t n,
                  const int8_t* proj, uint32_t* out, hipStream_t s);
// pats: npat x 16 bytes (first len used); out[r] = string r equals one of them
void probe_inlist16(bool mfma, const int64_t* off, const uint8_t* chars, int64_t n, const uint8_t* pats, int npat,
                    int len, uint8_t* out, hipStream_t s);

// ---- nested.hip (LIST rows: [n, 2] int64 (start, length) into a child column) ---
void list_element_idx(const int64_t* se, const uint8_t* valid, const int64_t* pos, const uint8_t* pos_valid,
                      int64_t pos_const, int64_t n, int64_t child_n, int64_t* out, hipStream_t s);
void interleave_idx(int64_t n, int k, int64_t* out, hipStream_t s);
void list_slots(int64_t n, int64_t k, int64_t* se, hipStream_t s);

// ---- json.hip (NDJSON records; rows split by csv_rows with no quote) ------------
// names / name_off: the schema's field names, packed (ncols <= 64); cols as csv_parse
void json_parse(const uint8_t* buf, int64_t start, const int64_t* rows_end, int64_t nrows, const CsvColumn* cols,
                int ncols, const uint8_t* names, const int32_t* name_off, int* err, hipStream_t stream);
void json_str_copy(const int64_t* pos, const int64_t* len_flag, const int64_t* off, int64_t n, uint8_t* out,
                   hipStream_t stream);

// ---- ranges.hip ----------------------------------------------------------------
// big: non-decreasing int32/int64 keys; per probe key q[i]: big[lo[i] .. lo[i]+cnt[i]) == q[i]
// fence (optional): big[j * kFence] for j < nf (ops/hashing.py search_fence)
constexpr int64_t kFence = 256;
void sorted_ranges(const void* big, bool key64, int64_t nb, const void* q, const uint8_t* qvalid, int64_t nq,
                   int64_t* lo, int64_t* cnt, const void* fence, int64_t nf, hipStream_t stream);
// off: exclusive offsets [ns] of the range lengths (total = sum); pairs (s, lo[s] + k) for k < len(s)
void expand_ranges(const int64_t* off, const int64_t* lo, int64_t ns, int64_t total, void* sidx, void* bidx,
                   bool out64, hipStream_t stream);
// second equality key inside the first key's ranges: offsets == null -> counts[ns] of matches,
// else pairs written at offsets (exclusive scan of those counts)
// lower-bound table first[k-kmin] (kmax-kmin+2 entries) of a sorted key column, and range lookups in it
void dense_index_build(const void* big, bool key64, int64_t nb, int64_t kmin, int64_t kmax, void* first, bool first64,
                       int32_t* long_gap, hipStream_t stream);
void dense_ranges(const void* first, bool first64, int64_t kmin, int64_t kmax, const void* q, bool key64,
                  const uint8_t* qvalid, int64_t nq, int64_t* lo, int64_t* cnt, hipStream_t stream);
// probe keys into DISTINCT sorted keys (nb < 2^31): hit[i] 0/1 and pos[i] (int32 row, 0 on a miss);
// first != null: through the dense lower-bound table, else a (fenced) binary search of big
void unique_lookup(const void* big, bool key64, int64_t nb, const void* first, bool first64, int64_t kmin,
                   int64_t kmax, const void* q, const uint8_t* qvalid, int64_t nq, uint8_t* hit, int32_t* pos,
                   const void* fence, int64_t nf, hipStream_t stream);
// hit[i] = exists k in [lo[i], lo[i]+cnt[i]) with big2[k] OP small2[i] (op: 0 =, 1 <>, 2 <, 3 <=, 4 >, 5 >=)
void sorted_exists(const void* big2, const void* small2, bool key64, const int64_t* lo, const int64_t* cnt,
                   int64_t ns, int op, const uint8_t* mask, uint8_t* hit, hipStream_t stream);
void sorted_match(const void* big2, const void* small2, bool key64, const int64_t* lo, const int64_t* cnt,
                  int64_t ns, int32_t* counts, const int64_t* offsets, void* sidx, void* bidx, bool out64,
                  int64_t out_cap, int32_t* first, hipStream_t stream);
// the (small row, big row) pairs of sorted ranges whose big row is set in
// ``mask`` (the big side's filter): pass 1 counts (offsets null), pass 2 writes
void sorted_masked(const uint8_t* mask, const int64_t* lo, const int64_t* cnt, int64_t ns, int32_t* counts,
                   const int64_t* offsets, void* sidx, void* bidx, bool out64, int64_t out_cap, hipStream_t stream);

// ---- parquet.hip ---------------------------------------------------------------
enum PqPhys : int { PQ_PHYS_BOOLEAN = 0, PQ_PHYS_INT32 = 1, PQ_PHYS_INT64 = 2, PQ_PHYS_INT96 = 3, PQ_PHYS_FLOAT = 4,
                    PQ_PHYS_DOUBLE = 5, PQ_PHYS_BYTE_ARRAY = 6, PQ_PHYS_FLBA = 7 };
enum PqPageKind : int { PQ_PAGE_DATA_V1 = 0, PQ_PAGE_DATA_V2 = 1, PQ_PAGE_DICT = 2 };
enum PqPageFlags : int { PQ_DATA_IN_DEC = 1, PQ_DICT_IN_DEC = 2 };
enum PqConv : int { PQ_CONV_COPY = 0, PQ_CONV_NARROW = 1, PQ_CONV_SEXT = 2, PQ_CONV_ZEXT = 3, PQ_CONV_F2D = 4,
                    PQ_CONV_FLBA = 5, PQ_CONV_MUL = 6, PQ_CONV_DIV = 7, PQ_CONV_BOOL = 8 };

// One page of a column, planned on the host (csrc/io/parquet_meta.cpp).
// Offsets are into the staged raw buffer, or the decompression buffer when
// the matching PQ_*_IN_DEC flag is set.
struct PqPage {
  int64_t data_off;    // payload (values; v1 pages start with the level streams)
  int64_t levels_off;  // v2: definition levels (raw buffer); -1 otherwise
  int64_t dict_off;    // the chunk's dictionary payload; -1 if none
  int64_t out_row;     // first output row
  int64_t aux_off;     // DELTA_* / BYTE_STREAM_SPLIT pages: decoded values (decompression buffer); -1 otherwise
  int32_t size;        // payload bytes at data_off
  int32_t num_values;  // rows of the page (flat columns)
  int32_t levels_len;  // v2 definition-level bytes
  int32_t encoding;    // parquet Encoding of the values
  int32_t kind;        // PqPageKind
  int32_t flags;       // PqPageFlags
  int32_t dict_base;   // first global dictionary slot of the chunk
  int32_t dict_count;  // dictionary entries of the chunk
};
static_assert(sizeof(PqPage) == 72, "PqPage layout is shared with the host planner");

// A compressed page payload: raw -> decompression buffer, by codec
enum PqJobCodec : int { PQ_CODEC_SNAPPY = 1, PQ_CODEC_ZSTD = 6 };
struct PqSnappyJob {
  int64_t src_off;  // raw buffer
  int64_t dst_off;  // decompression buffer
  int32_t src_len, dst_len;
  int32_t codec;    // PqJobCodec (parquet CompressionCodec numbering)
  int32_t pad;
};
static_assert(sizeof(PqSnappyJob) == 32, "PqSnappyJob layout is shared with the host planner");

struct PqDecodeSpec {
  int32_t phys, type_len, out_width, conv;
  int64_t conv_k;   // PQ_CONV_MUL / PQ_CONV_DIV factor
  int32_t max_def, pad;
  void* out;        // fixed width values [rows]
  uint8_t* valid;   // [rows] or null (then the column must have no NULLs)
  uint32_t* scratch;  // [rows] compact value index -> dictionary index / byte offset
  int64_t* str_len;   // strings, plain output: per-row length
  int64_t* str_pos;   // ... and address of the bytes
  int32_t* codes;     // strings, dictionary output: global dictionary slot per row
  int64_t* dict_len;  // [dictionary entries] (BYTE_ARRAY dictionaries)
  int64_t* dict_pos;
  const uint8_t* raw;
  const uint8_t* dec;
  int* error;         // first error code (0 = ok)
};

void pq_snappy(const PqSnappyJob* jobs, int64_t njobs, const uint8_t* raw, uint8_t* dec, int* error,
               hipStream_t stream);
// zstd.hip: ZSTD pages, one 64-lane workgroup each; `lit` holds `slots` literal
// buffers of 128 KiB (slots = pq_zstd_slots(njobs) workgroups run at a time)
constexpr int64_t kZstdMaxSlots = 1024;
int64_t pq_zstd_slots(int64_t njobs);
void pq_zstd(const PqSnappyJob* jobs, int64_t njobs, const uint8_t* raw, uint8_t* dec, uint8_t* lit, int64_t slots,
             int* error, hipStream_t stream);
// host reference decoder (same code, one lane): 0 or a zstd error code (20..24)
int zstd_decompress_host(const uint8_t* src, int64_t slen, uint8_t* dst, int64_t dcap);
// pages of several columns in one launch: page_col[i] indexes specs[] (device arrays)
void pq_dict_strings(const PqPage* pages, int64_t npages, const int32_t* page_col, const PqDecodeSpec* specs,
                     hipStream_t stream);
void pq_decode(const PqPage* pages, int64_t npages, const int32_t* page_col, const PqDecodeSpec* specs,
               hipStream_t stream);
void pq_str_copy(const int64_t* pos, const int64_t* off, int64_t n, uint8_t* out, hipStream_t stream);

// ---- window.hip (window functions over rows sorted by partition / order keys)
enum WinVal { kWinI64 = 0, kWinI32 = 1, kWinF64 = 2, kWinOne = 3, kWinHeadIdx = 4, kWinHead2 = 5 };
enum WinFn {
  kWinRowNumber = 0, kWinRank = 1, kWinDenseRank = 2, kWinPercentRank = 3, kWinCumeDist = 4, kWinNtile = 5,
  kWinLag = 10, kWinFirst = 11, kWinLast = 12, kWinNth = 13
};
int64_t win_scan_tiles(int64_t n);
// op: 0 sum i64, 1 sum f64, 2 min i64, 3 max i64, 4 min f64, 5 max f64; tflag/tval: win_scan_tiles(n) slots
void win_seg_scan(const void* ids, bool ids64, const void* ids2, bool ids2_64, const void* vals, int vkind,
                  const uint8_t* valid, int64_t n, int op, bool reverse, int* tflag, int64_t* tval, int64_t* out,
                  int* err, hipStream_t s);
void win_bounds(int64_t n, const int64_t* seg_start, const int64_t* seg_end, const int64_t* peer_start,
                const int64_t* peer_end, int unit, int skind, int64_t soff_i, double soff_f, int ekind,
                int64_t eoff_i, double eoff_f, const void* key, bool key_f64, const uint8_t* key_valid, bool desc,
                const int64_t* gnum, const int64_t* gpos, int64_t ngroups, int64_t* lo, int64_t* hi,
                hipStream_t s);
void win_frame_sum(const int64_t* psum, bool f64, const int64_t* pcnt, const int64_t* lo, const int64_t* hi,
                   int64_t n, int64_t* sum_out, int64_t* cnt_out, hipStream_t s);
// sparse table [levels][n] of min / max (floats as ordered int64) and its O(1) frame queries
void win_sparse_build(const int64_t* vals, bool f64, const uint8_t* valid, int64_t n, bool is_max, int levels,
                      int64_t* table, hipStream_t s);
void win_sparse_query(const int64_t* table, int levels, int64_t n, const int64_t* lo, const int64_t* hi,
                      const int64_t* pcnt, bool is_max, bool f64, int64_t* out, uint8_t* out_valid, hipStream_t s);
void win_frame_minmax(const int64_t* vals, bool f64, bool is_max, const uint8_t* valid, const int64_t* lo,
                      const int64_t* hi, int64_t n, int64_t* out, uint8_t* out_valid, hipStream_t s);
void win_rank(int fn, int64_t arg, int64_t n, const int64_t* seg_start, const int64_t* seg_end,
              const int64_t* peer_start, const int64_t* peer_end, const int64_t* dense, int64_t* out,
              hipStream_t s);
void win_index(int fn, int64_t arg, int64_t n, const int64_t* seg_start, const int64_t* seg_end, const int64_t* lo,
               const int64_t* hi, int64_t* out, hipStream_t s);

// ---- strfunc.hip (scalar string functions over plain UTF-8 columns)
enum StrFnCode {
  kSfTrim = 0, kSfReplace = 1, kSfLpad = 2, kSfRpad = 3, kSfReverse = 4, kSfRepeat = 5, kSfLeft = 6, kSfRight = 7,
  kSfInitcap = 8, kSfTranslate = 9, kSfSplitPart = 10,
  kSfStrpos = 20, kSfAscii = 21, kSfOctetLength = 22
};
struct StrFnArgs {
  int fn;
  int64_t n1;              // trim mode bits (1 left, 2 right) / pad length / repeat count / left-right n / part
  const uint8_t* a;        // device bytes: trim set / search / fill / from-chars / delimiter
  int64_t alen;
  const uint8_t* b;        // device bytes: replacement / to-chars
  int64_t blen;
};
void str_fn_lengths(const StrFnArgs& a, const int64_t* off, const uint8_t* chars, int64_t n, int64_t* len,
                    hipStream_t s);
// out_cap: bytes of ``out``; a row whose new_off range passes it is skipped
// (new_off may come from a replayed readback that does not match the data)
void str_fn_copy(const StrFnArgs& a, const int64_t* off, const uint8_t* chars, int64_t n, const int64_t* new_off,
                 uint8_t* out, int64_t out_cap, hipStream_t s);
void str_fn_int(int fn, const uint8_t* pat, int64_t plen, const int64_t* off, const uint8_t* chars, int64_t n,
                int32_t* out, hipStream_t s);

}  // namespace kern
}  // namespace igloo
