// pybind11 module `igloo_amd._native`: SQL parser + gfx950 kernel launchers +
// device runtime. Pointer arguments are passed as integers (torch
// tensor.data_ptr()); shape/dtype validation happens in igloo_amd/ops before
// any launch, so this layer is a thin, allocation-free trampoline.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>
#include <memory>
#include <vector>

#include "io/parquet_meta.h"
#include "kernels/kernels.h"
#include "runtime/runtime.h"
#include "sql/ast.h"
#include "sql/ast_py.h"

namespace py = pybind11;
using namespace igloo;

namespace {

template <typename T>
T* P(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

py::list parse(const std::string& text) {
  py::list out;
  try {
    for (auto& st : sql::parse_sql(text)) out.append(sql::to_python(st));
  } catch (const sql::ParseError& e) {
    PyErr_SetString(PyExc_SyntaxError, e.what());
    throw py::error_already_set();
  }
  return out;
}

py::list tokenize(const std::string& text) {
  py::list out;
  static const char* names[] = {"ident", "quoted_ident", "keyword", "number", "string", "op", "end"};
  try {
    for (auto& t : sql::tokenize(text)) out.append(py::make_tuple(names[t.kind], t.text, t.pos));
  } catch (const sql::ParseError& e) {
    PyErr_SetString(PyExc_SyntaxError, e.what());
    throw py::error_already_set();
  }
  return out;
}

py::dict leaf_dict(const io::PqLeaf& l) {
  py::dict d;
  d["name"] = l.name;
  d["type"] = l.type;
  d["type_length"] = l.type_length;
  d["max_def"] = l.max_def;
  d["max_rep"] = l.max_rep;
  d["converted_type"] = l.converted_type;
  d["logical"] = l.logical;
  d["scale"] = l.scale;
  d["precision"] = l.precision;
  return d;
}

py::dict chunk_dict(const io::PqChunk& c) {
  py::dict d;
  d["type"] = c.type;
  d["codec"] = c.codec;
  d["num_values"] = c.num_values;
  d["start"] = c.start();
  d["length"] = c.total_compressed;
  d["uncompressed"] = c.total_uncompressed;
  d["data_page_offset"] = c.data_page_offset;
  d["dictionary_page_offset"] = c.dictionary_page_offset;
  d["encodings"] = c.encodings;
  d["external"] = c.external;
  d["null_count"] = c.stats.has_nulls ? py::object(py::int_(c.stats.null_count)) : py::object(py::none());
  d["min"] = c.stats.has_min ? py::object(py::bytes(c.stats.min)) : py::object(py::none());
  d["max"] = c.stats.has_max ? py::object(py::bytes(c.stats.max)) : py::object(py::none());
  return d;
}

py::dict page_header_dict(const io::PqPageHeader& h) {
  py::dict d;
  d["type"] = h.type;
  d["header_len"] = h.header_len;
  d["compressed"] = h.compressed;
  d["uncompressed"] = h.uncompressed;
  d["num_values"] = h.num_values;
  d["encoding"] = h.encoding;
  d["def_encoding"] = h.def_encoding;
  d["num_nulls"] = h.num_nulls;
  d["num_rows"] = h.num_rows;
  d["def_len"] = h.def_len;
  d["rep_len"] = h.rep_len;
  d["is_compressed"] = h.is_compressed;
  return d;
}

kern::PqDecodeSpec decode_spec(const py::dict& d, bool need_output = true) {
  kern::PqDecodeSpec s{};
  s.phys = d["phys"].cast<int>();
  s.type_len = d["type_len"].cast<int>();
  s.out_width = d["out_width"].cast<int>();
  s.conv = d["conv"].cast<int>();
  s.conv_k = d["conv_k"].cast<int64_t>();
  s.max_def = d["max_def"].cast<int>();
  s.out = P<void>(d["out"].cast<uintptr_t>());
  s.valid = P<uint8_t>(d["valid"].cast<uintptr_t>());
  s.scratch = P<uint32_t>(d["scratch"].cast<uintptr_t>());
  s.str_len = P<int64_t>(d["str_len"].cast<uintptr_t>());
  s.str_pos = P<int64_t>(d["str_pos"].cast<uintptr_t>());
  s.codes = P<int32_t>(d["codes"].cast<uintptr_t>());
  s.dict_len = P<int64_t>(d["dict_len"].cast<uintptr_t>());
  s.dict_pos = P<int64_t>(d["dict_pos"].cast<uintptr_t>());
  s.raw = P<const uint8_t>(d["raw"].cast<uintptr_t>());
  s.dec = P<const uint8_t>(d["dec"].cast<uintptr_t>());
  s.error = P<int>(d["error"].cast<uintptr_t>());
  if (s.max_def < 0 || s.max_def > 1 || s.phys < 0 || s.phys > kern::PQ_PHYS_FLBA || !s.raw || !s.error)
    throw std::runtime_error("pq_decode: bad spec");
  if (need_output && (s.phys == kern::PQ_PHYS_BYTE_ARRAY ? !(s.codes || (s.str_len && s.str_pos)) : !s.out))
    throw std::runtime_error("pq_decode: missing output buffer");
  return s;
}

}  // namespace

namespace igloo {
void register_jit(py::module_& m);  // runtime/jit.cpp
void register_arrow_device(py::module_& m);  // runtime/arrow_device.cpp
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "igloo MI355X native core: SQL frontend, gfx950 kernels, device runtime";
  m.attr("ARCH") = "gfx950";
  m.attr("MAX_AGGS") = kern::kMaxAggs;
  m.attr("MAX_GATHER_COLS") = kern::kMaxGatherCols;
  m.attr("MAX_PARTS") = kern::kMaxParts;
  igloo::register_jit(m);
  igloo::register_arrow_device(m);

  // ------------------------------------------------------------------ SQL
  m.def("parse_sql", &parse, "Parse SQL text into a list of statement ASTs (dicts)");
  m.def("tokenize", &tokenize);

  // -------------------------------------------------------------- runtime
  m.def("device_count", &rt::device_count);
  m.def("device_info", [](int dev) {
    auto d = rt::device_info(dev);
    py::dict r;
    r["device"] = d.device;
    r["name"] = d.name;
    r["arch"] = d.arch;
    r["total_mem"] = d.total_mem;
    r["free_mem"] = d.free_mem;
    r["cu_count"] = d.cu_count;
    r["wave_size"] = d.wave_size;
    r["lds_per_block"] = d.lds_per_block;
    r["l2_bytes"] = d.l2_bytes;
    r["clock_khz"] = d.clock_khz;
    return r;
  });
  py::class_<rt::PinnedPool>(m, "PinnedPool")
      .def(py::init<size_t>())
      .def("acquire",
           [](rt::PinnedPool& p, size_t bytes) {
             size_t got = 0;
             void* ptr = p.acquire(bytes, &got);
             return py::make_tuple((uintptr_t)ptr, got);
           })
      .def("release", [](rt::PinnedPool& p, uintptr_t ptr, size_t bytes) { p.release((void*)ptr, bytes); })
      .def_property_readonly("cached_bytes", &rt::PinnedPool::cached_bytes);

  // ------------------------------------------------------- select / scan
  m.def("select_num_tiles", &kern::select_num_tiles);
  // ---- pack.hip
  auto pack_spec = [](const std::vector<std::tuple<uintptr_t, uintptr_t, int, int>>& cols, int row_bytes) {
    if (cols.size() > (size_t)kern::kMaxPackCols) throw std::runtime_error("pack: too many columns");
    kern::PackSpec spec{};
    spec.ncols = (int32_t)cols.size();
    spec.row_bytes = row_bytes;
    for (size_t i = 0; i < cols.size(); ++i) {
      spec.cols[i].src = P<const void>(std::get<0>(cols[i]));
      spec.cols[i].dst = P<void>(std::get<1>(cols[i]));
      spec.cols[i].width = std::get<2>(cols[i]);
      spec.cols[i].offset = std::get<3>(cols[i]);
      if (spec.cols[i].offset + spec.cols[i].width > row_bytes) throw std::runtime_error("pack: field outside row");
    }
    return spec;
  };
  m.def("pack_rows", [pack_spec](std::vector<std::tuple<uintptr_t, uintptr_t, int, int>> cols, int row_bytes,
                                 uintptr_t perm, bool perm64, int64_t n, uintptr_t out, uintptr_t s) {
    kern::pack_rows(pack_spec(cols, row_bytes), P<const void>(perm), perm64, n, P<uint8_t>(out), S(s));
  });
  m.def("unpack_rows", [pack_spec](std::vector<std::tuple<uintptr_t, uintptr_t, int, int>> cols, int row_bytes,
                                   uintptr_t in, int64_t n, uintptr_t s) {
    kern::unpack_rows(pack_spec(cols, row_bytes), P<const uint8_t>(in), n, S(s));
  });
  // ---- util.hip
  m.def("column_stats", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, uintptr_t out, uintptr_t s) {
    kern::column_stats(P<const void>(keys), key64, P<const uint8_t>(valid), n, P<long long>(out), S(s));
  });
  m.def("run_bounds", [](uintptr_t keys, bool key64, int64_t n, uintptr_t out, uintptr_t s) {
    kern::run_bounds(P<const void>(keys), key64, n, P<uint8_t>(out), S(s));
  });
  // ---- sort.hip
  m.def("radix_sort_ws_bytes", &kern::radix_sort_ws_bytes);
  m.def("radix_sort_pairs", [](uintptr_t k0, uintptr_t k1, bool key64, uintptr_t v0, uintptr_t v1, bool val64,
                               int64_t n, int begin_bit, int end_bit, uintptr_t ws, uintptr_t s) {
    return kern::radix_sort_pairs(P<void>(k0), P<void>(k1), key64, P<void>(v0), P<void>(v1), val64, n, begin_bit,
                                  end_bit, P<void>(ws), S(s));
  });
  m.def("sort_key_pack", [](std::vector<std::tuple<uintptr_t, uintptr_t, uint64_t, uint64_t, int, int, int, int, int>> cols,
                            uintptr_t perm, bool perm64, int64_t n, uintptr_t out, bool out32, uintptr_t s) {
    if (cols.empty() || cols.size() > (size_t)kern::kMaxSortCols) throw std::runtime_error("sort_key_pack: bad column count");
    kern::SortKeySpec spec{};
    spec.ncols = (int32_t)cols.size();
    int total = 0;
    for (size_t i = 0; i < cols.size(); ++i) {
      auto& c = spec.cols[i];
      const auto& t = cols[i];
      c.ptr = P<const void>(std::get<0>(t));
      c.valid = P<const uint8_t>(std::get<1>(t));
      c.lo = std::get<2>(t);
      c.span = std::get<3>(t);
      c.kind = std::get<4>(t);
      c.width = std::get<5>(t);
      c.bits = std::get<6>(t);
      c.desc = std::get<7>(t);
      c.nulls_first = std::get<8>(t);
      if (c.bits < 0 || c.bits > 64) throw std::runtime_error("sort_key_pack: bad field width");
      total += c.bits + (c.valid ? 1 : 0);
    }
    if (total > (out32 ? 32 : 64)) throw std::runtime_error("sort_key_pack: key fields exceed the key width");
    kern::sort_key_pack(spec, P<const void>(perm), perm64, n, P<void>(out), out32, S(s));
  });
  m.def("radix_digit_hist", [](uintptr_t keys, bool key64, int64_t n, int shift, uint64_t prefix, int pshift,
                               uintptr_t hist, uintptr_t s) {
    kern::radix_digit_hist(P<const void>(keys), key64, n, shift, prefix, pshift, P<unsigned long long>(hist), S(s));
  });
  m.def("radix_le_mask", [](uintptr_t keys, bool key64, int64_t n, uint64_t bound, uintptr_t mask, uintptr_t s) {
    kern::radix_le_mask(P<const void>(keys), key64, n, bound, P<uint8_t>(mask), S(s));
  });
  m.def("select_count", [](uintptr_t mask, int64_t n, uintptr_t tiles, uintptr_t total, uintptr_t s) {
    kern::select_count(P<const uint8_t>(mask), n, P<int64_t>(tiles), P<int64_t>(total), S(s));
  });
  // tile counts a fused scan wrote with its mask -> exclusive offsets in place + total
  m.def("select_scan_counts", [](uintptr_t counts, int64_t tiles, uintptr_t total, uintptr_t s) {
    if (!counts || !total || tiles <= 0) throw std::runtime_error("select_scan_counts: bad arguments");
    kern::scan_counts(P<int64_t>(counts), tiles, P<int64_t>(total), S(s));
  });
  m.def("select_write", [](uintptr_t mask, int64_t n, uintptr_t tiles, uintptr_t out, bool idx64, int64_t cap,
                           uintptr_t s) {
    kern::select_write(P<const uint8_t>(mask), n, P<const int64_t>(tiles), P<void>(out), idx64, cap, S(s));
  });
  m.def("select_compact", [](uintptr_t mask, int64_t n, uintptr_t tiles,
                             const std::vector<std::tuple<uintptr_t, uintptr_t, int, uintptr_t, uintptr_t>>& cols,
                             uintptr_t idx, bool idx64, int64_t cap, uintptr_t s) {
    kern::CompactArgs a{};
    if ((int)cols.size() > kern::kMaxCompactCols) throw std::runtime_error("select_compact: too many columns");
    for (size_t j = 0; j < cols.size(); ++j) {
      auto& c = cols[j];
      a.cols[j] = {P<void>(std::get<0>(c)), P<void>(std::get<1>(c)), std::get<2>(c), P<uint8_t>(std::get<3>(c)),
                   P<uint8_t>(std::get<4>(c))};
    }
    a.ncols = (int)cols.size();
    a.idx = P<void>(idx);
    a.idx64 = idx64;
    kern::select_compact(P<uint8_t>(mask), n, P<int64_t>(tiles), a, cap, S(s));
  });
  m.def("scan_workspace_tiles", &kern::scan_workspace_tiles);
  m.def("exclusive_scan", [](uintptr_t in, bool in64, int64_t n, uintptr_t out, uintptr_t ws, uintptr_t total, uintptr_t s) {
    kern::exclusive_scan(P<const void>(in), in64, n, P<int64_t>(out), P<int64_t>(ws), P<int64_t>(total), S(s));
  });

  // ------------------------------------------------------------ hash tables
  m.def("join_build", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, uintptr_t tkeys, uintptr_t thead,
                         bool rid64, int64_t cap, int64_t kmin, bool direct, uintptr_t dups, uintptr_t bits,
                         uint64_t bmask, uintptr_t s) {
    if (n > 0 && (!keys || !thead || !dups || (!direct && !tkeys))) throw std::runtime_error("join_build: null buffer");
    kern::join_build(P<const void>(keys), key64, P<const uint8_t>(valid), n, P<int64_t>(tkeys), P<void>(thead), rid64,
                     cap, kmin, direct, P<unsigned long long>(dups), P<uint32_t>(bits), bmask, S(s));
  });
  m.def("join_csr_count", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, uintptr_t tkeys, uintptr_t cnt,
                             bool rid64, int64_t cap, int64_t kmin, bool direct, uintptr_t s) {
    if (n > 0 && (!keys || !cnt || (!direct && !tkeys))) throw std::runtime_error("join_csr_count: null buffer");
    kern::join_csr_count(P<const void>(keys), key64, P<const uint8_t>(valid), n, P<const int64_t>(tkeys),
                         P<void>(cnt), rid64, cap, kmin, direct, S(s));
  });
  m.def("join_csr_scatter", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, uintptr_t tkeys, uintptr_t cnt,
                               uintptr_t cstart, uintptr_t crows, bool rid64, int64_t cap, int64_t kmin, bool direct,
                               uintptr_t s) {
    if (n > 0 && (!keys || !cnt || !cstart || !crows || (!direct && !tkeys)))
      throw std::runtime_error("join_csr_scatter: null buffer");
    kern::join_csr_scatter(P<const void>(keys), key64, P<const uint8_t>(valid), n, P<const int64_t>(tkeys),
                           P<void>(cnt), P<const void>(cstart), P<void>(crows), rid64, cap, kmin, direct, S(s));
  });
  m.def("join_probe", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t m_, uintptr_t tkeys, uintptr_t thead,
                         uintptr_t cstart, uintptr_t crows, bool rid64, int64_t cap, int64_t kmin, bool direct,
                         uintptr_t counts, uintptr_t first, uintptr_t matched, uintptr_t bits, uint64_t bmask,
                         uintptr_t s) {
    if (m_ > 0 && (!keys || !thead || (!direct && !tkeys) || (!cstart != !crows)))
      throw std::runtime_error("join_probe: null buffer");
    kern::join_probe(P<const void>(keys), key64, P<const uint8_t>(valid), m_, P<const int64_t>(tkeys),
                     P<const void>(thead), P<const void>(cstart), P<const void>(crows), rid64, cap, kmin, direct,
                     P<int32_t>(counts), P<void>(first), P<uint8_t>(matched), P<const uint32_t>(bits), bmask, S(s));
  });
  m.def("probe_hit_tiles", [](int64_t m_) { return kern::probe_hit_tiles(m_); });
  m.def("probe_hits", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t m_, uintptr_t tkeys, uintptr_t thead,
                         bool rid64, int64_t cap, int64_t kmin, bool direct, uintptr_t bits, uint64_t bmask,
                         bool negate, uintptr_t words, uintptr_t tile_counts, uintptr_t s) {
    if (m_ > 0 && (!keys || !thead || !words || !tile_counts || (!direct && !tkeys)))
      throw std::runtime_error("probe_hits: null buffer");
    kern::probe_hits(P<const void>(keys), key64, P<const uint8_t>(valid), m_, P<const int64_t>(tkeys),
                     P<const void>(thead), rid64, cap, kmin, direct, P<const uint32_t>(bits), bmask, negate,
                     P<unsigned long long>(words), P<int64_t>(tile_counts), S(s));
  });
  m.def("set_probe_grid_cap", &kern::set_probe_grid_cap);
  m.def("set_probe_bits", &kern::set_probe_bits);
  m.def("probe_write", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t m_, uintptr_t tkeys, uintptr_t thead,
                          bool rid64, int64_t cap, int64_t kmin, bool direct, uintptr_t words, uintptr_t tile_off,
                          uintptr_t out_probe, bool out64, uintptr_t out_build, int64_t out_cap, uintptr_t s) {
    if (m_ > 0 && (!keys || !thead || !words || !tile_off || !out_probe || (!direct && !tkeys)))
      throw std::runtime_error("probe_write: null buffer");
    kern::probe_write(P<const void>(keys), key64, P<const uint8_t>(valid), m_, P<const int64_t>(tkeys),
                      P<const void>(thead), rid64, cap, kmin, direct, P<const unsigned long long>(words),
                      P<const int64_t>(tile_off), P<void>(out_probe), out64, P<void>(out_build), out_cap, S(s));
  });
  m.def("join_expand", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t m_, uintptr_t tkeys, uintptr_t thead,
                          uintptr_t cstart, uintptr_t crows, bool rid64, int64_t cap, int64_t kmin, bool direct,
                          uintptr_t offsets, uintptr_t out_probe, uintptr_t out_build, uintptr_t bits, uint64_t bmask,
                          int64_t out_cap, uintptr_t s) {
    if (m_ > 0 && (!keys || !thead || !offsets || !out_probe || !out_build || (!direct && !tkeys)))
      throw std::runtime_error("join_expand: null buffer");
    kern::join_expand(P<const void>(keys), key64, P<const uint8_t>(valid), m_, P<const int64_t>(tkeys),
                      P<const void>(thead), P<const void>(cstart), P<const void>(crows), rid64, cap, kmin, direct,
                      P<const int64_t>(offsets), P<int32_t>(out_probe), P<void>(out_build), P<const uint32_t>(bits),
                      bmask, out_cap, S(s));
  });
  // fused scan kernels. cols: [(ptr, width)], terms: [(col, kind, lo, hi, set)],
  // keys: [(col, lo, mul)], aggs: [(op, checked, [(col, a, b)], dst, dst2, shared)]
  using FfCols = std::vector<std::pair<uintptr_t, int64_t>>;
  using FfTerms = std::vector<std::tuple<int, int, int64_t, int64_t, uint64_t>>;
  using FfKeys = std::vector<std::tuple<int, int64_t, int64_t>>;
  using FfAggs = std::vector<std::tuple<int, int, std::vector<std::tuple<int64_t, int64_t, int64_t>>, uintptr_t,
                                        uintptr_t, int, int>>;
  auto make_ff = [](const FfCols& cols, const FfTerms& terms, uintptr_t mask) {
    if (cols.size() > (size_t)kern::kFfMaxCols || terms.size() > (size_t)kern::kFfMaxTerms)
      throw std::runtime_error("fused scan: too many columns / terms");
    kern::FfSpec f{};
    f.ncols = (int32_t)cols.size();
    for (size_t i = 0; i < cols.size(); ++i) {
      f.cols[i].ptr = reinterpret_cast<const void*>(cols[i].first);
      f.cols[i].width = cols[i].second;
      const int64_t w = f.cols[i].width;  // signed 1/2/4/8-byte integer columns
      if (!(w == 1 || w == 2 || w == 4 || w == 8) || (cols[i].first % (w < 4 ? 4 : w)) != 0)
        throw std::runtime_error("fused scan: bad column width / alignment");
    }
    f.nterms = (int32_t)terms.size();
    for (size_t i = 0; i < terms.size(); ++i) {
      auto [col, kind, lo, hi, set] = terms[i];
      // kind = base kind (0 range, 1 not-range, 2 code set, 3 col-col range) | OR-group << 8 (0: top level)
      const int base = kind & 0xff, grp = kind >> 8;
      if (col < 0 || col >= f.ncols || kind < 0 || base > 3 || grp > 31 || (base == 3 && (int64_t)set >= f.ncols))
        throw std::runtime_error("fused scan: bad term");
      f.terms[i] = kern::FfTerm{col, kind, lo, hi, set};
    }
    f.mask = P<const uint8_t>(mask);
    return f;
  };
  m.def("ff_mask", [make_ff](const FfCols& cols, const FfTerms& terms, uintptr_t mask, int64_t n, uintptr_t out,
                             uintptr_t s) {
    kern::FfSpec f = make_ff(cols, terms, mask);
    kern::ff_mask(f, n, P<uint8_t>(out), S(s));
  });
  m.def("ff_aggregate", [make_ff](const FfCols& cols, const FfTerms& terms, uintptr_t mask, const FfKeys& keys,
                                  int ngroups, const FfAggs& aggs, uintptr_t counts, uintptr_t overflow, int64_t n,
                                  uintptr_t s) {
    kern::FfSpec f = make_ff(cols, terms, mask);
    if (keys.size() > 2 || ngroups < 1 || ngroups > kern::kFfMaxGroups || aggs.size() > (size_t)kern::kFfMaxAggs)
      throw std::runtime_error("fused aggregate: shape out of range");
    f.nkeys = (int32_t)keys.size();
    for (size_t i = 0; i < keys.size(); ++i) {
      auto [col, lo, mul] = keys[i];
      if (col < 0 || col >= f.ncols) throw std::runtime_error("fused aggregate: bad key column");
      f.key_col[i] = col;
      f.key_lo[i] = lo;
      f.key_mul[i] = mul;
    }
    f.ngroups = ngroups;
    f.naggs = (int32_t)aggs.size();
    for (size_t i = 0; i < aggs.size(); ++i) {
      auto& [op, checked, facs, dst, dst2, shared, vbits] = aggs[i];
      if (op < 0 || op > 3 || facs.size() > (size_t)kern::kFfMaxFactors)
        throw std::runtime_error("fused aggregate: bad aggregate");
      if (shared < 0 || shared > (int)facs.size() || (shared > 0 && (i == 0 || f.aggs[i - 1].nfac != shared)))
        throw std::runtime_error("fused aggregate: bad shared prefix");
      kern::FfAgg& A = f.aggs[i];
      A.op = op;
      A.checked = checked;
      A.shared = shared;
      A.nfac = (int32_t)facs.size();
      for (size_t k = 0; k < facs.size(); ++k) {
        auto [col, a, b] = facs[k];
        if (col >= f.ncols) throw std::runtime_error("fused aggregate: bad factor column");
        A.f[k] = kern::FfFactor{col, a, b};
      }
      A.dst = P<int64_t>(dst);
      A.dst2 = P<int64_t>(dst2);
      A.vbits = vbits > 0 && vbits < 64 ? vbits : 64;
    }
    f.counts = P<int64_t>(counts);
    f.overflow = P<int>(overflow);
    kern::ff_aggregate(f, n, S(s));
  });
  m.def("ff_set_mfma", [](bool on) { return kern::ff_set_mfma(on); });
  m.attr("HLL_REGISTERS") = kern::kHllRegisters;
  m.def("hll_blocks", [](int64_t n) { return kern::hll_blocks(n); });
  m.def("hll_sketch", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, uintptr_t block_regs, uintptr_t regs,
                         uintptr_t s) {
    kern::hll_sketch(P<const void>(keys), key64, P<const uint8_t>(valid), n, P<uint8_t>(block_regs),
                     P<uint8_t>(regs), S(s));
  });
  m.def("groupby_build", [](uintptr_t keys, bool key64, int64_t n, uintptr_t tkeys, uintptr_t trow, int64_t cap,
                            int64_t kmin, bool direct, uintptr_t s) {
    kern::groupby_build(P<const void>(keys), key64, n, P<int64_t>(tkeys), P<int32_t>(trow), cap, kmin, direct, S(s));
  });
  m.def("groupby_occupied", [](uintptr_t trow, int64_t cap, uintptr_t occ, uintptr_t gid_of_slot, uintptr_t s) {
    kern::groupby_occupied(P<const int32_t>(trow), cap, P<uint8_t>(occ), P<int32_t>(gid_of_slot), S(s));
  });
  m.def("groupby_assign", [](uintptr_t slots, bool slots64, int64_t g, int64_t cap, uintptr_t trow,
                             uintptr_t gid_of_slot, uintptr_t rep_row, uintptr_t s) {
    kern::groupby_assign(P<const void>(slots), slots64, g, cap, P<const int32_t>(trow), P<int32_t>(gid_of_slot),
                         P<int32_t>(rep_row), S(s));
  });
  m.def("groupby_lookup", [](uintptr_t keys, bool key64, int64_t n, uintptr_t tkeys, uintptr_t gid_of_slot,
                             int64_t cap, int64_t kmin, bool direct, uintptr_t gid, uintptr_t s) {
    kern::groupby_lookup(P<const void>(keys), key64, n, P<const int64_t>(tkeys), P<const int32_t>(gid_of_slot), cap,
                         kmin, direct, P<int32_t>(gid), S(s));
  });

  // ------------------------------------------------------------ aggregation
  m.def("agg_lds_max_groups", &kern::agg_lds_max_groups);
  // descs: list of (op, src64, src, valid, dst, dst2)
  m.def("agg_update", [](uintptr_t gid, int64_t n, int ngroups, const std::vector<std::tuple<int, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t>>& descs, uintptr_t s, bool sorted_gids) {
    std::vector<kern::AggDesc> d;
    for (auto& t : descs)
      d.push_back({std::get<0>(t), std::get<1>(t), P<const void>(std::get<2>(t)), P<const uint8_t>(std::get<3>(t)),
                   P<void>(std::get<4>(t)), P<void>(std::get<5>(t))});
    kern::agg_update(P<const int32_t>(gid), n, ngroups, d.data(), (int)d.size(), S(s), sorted_gids);
  }, py::arg("gid"), py::arg("n"), py::arg("ngroups"), py::arg("descs"), py::arg("s"), py::arg("sorted_gids") = false);
  m.def("agg_part_buckets", [](int64_t ngroups, int nagg) { return kern::agg_part_buckets(ngroups, nagg); });
  m.def("agg_part_blocks", []() { return kern::agg_part_blocks(); });
  // phase 0 / 1 / 2 of the radix-partitioned aggregate; vals: one pointer per desc (0: COUNT(*))
  m.def("agg_partitioned", [](uintptr_t gid, int64_t n, int64_t ngroups,
                              const std::vector<std::tuple<int, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t>>& descs,
                              int phase, uintptr_t cnt, uintptr_t off, uintptr_t total, uintptr_t pg,
                              const std::vector<uintptr_t>& vals, uintptr_t s) {
    if (!gid || n >= (int64_t(1) << 31) || ngroups <= 0 || ngroups >= (int64_t(1) << 31) || phase < 0 || phase > 2 ||
        descs.empty() || descs.size() > 8 || vals.size() != descs.size() || (phase == 0 && !cnt) ||
        (phase >= 1 && (!off || !pg)) || (phase == 2 && !total))
      throw std::runtime_error("agg_partitioned: bad arguments");
    std::vector<kern::AggDesc> d;
    for (auto& t : descs)
      d.push_back({std::get<0>(t), std::get<1>(t), P<const void>(std::get<2>(t)), P<const uint8_t>(std::get<3>(t)),
                   P<void>(std::get<4>(t)), P<void>(std::get<5>(t))});
    std::vector<int64_t*> v;
    for (auto x : vals) v.push_back(P<int64_t>(x));
    kern::agg_partitioned(P<const int32_t>(gid), n, ngroups, d.data(), (int)d.size(), phase, P<int32_t>(cnt),
                          P<const int64_t>(off), P<const int64_t>(total), P<uint16_t>(pg), v.data(), S(s));
  });
  m.def("sorted_having", [](uintptr_t keys, bool key64, int64_t n,
                            const std::vector<std::tuple<int, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t>>& descs,
                            int hagg, int hop, long long hlo, long long hhi, double hf, uintptr_t rep, int64_t cap,
                            uintptr_t counter, uintptr_t s) {
    std::vector<kern::AggDesc> d;
    for (auto& t : descs)
      d.push_back({std::get<0>(t), std::get<1>(t), P<const void>(std::get<2>(t)), P<const uint8_t>(std::get<3>(t)),
                   P<void>(std::get<4>(t)), P<void>(std::get<5>(t))});
    kern::sorted_having(P<const void>(keys), key64, n, d.data(), (int)d.size(), hagg, hop, hlo, hhi, hf,
                        P<int64_t>(rep), cap, P<unsigned long long>(counter), S(s));
  });
  m.def("fill_runs", [](uintptr_t starts, bool starts64, int64_t nruns, int64_t n, uintptr_t gid, uintptr_t s) {
    kern::fill_runs(P<const void>(starts), starts64, nruns, n, P<int32_t>(gid), S(s));
  });

  // ----------------------------------------------------------------- gather
  // descs: list of (src, dst, elem_bytes, src_valid, dst_valid, src_rows)
  m.def("gather_multi", [](uintptr_t idx, bool idx64, int64_t n, const std::vector<std::tuple<uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, int64_t>>& descs, uintptr_t s) {
    std::vector<kern::GatherDesc> d;
    for (auto& t : descs)
      d.push_back({P<const void>(std::get<0>(t)), P<void>(std::get<1>(t)), std::get<2>(t),
                   P<const uint8_t>(std::get<3>(t)), P<uint8_t>(std::get<4>(t)), std::get<5>(t)});
    kern::gather_multi(P<const void>(idx), idx64, n, d.data(), (int)d.size(), S(s));
  });
  m.def("gather_packed", [](uintptr_t idx, bool idx64, int64_t n, uintptr_t src, int64_t rows, int row_bytes,
                            const std::vector<std::tuple<uintptr_t, int, int, int, int>>& fields, uintptr_t s) {
    std::vector<kern::PackedField> f;
    for (auto& t : fields)
      f.push_back({P<void>(std::get<0>(t)), std::get<1>(t), std::get<2>(t), std::get<3>(t), std::get<4>(t)});
    kern::gather_packed(P<const void>(idx), idx64, n, P<const uint8_t>(src), rows, row_bytes, f.data(), (int)f.size(),
                        S(s));
  });
  m.def("str_gather_lengths", [](uintptr_t off, int64_t rows, uintptr_t idx, bool idx64, int64_t n, uintptr_t len,
                                 uintptr_t s) {
    kern::str_gather_lengths(P<const int64_t>(off), rows, P<const void>(idx), idx64, n, P<int64_t>(len), S(s));
  });
  m.def("str_gather_copy", [](uintptr_t off, int64_t rows, uintptr_t chars, uintptr_t idx, bool idx64, int64_t n,
                              uintptr_t new_off, uintptr_t out, int64_t out_cap, uintptr_t s) {
    kern::str_gather_copy(P<const int64_t>(off), rows, P<const uint8_t>(chars), P<const void>(idx), idx64, n,
                          P<const int64_t>(new_off), P<uint8_t>(out), out_cap, S(s));
  });

  // ---------------------------------------------------------------- strings
  m.def("str_like", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t pat, uintptr_t kind, int mlen, bool ci,
                       bool neg, uintptr_t out, uintptr_t s) {
    kern::str_like(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(pat), P<const uint8_t>(kind),
                   mlen, ci, neg, P<uint8_t>(out), S(s));
  });
  m.def("str_case", [](uintptr_t in, int64_t nbytes, bool up, uintptr_t out, uintptr_t flag, uintptr_t s) {
    kern::str_case(P<const uint8_t>(in), nbytes, up, P<uint8_t>(out), P<int>(flag), S(s));
  });
  m.def("str_substr_lengths", [](uintptr_t off, uintptr_t chars, int64_t n, int64_t start, int64_t len, bool has_len,
                                 uintptr_t out, uintptr_t s) {
    kern::str_substr_lengths(P<const int64_t>(off), P<const uint8_t>(chars), n, start, len, has_len, P<int64_t>(out), S(s));
  });
  m.def("str_substr_copy", [](uintptr_t off, uintptr_t chars, int64_t n, int64_t start, int64_t len, bool has_len,
                              uintptr_t new_off, uintptr_t out, uintptr_t s) {
    kern::str_substr_copy(P<const int64_t>(off), P<const uint8_t>(chars), n, start, len, has_len,
                          P<const int64_t>(new_off), P<uint8_t>(out), S(s));
  });
  m.def("mark_slot_rows", [](uintptr_t trow, int64_t cap, int64_t n, uintptr_t mark, uintptr_t s) {
    kern::mark_slot_rows(P<const int32_t>(trow), cap, n, P<uint8_t>(mark), S(s));
  });
  m.def("pack_bits", [](std::vector<uintptr_t> cols, std::vector<bool> is64, std::vector<int64_t> lo,
                        std::vector<int> shift, int64_t n, uintptr_t out, uintptr_t s) {
    std::vector<const void*> c(cols.size());
    std::unique_ptr<bool[]> w(new bool[cols.size()]);
    for (size_t i = 0; i < cols.size(); ++i) {
      c[i] = reinterpret_cast<const void*>(cols[i]);
      w[i] = is64[i];
    }
    kern::pack_bits(c.data(), w.get(), lo.data(), shift.data(), (int)cols.size(), n, P<int64_t>(out), S(s));
  });
  m.def("differs_from_rep", [](uintptr_t a, int elem_bytes, uintptr_t rep, bool rep64, int64_t n, uintptr_t flag,
                               uintptr_t s) {
    kern::differs_from_rep(P<const void>(a), elem_bytes, P<const void>(rep), rep64, n, P<int>(flag), S(s));
  });
  m.def("mark_keys", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, int64_t kmin, int64_t dom,
                        uintptr_t marks, uintptr_t s) {
    kern::mark_keys(P<const void>(keys), key64, P<const uint8_t>(valid), n, kmin, dom, P<uint8_t>(marks), S(s));
  });
  m.def("probe_marks", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, int64_t base, int64_t dom,
                          uintptr_t marks, bool negate, uintptr_t out, uintptr_t s) {
    kern::probe_marks(P<const void>(keys), key64, P<const uint8_t>(valid), n, base, dom, P<const uint8_t>(marks),
                      negate, P<uint8_t>(out), S(s));
  });
  m.def("const_ints", [](uintptr_t out, std::vector<int64_t> vals, uintptr_t s) {
    kern::const_ints(P<int64_t>(out), vals.data(), (int64_t)vals.size(), S(s));
  });
  m.def("end_capture", [](uintptr_t s) { kern::end_capture(S(s)); });
  m.def("str_char_length", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t out, uintptr_t s) {
    kern::str_char_length(P<const int64_t>(off), P<const uint8_t>(chars), n, P<int32_t>(out), S(s));
  });
  m.def("str_concat2_lengths", [](uintptr_t oa, bool ba, uintptr_t ob, bool bb, int64_t n, uintptr_t len, uintptr_t s) {
    kern::str_concat2_lengths(P<const int64_t>(oa), ba, P<const int64_t>(ob), bb, n, P<int64_t>(len), S(s));
  });
  m.def("str_concat2_copy", [](uintptr_t oa, uintptr_t ca, bool ba, uintptr_t ob, uintptr_t cb, bool bb, int64_t n,
                               uintptr_t off, uintptr_t out, uintptr_t s) {
    kern::str_concat2_copy(P<const int64_t>(oa), P<const uint8_t>(ca), ba, P<const int64_t>(ob), P<const uint8_t>(cb),
                           bb, n, P<const int64_t>(off), P<uint8_t>(out), S(s));
  });
  m.def("fmt_lengths", [](uintptr_t vals, int kind, int64_t n, int scale, uintptr_t valid, uintptr_t len, uintptr_t s) {
    kern::fmt_lengths(P<const void>(vals), kind, n, scale, P<const uint8_t>(valid), P<int64_t>(len), S(s));
  });
  m.def("fmt_write", [](uintptr_t vals, int kind, int64_t n, int scale, uintptr_t valid, uintptr_t off, uintptr_t out,
                        uintptr_t s) {
    kern::fmt_write(P<const void>(vals), kind, n, scale, P<const uint8_t>(valid), P<const int64_t>(off), P<uint8_t>(out),
                    S(s));
  });
  m.def("str_parse", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t valid, int kind, int scale, uintptr_t out,
                        uintptr_t err, uintptr_t s) {
    kern::str_parse(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(valid), kind, scale,
                    P<void>(out), P<int>(err), S(s));
  });
  m.def("wide_fits", [](uintptr_t lo, uintptr_t hi, int64_t n, uintptr_t flag, uintptr_t s) {
    kern::wide_fits(P<const int64_t>(lo), P<const int64_t>(hi), n, P<int>(flag), S(s));
  });
  m.def("avg_wide", [](uintptr_t sums, bool wide, uintptr_t cnt, int64_t n, int64_t up, uintptr_t out, uintptr_t s) {
    kern::avg_wide(P<const int64_t>(sums), wide, P<const int64_t>(cnt), n, up, P<int64_t>(out), S(s));
  });
  m.def("str_prefix_keys", [](uintptr_t off, uintptr_t chars, int64_t n, int chunks, uintptr_t out, uintptr_t s) {
    kern::str_prefix_keys(P<const int64_t>(off), P<const uint8_t>(chars), n, chunks, P<int64_t>(out), S(s));
  });
  m.def("str_hash64", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t valid, uintptr_t out, uintptr_t s) {
    kern::str_hash64(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(valid), P<int64_t>(out), S(s));
  });
  m.def("str_like_segments", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t seg, uintptr_t seg_off, int nseg,
                                 bool anchor_start, bool anchor_end, bool negate, uintptr_t out, int64_t nbytes,
                                 int min_seg, uintptr_t s) {
    kern::str_like_segments(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(seg),
                            P<const int32_t>(seg_off), nseg, anchor_start, anchor_end, negate, P<uint8_t>(out), nbytes,
                            min_seg, S(s));
  });
  m.def("str_eq_rows", [](uintptr_t aoff, uintptr_t achars, uintptr_t ai, uintptr_t boff, uintptr_t bchars, uintptr_t bi,
                          bool idx64, int64_t n, uintptr_t mism, uintptr_t s) {
    kern::str_eq_rows(P<const int64_t>(aoff), P<const uint8_t>(achars), P<const void>(ai), P<const int64_t>(boff),
                      P<const uint8_t>(bchars), P<const void>(bi), idx64, n, P<int>(mism), S(s));
  });
  m.def("str_in_set", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t vb, uintptr_t voff, uintptr_t vmode,
                         int nv, uintptr_t out, uintptr_t s) {
    if (n > 0 && (!off || !out || nv < 0 || (nv > 0 && (!vb || !voff || !vmode))))
      throw std::runtime_error("str_in_set: bad arguments");
    kern::str_in_set(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(vb), P<const int32_t>(voff),
                     P<const uint8_t>(vmode), nv, P<uint8_t>(out), S(s));
  });
  m.def("str_cmp_const", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t c, int64_t cn, int op, uintptr_t out,
                            uintptr_t s) {
    kern::str_cmp_const(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint8_t>(c), cn, op,
                        P<uint8_t>(out), S(s));
  });
  m.def("str_prefix_key", [](uintptr_t off, uintptr_t chars, int64_t n, int64_t skip, uintptr_t out, uintptr_t s) {
    kern::str_prefix_key(P<const int64_t>(off), P<const uint8_t>(chars), n, skip, P<int64_t>(out), S(s));
  });

  // -------------------------------------------------------------------- csv
  m.attr("CSV_TILE") = kern::kCsvTile;
  m.attr("CSV_COLUMN_BYTES") = (int)sizeof(kern::CsvColumn);
  m.def("csv_num_tiles", &kern::csv_num_tiles);
  m.def("csv_quote_parity", [](uintptr_t buf, int64_t n, int quote, uintptr_t tile_par, uintptr_t s) {
    kern::csv_quote_parity(P<const uint8_t>(buf), n, (uint8_t)quote, P<uint8_t>(tile_par), S(s));
  });
  m.def("csv_rows", [](uintptr_t buf, int64_t n, int64_t start, int quote, uintptr_t tile_state, uintptr_t tile_rows,
                       uintptr_t tile_off, uintptr_t rows_end, uintptr_t s) {
    kern::csv_rows(P<const uint8_t>(buf), n, start, (uint8_t)quote, P<const uint8_t>(tile_state),
                   P<int64_t>(tile_rows), P<const int64_t>(tile_off), P<int64_t>(rows_end), S(s));
  });
  // cols: [(kind, scale, out, len, valid)] -> packed CsvColumn array (upload, then pass to csv_parse)
  m.def("csv_pack_columns", [](const std::vector<std::tuple<int, int, uintptr_t, uintptr_t, uintptr_t>>& cols) {
    std::vector<kern::CsvColumn> v;
    for (auto& [kind, scale, out, len, valid] : cols) {
      if (kind < kern::CSV_SKIP || kind > kern::CSV_UTF8) throw std::runtime_error("csv: bad column kind");
      if (kind != kern::CSV_SKIP && !out) throw std::runtime_error("csv: missing output buffer");
      if (kind == kern::CSV_UTF8 && !len) throw std::runtime_error("csv: missing length buffer");
      v.push_back({kind, scale, P<void>(out), P<int64_t>(len), P<uint8_t>(valid)});
    }
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(kern::CsvColumn));
  });
  m.def("csv_parse", [](uintptr_t buf, int64_t start, uintptr_t rows_end, int64_t nrows, uintptr_t cols, int ncols,
                        int delim, int quote, uintptr_t err, uintptr_t s) {
    kern::csv_parse(P<const uint8_t>(buf), start, P<const int64_t>(rows_end), nrows,
                    P<const kern::CsvColumn>(cols), ncols, (uint8_t)delim, (uint8_t)quote, P<int>(err), S(s));
  });
  m.def("csv_str_lengths", [](uintptr_t len_flag, int64_t n, uintptr_t len, uintptr_t s) {
    kern::csv_str_lengths(P<const int64_t>(len_flag), n, P<int64_t>(len), S(s));
  });
  m.def("csv_str_copy", [](uintptr_t pos, uintptr_t len_flag, uintptr_t off, int64_t n, int quote, uintptr_t out,
                           uintptr_t s) {
    kern::csv_str_copy(P<const int64_t>(pos), P<const int64_t>(len_flag), P<const int64_t>(off), n, (uint8_t)quote,
                       P<uint8_t>(out), S(s));
  });

  m.def("strfmt_lengths", [](const std::string& fmt, bool is_date, uintptr_t v, int64_t n, uintptr_t len,
                             uintptr_t s) {
    kern::strfmt_lengths(reinterpret_cast<const uint8_t*>(fmt.data()), (int)fmt.size(), is_date, P<const void>(v), n,
                         P<int64_t>(len), S(s));
  });
  m.def("strfmt_write", [](const std::string& fmt, bool is_date, uintptr_t v, int64_t n, uintptr_t off,
                           int64_t out_cap, uintptr_t out, uintptr_t s) {
    kern::strfmt_write(reinterpret_cast<const uint8_t*>(fmt.data()), (int)fmt.size(), is_date, P<const void>(v), n,
                       P<const int64_t>(off), out_cap, P<uint8_t>(out), S(s));
  });
  m.def("regex_lds_bytes", &kern::regex_lds_bytes);
  m.def("regex_dfa_match", [](uintptr_t off, uintptr_t chars, int64_t n, uintptr_t table, uintptr_t cls,
                              uintptr_t flags, int nstates, int nclasses, int start, bool anchored_end, bool negate,
                              uintptr_t out, uintptr_t s) {
    kern::regex_dfa_match(P<const int64_t>(off), P<const uint8_t>(chars), n, P<const uint16_t>(table),
                          P<const uint8_t>(cls), P<const uint8_t>(flags), nstates, nclasses, start, anchored_end,
                          negate, P<uint8_t>(out), S(s));
  });
  m.def("probe_hash16", [](bool mfma, uintptr_t k0, uintptr_t k1, uintptr_t k2, uintptr_t k3, int64_t n,
                           uintptr_t proj, uintptr_t out, uintptr_t s) {
    kern::probe_hash16(mfma, P<const int32_t>(k0), P<const int32_t>(k1), P<const int32_t>(k2), P<const int32_t>(k3),
                       n, P<const int8_t>(proj), P<uint32_t>(out), S(s));
  });
  m.def("probe_inlist16", [](bool mfma, uintptr_t off, uintptr_t chars, int64_t n, const std::string& pats, int npat,
                             int len, uintptr_t out, uintptr_t s) {
    if ((int64_t)pats.size() < 16 * npat) throw std::runtime_error("probe_inlist16: 16 bytes per pattern");
    kern::probe_inlist16(mfma, P<const int64_t>(off), P<const uint8_t>(chars), n,
                         reinterpret_cast<const uint8_t*>(pats.data()), npat, len, P<uint8_t>(out), S(s));
  });
  m.def("digest_width", &kern::digest_width);
  m.def("digest_hex", [](int algo, uintptr_t off, uintptr_t chars, int64_t n, uintptr_t out, uintptr_t s) {
    kern::digest_hex(algo, P<const int64_t>(off), P<const uint8_t>(chars), n, P<uint8_t>(out), S(s));
  });
  m.def("uuid_v4", [](uint64_t seed, int64_t n, uintptr_t out, uintptr_t s) {
    kern::uuid_v4(seed, n, P<uint8_t>(out), S(s));
  });
  m.def("list_element_idx", [](uintptr_t se, uintptr_t valid, uintptr_t pos, uintptr_t pos_valid, int64_t pos_const,
                               int64_t n, int64_t child_n, uintptr_t out, uintptr_t s) {
    kern::list_element_idx(P<const int64_t>(se), P<const uint8_t>(valid), P<const int64_t>(pos),
                           P<const uint8_t>(pos_valid), pos_const, n, child_n, P<int64_t>(out), S(s));
  });
  m.def("interleave_idx", [](int64_t n, int k, uintptr_t out, uintptr_t s) {
    kern::interleave_idx(n, k, P<int64_t>(out), S(s));
  });
  m.def("list_slots", [](int64_t n, int64_t k, uintptr_t se, uintptr_t s) {
    kern::list_slots(n, k, P<int64_t>(se), S(s));
  });
  m.def("json_parse", [](uintptr_t buf, int64_t start, uintptr_t rows_end, int64_t nrows, uintptr_t cols, int ncols,
                         uintptr_t names, uintptr_t name_off, uintptr_t err, uintptr_t s) {
    if (ncols > 64) throw std::runtime_error("json_parse: at most 64 fields");
    kern::json_parse(P<const uint8_t>(buf), start, P<const int64_t>(rows_end), nrows, P<const kern::CsvColumn>(cols),
                     ncols, P<const uint8_t>(names), P<const int32_t>(name_off), P<int>(err), S(s));
  });
  m.def("json_str_copy", [](uintptr_t pos, uintptr_t len_flag, uintptr_t off, int64_t n, uintptr_t out, uintptr_t s) {
    kern::json_str_copy(P<const int64_t>(pos), P<const int64_t>(len_flag), P<const int64_t>(off), n, P<uint8_t>(out),
                        S(s));
  });

  // ----------------------------------------------------------- sorted joins
  m.def("sorted_ranges", [](uintptr_t big, bool key64, int64_t nb, uintptr_t q, uintptr_t qvalid, int64_t nq,
                            uintptr_t lo, uintptr_t cnt, uintptr_t fence, int64_t nf, uintptr_t s) {
    kern::sorted_ranges(P<const void>(big), key64, nb, P<const void>(q), P<const uint8_t>(qvalid), nq, P<int64_t>(lo),
                        P<int64_t>(cnt), P<const void>(fence), nf, S(s));
  });
  m.attr("SEARCH_FENCE") = kern::kFence;
  m.attr("STATS_SLOTS") = kern::kStatsSlots;
  m.def("expand_ranges", [](uintptr_t off, uintptr_t lo, int64_t ns, int64_t total, uintptr_t sidx, uintptr_t bidx,
                            bool out64, uintptr_t s) {
    kern::expand_ranges(P<const int64_t>(off), P<const int64_t>(lo), ns, total, P<void>(sidx), P<void>(bidx), out64,
                        S(s));
  });

  m.def("dense_index_build", [](uintptr_t big, bool key64, int64_t nb, int64_t kmin, int64_t kmax, uintptr_t first,
                                bool first64, uintptr_t long_gap, uintptr_t s) {
    if (nb <= 0 || kmax < kmin || !big || !first) throw std::runtime_error("dense_index_build: bad arguments");
    kern::dense_index_build(P<const void>(big), key64, nb, kmin, kmax, P<void>(first), first64, P<int32_t>(long_gap),
                            S(s));
  });
  m.def("dense_ranges", [](uintptr_t first, bool first64, int64_t kmin, int64_t kmax, uintptr_t q, bool key64,
                           uintptr_t qvalid, int64_t nq, uintptr_t lo, uintptr_t cnt, uintptr_t s) {
    if (nq > 0 && (!first || !q || !lo || !cnt)) throw std::runtime_error("dense_ranges: null buffer");
    kern::dense_ranges(P<const void>(first), first64, kmin, kmax, P<const void>(q), key64, P<const uint8_t>(qvalid), nq,
                       P<int64_t>(lo), P<int64_t>(cnt), S(s));
  });
  m.def("unique_lookup", [](uintptr_t big, bool key64, int64_t nb, uintptr_t first, bool first64, int64_t kmin,
                            int64_t kmax, uintptr_t q, uintptr_t qvalid, int64_t nq, uintptr_t hit, uintptr_t pos,
                            uintptr_t fence, int64_t nf, uintptr_t s) {
    if (nq > 0 && (!q || !hit || !pos || (!first && !big))) throw std::runtime_error("unique_lookup: null buffer");
    if (nb >= (int64_t{1} << 31)) throw std::runtime_error("unique_lookup: positions must fit int32");
    kern::unique_lookup(P<const void>(big), key64, nb, P<const void>(first), first64, kmin, kmax, P<const void>(q),
                        P<const uint8_t>(qvalid), nq, P<uint8_t>(hit), P<int32_t>(pos), P<const void>(fence), nf,
                        S(s));
  });
  m.def("key_histogram", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, int64_t kmin, int64_t span,
                            uintptr_t counts, uintptr_t s) {
    if (n > 0 && (!keys || !counts || span <= 0)) throw std::runtime_error("key_histogram: bad arguments");
    kern::key_histogram(P<const void>(keys), key64, P<const uint8_t>(valid), n, kmin, span, P<int32_t>(counts), S(s));
  });
  m.def("key_histogram_buckets", [](int64_t span) { return kern::key_histogram_buckets(span); });
  m.def("key_histogram_blocks", []() { return kern::key_histogram_blocks(); });
  m.def("key_histogram_partitioned", [](uintptr_t keys, bool key64, uintptr_t valid, int64_t n, int64_t kmin,
                                        int64_t span, int phase, uintptr_t cnt, uintptr_t off, int64_t total,
                                        uintptr_t part, uintptr_t counts, uintptr_t s) {
    if (span <= 0 || span > (int64_t(1) << 27) || n >= (int64_t(1) << 31) || phase < 0 || phase > 2 || !keys ||
        (phase == 0 && !cnt) || (phase >= 1 && (!off || !part)) || (phase == 2 && !counts))
      throw std::runtime_error("key_histogram_partitioned: bad arguments");
    kern::key_histogram_partitioned(P<const void>(keys), key64, P<const uint8_t>(valid), n, kmin, span, phase,
                                    P<int32_t>(cnt), P<const int64_t>(off), total, P<uint16_t>(part),
                                    P<int32_t>(counts), S(s));
  });
  m.def("sorted_exists", [](uintptr_t big2, uintptr_t small2, bool key64, uintptr_t lo, uintptr_t cnt, int64_t ns,
                            int op, uintptr_t mask, uintptr_t hit, uintptr_t s) {
    // op 6 (any row of the range set in mask) reads neither value column
    if (op < 0 || op > 6 || (op == 6 && !mask) || (ns > 0 && (!lo || !cnt || !hit || (op < 6 && (!big2 || !small2)))))
      throw std::runtime_error("sorted_exists: bad arguments");
    kern::sorted_exists(P<const void>(big2), P<const void>(small2), key64, P<const int64_t>(lo), P<const int64_t>(cnt),
                        ns, op, P<const uint8_t>(mask), P<uint8_t>(hit), S(s));
  });
  m.def("sorted_match", [](uintptr_t big2, uintptr_t small2, bool key64, uintptr_t lo, uintptr_t cnt, int64_t ns,
                           uintptr_t counts, uintptr_t offsets, uintptr_t sidx, uintptr_t bidx, bool out64,
                           int64_t out_cap, uintptr_t first, uintptr_t s) {
    if (ns > 0 && (!big2 || !small2 || !lo || !cnt || (!offsets && !counts) || (offsets && (!sidx || !bidx))))
      throw std::runtime_error("sorted_match: null buffer");
    kern::sorted_match(P<const void>(big2), P<const void>(small2), key64, P<const int64_t>(lo), P<const int64_t>(cnt),
                       ns, P<int32_t>(counts), P<const int64_t>(offsets), P<void>(sidx), P<void>(bidx), out64,
                       out_cap, P<int32_t>(first), S(s));
  });
  m.def("sorted_masked", [](uintptr_t mask, uintptr_t lo, uintptr_t cnt, int64_t ns, uintptr_t counts,
                            uintptr_t offsets, uintptr_t sidx, uintptr_t bidx, bool out64, int64_t out_cap,
                            uintptr_t s) {
    if (ns > 0 && (!mask || !lo || !cnt || (!offsets && !counts) || (offsets && (!sidx || !bidx))))
      throw std::runtime_error("sorted_masked: null buffer");
    kern::sorted_masked(P<const uint8_t>(mask), P<const int64_t>(lo), P<const int64_t>(cnt), ns, P<int32_t>(counts),
                        P<const int64_t>(offsets), P<void>(sidx), P<void>(bidx), out64, out_cap, S(s));
  });

  // -------------------------------------------------------------- partition
  m.def("partition_run_blocks", &kern::partition_run_blocks);
  m.def("partition_run", [](uintptr_t keys, bool key64, int64_t n, int nparts, uintptr_t ws, uintptr_t total,
                            uintptr_t perm, bool perm64, uintptr_t s) {
    kern::partition_run(P<const void>(keys), key64, n, nparts, P<int64_t>(ws), P<int64_t>(total), P<void>(perm),
                        perm64, S(s));
  });
  m.def("partition_ids", [](uintptr_t keys, bool key64, int64_t n, int nparts, uintptr_t out, uintptr_t s) {
    kern::partition_ids(P<const void>(keys), key64, n, nparts, P<int32_t>(out), S(s));
  });
  m.def("str_fn_lengths", [](int fn, int64_t n1, uintptr_t a, int64_t alen, uintptr_t b, int64_t blen, uintptr_t off,
                             uintptr_t chars, int64_t n, uintptr_t len, uintptr_t s) {
    kern::StrFnArgs args{fn, n1, P<uint8_t>(a), alen, P<uint8_t>(b), blen};
    kern::str_fn_lengths(args, P<int64_t>(off), P<uint8_t>(chars), n, P<int64_t>(len), S(s));
  });
  m.def("str_fn_copy", [](int fn, int64_t n1, uintptr_t a, int64_t alen, uintptr_t b, int64_t blen, uintptr_t off,
                          uintptr_t chars, int64_t n, uintptr_t new_off, uintptr_t out, int64_t out_cap,
                          uintptr_t s) {
    kern::StrFnArgs args{fn, n1, P<uint8_t>(a), alen, P<uint8_t>(b), blen};
    kern::str_fn_copy(args, P<int64_t>(off), P<uint8_t>(chars), n, P<int64_t>(new_off), P<uint8_t>(out), out_cap,
                      S(s));
  });
  m.def("str_fn_int", [](int fn, uintptr_t pat, int64_t plen, uintptr_t off, uintptr_t chars, int64_t n, uintptr_t out,
                         uintptr_t s) {
    kern::str_fn_int(fn, P<uint8_t>(pat), plen, P<int64_t>(off), P<uint8_t>(chars), n, P<int32_t>(out), S(s));
  });
  m.def("win_scan_tiles", &kern::win_scan_tiles);
  m.def("win_seg_scan", [](uintptr_t ids, bool ids64, uintptr_t ids2, bool ids2_64, uintptr_t vals, int vkind,
                           uintptr_t valid, int64_t n, int op, bool reverse, uintptr_t tflag, uintptr_t tval,
                           uintptr_t out, uintptr_t err, uintptr_t s) {
    kern::win_seg_scan(P<void>(ids), ids64, P<void>(ids2), ids2_64, P<void>(vals), vkind, P<uint8_t>(valid), n, op,
                       reverse, P<int>(tflag), P<int64_t>(tval), P<int64_t>(out), P<int>(err), S(s));
  });
  m.def("win_bounds", [](int64_t n, uintptr_t ss, uintptr_t se, uintptr_t ps, uintptr_t pe, int unit, int skind,
                         int64_t soff_i, double soff_f, int ekind, int64_t eoff_i, double eoff_f, uintptr_t key,
                         bool key_f64, uintptr_t key_valid, bool desc, uintptr_t gnum, uintptr_t gpos,
                         int64_t ngroups, uintptr_t lo, uintptr_t hi, uintptr_t s) {
    kern::win_bounds(n, P<int64_t>(ss), P<int64_t>(se), P<int64_t>(ps), P<int64_t>(pe), unit, skind, soff_i, soff_f,
                     ekind, eoff_i, eoff_f, P<void>(key), key_f64, P<uint8_t>(key_valid), desc, P<int64_t>(gnum),
                     P<int64_t>(gpos), ngroups, P<int64_t>(lo), P<int64_t>(hi), S(s));
  });
  m.def("win_frame_sum", [](uintptr_t psum, bool f64, uintptr_t pcnt, uintptr_t lo, uintptr_t hi, int64_t n,
                            uintptr_t sum_out, uintptr_t cnt_out, uintptr_t s) {
    kern::win_frame_sum(P<int64_t>(psum), f64, P<int64_t>(pcnt), P<int64_t>(lo), P<int64_t>(hi), n,
                        P<int64_t>(sum_out), P<int64_t>(cnt_out), S(s));
  });
  m.def("win_sparse_build", [](uintptr_t vals, bool f64, uintptr_t valid, int64_t n, bool is_max, int levels,
                               uintptr_t table, uintptr_t s) {
    kern::win_sparse_build(P<int64_t>(vals), f64, P<uint8_t>(valid), n, is_max, levels, P<int64_t>(table), S(s));
  });
  m.def("win_sparse_query", [](uintptr_t table, int levels, int64_t n, uintptr_t lo, uintptr_t hi, uintptr_t pcnt,
                               bool is_max, bool f64, uintptr_t out, uintptr_t out_valid, uintptr_t s) {
    kern::win_sparse_query(P<int64_t>(table), levels, n, P<int64_t>(lo), P<int64_t>(hi), P<int64_t>(pcnt), is_max,
                           f64, P<int64_t>(out), P<uint8_t>(out_valid), S(s));
  });
  m.def("win_frame_minmax", [](uintptr_t vals, bool f64, bool is_max, uintptr_t valid, uintptr_t lo, uintptr_t hi,
                               int64_t n, uintptr_t out, uintptr_t out_valid, uintptr_t s) {
    kern::win_frame_minmax(P<int64_t>(vals), f64, is_max, P<uint8_t>(valid), P<int64_t>(lo), P<int64_t>(hi), n,
                           P<int64_t>(out), P<uint8_t>(out_valid), S(s));
  });
  m.def("win_rank", [](int fn, int64_t arg, int64_t n, uintptr_t ss, uintptr_t se, uintptr_t ps, uintptr_t pe,
                       uintptr_t dense, uintptr_t out, uintptr_t s) {
    kern::win_rank(fn, arg, n, P<int64_t>(ss), P<int64_t>(se), P<int64_t>(ps), P<int64_t>(pe), P<int64_t>(dense),
                   P<int64_t>(out), S(s));
  });
  m.def("win_index", [](int fn, int64_t arg, int64_t n, uintptr_t ss, uintptr_t se, uintptr_t lo, uintptr_t hi,
                        uintptr_t out, uintptr_t s) {
    kern::win_index(fn, arg, n, P<int64_t>(ss), P<int64_t>(se), P<int64_t>(lo), P<int64_t>(hi), P<int64_t>(out),
                    S(s));
  });
  m.def("date_part", [](uintptr_t days, int64_t n, int field, uintptr_t out, uintptr_t s) {
    kern::date_part(P<const int32_t>(days), n, field, P<int32_t>(out), S(s));
  });

  // ---------------------------------------------------------------- parquet
  m.def("pq_file_meta", [](const std::string& path) {
    io::PqFileMeta meta;
    {
      py::gil_scoped_release rel;
      meta = io::read_file_meta(path);
    }
    py::dict d;
    d["version"] = meta.version;
    d["num_rows"] = meta.num_rows;
    d["created_by"] = meta.created_by;
    py::list leaves, groups;
    for (auto& l : meta.leaves) leaves.append(leaf_dict(l));
    for (auto& g : meta.row_groups) {
      py::dict gd;
      gd["num_rows"] = g.num_rows;
      py::list cs;
      for (auto& c : g.chunks) cs.append(chunk_dict(c));
      gd["chunks"] = cs;
      groups.append(gd);
    }
    d["leaves"] = leaves;
    d["row_groups"] = groups;
    return d;
  }, "Parse a Parquet footer (native Thrift compact decoder)");
  m.def("pq_page_headers", [](uintptr_t host, int64_t n) {
    py::list out;
    for (auto& h : io::parse_chunk_pages(P<const uint8_t>(host), (size_t)n)) out.append(page_header_dict(h));
    return out;
  });
  m.def("pq_pread", [](const std::string& path, const std::vector<std::tuple<int64_t, int64_t, uintptr_t>>& ranges,
                       int threads) {
    std::vector<io::ReadRange> rs;
    for (auto& [off, len, dst] : ranges) {
      if (off < 0 || len < 0 || !dst) throw std::runtime_error("pq_pread: bad range");
      rs.push_back({off, len, P<uint8_t>(dst)});
    }
    py::gil_scoped_release rel;
    io::pread_ranges(path, rs, threads);
  });
  m.def("pq_plan", [](uintptr_t host, const std::vector<std::tuple<int64_t, int64_t, int, int64_t, int64_t>>& chunks,
                      int phys, int max_def, int max_rep, int64_t dec_base, int type_len) {
    std::vector<io::PqChunkIn> cs;
    for (auto& [off, len, codec, first, rows] : chunks) cs.push_back({off, len, codec, first, rows});
    io::PqPlan plan;
    {
      py::gil_scoped_release rel;
      plan = io::plan_column(P<const uint8_t>(host), cs, phys, max_def, max_rep, dec_base, type_len);
    }
    py::dict d;
    d["pages"] = py::bytes((const char*)plan.pages.data(), plan.pages.size());
    d["jobs"] = py::bytes((const char*)plan.jobs.data(), plan.jobs.size());
    d["num_pages"] = plan.num_pages;
    d["num_jobs"] = plan.num_jobs;
    d["num_zstd_jobs"] = plan.num_zstd_jobs;
    d["num_dict_pages"] = plan.num_dict_pages;
    d["dec_bytes"] = plan.dec_bytes;
    d["dict_entries"] = plan.dict_entries;
    d["plain_pages"] = plan.plain_pages;
    d["max_page_values"] = plan.max_page_values;
    d["unsupported"] = plan.unsupported;
    return d;
  }, "Plan GPU decode descriptors for one column's chunks staged at `host`",
     py::arg("host"), py::arg("chunks"), py::arg("phys"), py::arg("max_def"), py::arg("max_rep"),
     py::arg("dec_base") = 0, py::arg("type_len") = 0);
  m.def("pq_pack_spec", [](const py::dict& spec, bool need_output) {
    kern::PqDecodeSpec sp = decode_spec(spec, need_output);
    return py::bytes(reinterpret_cast<const char*>(&sp), sizeof(sp));
  }, "Validated binary PqDecodeSpec (concatenate one per column and upload)");
  m.attr("PQ_SPEC_BYTES") = (int)sizeof(kern::PqDecodeSpec);
  m.def("pq_zstd_slots", &kern::pq_zstd_slots);
  m.def("pq_zstd", [](uintptr_t jobs, int64_t njobs, uintptr_t raw, uintptr_t dec, uintptr_t lit, int64_t slots,
                      uintptr_t err, uintptr_t s) {
    if (njobs > 0 && (!jobs || !raw || !dec || !lit || !err)) throw std::runtime_error("pq_zstd: null buffer");
    kern::pq_zstd(P<const kern::PqSnappyJob>(jobs), njobs, P<const uint8_t>(raw), P<uint8_t>(dec), P<uint8_t>(lit),
                  slots, P<int>(err), S(s));
  });
  // host reference: decompress `src` (bytes) into exactly `size` bytes; (error code, output)
  m.def("zstd_decompress_host", [](py::bytes src, int64_t size) {
    std::string in = src;
    std::string out((size_t)size, '\0');
    int e;
    {
      py::gil_scoped_release nogil;
      e = kern::zstd_decompress_host((const uint8_t*)in.data(), (int64_t)in.size(), (uint8_t*)out.data(), size);
    }
    return py::make_tuple(e, py::bytes(out));
  });
  m.def("pq_snappy", [](uintptr_t jobs, int64_t njobs, uintptr_t raw, uintptr_t dec, uintptr_t err, uintptr_t s) {
    if (njobs > 0 && (!jobs || !raw || !dec || !err)) throw std::runtime_error("pq_snappy: null buffer");
    kern::pq_snappy(P<const kern::PqSnappyJob>(jobs), njobs, P<const uint8_t>(raw), P<uint8_t>(dec), P<int>(err), S(s));
  });
  m.def("pq_dict_strings", [](uintptr_t pages, int64_t npages, uintptr_t page_col, uintptr_t specs, uintptr_t s) {
    if (npages > 0 && (!pages || !page_col || !specs)) throw std::runtime_error("pq_dict_strings: null buffer");
    kern::pq_dict_strings(P<const kern::PqPage>(pages), npages, P<const int32_t>(page_col),
                          P<const kern::PqDecodeSpec>(specs), S(s));
  });
  m.def("pq_decode", [](uintptr_t pages, int64_t npages, uintptr_t page_col, uintptr_t specs, uintptr_t s) {
    if (npages > 0 && (!pages || !page_col || !specs)) throw std::runtime_error("pq_decode: null buffer");
    kern::pq_decode(P<const kern::PqPage>(pages), npages, P<const int32_t>(page_col),
                    P<const kern::PqDecodeSpec>(specs), S(s));
  });
  m.def("pq_str_copy", [](uintptr_t pos, uintptr_t off, int64_t n, uintptr_t out, uintptr_t s) {
    kern::pq_str_copy(P<const int64_t>(pos), P<const int64_t>(off), n, P<uint8_t>(out), S(s));
  });

  // ---------------------------------------------------------------- datagen
  // params: (kind, seed, row_base, min_len, max_len, vocab, vocab_off, vocab_n,
  //          inject, inject_len, inject_every, suffix_char, aux, row_ids)
  auto mkparams = [](const py::tuple& t) {
    kern::TextGenParams p;
    p.kind = t[0].cast<int>();
    p.seed = t[1].cast<uint64_t>();
    p.row_base = t[2].cast<int64_t>();
    p.min_len = t[3].cast<int>();
    p.max_len = t[4].cast<int>();
    p.vocab = P<const uint8_t>(t[5].cast<uintptr_t>());
    p.vocab_off = P<const int32_t>(t[6].cast<uintptr_t>());
    p.vocab_n = t[7].cast<int>();
    p.inject = P<const uint8_t>(t[8].cast<uintptr_t>());
    p.inject_len = t[9].cast<int>();
    p.inject_every = t[10].cast<int>();
    p.suffix_char = t[11].cast<int>();
    p.aux = P<const int32_t>(t[12].cast<uintptr_t>());
    p.row_ids = t.size() > 13 ? P<const int64_t>(t[13].cast<uintptr_t>()) : nullptr;
    return p;
  };
  m.def("textgen_lengths", [mkparams](const py::tuple& t, int64_t n, uintptr_t lens, bool device, uintptr_t s) {
    auto p = mkparams(t);
    py::gil_scoped_release rel;
    kern::textgen_lengths(p, n, P<int64_t>(lens), device, S(s));
  });
  m.def("textgen_write", [mkparams](const py::tuple& t, int64_t n, uintptr_t off, uintptr_t chars, bool device, uintptr_t s) {
    auto p = mkparams(t);
    py::gil_scoped_release rel;
    kern::textgen_write(p, n, P<const int64_t>(off), P<uint8_t>(chars), device, S(s));
  });
}
