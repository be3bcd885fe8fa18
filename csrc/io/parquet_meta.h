// Native Parquet metadata: Thrift compact-protocol decoding of the file footer
// (FileMetaData) and of the page headers inside a column chunk, a page planner
// that turns a column's chunks into GPU decode descriptors, and a
// multithreaded positional reader that stages column-chunk byte ranges into
// pinned host memory for one H2D copy.
//
// Parity: the reference reads Parquet through parquet-rs on a blocking thread
// (crates/engine/src/operators/parquet_scan.rs:47-58) and DataFusion's
// ListingTable+ParquetFormat (crates/engine/tests/integration_test.rs:46-56);
// here the host only parses metadata and moves bytes — decompression and page
// decoding run on the GPU (csrc/kernels/parquet.hip).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace igloo {
namespace io {

struct ParquetError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

enum PqType : int { PQ_BOOLEAN = 0, PQ_INT32 = 1, PQ_INT64 = 2, PQ_INT96 = 3, PQ_FLOAT = 4, PQ_DOUBLE = 5,
                    PQ_BYTE_ARRAY = 6, PQ_FLBA = 7 };
enum PqCodec : int { PQ_UNCOMPRESSED = 0, PQ_SNAPPY = 1, PQ_GZIP = 2, PQ_LZO = 3, PQ_BROTLI = 4, PQ_LZ4 = 5,
                     PQ_ZSTD = 6, PQ_LZ4_RAW = 7 };
enum PqPageType : int { PQ_DATA_PAGE = 0, PQ_INDEX_PAGE = 1, PQ_DICTIONARY_PAGE = 2, PQ_DATA_PAGE_V2 = 3 };
enum PqEncoding : int { PQ_PLAIN = 0, PQ_PLAIN_DICTIONARY = 2, PQ_RLE = 3, PQ_BIT_PACKED = 4,
                        PQ_DELTA_BINARY_PACKED = 5, PQ_DELTA_LENGTH_BYTE_ARRAY = 6, PQ_DELTA_BYTE_ARRAY = 7,
                        PQ_RLE_DICTIONARY = 8, PQ_BYTE_STREAM_SPLIT = 9 };

struct PqStats {
  bool has_min = false, has_max = false, has_nulls = false;
  std::string min, max;  // plain-encoded little-endian (fixed) or raw bytes
  int64_t null_count = 0;
};

// A leaf column of the (flattened) schema.
struct PqLeaf {
  std::string name;        // dotted path
  int type = -1;           // PqType
  int type_length = 0;     // FIXED_LEN_BYTE_ARRAY width
  int max_def = 0, max_rep = 0;
  int converted_type = -1;
  int scale = 0, precision = 0;
  std::string logical;     // "", "string", "decimal", "date", "timestamp_ms/us/ns", "int8/16/32/64", "uint..."
};

struct PqChunk {
  int type = -1;
  int codec = 0;
  int64_t num_values = 0;
  int64_t total_compressed = 0, total_uncompressed = 0;
  int64_t data_page_offset = -1, dictionary_page_offset = -1;
  bool external = false;  // ColumnChunk.file_path set: data lives in another file
  std::vector<int> encodings;
  PqStats stats;
  // first byte of the chunk (dictionary page when there is one)
  int64_t start() const {
    return (dictionary_page_offset > 0 && dictionary_page_offset < data_page_offset) ? dictionary_page_offset
                                                                                      : data_page_offset;
  }
};

struct PqRowGroup {
  int64_t num_rows = 0;
  std::vector<PqChunk> chunks;  // one per leaf
};

struct PqFileMeta {
  int32_t version = 0;
  int64_t num_rows = 0;
  std::string created_by;
  std::vector<PqLeaf> leaves;
  std::vector<PqRowGroup> row_groups;
};

struct PqPageHeader {
  int type = -1;
  int32_t header_len = 0;  // bytes of the Thrift header
  int32_t compressed = 0, uncompressed = 0;
  int32_t num_values = 0;
  int32_t encoding = 0;
  int32_t def_encoding = 3, rep_encoding = 3;
  // v2
  int32_t num_nulls = 0, num_rows = 0;
  int32_t def_len = 0, rep_len = 0;
  bool is_compressed = true;
};

PqFileMeta parse_file_meta(const uint8_t* p, size_t n);
PqFileMeta read_file_meta(const std::string& path);
PqPageHeader parse_page_header(const uint8_t* p, size_t n);
// Every page header of a column chunk whose bytes are [p, p+n).
std::vector<PqPageHeader> parse_chunk_pages(const uint8_t* p, size_t n);

struct ReadRange {
  int64_t file_offset;
  int64_t length;
  uint8_t* dst;
};
// Positional reads of `ranges` from `path` on up to `threads` threads.
void pread_ranges(const std::string& path, const std::vector<ReadRange>& ranges, int threads);

// ---- page planning -----------------------------------------------------------
// One column's chunks, staged back to back in one host buffer (mirrored 1:1 in
// a device "raw" buffer). The planner walks the page headers and emits the
// device descriptors of csrc/kernels/kernels.h (PqPage / PqSnappyJob); page
// payloads that need decompression get a slot in a device "dec" buffer.
struct PqChunkIn {
  int64_t buf_off;    // chunk start inside the staged buffer
  int64_t length;     // chunk bytes
  int codec;
  int64_t first_row;  // output row of the chunk's first value
  int64_t num_rows;
};

struct PqPlan {
  std::vector<uint8_t> pages;  // packed kern::PqPage
  std::vector<uint8_t> jobs;   // packed kern::PqSnappyJob
  int64_t num_pages = 0, num_jobs = 0, num_dict_pages = 0;
  int64_t num_zstd_jobs = 0;   // of num_jobs
  int64_t dec_bytes = 0;     // device bytes needed for decompressed payloads
  int64_t dict_entries = 0;  // sum of dictionary sizes over chunks
  int64_t plain_pages = 0;   // data pages not dictionary-encoded
  int64_t max_page_values = 0;
  std::string unsupported;   // non-empty: this column needs the host decoder
};

// dec_base: first free byte of the (shared) decompression buffer; plan.dec_bytes
// is returned as the end of this column's slots (dec_base included).
PqPlan plan_column(const uint8_t* host, const std::vector<PqChunkIn>& chunks, int phys_type, int max_def,
                   int max_rep, int64_t dec_base = 0, int type_len = 0);

}  // namespace io
}  // namespace igloo
