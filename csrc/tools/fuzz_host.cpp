// Host-side robustness driver for the native front end, built with
// AddressSanitizer + UndefinedBehaviorSanitizer (scripts/sanitize_host.sh).
//
// GPU ASan is not available on the MI355X pool, so the sanitizer coverage the
// survey asks for runs on the host code that parses untrusted
// input: the SQL lexer/parser (csrc/sql/parser.cpp) and the Parquet footer /
// page-header Thrift decoders (csrc/io/parquet_meta.cpp). Inputs:
//   * every SQL statement of a corpus file (one statement per blank-line
//     separated block), each also truncated at every byte and with seeded
//     random byte flips;
//   * the footer of every Parquet file named on the command line, whole,
//     truncated at every byte and with seeded byte flips, plus the first page
//     header of each file under the same mutations.
// Parse errors are expected; any sanitizer report aborts the run (non-zero exit).
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "io/parquet_meta.h"
#include "sql/ast.h"

using namespace igloo;

static int g_ok = 0, g_err = 0;

static void try_sql(const std::string& s) {
  try {
    auto v = sql::parse_sql(s);
    g_ok += (int)v.size() > 0;
  } catch (const std::exception&) {
    ++g_err;
  }
}

static void try_footer(const std::vector<uint8_t>& b) {
  try {
    auto m = io::parse_file_meta(b.data(), b.size());
    g_ok += m.num_rows >= 0;
  } catch (const std::exception&) {
    ++g_err;
  }
}

static void try_page(const std::vector<uint8_t>& b) {
  try {
    auto h = io::parse_page_header(b.data(), b.size());
    (void)h;
    ++g_ok;
  } catch (const std::exception&) {
    ++g_err;
  }
}

template <class F>
static void mutate(const std::string& base, std::mt19937& rng, int flips, F&& f) {
  for (size_t i = 0; i <= base.size(); i += (base.size() > 4096 ? base.size() / 2048 : 1)) f(base.substr(0, i));
  for (int k = 0; k < flips && !base.empty(); ++k) {
    std::string m = base;
    int n = 1 + (int)(rng() % 4);
    for (int j = 0; j < n; ++j) m[rng() % m.size()] = (char)(rng() & 0xFF);
    f(m);
  }
}

static std::vector<uint8_t> read_file(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s sql_corpus.txt [file.parquet ...]\n", argv[0]);
    return 2;
  }
  std::mt19937 rng(20251017);
  std::ifstream in(argv[1]);
  std::stringstream ss;
  ss << in.rdbuf();
  std::string text = ss.str(), cur;
  std::vector<std::string> stmts;
  std::istringstream lines(text);
  for (std::string line; std::getline(lines, line);) {
    if (line.find_first_not_of(" \t\r") == std::string::npos) {
      if (!cur.empty()) stmts.push_back(cur);
      cur.clear();
    } else {
      cur += line + "\n";
    }
  }
  if (!cur.empty()) stmts.push_back(cur);
  for (auto& s : stmts) mutate(s, rng, 200, [](const std::string& m) { try_sql(m); });
  std::printf("sql: %zu statements, %d parsed, %d rejected\n", stmts.size(), g_ok, g_err);
  int files = 0;
  for (int a = 2; a < argc; ++a) {
    auto b = read_file(argv[a]);
    if (b.size() < 12) continue;
    uint32_t flen = (uint32_t)b[b.size() - 8] | ((uint32_t)b[b.size() - 7] << 8) | ((uint32_t)b[b.size() - 6] << 16) |
                    ((uint32_t)b[b.size() - 5] << 24);
    if (flen + 8 > b.size()) continue;
    std::string footer(b.end() - 8 - flen, b.end() - 8);
    mutate(footer, rng, 500, [](const std::string& m) { try_footer(std::vector<uint8_t>(m.begin(), m.end())); });
    std::string page(b.begin() + 4, b.begin() + std::min<size_t>(b.size() - 8, 4 + 256));
    mutate(page, rng, 500, [](const std::string& m) { try_page(std::vector<uint8_t>(m.begin(), m.end())); });
    ++files;
  }
  std::printf("parquet: %d files; total %d parsed, %d rejected; no sanitizer reports\n", files, g_ok, g_err);
  return 0;
}
