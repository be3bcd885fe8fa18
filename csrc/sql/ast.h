// SQL abstract syntax tree produced by the native lexer/parser.
//
// Parity: replaces the reference's use of sqlparser-rs through DataFusion
// (reference crates/engine/src/parser.rs:7-12, GenericDialect) with a
// hand-written recursive-descent parser. The tree is a small generic node
// type so the binder (Python side, igloo_amd/sql/binder.py) can walk it
// without a per-node binding class.
#pragma once

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace igloo {
namespace sql {

struct Node;
using NodeP = std::shared_ptr<Node>;

struct Node {
  std::string kind;                        // e.g. "select", "bin", "col", "lit"
  std::string str;                         // operator / name / literal text
  std::vector<NodeP> kids;                 // positional children
  std::map<std::string, NodeP> attrs;      // named children (may be null)
  std::map<std::string, std::string> flags;  // small string attributes
  int pos = 0;                             // byte offset in the source text

  Node() = default;
  Node(std::string k, std::string s = {}) : kind(std::move(k)), str(std::move(s)) {}
};

inline NodeP make(const std::string& kind, const std::string& s = {}) {
  return std::make_shared<Node>(kind, s);
}

struct ParseError : std::runtime_error {
  int pos;
  ParseError(const std::string& msg, int p) : std::runtime_error(msg), pos(p) {}
};

// Parse a string holding one or more ';'-separated statements.
std::vector<NodeP> parse_sql(const std::string& text);

// Token stream exposed for tests / tooling.
struct Token {
  enum Kind { Ident, QuotedIdent, Keyword, Number, String, Op, End } kind;
  std::string text;  // keywords upper-cased; identifiers lower-cased (unquoted)
  int pos;
};
std::vector<Token> tokenize(const std::string& text);

}  // namespace sql
}  // namespace igloo
