// Hand-written SQL lexer + recursive-descent parser.
//
// Covers the DataFusion-compatible surface the reference relies on
// (reference crates/engine/src/lib.rs:54-57 feeds arbitrary SQL to
// DataFusion; crates/engine/src/parser.rs:7-12 parses with GenericDialect):
// SELECT [DISTINCT] ... FROM ... [JOIN ... ON/USING] WHERE ... GROUP BY ...
// HAVING ... ORDER BY ... [NULLS FIRST|LAST] LIMIT/OFFSET, WITH CTEs,
// UNION/INTERSECT/EXCEPT, scalar/IN/EXISTS subqueries, CASE, CAST, '::',
// EXTRACT, SUBSTRING(x FROM a FOR b), DATE/INTERVAL literals, LIKE/ILIKE,
// BETWEEN, IN-lists, IS [NOT] NULL, plus EXPLAIN [ANALYZE], SET,
// CREATE EXTERNAL TABLE ... STORED AS ... LOCATION, SHOW TABLES, DROP TABLE.
#include "ast.h"

#include <algorithm>
#include <cctype>
#include <set>

namespace igloo {
namespace sql {

namespace {

const std::set<std::string>& reserved() {
  static const std::set<std::string> kw = {
      "SELECT", "FROM",  "WHERE",   "GROUP",  "BY",     "HAVING",   "ORDER",  "LIMIT",
      "OFFSET", "UNION", "INTERSECT", "EXCEPT", "JOIN", "INNER",    "LEFT",   "RIGHT",
      "FULL",   "OUTER", "CROSS",   "ON",     "USING",  "AS",       "AND",    "OR",
      "NOT",    "IN",    "IS",      "NULL",   "LIKE",   "ILIKE",    "BETWEEN", "CASE",
      "WHEN",   "THEN",  "ELSE",    "END",    "EXISTS", "DISTINCT", "ALL",    "WITH",
      "ASC",    "DESC",  "NULLS",   "NATURAL", "SEMI",  "ANTI",     "FETCH",  "WINDOW",
      "QUALIFY", "TRUE", "FALSE",   "INTERVAL", "DATE", "TIMESTAMP", "CAST",   "EXTRACT",
      "SUBSTRING", "ESCAPE", "SET", "EXPLAIN", "VALUES", "CREATE", "DROP", "SHOW",
      "FIRST", "LAST"};
  return kw;
}

std::string upper(std::string s) {
  for (auto& c : s) c = (char)std::toupper((unsigned char)c);
  return s;
}
std::string lower(std::string s) {
  for (auto& c : s) c = (char)std::tolower((unsigned char)c);
  return s;
}

}  // namespace

std::vector<Token> tokenize(const std::string& t) {
  std::vector<Token> out;
  size_t i = 0, n = t.size();
  while (i < n) {
    char c = t[i];
    if (std::isspace((unsigned char)c)) { ++i; continue; }
    if (c == '-' && i + 1 < n && t[i + 1] == '-') {  // line comment
      while (i < n && t[i] != '\n') ++i;
      continue;
    }
    if (c == '/' && i + 1 < n && t[i + 1] == '*') {  // block comment
      size_t j = t.find("*/", i + 2);
      if (j == std::string::npos) throw ParseError("unterminated block comment", (int)i);
      i = j + 2;
      continue;
    }
    int start = (int)i;
    if (std::isalpha((unsigned char)c) || c == '_') {
      size_t j = i;
      while (j < n && (std::isalnum((unsigned char)t[j]) || t[j] == '_' || t[j] == '$')) ++j;
      std::string w = t.substr(i, j - i);
      std::string u = upper(w);
      if (reserved().count(u))
        out.push_back({Token::Keyword, u, start});
      else
        out.push_back({Token::Ident, lower(w), start});
      i = j;
      continue;
    }
    if (std::isdigit((unsigned char)c) || (c == '.' && i + 1 < n && std::isdigit((unsigned char)t[i + 1]))) {
      size_t j = i;
      while (j < n && std::isdigit((unsigned char)t[j])) ++j;
      if (j < n && t[j] == '.') {
        ++j;
        while (j < n && std::isdigit((unsigned char)t[j])) ++j;
      }
      if (j < n && (t[j] == 'e' || t[j] == 'E')) {
        size_t k = j + 1;
        if (k < n && (t[k] == '+' || t[k] == '-')) ++k;
        if (k < n && std::isdigit((unsigned char)t[k])) {
          j = k;
          while (j < n && std::isdigit((unsigned char)t[j])) ++j;
        }
      }
      out.push_back({Token::Number, t.substr(i, j - i), start});
      i = j;
      continue;
    }
    if (c == '\'') {
      std::string s;
      size_t j = i + 1;
      for (;;) {
        if (j >= n) throw ParseError("unterminated string literal", start);
        if (t[j] == '\'') {
          if (j + 1 < n && t[j + 1] == '\'') { s += '\''; j += 2; continue; }
          ++j;
          break;
        }
        s += t[j++];
      }
      out.push_back({Token::String, s, start});
      i = j;
      continue;
    }
    if (c == '"' || c == '`') {
      char q = c;
      size_t j = t.find(q, i + 1);
      if (j == std::string::npos) throw ParseError("unterminated quoted identifier", start);
      out.push_back({Token::QuotedIdent, t.substr(i + 1, j - i - 1), start});
      i = j + 1;
      continue;
    }
    if (c == '$' && i + 1 < n && std::isdigit((unsigned char)t[i + 1])) {  // $n statement parameter
      size_t j = i + 1;
      while (j < n && std::isdigit((unsigned char)t[j])) ++j;
      out.push_back({Token::Op, t.substr(i, j - i), start});
      i = j;
      continue;
    }
    if (t.compare(i, 3, "!~*") == 0) {
      out.push_back({Token::Op, "!~*", start});
      i += 3;
      continue;
    }
    static const char* ops2[] = {"<>", "!=", "<=", ">=", "||", "::", "==", "~*", "!~"};
    bool matched = false;
    for (auto op : ops2) {
      if (t.compare(i, 2, op) == 0) {
        out.push_back({Token::Op, std::string(op) == "==" ? "=" : op, start});
        i += 2;
        matched = true;
        break;
      }
    }
    if (matched) continue;
    if (std::string("+-*/%=<>(),.;~[]").find(c) != std::string::npos) {
      out.push_back({Token::Op, std::string(1, c), start});
      ++i;
      continue;
    }
    throw ParseError(std::string("unexpected character '") + c + "'", start);
  }
  out.push_back({Token::End, "", (int)n});
  return out;
}

namespace {

class Parser {
 public:
  explicit Parser(const std::string& text) : toks_(tokenize(text)) {}

  std::vector<NodeP> statements() {
    std::vector<NodeP> out;
    while (true) {
      while (acceptOp(";")) {}
      if (peek().kind == Token::End) break;
      out.push_back(statement());
      if (peek().kind != Token::End && !isOp(";"))
        fail("expected end of statement");
    }
    return out;
  }

 private:
  std::vector<Token> toks_;
  size_t p_ = 0;

  const Token& peek(int k = 0) const { return toks_[std::min(p_ + k, toks_.size() - 1)]; }
  const Token& next() { return toks_[p_ < toks_.size() - 1 ? p_++ : p_]; }
  [[noreturn]] void fail(const std::string& msg) const {
    const Token& t = peek();
    std::string near = t.kind == Token::End ? "end of input" : "'" + t.text + "'";
    throw ParseError(msg + " near " + near + " at position " + std::to_string(t.pos), t.pos);
  }
  bool isKw(const char* k, int off = 0) const {
    return peek(off).kind == Token::Keyword && peek(off).text == k;
  }
  bool isWord(const char* w, int off = 0) const {  // non-reserved keyword, e.g. TABLE
    return peek(off).kind == Token::Ident && peek(off).text == lower(w);
  }
  bool isOp(const char* o, int off = 0) const {
    return peek(off).kind == Token::Op && peek(off).text == o;
  }
  bool acceptKw(const char* k) {
    if (isKw(k)) { ++p_; return true; }
    return false;
  }
  bool acceptWord(const char* w) {
    if (isWord(w)) { ++p_; return true; }
    return false;
  }
  bool acceptOp(const char* o) {
    if (isOp(o)) { ++p_; return true; }
    return false;
  }
  void expectKw(const char* k) {
    if (!acceptKw(k)) fail(std::string("expected ") + k);
  }
  void expectWord(const char* w) {
    if (!acceptWord(w)) fail(std::string("expected ") + upper(w));
  }
  void expectOp(const char* o) {
    if (!acceptOp(o)) fail(std::string("expected '") + o + "'");
  }
  std::string ident() {
    const Token& t = peek();
    if (t.kind == Token::Ident || t.kind == Token::QuotedIdent) { ++p_; return t.text; }
    // a few reserved words are fine as identifiers in name position
    if (t.kind == Token::Keyword && (t.text == "FIRST" || t.text == "LAST" || t.text == "DATE")) {
      ++p_;
      return lower(t.text);
    }
    fail("expected identifier");
  }
  NodeP list(std::vector<NodeP> v) {
    auto n = make("list");
    n->kids = std::move(v);
    return n;
  }

  // ---------------------------------------------------------------- statements
  NodeP statement() {
    int pos = peek().pos;
    NodeP n;
    if (acceptKw("EXPLAIN")) {
      n = make("explain");
      if (acceptWord("analyze")) n->flags["analyze"] = "1";
      if (acceptWord("verbose")) n->flags["verbose"] = "1";
      n->kids.push_back(statement());
    } else if (acceptKw("SET")) {
      n = make("set");
      std::string name = ident();
      while (acceptOp(".")) name += "." + ident();
      n->str = name;
      if (!acceptOp("=")) expectWord("to");
      n->kids.push_back(expr());
    } else if (acceptKw("SHOW")) {
      n = make("show");
      if (acceptWord("all")) {
        n->str = "all";
      } else {
        n->str = ident();
        if (n->str == "columns" || n->str == "fields") {
          if (!acceptKw("FROM")) expectKw("IN");
          std::string t = ident();
          while (acceptOp(".")) t += "." + ident();
          n->flags["table"] = t;
          n->str = "columns";
        } else {
          while (acceptOp(".")) n->str += "." + ident();
        }
      }
    } else if (isWord("describe") || (isKw("DESC") && peek(1).kind != Token::End)) {
      ++p_;
      n = make("describe");
      std::string t = ident();
      while (acceptOp(".")) t += "." + ident();
      n->str = t;
    } else if (acceptWord("insert")) {
      acceptWord("into");
      n = make("insert");
      std::string t = ident();
      while (acceptOp(".")) t += "." + ident();
      n->str = t;
      if (isOp("(") && (peek(1).kind == Token::Ident || peek(1).kind == Token::QuotedIdent)) {
        ++p_;
        std::vector<NodeP> cols;
        do cols.push_back(make("name", ident()));
        while (acceptOp(","));
        expectOp(")");
        n->attrs["columns"] = list(cols);
      }
      n->attrs["query"] = query();
    } else if (acceptWord("truncate")) {
      acceptWord("table");
      n = make("truncate", ident());
    } else if (acceptKw("CREATE")) {
      n = createStmt();
    } else if (acceptWord("copy")) {
      // COPY (query) | table TO 'path' [STORED AS fmt] [OPTIONS (k v, ...)]
      n = make("copy");
      if (acceptOp("(")) {
        n->attrs["query"] = query();
        expectOp(")");
      } else {
        std::string t = ident();
        while (acceptOp(".")) t += "." + ident();
        n->str = t;
      }
      expectWord("to");
      if (peek().kind != Token::String) fail("expected target path string");
      n->flags["path"] = next().text;
      for (;;) {
        if (acceptWord("stored")) {
          expectKw("AS");
          n->flags["stored_as"] = upper(ident());
        } else if (acceptWord("options") || (isOp("(") && !n->flags.count("opts"))) {
          n->flags["opts"] = "1";
          expectOp("(");
          do {
            std::string k = peek().kind == Token::String ? next().text : ident();
            while (acceptOp(".")) k += "." + ident();
            std::string v = next().text;
            n->flags["opt." + lower(k)] = v;
          } while (acceptOp(","));
          expectOp(")");
        } else {
          break;
        }
      }
    } else if (acceptWord("prepare")) {
      // PREPARE name [(type, ...)] AS statement
      n = make("prepare", ident());
      if (acceptOp("(")) {
        std::vector<NodeP> ts;
        do ts.push_back(make("name", typeName()));
        while (acceptOp(","));
        expectOp(")");
        n->attrs["types"] = list(ts);
      }
      expectKw("AS");
      n->kids.push_back(statement());
    } else if (acceptWord("execute")) {
      n = make("execute", ident());
      std::vector<NodeP> args;
      if (acceptOp("(")) {
        if (!acceptOp(")")) {
          do args.push_back(expr());
          while (acceptOp(","));
          expectOp(")");
        }
      }
      n->attrs["args"] = list(args);
    } else if (acceptWord("deallocate")) {
      acceptWord("prepare");
      n = make("deallocate", ident());
    } else if (acceptKw("DROP")) {
      if (acceptWord("view")) n = make("drop_view");
      else { expectWord("table"); n = make("drop_table"); }
      if (acceptWord("if")) { expectKw("EXISTS"); n->flags["if_exists"] = "1"; }
      n->str = ident();
    } else {
      n = query();
    }
    n->pos = pos;
    return n;
  }

  NodeP createStmt() {
    bool replace = false;
    if (acceptKw("OR")) { expectWord("replace"); replace = true; }
    bool external = acceptWord("external");
    if (acceptWord("view")) {
      auto n = make("create_view");
      if (replace) n->flags["replace"] = "1";
      if (acceptWord("if")) { expectKw("NOT"); expectKw("EXISTS"); n->flags["if_not_exists"] = "1"; }
      n->str = ident();
      if (isOp("(")) {
        ++p_;
        std::vector<NodeP> cols;
        do cols.push_back(make("name", ident()));
        while (acceptOp(","));
        expectOp(")");
        n->attrs["columns"] = list(cols);
      }
      expectKw("AS");
      n->attrs["query"] = query();
      return n;
    }
    expectWord("table");
    auto n = make(external ? "create_external_table" : "create_table");
    if (acceptWord("if")) { expectKw("NOT"); expectKw("EXISTS"); n->flags["if_not_exists"] = "1"; }
    n->str = ident();
    std::vector<NodeP> cols;
    if (acceptOp("(")) {
      do {
        auto c = make("coldef", ident());
        c->flags["type"] = typeName();
        if (acceptKw("NOT")) { expectKw("NULL"); c->flags["not_null"] = "1"; }
        else acceptKw("NULL");
        cols.push_back(c);
      } while (acceptOp(","));
      expectOp(")");
    }
    n->attrs["columns"] = list(cols);
    for (;;) {
      if (acceptWord("stored")) {
        expectKw("AS");
        n->flags["stored_as"] = upper(ident());
      } else if (acceptKw("WITH")) {
        expectWord("header");
        expectWord("row");
        n->flags["header"] = "1";
      } else if (acceptWord("location")) {
        if (peek().kind != Token::String) fail("expected location string");
        n->flags["location"] = next().text;
      } else if (acceptWord("delimiter")) {
        n->flags["delimiter"] = next().text;
      } else if (acceptWord("options")) {
        expectOp("(");
        do {
          std::string k = peek().kind == Token::String ? next().text : ident();
          std::string v = next().text;
          n->flags["opt." + k] = v;
        } while (acceptOp(","));
        expectOp(")");
      } else if (acceptKw("AS")) {
        n->attrs["query"] = query();
      } else {
        break;
      }
    }
    return n;
  }

  std::string typeName() {
    std::string t;
    if (peek().kind == Token::Keyword && (peek().text == "DATE" || peek().text == "TIMESTAMP" || peek().text == "INTERVAL"))
      t = next().text;
    else
      t = upper(ident());
    if (t == "DOUBLE") acceptWord("precision");
    if (t == "CHARACTER" && acceptWord("varying")) t = "VARCHAR";
    if (acceptOp("(")) {
      t += "(";
      t += next().text;
      while (acceptOp(",")) t += "," + next().text;
      expectOp(")");
      t += ")";
    }
    return t;
  }

  // --------------------------------------------------------------------- query
  NodeP query() {
    auto q = make("query");
    q->pos = peek().pos;
    if (acceptKw("WITH")) {
      if (acceptWord("recursive")) q->flags["recursive"] = "1";
      std::vector<NodeP> ctes;
      do {
        auto c = make("cte", ident());
        if (acceptOp("(")) {
          std::vector<NodeP> cols;
          do cols.push_back(make("name", ident()));
          while (acceptOp(","));
          expectOp(")");
          c->attrs["columns"] = list(cols);
        }
        expectKw("AS");
        expectOp("(");
        c->attrs["query"] = query();
        expectOp(")");
        ctes.push_back(c);
      } while (acceptOp(","));
      q->attrs["with"] = list(ctes);
    }
    q->attrs["body"] = setExpr();
    if (acceptKw("ORDER")) {
      expectKw("BY");
      std::vector<NodeP> items;
      do items.push_back(orderItem());
      while (acceptOp(","));
      q->attrs["order"] = list(items);
    }
    for (;;) {
      if (acceptKw("LIMIT")) {
        if (acceptKw("ALL")) continue;
        q->attrs["limit"] = expr();
      } else if (acceptKw("OFFSET")) {
        q->attrs["offset"] = expr();
        if (!acceptWord("rows")) acceptWord("row");
      } else if (acceptKw("FETCH")) {
        if (!acceptKw("FIRST")) expectWord("next");
        q->attrs["limit"] = expr();
        if (!acceptWord("rows")) acceptWord("row");
        expectWord("only");
      } else {
        break;
      }
    }
    return q;
  }

  NodeP orderItem() {
    auto o = make("order");
    o->kids.push_back(expr());
    if (acceptKw("DESC")) o->flags["desc"] = "1";
    else acceptKw("ASC");
    if (acceptKw("NULLS")) {
      if (acceptKw("FIRST")) o->flags["nulls"] = "first";
      else { expectKw("LAST"); o->flags["nulls"] = "last"; }
    }
    return o;
  }

  NodeP setExpr() {
    NodeP left = setTerm();
    for (;;) {
      std::string op;
      if (acceptKw("UNION")) op = "union";
      else if (acceptKw("EXCEPT")) op = "except";
      else break;
      if (acceptKw("ALL")) op += "_all";
      else acceptKw("DISTINCT");
      auto n = make("setop", op);
      n->kids = {left, setTerm()};
      left = n;
    }
    return left;
  }

  NodeP setTerm() {  // INTERSECT binds tighter than UNION/EXCEPT
    NodeP left = setPrimary();
    while (acceptKw("INTERSECT")) {
      std::string op = "intersect";
      if (acceptKw("ALL")) op += "_all";
      else acceptKw("DISTINCT");
      auto n = make("setop", op);
      n->kids = {left, setPrimary()};
      left = n;
    }
    return left;
  }

  NodeP setPrimary() {
    if (isOp("(")) {
      // parenthesised query
      ++p_;
      NodeP q = query();
      expectOp(")");
      auto n = make("subquery_body");
      n->attrs["query"] = q;
      return n;
    }
    if (acceptKw("VALUES")) return valuesBody();
    return select();
  }

  NodeP valuesBody() {
    auto v = make("values");
    do {
      expectOp("(");
      std::vector<NodeP> row;
      do row.push_back(expr());
      while (acceptOp(","));
      expectOp(")");
      v->kids.push_back(list(row));
    } while (acceptOp(","));
    return v;
  }

  NodeP select() {
    int pos = peek().pos;
    expectKw("SELECT");
    auto s = make("select");
    s->pos = pos;
    if (acceptKw("DISTINCT")) {
      if (acceptKw("ON")) {  // DISTINCT ON (expr, ...): first row per key
        expectOp("(");
        std::vector<NodeP> on;
        do on.push_back(expr());
        while (acceptOp(","));
        expectOp(")");
        s->attrs["distinct_on"] = list(on);
      } else {
        s->flags["distinct"] = "1";
      }
    } else {
      acceptKw("ALL");
    }
    std::vector<NodeP> items;
    do items.push_back(selectItem());
    while (acceptOp(","));
    s->attrs["items"] = list(items);
    if (acceptKw("FROM")) {
      std::vector<NodeP> from;
      do from.push_back(fromItem());
      while (acceptOp(","));
      s->attrs["from"] = list(from);
    }
    if (acceptKw("WHERE")) s->attrs["where"] = expr();
    if (acceptKw("GROUP")) {
      expectKw("BY");
      std::vector<NodeP> g;
      do g.push_back(groupItem());
      while (acceptOp(","));
      s->attrs["group"] = list(g);
    }
    if (acceptKw("HAVING")) s->attrs["having"] = expr();
    if (acceptKw("WINDOW")) {
      std::vector<NodeP> ws;
      do {
        std::string name = ident();
        expectKw("AS");
        expectOp("(");
        auto w = windowSpec();
        expectOp(")");
        auto d = make("window_def", name);
        d->attrs["spec"] = w;
        ws.push_back(d);
      } while (acceptOp(","));
      s->attrs["windows"] = list(ws);
    }
    if (acceptKw("QUALIFY")) s->attrs["qualify"] = expr();
    return s;
  }

  // GROUP BY item: expr | ROLLUP (...) | CUBE (...) | GROUPING SETS ((...), ...)
  NodeP groupItem() {
    if ((isWord("rollup") || isWord("cube")) && isOp("(", 1)) {
      auto n = make(next().text);
      expectOp("(");
      do n->kids.push_back(groupingElem());
      while (acceptOp(","));
      expectOp(")");
      return n;
    }
    if (isWord("grouping") && isWord("sets", 1)) {
      p_ += 2;
      auto n = make("grouping_sets");
      expectOp("(");
      do {
        if (isWord("rollup") || isWord("cube")) n->kids.push_back(groupItem());
        else n->kids.push_back(groupingElem());
      } while (acceptOp(","));
      expectOp(")");
      return n;
    }
    return expr();
  }

  // one grouping element: expr or a parenthesised (possibly empty) list
  NodeP groupingElem() {
    if (isOp("(")) {
      size_t save = p_;
      ++p_;
      if (acceptOp(")")) return list({});
      std::vector<NodeP> v;
      v.push_back(expr());
      if (acceptOp(",")) {
        do v.push_back(expr());
        while (acceptOp(","));
        expectOp(")");
        return list(v);
      }
      if (acceptOp(")")) return list(v);
      p_ = save;
    }
    return list({expr()});
  }

  NodeP selectItem() {
    // t.* / *
    if (isOp("*")) {
      ++p_;
      return make("star");
    }
    if ((peek().kind == Token::Ident || peek().kind == Token::QuotedIdent) && isOp(".", 1) && isOp("*", 2)) {
      auto s = make("star", next().text);
      p_ += 2;
      return s;
    }
    auto it = make("item");
    it->kids.push_back(expr());
    if (acceptKw("AS")) {
      it->flags["alias"] = peek().kind == Token::String ? next().text : ident();
    } else if (peek().kind == Token::Ident || peek().kind == Token::QuotedIdent) {
      it->flags["alias"] = ident();
    }
    return it;
  }

  void tableAlias(NodeP n) {
    if (acceptKw("AS")) {
      n->flags["alias"] = ident();
    } else if (peek().kind == Token::Ident || peek().kind == Token::QuotedIdent) {
      n->flags["alias"] = ident();
    } else {
      return;
    }
    if (isOp("(") && (peek(1).kind == Token::Ident || peek(1).kind == Token::QuotedIdent)) {
      ++p_;
      std::vector<NodeP> cols;
      do cols.push_back(make("name", ident()));
      while (acceptOp(","));
      expectOp(")");
      n->attrs["columns"] = list(cols);
    }
  }

  NodeP fromPrimary() {
    if (isOp("(")) {
      ++p_;
      if (isKw("SELECT") || isKw("WITH") || isKw("VALUES") || isOp("(")) {
        // could be a parenthesised join too: (a JOIN b)
        size_t save = p_;
        bool isQuery = isKw("SELECT") || isKw("WITH") || isKw("VALUES");
        if (!isQuery) {
          // look ahead: "((select" is a query; "(a join b)" is a join
          int depth = 0;
          size_t k = p_;
          while (k < toks_.size() && toks_[k].kind == Token::Op && toks_[k].text == "(") { ++depth; ++k; }
          isQuery = k < toks_.size() && toks_[k].kind == Token::Keyword &&
                    (toks_[k].text == "SELECT" || toks_[k].text == "WITH" || toks_[k].text == "VALUES");
          (void)depth;
        }
        if (isQuery) {
          auto n = make("subquery");
          n->attrs["query"] = query();
          expectOp(")");
          tableAlias(n);
          return n;
        }
        p_ = save;
      }
      NodeP j = fromItem();
      expectOp(")");
      if (j->kind == "table" || j->kind == "subquery") tableAlias(j);
      return j;
    }
    auto n = make("table");
    n->pos = peek().pos;
    std::string name = ident();
    while (acceptOp(".")) name += "." + ident();
    n->str = name;
    if (isOp("(")) {  // table function: generate_series(a, b [, step]), range(...), unnest(list)
      ++p_;
      n->kind = "table_func";
      if (!acceptOp(")")) {
        do n->kids.push_back(expr());
        while (acceptOp(","));
        expectOp(")");
      }
    }
    tableAlias(n);
    return n;
  }

  NodeP fromItem() {
    NodeP left = fromPrimary();
    for (;;) {
      std::string type;
      bool natural = acceptKw("NATURAL");
      if (acceptKw("CROSS")) { expectKw("JOIN"); type = "cross"; }
      else if (acceptKw("INNER")) { expectKw("JOIN"); type = "inner"; }
      else if (acceptKw("JOIN")) type = "inner";
      else if (acceptKw("LEFT")) {
        if (acceptKw("SEMI")) type = "left_semi";
        else if (acceptKw("ANTI")) type = "left_anti";
        else { acceptKw("OUTER"); type = "left"; }
        expectKw("JOIN");
      } else if (acceptKw("RIGHT")) {
        if (acceptKw("SEMI")) type = "right_semi";
        else if (acceptKw("ANTI")) type = "right_anti";
        else { acceptKw("OUTER"); type = "right"; }
        expectKw("JOIN");
      } else if (acceptKw("FULL")) { acceptKw("OUTER"); expectKw("JOIN"); type = "full"; }
      else {
        if (natural) fail("expected JOIN after NATURAL");
        break;
      }
      auto j = make("join", type);
      if (natural) j->flags["natural"] = "1";
      j->kids = {left, fromPrimary()};
      if (type != "cross" && !natural) {
        if (acceptKw("ON")) j->attrs["on"] = expr();
        else if (acceptKw("USING")) {
          expectOp("(");
          std::vector<NodeP> cols;
          do cols.push_back(make("name", ident()));
          while (acceptOp(","));
          expectOp(")");
          j->attrs["using"] = list(cols);
        } else {
          fail("expected ON or USING");
        }
      }
      left = j;
    }
    return left;
  }

  // --------------------------------------------------------------- expressions
  NodeP expr() { return orExpr(); }

  NodeP bin(const std::string& op, NodeP l, NodeP r) {
    auto n = make("bin", op);
    n->pos = l->pos;
    n->kids = {l, r};
    return n;
  }

  NodeP orExpr() {
    NodeP l = andExpr();
    while (acceptKw("OR")) l = bin("or", l, andExpr());
    return l;
  }
  NodeP andExpr() {
    NodeP l = notExpr();
    while (acceptKw("AND")) l = bin("and", l, notExpr());
    return l;
  }
  NodeP notExpr() {
    if (isKw("NOT") && !isKw("EXISTS", 1)) {
      ++p_;
      auto n = make("un", "not");
      n->kids.push_back(notExpr());
      return n;
    }
    return predicate();
  }

  NodeP predicate() {
    NodeP l = comparison();
    for (;;) {
      int save = (int)p_;
      bool neg = acceptKw("NOT");
      if (acceptKw("BETWEEN")) {
        auto n = make("between");
        if (neg) n->flags["neg"] = "1";
        acceptWord("symmetric");
        NodeP lo = additive();
        expectKw("AND");
        NodeP hi = additive();
        n->kids = {l, lo, hi};
        l = n;
      } else if (acceptKw("IN")) {
        expectOp("(");
        if (isKw("SELECT") || isKw("WITH") || isKw("VALUES")) {
          auto n = make("insub");
          if (neg) n->flags["neg"] = "1";
          n->kids.push_back(l);
          n->attrs["query"] = query();
          expectOp(")");
          l = n;
        } else {
          auto n = make("inlist");
          if (neg) n->flags["neg"] = "1";
          n->kids.push_back(l);
          do n->kids.push_back(expr());
          while (acceptOp(","));
          expectOp(")");
          l = n;
        }
      } else if (isWord("similar") && isWord("to", 1)) {
        p_ += 2;
        auto n = make("similar");
        if (neg) n->flags["neg"] = "1";
        n->kids = {l, additive()};
        if (acceptKw("ESCAPE")) n->attrs["escape"] = primary();
        l = n;
      } else if (isKw("LIKE") || isKw("ILIKE")) {
        auto n = make("like");
        if (next().text == "ILIKE") n->flags["ilike"] = "1";
        if (neg) n->flags["neg"] = "1";
        n->kids = {l, additive()};
        if (acceptKw("ESCAPE")) n->attrs["escape"] = primary();
        l = n;
      } else if (!neg && acceptKw("IS")) {
        bool isneg = acceptKw("NOT");
        if (acceptKw("NULL")) {
          auto n = make("isnull");
          if (isneg) n->flags["neg"] = "1";
          n->kids.push_back(l);
          l = n;
        } else if (acceptKw("TRUE") || acceptKw("FALSE")) {
          auto n = make("istruth", toks_[p_ - 1].text == "TRUE" ? "true" : "false");
          if (isneg) n->flags["neg"] = "1";
          n->kids.push_back(l);
          l = n;
        } else if (acceptKw("DISTINCT")) {
          expectKw("FROM");
          auto n = make("bin", isneg ? "is_not_distinct_from" : "is_distinct_from");
          n->kids = {l, comparison()};
          l = n;
        } else {
          fail("expected NULL, TRUE, FALSE or DISTINCT FROM after IS");
        }
      } else {
        p_ = save;
        break;
      }
    }
    return l;
  }

  NodeP comparison() {
    NodeP l = concat();
    for (;;) {
      const char* ops[] = {"=", "<>", "!=", "<", "<=", ">", ">=", "~", "~*", "!~", "!~*"};
      std::string op;
      for (auto o : ops)
        if (isOp(o)) { op = o; break; }
      if (op.empty()) break;
      ++p_;
      if (op == "!=") op = "<>";
      // quantified comparison: x > ALL (subquery) / ANY
      l = bin(op, l, concat());
    }
    return l;
  }

  NodeP concat() {
    NodeP l = additive();
    while (acceptOp("||")) l = bin("||", l, additive());
    return l;
  }
  NodeP additive() {
    NodeP l = multiplicative();
    for (;;) {
      if (acceptOp("+")) l = bin("+", l, multiplicative());
      else if (acceptOp("-")) l = bin("-", l, multiplicative());
      else break;
    }
    return l;
  }
  NodeP multiplicative() {
    NodeP l = unary();
    for (;;) {
      if (acceptOp("*")) l = bin("*", l, unary());
      else if (acceptOp("/")) l = bin("/", l, unary());
      else if (acceptOp("%")) l = bin("%", l, unary());
      else break;
    }
    return l;
  }
  NodeP unary() {
    if (acceptOp("-")) {
      NodeP x = unary();
      if (x->kind == "lit" && (x->flags["type"] == "int" || x->flags["type"] == "dec" || x->flags["type"] == "float")) {
        x->str = x->str[0] == '-' ? x->str.substr(1) : "-" + x->str;
        return x;
      }
      auto n = make("un", "-");
      n->kids.push_back(x);
      return n;
    }
    if (acceptOp("+")) return unary();
    return postfix();
  }
  NodeP postfix() {
    NodeP x = primary();
    for (;;) {
      if (acceptOp("::")) {
        auto c = make("cast");
        c->kids.push_back(x);
        c->flags["type"] = typeName();
        x = c;
      } else if (acceptOp("[")) {  // list element (1-based) or struct field by name
        auto f = make("func", "array_element");
        f->pos = x->pos;
        f->kids = {x, expr()};
        expectOp("]");
        x = f;
      } else {
        return x;
      }
    }
  }

  NodeP arrayLiteral() {  // [a, b, ...] -> make_array(a, b, ...)
    expectOp("[");
    auto f = make("func", "make_array");
    if (!acceptOp("]")) {
      do f->kids.push_back(expr());
      while (acceptOp(","));
      expectOp("]");
    }
    return f;
  }

  NodeP lit(const std::string& type, const std::string& s) {
    auto n = make("lit", s);
    n->flags["type"] = type;
    return n;
  }

  NodeP primary() {
    const Token& t = peek();
    int pos = t.pos;
    NodeP n = primaryInner();
    n->pos = pos;
    return n;
  }

  NodeP primaryInner() {
    const Token& t = peek();
    switch (t.kind) {
      case Token::Number: {
        ++p_;
        bool isdec = t.text.find('.') != std::string::npos;
        bool isexp = t.text.find_first_of("eE") != std::string::npos;
        return lit(isexp ? "float" : isdec ? "dec" : "int", t.text);
      }
      case Token::String:
        ++p_;
        return lit("str", t.text);
      case Token::Op:
        if (t.text == "[") return arrayLiteral();
        if (t.text.size() > 1 && t.text[0] == '$') {  // $n parameter of a prepared statement
          ++p_;
          return make("param", t.text.substr(1));
        }
        if (t.text == "(") {
          ++p_;
          if (isKw("SELECT") || isKw("WITH")) {
            auto n = make("subq");
            n->attrs["query"] = query();
            expectOp(")");
            return n;
          }
          NodeP e = expr();
          if (acceptOp(",")) {  // row constructor (a, b)
            auto r = make("row");
            r->kids.push_back(e);
            do r->kids.push_back(expr());
            while (acceptOp(","));
            expectOp(")");
            return r;
          }
          expectOp(")");
          auto n = make("paren");
          n->kids.push_back(e);
          return n;
        }
        fail("unexpected operator");
      case Token::Keyword: {
        const std::string& k = t.text;
        if (k == "NULL") { ++p_; return lit("null", ""); }
        if (k == "TRUE" || k == "FALSE") { ++p_; return lit("bool", k == "TRUE" ? "true" : "false"); }
        if (k == "DATE" && peek(1).kind == Token::String) { ++p_; return lit("date", next().text); }
        if (k == "TIMESTAMP" && peek(1).kind == Token::String) { ++p_; return lit("timestamp", next().text); }
        if (k == "INTERVAL") {
          ++p_;
          std::string v;
          if (peek().kind == Token::String) v = next().text;
          else if (peek().kind == Token::Number) v = next().text;
          else fail("expected interval value");
          auto n = lit("interval", v);
          // optional unit after the quoted value: interval '3' month
          if (peek().kind == Token::Ident) {
            std::string u = peek().text;
            static const std::set<std::string> units = {
                "year", "years", "month", "months", "day", "days", "week", "weeks",
                "hour", "hours", "minute", "minutes", "second", "seconds"};
            if (units.count(u)) {
              ++p_;
              n->flags["unit"] = u;
              // TPC-H spelling: interval '90' day (3)
              if (isOp("(") && peek(1).kind == Token::Number && isOp(")", 2)) p_ += 3;
            }
          }
          return n;
        }
        if (k == "CASE") return caseExpr();
        if (k == "CAST") {
          ++p_;
          expectOp("(");
          auto c = make("cast");
          c->kids.push_back(expr());
          expectKw("AS");
          c->flags["type"] = typeName();
          expectOp(")");
          return c;
        }
        if (k == "EXTRACT") {
          ++p_;
          expectOp("(");
          auto e = make("extract");
          std::string field = peek().kind == Token::String ? next().text : (peek().kind == Token::Keyword ? next().text : ident());
          e->str = lower(field);
          expectKw("FROM");
          e->kids.push_back(expr());
          expectOp(")");
          return e;
        }
        if (k == "SUBSTRING") {
          ++p_;
          expectOp("(");
          auto s = make("func", "substr");
          s->kids.push_back(expr());
          if (acceptKw("FROM") || acceptOp(",")) {
            s->kids.push_back(expr());
            if (acceptWord("for") || acceptOp(",")) s->kids.push_back(expr());
          }
          expectOp(")");
          return s;
        }
        if (k == "EXISTS" || (k == "NOT" && isKw("EXISTS", 1))) {
          bool neg = k == "NOT";
          if (neg) ++p_;
          ++p_;
          expectOp("(");
          auto e = make("exists");
          if (neg) e->flags["neg"] = "1";
          e->attrs["query"] = query();
          expectOp(")");
          return e;
        }
        if (k == "LEFT" || k == "RIGHT") {  // string functions left(s, n) / right(s, n)
          if (isOp("(", 1)) {
            ++p_;
            return funcCall(lower(k));
          }
        }
        if (k == "FIRST" || k == "LAST") {
          ++p_;
          return colRef(lower(k));
        }
        fail("unexpected keyword");
      }
      case Token::Ident:
      case Token::QuotedIdent: {
        std::string name = next().text;
        if (name == "array" && t.kind == Token::Ident && isOp("[")) return arrayLiteral();
        if (isOp("(") && t.kind == Token::Ident) {
          if (name == "trim") return trimCall();
          if (name == "position") {  // POSITION(needle IN haystack) -> strpos(haystack, needle)
            ++p_;
            NodeP needle = additive();
            expectKw("IN");
            NodeP hay = expr();
            expectOp(")");
            auto f = make("func", "strpos");
            f->kids = {hay, needle};
            return f;
          }
          return funcCall(name);
        }
        return colRef(name);
      }
      default:
        fail("unexpected end of input");
    }
  }

  NodeP colRef(const std::string& first) {
    auto c = make("col");
    std::vector<NodeP> parts{make("name", first)};
    while (isOp(".") && (peek(1).kind == Token::Ident || peek(1).kind == Token::QuotedIdent)) {
      ++p_;
      parts.push_back(make("name", next().text));
    }
    c->kids = parts;
    c->str = parts.back()->str;
    return c;
  }

  NodeP funcCall(const std::string& name) {
    expectOp("(");
    auto f = make("func", name);
    if (acceptOp("*")) {
      f->flags["star"] = "1";
      expectOp(")");
    } else if (acceptOp(")")) {
      // no args
    } else {
      if (acceptKw("DISTINCT")) f->flags["distinct"] = "1";
      else acceptKw("ALL");
      do f->kids.push_back(expr());
      while (acceptOp(","));
      if (acceptKw("ORDER")) {  // ordered aggregate: array_agg(x ORDER BY y)
        expectKw("BY");
        std::vector<NodeP> os;
        do os.push_back(orderItem());
        while (acceptOp(","));
        f->attrs["order"] = list(os);
      }
      expectOp(")");
    }
    if (acceptWord("within")) {  // ordered-set aggregate: percentile_cont(q) WITHIN GROUP (ORDER BY x)
      expectKw("GROUP");
      expectOp("(");
      expectKw("ORDER");
      expectKw("BY");
      std::vector<NodeP> os;
      do os.push_back(orderItem());
      while (acceptOp(","));
      expectOp(")");
      f->attrs["within_group"] = list(os);
    }
    if (acceptWord("filter")) {
      expectOp("(");
      expectKw("WHERE");
      f->attrs["filter"] = expr();
      expectOp(")");
    }
    if (acceptWord("over")) {
      if (isOp("(")) {
        ++p_;
        f->attrs["over"] = windowSpec();
        expectOp(")");
      } else {
        auto w = make("window", ident());  // named window (WINDOW clause)
        f->attrs["over"] = w;
      }
    }
    return f;
  }

  // ( [base] [PARTITION BY ...] [ORDER BY ...] [frame] ) -- body without parens
  NodeP windowSpec() {
    auto w = make("window");
    if ((peek().kind == Token::Ident || peek().kind == Token::QuotedIdent) && !isWord("partition") &&
        !isWord("rows") && !isWord("range") && !isWord("groups"))
      w->str = ident();  // OVER (w ORDER BY ...) refines a named window
    if (acceptWord("partition")) {
      expectKw("BY");
      std::vector<NodeP> ps;
      do ps.push_back(expr());
      while (acceptOp(","));
      w->attrs["partition"] = list(ps);
    }
    if (acceptKw("ORDER")) {
      expectKw("BY");
      std::vector<NodeP> os;
      do os.push_back(orderItem());
      while (acceptOp(","));
      w->attrs["order"] = list(os);
    }
    std::string unit;
    if (acceptWord("rows")) unit = "rows";
    else if (acceptWord("range")) unit = "range";
    else if (acceptWord("groups")) unit = "groups";
    if (!unit.empty()) {
      auto fr = make("frame", unit);
      if (acceptKw("BETWEEN")) {
        fr->kids.push_back(frameBound());
        expectKw("AND");
        fr->kids.push_back(frameBound());
      } else {
        fr->kids.push_back(frameBound());
        fr->kids.push_back(make("bound", "current"));
      }
      if (acceptWord("exclude")) {
        if (acceptWord("no")) expectWord("others");
        else fail("only EXCLUDE NO OTHERS is supported");
      }
      w->attrs["frame"] = fr;
    }
    return w;
  }

  NodeP frameBound() {
    if (acceptWord("unbounded")) {
      if (acceptWord("preceding")) return make("bound", "unbounded_preceding");
      expectWord("following");
      return make("bound", "unbounded_following");
    }
    if (acceptWord("current")) {
      expectWord("row");
      return make("bound", "current");
    }
    NodeP off = additive();
    NodeP b;
    if (acceptWord("preceding")) b = make("bound", "preceding");
    else { expectWord("following"); b = make("bound", "following"); }
    b->kids.push_back(off);
    return b;
  }

  // TRIM([LEADING|TRAILING|BOTH] [chars] FROM s) / trim(s [, chars])
  NodeP trimCall() {
    expectOp("(");
    std::string fn = "btrim";
    if (acceptWord("leading")) fn = "ltrim";
    else if (acceptWord("trailing")) fn = "rtrim";
    else acceptWord("both");
    auto f = make("func", fn);
    if (acceptKw("FROM")) {
      f->kids.push_back(expr());
    } else {
      NodeP first = expr();
      if (acceptKw("FROM")) {
        f->kids = {expr(), first};
      } else if (acceptOp(",")) {
        f->kids = {first, expr()};
      } else {
        f->kids = {first};
      }
    }
    expectOp(")");
    return f;
  }

  NodeP caseExpr() {
    expectKw("CASE");
    auto c = make("case");
    if (!isKw("WHEN")) c->attrs["operand"] = expr();
    while (acceptKw("WHEN")) {
      NodeP w = expr();
      expectKw("THEN");
      NodeP th = expr();
      c->kids.push_back(w);
      c->kids.push_back(th);
    }
    if (c->kids.empty()) fail("CASE requires at least one WHEN");
    if (acceptKw("ELSE")) c->attrs["else"] = expr();
    expectKw("END");
    return c;
  }
};

}  // namespace

std::vector<NodeP> parse_sql(const std::string& text) {
  Parser p(text);
  return p.statements();
}

}  // namespace sql
}  // namespace igloo
