// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the reference's condition machinery for validate rules:
//   * JMESPath subset of github.com/kyverno/go-jmespath v0.4.1-0.20231124160150-95e59c162877
//     (go.mod:33; third-party, absent here): fields, quoted fields, sub-expressions, index,
//     flatten `[]`, list / value projections `[*]` `.*`, filters `[?a == b]`, multi-select
//     lists, `||` `&&` `!` `|`, comparators, `@`, raw-string and JSON literals, and the
//     functions keys / length / contains / to_string / starts_with / ends_with / values.
//     Upstream JMESPath semantics (a missing field is null, projections drop nulls) plus the
//     fork's NotFoundError ("Unknown key \"k\" in path", pinned by
//     pkg/engine/validation_test.go:1997-2054 and pkg/engine/context/deferred_test.go:68-80).
//     Where the fork raises it is not visible here: this restatement raises it only for an
//     expression that is a plain chain of field / index accesses (the form every pinning
//     test uses) and `||` catches it on its left (the documented default-value idiom the
//     chart policies rely on). Other placements are PARITY UNPINNED.
//   * variable substitution in condition keys / values: pkg/engine/variables/vars.go
//     substituteVariablesIfAny :311-389, substituteVarInPattern :403-420,
//     replaceBracesAndTrimSpaces :422-427; context.Query pkg/engine/context/evaluate.go:11-32
//   * conditions: variables/evaluate.go:14-125 (Evaluate, evaluateAnyAllConditions,
//     evaluateOldConditions); operators variables/operator/{equal,notequal,anyin,anynotin,
//     allin,allnotin,in,notin}.go and operator.go parseDuration :79-138
//   * handlers: preconditions (engine.go:278-286, validate_resource.go:121-135), deny
//     (validate_resource.go:268-279), foreach (:186-254, utils/foreach.go:12-63)
// Background / CLI context: request.operation = "CREATE", request.object = the resource.
#pragma once
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "image.hpp"
#include "json_dom.hpp"
#include "pattern.hpp"
#include "wildcard.hpp"

namespace oracle {
namespace cond {

struct Unsupported : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct NotFound {  // go-jmespath fork NotFoundError
  std::string key;
};
struct EvalError {  // any other evaluation / substitution error => rule ERROR
  std::string msg;
  bool restated = false;  // msg is the reference's error text (else a description only)
};

// ---- values -------------------------------------------------------------------------
// The context is JSON: numbers are float64 (encoding/json). Null is a null JPtr.
inline JPtr mk_null() { return nullptr; }
inline JPtr mk_str(const std::string& s) {
  auto v = std::make_shared<JVal>();
  v->t = JT::Str;
  v->s = s;
  return v;
}
inline JPtr mk_num(double f) {
  auto v = std::make_shared<JVal>();
  v->t = JT::Float;
  v->f = f;
  return v;
}
inline JPtr mk_bool(bool b) {
  auto v = std::make_shared<JVal>();
  v->t = JT::Bool;
  v->b = b;
  return v;
}
inline JPtr mk_arr(std::vector<JPtr> a) {
  auto v = std::make_shared<JVal>();
  v->t = JT::Arr;
  v->a = std::move(a);
  return v;
}
inline bool is_null(const JPtr& v) { return !v || v->t == JT::Null; }
// resource / policy JSON -> context JSON (whole numbers become float64)
inline JPtr to_ctx(const JVal& v) {
  auto o = std::make_shared<JVal>(v);
  if (o->t == JT::Int) o->t = JT::Float, o->f = (double)o->i;
  for (auto& e : o->a) e = e ? to_ctx(*e) : nullptr;
  for (auto& kv : o->o) kv.second = kv.second ? to_ctx(*kv.second) : nullptr;
  return o;
}
inline bool is_false(const JPtr& v) {  // JMESPath false-like values
  if (is_null(v)) return true;
  switch (v->t) {
    case JT::Bool: return !v->b;
    case JT::Str: return v->s.empty();
    case JT::Arr: return v->a.empty();
    case JT::Obj: return v->o.empty();
    default: return false;
  }
}
inline bool deep_equal(const JPtr& x, const JPtr& y) {  // reflect.DeepEqual on JSON values
  if (is_null(x) || is_null(y)) return is_null(x) && is_null(y);
  if (x->t != y->t) return false;
  switch (x->t) {
    case JT::Bool: return x->b == y->b;
    case JT::Float: return x->f == y->f;
    case JT::Str: return x->s == y->s;
    case JT::Arr:
      if (x->a.size() != y->a.size()) return false;
      for (size_t i = 0; i < x->a.size(); ++i)
        if (!deep_equal(x->a[i], y->a[i])) return false;
      return true;
    case JT::Obj: {
      if (x->o.size() != y->o.size()) return false;
      for (auto& kv : x->o) {
        const JVal* o = y->get(kv.first.c_str());
        bool found = false;
        for (auto& kv2 : y->o)
          if (kv2.first == kv.first) {
            found = true;
            if (!deep_equal(kv.second, kv2.second)) return false;
          }
        (void)o;
        if (!found) return false;
      }
      return true;
    }
    default: return false;
  }
}

// fmt.Sprint(float64): the %v verb is strconv.AppendFloat(v, 'g', -1, 64) (fmt/print.go
// fmtFloat), whose shortest form switches to %e when exp < -4 || exp >= 6 (strconv/ftoa.go:
// "if precision was the shortest possible, use precision 6 for this decision"): 1e+06, 123456.
inline void shortest_digits(double v, std::string* d, int* dp) {
  // go_format_E: "d.dddE+XX" shortest round-trip digits
  std::string e = pat::go_format_E(v);
  size_t E = e.find('E');
  std::string m = e.substr(0, E);
  int ex = atoi(e.c_str() + E + 1);
  d->clear();
  for (char c : m)
    if (c >= '0' && c <= '9') *d += c;
  *dp = ex + 1;
}
inline std::string go_sprint_float(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return std::signbit(v) ? "-0" : "0";
  std::string sign = v < 0 ? "-" : "";
  std::string d;
  int dp;
  shortest_digits(std::fabs(v), &d, &dp);
  const int nd = (int)d.size(), exp = dp - 1;
  if (exp < -4 || exp >= 6) {
    std::string o = sign + d.substr(0, 1);
    if (nd > 1) o += "." + d.substr(1);
    char buf[16];
    snprintf(buf, sizeof buf, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    return o + buf;
  }
  if (dp <= 0) return sign + "0." + std::string(-dp, '0') + d;
  if (dp >= nd) return sign + d + std::string(dp - nd, '0');
  return sign + d.substr(0, dp) + "." + d.substr(dp);
}
// fmt.Sprint of a JSON value (%v): maps print as map[k:v ...] with sorted keys.
inline std::string go_sprint(const JPtr& v) {
  if (is_null(v)) return "<nil>";
  switch (v->t) {
    case JT::Bool: return v->b ? "true" : "false";
    case JT::Float: return go_sprint_float(v->f);
    case JT::Int: return std::to_string(v->i);
    case JT::Str: return v->s;
    case JT::Arr: {
      std::string o = "[";
      for (size_t i = 0; i < v->a.size(); ++i) o += (i ? " " : "") + go_sprint(v->a[i]);
      return o + "]";
    }
    case JT::Obj: {
      std::map<std::string, std::string> m;
      for (auto& kv : v->o) m[kv.first] = go_sprint(kv.second);
      std::string o = "map[";
      bool first = true;
      for (auto& kv : m) o += (first ? "" : " ") + kv.first + ":" + kv.second, first = false;
      return o + "]";
    }
    default: return "<nil>";
  }
}
// encoding/json Marshal (compact; float64 'f' in [1e-6, 1e21) else 'e'; HTML-escaped < > &)
inline std::string json_quote(const std::string& s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '<': o += "\\u003c"; break;
      case '>': o += "\\u003e"; break;
      case '&': o += "\\u0026"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
    }
  }
  return o + "\"";
}
inline std::string json_float(double f) {
  const double a = std::fabs(f);
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    std::string d;
    int dp;
    shortest_digits(a, &d, &dp);
    const int exp = dp - 1;
    std::string o = (f < 0 ? "-" : "") + d.substr(0, 1);
    if (d.size() > 1) o += "." + d.substr(1);
    char buf[16];
    snprintf(buf, sizeof buf, "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    return o + buf;
  }
  if (f == 0) return "0";
  std::string d;
  int dp;
  shortest_digits(a, &d, &dp);
  const int nd = (int)d.size();
  std::string o = f < 0 ? "-" : "";
  if (dp <= 0) return o + "0." + std::string(-dp, '0') + d;
  if (dp >= nd) return o + d + std::string(dp - nd, '0');
  return o + d.substr(0, dp) + "." + d.substr(dp);
}
inline std::string json_marshal(const JPtr& v) {
  if (is_null(v)) return "null";
  switch (v->t) {
    case JT::Bool: return v->b ? "true" : "false";
    case JT::Float: return json_float(v->f);
    case JT::Int: return std::to_string(v->i);
    case JT::Str: return json_quote(v->s);
    case JT::Arr: {
      std::string o = "[";
      for (size_t i = 0; i < v->a.size(); ++i) o += (i ? "," : "") + json_marshal(v->a[i]);
      return o + "]";
    }
    case JT::Obj: {  // Go marshals map[string]interface{} with sorted keys
      std::map<std::string, std::string> m;
      for (auto& kv : v->o) m[kv.first] = json_marshal(kv.second);
      std::string o = "{";
      bool first = true;
      for (auto& kv : m) o += (first ? "" : ",") + json_quote(kv.first) + ":" + kv.second, first = false;
      return o + "}";
    }
    default: return "null";
  }
}

// ---- JMESPath subset ----------------------------------------------------------------------
enum Tok {
  T_EOF, T_ID, T_QID, T_NUM, T_DOT, T_STAR, T_FLAT, T_FILTER, T_LBRACK, T_RBRACK, T_COMMA, T_COLON,
  T_LPAREN, T_RPAREN, T_LBRACE, T_RBRACE, T_CUR, T_OR, T_AND, T_PIPE, T_NOT, T_EQ, T_NE, T_LT, T_LE,
  T_GT, T_GE, T_LIT, T_RAW, T_EXPREF
};
struct Token {
  Tok t;
  std::string s;
  long n = 0;
  JPtr lit;
};
inline std::vector<Token> lex(const std::string& q) {
  std::vector<Token> out;
  size_t i = 0;
  auto err = [&](const char* m) { throw EvalError{std::string("incorrect query ") + q + ": " + m}; };
  while (i < q.size()) {
    char c = q[i];
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
      ++i;
      continue;
    }
    if (isalpha((unsigned char)c) || c == '_') {
      size_t j = i;
      while (j < q.size() && (isalnum((unsigned char)q[j]) || q[j] == '_')) ++j;
      out.push_back({T_ID, q.substr(i, j - i)});
      i = j;
      continue;
    }
    if (isdigit((unsigned char)c) || (c == '-' && i + 1 < q.size() && isdigit((unsigned char)q[i + 1]))) {
      size_t j = i + 1;
      while (j < q.size() && isdigit((unsigned char)q[j])) ++j;
      Token t{T_NUM, q.substr(i, j - i)};
      t.n = atol(t.s.c_str());
      out.push_back(t);
      i = j;
      continue;
    }
    if (c == '"') {  // quoted identifier: a JSON string
      size_t j = i + 1;
      while (j < q.size() && q[j] != '"') j += q[j] == '\\' ? 2 : 1;
      if (j >= q.size()) err("unclosed quoted identifier");
      JPtr s = parse_json(q.substr(i, j + 1 - i));
      out.push_back({T_QID, s->s});
      i = j + 1;
      continue;
    }
    if (c == '\'') {  // raw string literal
      std::string s;
      size_t j = i + 1;
      while (j < q.size() && q[j] != '\'') {
        if (q[j] == '\\' && j + 1 < q.size() && q[j + 1] == '\'') {
          s += '\'';
          j += 2;
        } else {
          s += q[j++];
        }
      }
      if (j >= q.size()) err("unclosed raw string");
      Token t{T_RAW, s};
      t.lit = mk_str(s);
      out.push_back(t);
      i = j + 1;
      continue;
    }
    if (c == '`') {  // JSON literal
      std::string s;
      size_t j = i + 1;
      while (j < q.size() && q[j] != '`') {
        if (q[j] == '\\' && j + 1 < q.size() && q[j + 1] == '`') {
          s += '`';
          j += 2;
        } else {
          s += q[j++];
        }
      }
      if (j >= q.size()) err("unclosed JSON literal");
      Token t{T_LIT, s};
      try {
        JParser p(s.data(), s.size());
        t.lit = to_ctx(*p.parse());
        if (!p.at_end()) throw std::runtime_error("trailing");
      } catch (const std::exception&) {
        t.lit = mk_str(s);  // go-jmespath: an invalid JSON literal is a (deprecated) string
      }
      out.push_back(t);
      i = j + 1;
      continue;
    }
    auto two = [&](char a, char b) { return c == a && i + 1 < q.size() && q[i + 1] == b; };
    if (two('[', ']')) { out.push_back({T_FLAT}); i += 2; continue; }
    if (two('[', '?')) { out.push_back({T_FILTER}); i += 2; continue; }
    if (two('|', '|')) { out.push_back({T_OR}); i += 2; continue; }
    if (two('&', '&')) { out.push_back({T_AND}); i += 2; continue; }
    if (two('=', '=')) { out.push_back({T_EQ}); i += 2; continue; }
    if (two('!', '=')) { out.push_back({T_NE}); i += 2; continue; }
    if (two('<', '=')) { out.push_back({T_LE}); i += 2; continue; }
    if (two('>', '=')) { out.push_back({T_GE}); i += 2; continue; }
    switch (c) {
      case '.': out.push_back({T_DOT}); break;
      case '*': out.push_back({T_STAR}); break;
      case '[': out.push_back({T_LBRACK}); break;
      case ']': out.push_back({T_RBRACK}); break;
      case ',': out.push_back({T_COMMA}); break;
      case ':': out.push_back({T_COLON}); break;
      case '(': out.push_back({T_LPAREN}); break;
      case ')': out.push_back({T_RPAREN}); break;
      case '{': out.push_back({T_LBRACE}); break;
      case '}': out.push_back({T_RBRACE}); break;
      case '@': out.push_back({T_CUR}); break;
      case '|': out.push_back({T_PIPE}); break;
      case '!': out.push_back({T_NOT}); break;
      case '<': out.push_back({T_LT}); break;
      case '>': out.push_back({T_GT}); break;
      case '&': out.push_back({T_EXPREF}); break;
      default: err("unknown character");
    }
    ++i;
  }
  out.push_back({T_EOF});
  return out;
}

enum NT { N_FIELD, N_SUB, N_INDEX, N_FLATTEN, N_PROJ, N_VPROJ, N_FILTER, N_MSL, N_OR, N_AND, N_NOT, N_PIPE,
          N_CUR, N_LIT, N_FUNC, N_CMP };
struct Node {
  NT t;
  std::string s;  // field name / function name
  long n = 0;     // index / comparator token
  JPtr lit;
  std::vector<std::shared_ptr<Node>> k;
};
using NPtr = std::shared_ptr<Node>;
inline NPtr nd(NT t, std::vector<NPtr> k = {}) {
  auto n = std::make_shared<Node>();
  n->t = t;
  n->k = std::move(k);
  return n;
}

// go-jmespath parser.go (Pratt parser, binding powers as upstream)
class Parser {
 public:
  explicit Parser(const std::string& q) : q_(q), t_(lex(q)) {}
  NPtr parse() {
    NPtr e = expr(0);
    if (cur().t != T_EOF) fail("unexpected token");
    return e;
  }

 private:
  std::string q_;
  std::vector<Token> t_;
  size_t i_ = 0;
  [[noreturn]] void fail(const char* m) { throw EvalError{"incorrect query " + q_ + ": " + m}; }
  const Token& cur() const { return t_[i_]; }
  const Token& peek(size_t k = 1) const { return t_[std::min(i_ + k, t_.size() - 1)]; }
  void adv() { ++i_; }
  void match(Tok t) {
    if (cur().t != t) fail("unexpected token");
    adv();
  }
  static int bp(Tok t) {
    switch (t) {
      case T_PIPE: return 1;
      case T_OR: return 2;
      case T_AND: return 3;
      case T_EQ: case T_NE: case T_LT: case T_LE: case T_GT: case T_GE: return 5;
      case T_FLAT: return 9;
      case T_STAR: return 20;
      case T_FILTER: return 21;
      case T_DOT: return 40;
      case T_NOT: return 45;
      case T_LBRACE: return 50;
      case T_LBRACK: return 55;
      case T_LPAREN: return 60;
      default: return 0;
    }
  }
  NPtr expr(int rbp) {
    Token tk = cur();
    adv();
    NPtr left = nud(tk);
    while (rbp < bp(cur().t)) {
      Token t2 = cur();
      adv();
      left = led(t2, left);
    }
    return left;
  }
  NPtr field(const std::string& s) {
    NPtr n = nd(N_FIELD);
    n->s = s;
    return n;
  }
  NPtr nud(const Token& tk) {
    switch (tk.t) {
      case T_LIT:
      case T_RAW: {
        NPtr n = nd(N_LIT);
        n->lit = tk.lit;
        return n;
      }
      case T_ID: return field(tk.s);
      case T_QID: {
        if (cur().t == T_LPAREN) fail("quoted identifier cannot be a function name");
        return field(tk.s);
      }
      case T_STAR: {
        NPtr rhs = cur().t == T_EOF ? nd(N_CUR) : proj_rhs(bp(T_STAR));
        return nd(N_VPROJ, {nd(N_CUR), rhs});
      }
      case T_FILTER: return filter(nd(N_CUR));
      case T_FLAT: return nd(N_PROJ, {nd(N_FLATTEN, {nd(N_CUR)}), proj_rhs(bp(T_FLAT))});
      case T_LBRACK: {
        if (cur().t == T_NUM || cur().t == T_COLON) {
          NPtr ix = index_expr();
          return nd(N_INDEX, {nd(N_CUR), ix});
        }
        if (cur().t == T_STAR && peek().t == T_RBRACK) {
          adv();
          adv();
          return nd(N_PROJ, {nd(N_CUR), proj_rhs(bp(T_STAR))});
        }
        return msl();
      }
      case T_CUR: return nd(N_CUR);
      case T_NOT: return nd(N_NOT, {expr(bp(T_NOT))});
      case T_LPAREN: {
        NPtr e = expr(0);
        match(T_RPAREN);
        return e;
      }
      case T_LBRACE: throw Unsupported("JMESPath multi-select hash");
      case T_EXPREF: throw Unsupported("JMESPath expression reference");
      default: fail("unexpected token");
    }
  }
  NPtr index_expr() {  // after '[': a number then ']' (slices unsupported)
    if (cur().t != T_NUM || peek().t != T_RBRACK) throw Unsupported("JMESPath slice");
    NPtr ix = nd(N_LIT);
    ix->n = cur().n;
    adv();
    adv();
    return ix;
  }
  NPtr msl() {  // multi-select list, '[' consumed
    std::vector<NPtr> k;
    for (;;) {
      k.push_back(expr(0));
      if (cur().t == T_RBRACK) break;
      match(T_COMMA);
    }
    match(T_RBRACK);
    return nd(N_MSL, k);
  }
  NPtr filter(NPtr left) {  // '[?' consumed
    NPtr c = expr(0);
    match(T_RBRACK);
    NPtr rhs = cur().t == T_FLAT ? nd(N_CUR) : proj_rhs(bp(T_FILTER));
    return nd(N_FILTER, {left, rhs, c});
  }
  NPtr proj_rhs(int b) {
    if (bp(cur().t) < 10) return nd(N_CUR);
    if (cur().t == T_LBRACK || cur().t == T_FILTER) return expr(b);
    if (cur().t == T_DOT) {
      adv();
      return dot_rhs(b);
    }
    fail("bad projection");
  }
  NPtr dot_rhs(int b) {
    if (cur().t == T_ID || cur().t == T_QID || cur().t == T_STAR) return expr(b);
    if (cur().t == T_LBRACK) {
      adv();
      return msl();
    }
    if (cur().t == T_LBRACE) throw Unsupported("JMESPath multi-select hash");
    fail("bad dot");
  }
  NPtr led(const Token& tk, NPtr left) {
    switch (tk.t) {
      case T_DOT: {
        if (cur().t != T_STAR) return nd(N_SUB, {left, dot_rhs(bp(T_DOT))});
        adv();
        return nd(N_VPROJ, {left, proj_rhs(bp(T_DOT))});
      }
      case T_PIPE: return nd(N_PIPE, {left, expr(bp(T_PIPE))});
      case T_OR: return nd(N_OR, {left, expr(bp(T_OR))});
      case T_AND: return nd(N_AND, {left, expr(bp(T_AND))});
      case T_LPAREN: {
        if (left->t != N_FIELD) fail("bad function call");
        NPtr f = nd(N_FUNC);
        f->s = left->s;
        while (cur().t != T_RPAREN) {
          f->k.push_back(expr(0));
          if (cur().t == T_COMMA) adv();
        }
        match(T_RPAREN);
        static const std::set<std::string> ok = {"keys", "length", "contains", "to_string", "starts_with",
                                                 "ends_with", "values", "not_null"};
        if (!ok.count(f->s)) throw Unsupported("JMESPath function " + f->s);
        return f;
      }
      case T_FILTER: return filter(left);
      case T_FLAT: return nd(N_PROJ, {nd(N_FLATTEN, {left}), proj_rhs(bp(T_FLAT))});
      case T_LBRACK: {
        if (cur().t == T_NUM || cur().t == T_COLON) return nd(N_INDEX, {left, index_expr()});
        match(T_STAR);
        match(T_RBRACK);
        return nd(N_PROJ, {left, proj_rhs(bp(T_STAR))});
      }
      case T_EQ: case T_NE: case T_LT: case T_LE: case T_GT: case T_GE: {
        NPtr n = nd(N_CMP, {left, expr(bp(tk.t))});
        n->n = tk.t;
        return n;
      }
      default: fail("unexpected token");
    }
  }
};

// A plain chain of field / index accesses from the root (where NotFoundError is raised). The
// parser binds an index to the field before it (`a.b[0].c` = SUB(SUB(a, INDEX(b, 0)), c)), so
// the right side of a SUB is a field or an indexed field.
inline bool plain_chain(const Node& n) {
  if (n.t == N_FIELD) return true;
  if (n.t == N_SUB) return plain_chain(*n.k[0]) && plain_chain(*n.k[1]);
  if (n.t == N_INDEX) return plain_chain(*n.k[0]);
  return false;
}

struct Interp {
  bool strict = false;  // raise NotFound on a missing member (plain chains only)
  JPtr eval(const Node& n, const JPtr& v) {
    switch (n.t) {
      case N_CUR: return v;
      case N_LIT: return n.lit;
      case N_FIELD: {
        if (is_null(v) || v->t != JT::Obj) return nullptr;
        for (auto& kv : v->o)
          if (kv.first == n.s) return kv.second;
        if (strict) throw NotFound{n.s};
        return nullptr;
      }
      case N_SUB: return eval(*n.k[1], eval(*n.k[0], v));
      case N_INDEX: {
        JPtr l = eval(*n.k[0], v);
        if (is_null(l) || l->t != JT::Arr) return nullptr;
        long i = n.k[1]->n;
        if (i < 0) i += (long)l->a.size();
        if (i < 0 || i >= (long)l->a.size()) return nullptr;
        return l->a[i];
      }
      case N_FLATTEN: {
        JPtr l = eval(*n.k[0], v);
        if (is_null(l) || l->t != JT::Arr) return nullptr;
        std::vector<JPtr> o;
        for (auto& e : l->a)
          if (!is_null(e) && e->t == JT::Arr) o.insert(o.end(), e->a.begin(), e->a.end());
          else o.push_back(e);
        return mk_arr(o);
      }
      case N_PROJ: {
        JPtr l = eval(*n.k[0], v);
        if (is_null(l) || l->t != JT::Arr) return nullptr;
        std::vector<JPtr> o;
        for (auto& e : l->a) {
          JPtr r = eval(*n.k[1], e);
          if (!is_null(r)) o.push_back(r);
        }
        return mk_arr(o);
      }
      case N_VPROJ: {
        JPtr l = eval(*n.k[0], v);
        if (is_null(l) || l->t != JT::Obj) return nullptr;
        std::vector<JPtr> o;
        for (auto& kv : l->o) {  // Go map order: PARITY UNPINNED beyond set semantics
          JPtr r = eval(*n.k[1], kv.second);
          if (!is_null(r)) o.push_back(r);
        }
        return mk_arr(o);
      }
      case N_FILTER: {
        JPtr l = eval(*n.k[0], v);
        if (is_null(l) || l->t != JT::Arr) return nullptr;
        std::vector<JPtr> o;
        for (auto& e : l->a) {
          if (is_false(eval(*n.k[2], e))) continue;
          JPtr r = eval(*n.k[1], e);
          if (!is_null(r)) o.push_back(r);
        }
        return mk_arr(o);
      }
      case N_MSL: {
        if (is_null(v)) return nullptr;
        std::vector<JPtr> o;
        for (auto& k : n.k) o.push_back(eval(*k, v));
        return mk_arr(o);
      }
      case N_OR: {
        JPtr l;
        try {
          l = eval(*n.k[0], v);
        } catch (const NotFound&) {
          l = nullptr;
        }
        return is_false(l) ? eval(*n.k[1], v) : l;
      }
      case N_AND: {
        JPtr l = eval(*n.k[0], v);
        return is_false(l) ? l : eval(*n.k[1], v);
      }
      case N_NOT: return mk_bool(is_false(eval(*n.k[0], v)));
      case N_PIPE: return eval(*n.k[1], eval(*n.k[0], v));
      case N_CMP: {
        JPtr a = eval(*n.k[0], v), b = eval(*n.k[1], v);
        if (n.n == T_EQ) return mk_bool(deep_equal(a, b));
        if (n.n == T_NE) return mk_bool(!deep_equal(a, b));
        if (is_null(a) || is_null(b) || a->t != JT::Float || b->t != JT::Float) return nullptr;
        switch (n.n) {
          case T_LT: return mk_bool(a->f < b->f);
          case T_LE: return mk_bool(a->f <= b->f);
          case T_GT: return mk_bool(a->f > b->f);
          default: return mk_bool(a->f >= b->f);
        }
      }
      case N_FUNC: return call(n, v);
    }
    return nullptr;
  }
  [[noreturn]] static void type_err(const std::string& f) { throw EvalError{"invalid type for " + f}; }
  JPtr call(const Node& n, const JPtr& v) {
    std::vector<JPtr> a;
    for (auto& k : n.k) a.push_back(eval(*k, v));
    auto argc = [&](size_t c) {
      if (a.size() != c) throw EvalError{"invalid arity for " + n.s};
    };
    if (n.s == "keys" || n.s == "values") {
      argc(1);
      if (is_null(a[0]) || a[0]->t != JT::Obj) type_err(n.s);
      std::vector<JPtr> o;  // Go map iteration order: PARITY UNPINNED beyond set semantics
      for (auto& kv : a[0]->o) o.push_back(n.s == "keys" ? mk_str(kv.first) : kv.second);
      return mk_arr(o);
    }
    if (n.s == "length") {
      argc(1);
      if (is_null(a[0])) type_err(n.s);
      if (a[0]->t == JT::Str) {
        size_t c = 0;  // runes
        for (unsigned char ch : a[0]->s) c += (ch & 0xC0) != 0x80;
        return mk_num((double)c);
      }
      if (a[0]->t == JT::Arr) return mk_num((double)a[0]->a.size());
      if (a[0]->t == JT::Obj) return mk_num((double)a[0]->o.size());
      type_err(n.s);
    }
    if (n.s == "contains") {
      argc(2);
      if (is_null(a[0])) type_err(n.s);
      if (a[0]->t == JT::Arr) {
        for (auto& e : a[0]->a)
          if (deep_equal(e, a[1])) return mk_bool(true);
        return mk_bool(false);
      }
      if (a[0]->t == JT::Str) {
        if (is_null(a[1]) || a[1]->t != JT::Str) type_err(n.s);
        return mk_bool(a[0]->s.find(a[1]->s) != std::string::npos);
      }
      type_err(n.s);
    }
    if (n.s == "starts_with" || n.s == "ends_with") {
      argc(2);
      if (is_null(a[0]) || a[0]->t != JT::Str || is_null(a[1]) || a[1]->t != JT::Str) type_err(n.s);
      const std::string &s = a[0]->s, &p = a[1]->s;
      if (p.size() > s.size()) return mk_bool(false);
      return mk_bool(n.s == "starts_with" ? s.compare(0, p.size(), p) == 0
                                          : s.compare(s.size() - p.size(), p.size(), p) == 0);
    }
    if (n.s == "to_string") {
      argc(1);
      if (!is_null(a[0]) && a[0]->t == JT::Str) return a[0];
      return mk_str(json_marshal(a[0]));
    }
    if (n.s == "not_null") {
      for (auto& x : a)
        if (!is_null(x)) return x;
      return nullptr;
    }
    throw Unsupported("JMESPath function " + n.s);
  }
};

// Names an expression reads from the root of the JSON context. The restated context holds
// request.object, request.operation and the foreach element: anything else (images,
// request.userInfo, serviceAccountName, context entries, ...) is Unsupported.
inline void root_reads(const Node& n, std::vector<std::string>& out) {
  switch (n.t) {
    case N_FIELD: out.push_back(n.s); return;
    case N_SUB:
      if (n.k[0]->t == N_FIELD && n.k[0]->s == "request" && n.k[1]->t == N_FIELD) {
        out.push_back("request." + n.k[1]->s);
        return;
      }
      root_reads(*n.k[0], out);
      return;
    case N_INDEX: case N_FLATTEN: case N_PROJ: case N_VPROJ: case N_FILTER: case N_PIPE:
      root_reads(*n.k[0], out);
      return;
    case N_MSL: case N_OR: case N_AND: case N_CMP: case N_NOT: case N_FUNC:
      for (auto& k : n.k) root_reads(*k, out);
      return;
    case N_CUR: out.push_back("@"); return;
    case N_LIT: return;
  }
}
inline void check_roots(const Node& n) {
  std::vector<std::string> r;
  root_reads(n, r);
  for (auto& x : r)
    if (x != "request.object" && x != "request.operation" && x != "element" && x != "elementIndex" && x != "images" &&
        !(x.size() == 8 && x.compare(0, 7, "element") == 0 && x[7] >= '0' && x[7] <= '3') &&
        !(x.size() == 13 && x.compare(0, 12, "elementIndex") == 0 && x[12] >= '0' && x[12] <= '3'))
      throw Unsupported("context value " + x);
}
struct Query {
  NPtr ast;
  bool strict = false;
};
inline Query compile_query(const std::string& q) {
  Query o;
  std::string s = q;
  while (!s.empty() && isspace((unsigned char)s.back())) s.pop_back();
  size_t b = 0;
  while (b < s.size() && isspace((unsigned char)s[b])) ++b;
  s = s.substr(b);
  if (s.empty()) throw EvalError{"invalid query (nil)"};
  o.ast = Parser(s).parse();
  check_roots(*o.ast);
  o.strict = plain_chain(*o.ast);
  return o;
}
inline JPtr run_query(const Query& q, const JPtr& ctx) {
  Interp in;
  in.strict = q.strict;
  return in.eval(*q.ast, ctx);
}

// ---- variables in condition keys / values --------------------------------------------
// regex.RegexVariables `(^|[^\\])(\{\{(?:\{[^{}]*\}|[^{}])*\}\})`: one match = [start, end)
// of the `{{...}}` text (the preceding character is not part of it).
inline bool next_var(const std::string& s, size_t from, size_t* st, size_t* en) {
  for (size_t i = from; i + 1 < s.size(); ++i) {
    if (s[i] != '{' || s[i + 1] != '{') continue;
    if (i > 0 && s[i - 1] == '\\') continue;
    size_t j = i + 2;
    bool ok = false;
    while (j < s.size()) {
      if (s[j] == '}' && j + 1 < s.size() && s[j + 1] == '}') {
        ok = true;
        break;
      }
      if (s[j] == '{') {  // one nested {...} group without braces inside
        size_t k = j + 1;
        while (k < s.size() && s[k] != '{' && s[k] != '}') ++k;
        if (k >= s.size() || s[k] != '}') break;
        j = k + 1;
        continue;
      }
      if (s[j] == '}') break;
      ++j;
    }
    if (ok) {
      *st = i;
      *en = j + 2;
      return true;
    }
  }
  return false;
}
inline bool has_vars(const JVal& v) {
  if (v.t == JT::Str) {
    size_t a, b;
    return next_var(v.s, 0, &a, &b) || v.s.find("$(") != std::string::npos;
  }
  for (auto& e : v.a)
    if (e && has_vars(*e)) return true;
  for (auto& kv : v.o) {
    size_t a, b;
    if (next_var(kv.first, 0, &a, &b)) return true;
    if (kv.second && has_vars(*kv.second)) return true;
  }
  return false;
}

struct Ctx {
  JPtr root;  // {"request": {"operation", "object"}, "element", "elementIndex"}
};
inline std::string var_text(const std::string& v) {  // replaceBracesAndTrimSpaces
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) {
    if ((v[i] == '{' || v[i] == '}') && i + 1 < v.size() && v[i + 1] == v[i]) {
      ++i;
      continue;
    }
    s += v[i];
  }
  return pat::trim_space(s);
}
// vars.go:311-389 substituteVariablesIfAny over one string leaf at `path` (the JSON-pointer-like
// path jsonutils.traverse.go builds: "" at the root, "/<key>" / "/<index>" below). An error is
// the reference's text: ctx.Query wraps a search error as "JMESPath query failed: %w"
// (context/evaluate.go:27-31), which the type switch of :349-355 does not unwrap, so every
// resolver error is "failed to resolve <variable> at path <path>: <err>".
inline JPtr substitute_string(const std::string& in, const Ctx& c, const std::string& path = "") {
  std::string value = in;
  size_t st, en;
  for (int guard = 0; next_var(value, 0, &st, &en); ++guard) {
    if (guard > 64) throw EvalError{"too many variables"};
    const std::string v = value.substr(st, en - st);
    const std::string var = var_text(v);
    if (var == "@") throw Unsupported("{{@}} variables");
    if (var.find("{{") != std::string::npos) throw Unsupported("nested variables");
    JPtr r;
    const std::string pre = "failed to resolve " + var + " at path " + path + ": ";
    try {
      r = run_query(compile_query(var), c.root);
    } catch (const NotFound& nf) {
      throw EvalError{pre + "JMESPath query failed: Unknown key \"" + nf.key + "\" in path", true};
    } catch (const EvalError& e) {
      // "invalid query (nil)" (evaluate.go:17-19) is the reference's text; a parse or function
      // error would embed go-jmespath's own text, which is not restated
      throw EvalError{pre + e.msg, e.msg == "invalid query (nil)"};
    }
    if (value == v) return r;  // a whole-string variable keeps its JSON type
    const std::string sub = (!is_null(r) && r->t == JT::Str) ? r->s : json_marshal(r);
    value = value.substr(0, st) + sub + value.substr(en);
  }
  // escaped variables `\{{...}}` lose their backslash
  std::string o;
  for (size_t i = 0; i < value.size(); ++i) {
    if (value[i] == '\\' && i + 2 < value.size() && value[i + 1] == '{' && value[i + 2] == '{') continue;
    o += value[i];
  }
  return mk_str(o);
}
inline JPtr substitute(const JPtr& v, const Ctx& c, const std::string& path = "") {
  if (is_null(v)) return v;
  if (v->t == JT::Str) {  // a JSON null result as a node (substituted trees are walked as documents)
    JPtr r = substitute_string(v->s, c, path);
    if (!r) {
      r = std::make_shared<JVal>();
      r->t = JT::Null;
    }
    return r;
  }
  if (v->t == JT::Arr) {
    std::vector<JPtr> o;
    for (size_t i = 0; i < v->a.size(); ++i) o.push_back(substitute(v->a[i], c, path + "/" + std::to_string(i)));
    return mk_arr(o);
  }
  if (v->t == JT::Obj) {
    // jsonutils/traverse.go:90-117 traverseObject: every key goes through the action too
    // (OnlyForLeafsAndKeys, vars.go:311-313); a nil result keeps the key, another non-string
    // result is an error ("expected string after substituting variables in key"), a key that
    // changed is renamed (a rename onto another key of the map depends on Go's map order: not
    // restated)
    auto o = std::make_shared<JVal>();
    o->t = JT::Obj;
    std::set<std::string> seen;
    for (auto& kv : v->o) seen.insert(kv.first);
    for (auto& kv : v->o) {
      JPtr k = substitute_string(kv.first, c, path);  // a key's action sees its map's path
      std::string nk;
      if (is_null(k)) nk = kv.first;
      else if (k->t != JT::Str)
        throw EvalError{"expected string after substituting variables in key \"" + kv.first + "\"", true};
      else nk = k->s;
      if (nk != kv.first && seen.count(nk)) throw Unsupported("a substituted map key equal to another key of the map");
      seen.insert(nk);
      std::string kp;  // traverse.go:107: path + "/" + key with "/" escaped as "\/"
      for (char ch : kv.first) kp += ch == '/' ? std::string("\\/") : std::string(1, ch);
      o->o.push_back({nk, substitute(kv.second, c, path + "/" + kp)});
    }
    return o;
  }
  return v;
}

// ---- operators -------------------------------------------------------------------------
inline bool wmatch(const std::string& p, const std::string& s) { return wildcard_match(p, s); }
// operator.go:79-138 parseDuration; false = error
inline bool parse_duration2(const JPtr& key, const JPtr& value, double* ks, double* vs) {
  int64_t kd = 0, vd = 0;
  bool hk = false, hv = false;
  if (!is_null(key) && key->t == JT::Str && pat::go_parse_duration(key->s, &kd) && key->s != "0") hk = true;
  if (!is_null(value) && value->t == JT::Str && pat::go_parse_duration(value->s, &vd) && value->s != "0") hv = true;
  if (!hk && !hv) return false;
  auto num_dur = [](const JPtr& x, int64_t* d) {
    if (is_null(x) || x->t != JT::Float) return false;
    const double t = std::trunc(x->f);
    if (!(t >= -9.2e18 && t <= 9.2e18)) return false;  // Go conversion out of range: undefined
    *d = (int64_t)((uint64_t)(int64_t)t * 1000000000ull);  // time.Duration(f) * time.Second (wraps)
    return true;
  };
  if (!hk && !num_dur(key, &kd)) return false;
  if (!hv && !num_dur(value, &vd)) return false;
  auto secs = [](int64_t d) { return (double)(d / 1000000000) + (double)(d % 1000000000) / 1e9; };
  *ks = secs(kd);
  *vs = secs(vd);
  return true;
}
// equal.go / notequal.go
inline bool op_equals(const JPtr& key, const JPtr& value, bool negate) {
  if (is_null(key)) return false;
  switch (key->t) {
    case JT::Bool:
      if (is_null(value) || value->t != JT::Bool) return negate;
      return (key->b == value->b) != negate;
    case JT::Float: {
      if (is_null(value)) return negate;
      if (value->t == JT::Float) return (value->f == key->f) != negate;
      if (value->t == JT::Str) {
        double f;
        if (!pat::go_parse_float(value->s, &f)) return negate;
        return (f == key->f) != negate;
      }
      return negate;
    }
    case JT::Str: {
      double kd, vd;
      if (parse_duration2(key, value, &kd, &vd)) return (kd == vd) != negate;
      pat::Qty kq, vq;
      if (pat::go_parse_quantity(key->s, &kq) && !is_null(value) && value->t == JT::Str) {
        if (negate && value->s.empty()) return !wmatch(value->s, key->s);
        if (!pat::go_parse_quantity(value->s, &vq)) return false;
        return (pat::qty_cmp(kq, vq) == 0) != negate;
      }
      if (!is_null(value) && value->t == JT::Str) return wmatch(value->s, key->s) != negate;
      return negate;
    }
    case JT::Obj:
      if (is_null(value) || value->t != JT::Obj) return negate;
      return deep_equal(key, value) != negate;
    case JT::Arr:
      if (is_null(value) || value->t != JT::Arr) return negate;
      return deep_equal(key, value) != negate;
    default: return false;
  }
}
// value string forms of the set operators: InRange patterns are refused at compile time
inline bool json_string_array(const std::string& s, std::vector<std::string>* out, bool* invalid) {
  *invalid = false;
  JPtr v;
  try {
    JParser p(s.data(), s.size());
    v = p.parse();
    if (!p.at_end()) return false;
  } catch (const std::exception&) {
    return false;  // not valid JSON: the string itself
  }
  if (!v || v->t == JT::Null) return true;  // json.Unmarshal("null", &[]string) leaves a nil slice, no error
  if (v->t != JT::Arr) {
    *invalid = true;  // valid JSON but not a string array: Unmarshal error
    return true;
  }
  for (auto& e : v->a) {
    if (!e || e->t == JT::Null) {
      out->push_back("");  // null unmarshals into "" in a []string
      continue;
    }
    if (e->t != JT::Str) {
      *invalid = true;
      return true;
    }
    out->push_back(e->s);
  }
  return true;
}
enum SetOp { S_ANYIN, S_ALLIN, S_ANYNOTIN, S_ALLNOTIN };
// anyin.go / allin.go / anynotin.go / allnotin.go
inline bool op_set(SetOp op, const JPtr& key, const JPtr& value) {
  if (is_null(key)) return false;
  std::vector<std::string> keys;
  bool single = false;
  switch (key->t) {
    case JT::Str: keys = {key->s}, single = true; break;
    case JT::Float:
    case JT::Bool: keys = {go_sprint(key)}, single = true; break;
    case JT::Arr:
      for (auto& e : key->a) keys.push_back(go_sprint(e));
      break;
    default: return false;
  }
  const bool notin = op == S_ANYNOTIN || op == S_ALLNOTIN;
  auto found = [](const std::string& k, const std::vector<std::string>& vs) {
    for (auto& v : vs)
      if (wmatch(k, v) || wmatch(v, k)) return true;
    return false;
  };
  if (is_null(value)) return false;  // invalid type
  std::vector<std::string> vals;
  if (value->t == JT::Arr) {
    for (auto& e : value->a) vals.push_back(go_sprint(e));
  } else if (value->t == JT::Str) {
    const std::string& vs = value->s;
    // anyin.go:103-109 handleRange: pattern.Validate(key string, value) of an InRange value
    auto in_range = [&](const std::string& k, const std::string& pat) {
      JVal kv;
      kv.t = JT::Str, kv.s = k;
      return pat::validate_string_patterns(&kv, pat);
    };
    const bool range = pat::get_operator(vs) == pat::OP_IN_RANGE;
    if (single) {  // anyKeyExistsInArray / allKeyExistsInArray
      if (wmatch(vs, keys[0])) return !notin;
      if (range) return in_range(keys[0], vs) != notin;
      std::vector<std::string> arr;
      bool invalid;
      if (!json_string_array(vs, &arr, &invalid)) arr = {vs};
      else if (invalid) return false;
      bool ex = false;
      for (auto& a : arr)
        if (a == keys[0]) ex = true;
      return ex != notin;
    }
    if (keys.size() == 1 && keys[0] == vs) return !notin;
    if (range) {  // anySetExistsInArray / allSetExistsInArray (anyin.go:146-165, allin.go:133-155)
      std::string nr = vs;
      nr.replace(nr.find('-'), 1, "!-");  // strings.Replace(value, "-", "!-", 1) for AnyNotIn
      int hits = 0;
      for (auto& k : keys) hits += in_range(k, op == S_ANYNOTIN ? nr : vs) ? 1 : 0;
      if (op == S_ANYIN || op == S_ANYNOTIN) return hits > 0;
      if (op == S_ALLIN) return hits == (int)keys.size();
      return hits == 0;
    }
    bool invalid;
    if (!json_string_array(vs, &vals, &invalid)) vals = {vs};
    else if (invalid) return false;
    // string-array value: exact (wildcard) membership as for a list value below
  } else {
    return false;
  }
  if (single && value->t == JT::Arr) {  // a scalar key against a list value
    bool ex = false;
    for (auto& v : vals)
      if (wmatch(v, keys[0]) || wmatch(keys[0], v)) ex = true;
    return ex != notin;
  }
  switch (op) {
    case S_ANYIN:
      for (auto& k : keys)
        if (found(k, vals)) return true;
      return false;
    case S_ANYNOTIN:
      for (auto& k : keys)
        if (!found(k, vals)) return true;
      return false;
    case S_ALLIN:
      for (auto& k : keys)
        if (!found(k, vals)) return false;
      return true;
    default:  // S_ALLNOTIN
      for (auto& k : keys)
        if (found(k, vals)) return false;
      return true;
  }
}

// ---- numeric.go / duration.go (the GreaterThan* / LessThan* / Duration* operators) -------
// github.com/blang/semver/v4 v4.0.0 (go.mod; third-party, absent here) Parse and Compare, as
// numeric.go:158-163 uses them for string keys that are neither durations, quantities nor
// numbers. Restated from the published package: Major.Minor.Patch (decimal, no leading zero,
// ParseUint range), `-` prerelease identifiers (numeric without leading zero, or [0-9A-Za-z-]),
// `+` build identifiers (non-empty [0-9A-Za-z-]); build metadata never takes part in Compare.
struct SemVer {
  uint64_t mmp[3];
  std::vector<std::pair<bool, std::string>> pre;  // (is numeric, text); numeric texts compare by value
  std::vector<uint64_t> pre_num;
};
inline bool semver_uint(const std::string& s, uint64_t* out) {
  if (s.empty()) return false;
  for (char c : s)
    if (c < '0' || c > '9') return false;
  if (s.size() > 1 && s[0] == '0') return false;  // hasLeadingZeroes
  uint64_t x = 0;
  for (char c : s) {
    const uint64_t d = (uint64_t)(c - '0');
    if (x > (UINT64_MAX - d) / 10u) return false;  // strconv.ParseUint range error
    x = x * 10u + d;
  }
  *out = x;
  return true;
}
inline bool semver_alnum(const std::string& s) {
  for (char c : s)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '-')) return false;
  return true;
}
inline std::vector<std::string> split_all(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    size_t b = s.find(sep, a);
    out.push_back(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) return out;
    a = b + 1;
  }
}
inline bool semver_parse(const std::string& s, SemVer* v) {
  if (s.empty()) return false;
  const size_t d1 = s.find('.');
  if (d1 == std::string::npos) return false;
  const size_t d2 = s.find('.', d1 + 1);
  if (d2 == std::string::npos) return false;  // SplitN(s, ".", 3) needs three parts
  if (!semver_uint(s.substr(0, d1), &v->mmp[0]) || !semver_uint(s.substr(d1 + 1, d2 - d1 - 1), &v->mmp[1]))
    return false;
  std::string patch = s.substr(d2 + 1);
  std::vector<std::string> build, pre;
  const size_t bi = patch.find('+');
  if (bi != std::string::npos) {
    build = split_all(patch.substr(bi + 1), '.');
    patch = patch.substr(0, bi);
  }
  const size_t pi = patch.find('-');
  if (pi != std::string::npos) {
    pre = split_all(patch.substr(pi + 1), '.');
    patch = patch.substr(0, pi);
  }
  if (!semver_uint(patch, &v->mmp[2])) return false;
  v->pre.clear(), v->pre_num.clear();
  for (auto& p : pre) {  // NewPRVersion
    if (p.empty()) return false;
    bool digits = true;
    for (char c : p) digits = digits && c >= '0' && c <= '9';
    uint64_t n = 0;
    if (digits) {
      if (!semver_uint(p, &n)) return false;
    } else if (!semver_alnum(p)) {
      return false;
    }
    v->pre.push_back({digits, p});
    v->pre_num.push_back(n);
  }
  for (auto& b : build)
    if (b.empty() || !semver_alnum(b)) return false;
  return true;
}
inline int semver_cmp(const SemVer& a, const SemVer& b) {
  for (int i = 0; i < 3; ++i)
    if (a.mmp[i] != b.mmp[i]) return a.mmp[i] > b.mmp[i] ? 1 : -1;
  if (a.pre.empty() && b.pre.empty()) return 0;
  if (a.pre.empty()) return 1;
  if (b.pre.empty()) return -1;
  size_t i = 0;
  for (; i < a.pre.size() && i < b.pre.size(); ++i) {
    const bool an = a.pre[i].first, bn = b.pre[i].first;
    int c;
    if (an && !bn) c = -1;
    else if (!an && bn) c = 1;
    else if (an) c = a.pre_num[i] == b.pre_num[i] ? 0 : (a.pre_num[i] > b.pre_num[i] ? 1 : -1);
    else c = a.pre[i].second == b.pre[i].second ? 0 : (a.pre[i].second > b.pre[i].second ? 1 : -1);
    if (c) return c;
  }
  if (i == a.pre.size() && i == b.pre.size()) return 0;
  return i == a.pre.size() ? -1 : 1;
}
// compareByCondition (numeric.go:32-45) over a three-way result or two floats: `op` is the
// operator as written; only the canonical spelling matches (a differently-cased one reaches the
// handler through CreateOperatorHandler's lower-casing but falls to compareByCondition's default)
enum NumOp { N_GE, N_GT, N_LE, N_LT, N_NONE };
inline bool cmp_by(NumOp op, double k, double v) {
  switch (op) {
    case N_GE: return k >= v;
    case N_GT: return k > v;
    case N_LE: return k <= v;
    case N_LT: return k < v;
    default: return false;
  }
}
inline bool op_numeric_float(NumOp op, double key, const JPtr& value) {  // validateValueWithFloatPattern
  if (is_null(value)) return false;
  if (value->t == JT::Float) return cmp_by(op, key, value->f);
  if (value->t != JT::Str) return false;
  double kd, vd;
  if (parse_duration2(mk_num(key), value, &kd, &vd)) return cmp_by(op, kd, vd);
  double f;
  if (pat::go_parse_float(value->s, &f)) return cmp_by(op, key, f);
  return false;  // strconv.ParseInt cannot succeed where ParseFloat failed
}
inline bool op_numeric(NumOp op, const JPtr& key, const JPtr& value) {  // NumericOperatorHandler.Evaluate
  if (is_null(key)) return false;
  if (key->t == JT::Float) return op_numeric_float(op, key->f, value);
  if (key->t != JT::Str) return false;
  double kd, vd;  // validateValueWithStringPattern: duration, quantity, float, int, semver
  if (parse_duration2(key, value, &kd, &vd)) return cmp_by(op, kd, vd);
  pat::Qty kq, vq;
  if (pat::go_parse_quantity(key->s, &kq) && !is_null(value) && value->t == JT::Str &&
      pat::go_parse_quantity(value->s, &vq))
    return cmp_by(op, (double)pat::qty_cmp(kq, vq), 0.0);
  double f;
  if (pat::go_parse_float(key->s, &f)) return op_numeric_float(op, f, value);
  SemVer ks, vs;
  if (semver_parse(key->s, &ks)) {
    if (is_null(value) || value->t != JT::Str || !semver_parse(value->s, &vs)) return false;
    return cmp_by(op, (double)semver_cmp(ks, vs), 0.0);
  }
  return false;
}
// duration.go: time.Duration(number) * time.Second (float64 -> int64 truncation, wrapping
// multiplication) or time.ParseDuration of a string; int64 compares
inline bool dur_of(const JPtr& x, bool strings, int64_t* d) {
  if (is_null(x)) return false;
  if (x->t == JT::Float) {
    const double t = std::trunc(x->f);
    if (!(t >= -9.2e18 && t <= 9.2e18)) return false;  // Go conversion out of range: undefined
    *d = (int64_t)((uint64_t)(int64_t)t * 1000000000ull);
    return true;
  }
  return strings && x->t == JT::Str && pat::go_parse_duration(x->s, d);
}
inline bool op_duration(NumOp op, const JPtr& key, const JPtr& value) {  // DurationOperatorHandler
  int64_t kd, vd;
  if (is_null(key) || (key->t != JT::Float && key->t != JT::Str)) return false;
  if (!dur_of(key, true, &kd)) return false;  // a string key that is no duration: false
  if (!dur_of(value, true, &vd)) return false;
  switch (op) {
    case N_GE: return kd >= vd;
    case N_GT: return kd > vd;
    case N_LE: return kd <= vd;
    case N_LT: return kd < vd;
    default: return false;
  }
}

enum OpKind { O_EQ, O_NE, O_ANYIN, O_ALLIN, O_ANYNOTIN, O_ALLNOTIN, O_IN, O_NOTIN, O_NUM, O_DUR, O_BAD };
// CreateOperatorHandler (operator.go:27-67): dispatch on the lower-cased name; *num receives the
// compareByCondition operator (N_NONE when the spelling is not the canonical one)
inline OpKind parse_op(const std::string& o, NumOp* num = nullptr) {
  std::string l;
  for (char c : o) l += (char)tolower((unsigned char)c);
  if (l == "equal" || l == "equals") return O_EQ;
  if (l == "notequal" || l == "notequals") return O_NE;
  if (l == "anyin") return O_ANYIN;
  if (l == "allin") return O_ALLIN;
  if (l == "anynotin") return O_ANYNOTIN;
  if (l == "allnotin") return O_ALLNOTIN;
  if (l == "in") return O_IN;
  if (l == "notin") return O_NOTIN;
  static const char* const nums[4] = {"GreaterThanOrEquals", "GreaterThan", "LessThanOrEquals", "LessThan"};
  for (int d = 0; d < 2; ++d)
    for (int i = 0; i < 4; ++i) {
      const std::string canon = std::string(d ? "Duration" : "") + nums[i];
      std::string lc;
      for (char c : canon) lc += (char)tolower((unsigned char)c);
      if (l == lc) {
        if (num) *num = o == canon ? (NumOp)i : N_NONE;
        return d ? O_DUR : O_NUM;
      }
    }
  return O_BAD;  // no handler: "failed to create handler for condition operator" (evaluate.go:23-25)
}
// in.go / notin.go (deprecated): key in value list / string
inline bool op_in(const JPtr& key, const JPtr& value, bool notin) {
  if (is_null(key)) return false;
  // keyExistsInArray (in.go:60-92): 1 in, 0 not in, -1 invalid type (both operators false)
  auto key_in = [&](const std::string& k) -> int {
    if (is_null(value)) return -1;
    if (value->t == JT::Arr) {
      for (auto& e : value->a) {
        const std::string s = go_sprint(e);
        if (wmatch(s, k) || wmatch(k, s)) return 1;
      }
      return 0;
    }
    if (value->t == JT::Str) {
      if (wmatch(value->s, k)) return 1;
      std::vector<std::string> arr;
      bool invalid;
      // json.Unmarshal straight away (no json.Valid fallback as in anyin.go): text that is not
      // JSON is an Unmarshal error
      if (!json_string_array(value->s, &arr, &invalid) || invalid) return -1;
      for (auto& a : arr)
        if (a == k) return 1;
      return 0;
    }
    return -1;
  };
  switch (key->t) {
    case JT::Str:
    case JT::Float:
    case JT::Bool: {
      int r = key_in(key->t == JT::Str ? key->s : go_sprint(key));
      if (r < 0) return false;
      return (r == 1) != notin;
    }
    case JT::Arr: {
      // in.go:35-40: every key element is asserted to be a string (the reference panics
      // otherwise; restated as an evaluation error, PARITY UNPINNED)
      std::vector<std::string> keys;
      for (auto& e : key->a) {
        if (is_null(e) || e->t != JT::Str) throw EvalError{"In/NotIn key list element is not a string"};
        keys.push_back(e->s);
      }
      if (is_null(value)) return false;
      std::vector<std::string> vals;
      if (value->t == JT::Arr) {  // setExistsInArray (in.go:108-123): string elements only
        for (auto& e : value->a) {
          if (is_null(e) || e->t != JT::Str) return false;
          vals.push_back(e->s);
        }
      } else if (value->t == JT::Str) {
        // in.go:126-128: a one-element key equal to the value reports keyExists for both
        // operators, so NotIn is true there as well
        if (keys.size() == 1 && keys[0] == value->s) return true;
        bool invalid;
        if (!json_string_array(value->s, &vals, &invalid) || invalid) return false;
      } else {
        return false;
      }
      // isIn: every key is in the value set; isNotIn: some key is not (exact set lookups)
      bool all = true, any_missing = false;
      for (auto& k : keys) {
        bool f = false;
        for (auto& v : vals)
          if (v == k) f = true;
        all = all && f;
        any_missing = any_missing || !f;
      }
      return notin ? any_missing : all;
    }
    default: return false;
  }
}
inline bool apply_op(OpKind o, const JPtr& key, const JPtr& value, NumOp num = N_NONE) {
  switch (o) {
    case O_NUM: return op_numeric(num, key, value);
    case O_DUR: return op_duration(num, key, value);
    // evaluate.go:23-25: fmt.Errorf("...: %w", err) with the nil err of the value substitution
    case O_BAD: throw EvalError{"failed to create handler for condition operator: %!w(<nil>)", true};
    case O_EQ: return op_equals(key, value, false);
    case O_NE: return op_equals(key, value, true);
    case O_ANYIN: return op_set(S_ANYIN, key, value);
    case O_ALLIN: return op_set(S_ALLIN, key, value);
    case O_ANYNOTIN: return op_set(S_ANYNOTIN, key, value);
    case O_ALLNOTIN: return op_set(S_ALLNOTIN, key, value);
    case O_IN: return op_in(key, value, false);
    default: return op_in(key, value, true);
  }
}

// ---- conditions ------------------------------------------------------------------------
struct Condition {
  JPtr key, value;
  OpKind op;
  NumOp num = N_NONE;
  std::string message;  // kyvernov1.Condition.Message
};
struct AnyAll {
  bool has_any = false;
  std::vector<Condition> any, all;
};
struct Conditions {
  bool present = false;
  bool old_list = false;          // []Condition form
  std::vector<Condition> list;    // old form
  std::vector<AnyAll> blocks;     // AnyAllConditions (one block; a list of blocks for foreach deny?)
};
inline Condition parse_condition(const JVal& c) {
  Condition o;
  const JVal* k = c.get("key");
  const JVal* v = c.get("value");
  o.key = k ? to_ctx(*k) : nullptr;
  o.value = v ? to_ctx(*v) : nullptr;
  const JVal* op = c.get("operator");
  o.op = parse_op(op && op->t == JT::Str ? op->s : "", &o.num);
  const JVal* m = c.get("message");
  if (m && m->t == JT::Str) o.message = m->s;
  auto check = [](const JPtr& x) {
    if (x && x->t == JT::Str && x->s.find("$(") != std::string::npos) throw Unsupported("$(...) references");
  };
  check(o.key);
  check(o.value);
  if (o.value && o.value->t == JT::Str && has_vars(*o.value) && o.op >= O_ANYIN && o.op <= O_ALLNOTIN) {
    // a value substituted into a string could take the InRange form at run time; only a
    // whole-string variable (typed result) is accepted
    size_t a, b;
    next_var(o.value->s, 0, &a, &b);
    if (a != 0 || b != o.value->s.size()) throw Unsupported("partial variable in a set-operator value");
  }
  return o;
}
// utils.TransformConditions: a list => old form; a map with any/all => AnyAllConditions
inline Conditions parse_conditions(const JVal* j) {
  Conditions c;
  if (!j || j->is_null()) return c;
  c.present = true;
  if (j->t == JT::Arr) {
    c.old_list = true;
    for (auto& e : j->a) c.list.push_back(parse_condition(*e));
    return c;
  }
  if (j->t != JT::Obj) throw Unsupported("condition block");
  AnyAll b;
  const JVal* any = j->get("any");
  const JVal* all = j->get("all");
  if (any && any->t == JT::Arr) {
    b.has_any = true;
    for (auto& e : any->a) b.any.push_back(parse_condition(*e));
  } else if (any && !any->is_null()) {
    throw Unsupported("any block");
  }
  if (all && all->t == JT::Arr)
    for (auto& e : all->a) b.all.push_back(parse_condition(*e));
  else if (all && !all->is_null())
    throw Unsupported("all block");
  c.blocks.push_back(b);
  return c;
}
// evaluate.go:14-27: substitute key and value, then the operator; throws EvalError
inline bool eval_condition(const Condition& c, const Ctx& x) {
  JPtr k, v;
  try {
    k = substitute(c.key, x);
  } catch (const EvalError& e) {
    throw EvalError{"failed to substitute variables in condition key: " + e.msg, e.restated};
  }
  try {
    v = substitute(c.value, x);
  } catch (const EvalError& e) {
    throw EvalError{"failed to substitute variables in condition value: " + e.msg, e.restated};
  }
  return apply_op(c.op, k, v, c.num);
}
inline bool eval_conditions(const Conditions& c, const Ctx& x) {
  if (c.old_list) {
    for (auto& e : c.list)
      if (!eval_condition(e, x)) return false;
    return true;
  }
  for (auto& b : c.blocks) {
    bool any_ok = true, all_ok = true;
    if (b.has_any) {
      any_ok = false;
      for (auto& e : b.any)
        if (eval_condition(e, x)) {
          any_ok = true;
          break;
        }
    }
    for (auto& e : b.all)
      if (!eval_condition(e, x)) {
        all_ok = false;
        break;
      }
    if (!(any_ok && all_ok)) return false;
  }
  return true;
}

// stringutils.JoinNonEmpty (pkg/utils/strings)
inline std::string join_non_empty(const std::vector<std::string>& v, const std::string& sep) {
  std::string o;
  for (auto& x : v)
    if (!x.empty()) o += (o.empty() ? "" : sep) + x;
  return o;
}
// variables/evaluate.go:31-125 EvaluateConditions with its message: evaluateAnyAllConditions
// (the `any` block's messages up to its first true condition, the `all` block's up to its first
// false one; the true ones joined by "; " when both hold, else the false ones) or
// evaluateOldConditions (the first false condition's message, else the true ones joined by ";")
inline bool eval_conditions_msg(const Conditions& c, const Ctx& x, std::string* msg) {
  msg->clear();
  if (c.old_list) {
    std::vector<std::string> t;
    for (auto& e : c.list) {
      if (!eval_condition(e, x)) {
        *msg = e.message;
        return false;
      }
      t.push_back(e.message);
    }
    *msg = join_non_empty(t, ";");
    return true;
  }
  for (auto& b : c.blocks) {  // one block (utils.TransformConditions)
    bool any_ok = true, all_ok = true;
    std::vector<std::string> t, f;
    if (b.has_any) {
      any_ok = false;
      for (auto& e : b.any) {
        if (eval_condition(e, x)) {
          any_ok = true;
          t.push_back(e.message);
          break;
        }
        f.push_back(e.message);
      }
    }
    for (auto& e : b.all) {
      if (!eval_condition(e, x)) {
        all_ok = false;
        f.push_back(e.message);
        break;
      }
      t.push_back(e.message);
    }
    *msg = join_non_empty(any_ok && all_ok ? t : f, "; ");
    if (!(any_ok && all_ok)) return false;
  }
  return true;
}

// Compile-time check of every variable expression in a condition block: constructs this
// restatement does not cover throw Unsupported (a parse error stays a run-time ERROR).
inline void precompile_value(const JPtr& v) {
  if (is_null(v)) return;
  auto str = [](const std::string& s) {
    size_t st, en, from = 0;
    while (next_var(s, from, &st, &en)) {
      const std::string var = var_text(s.substr(st, en - st));
      if (var == "@") throw Unsupported("{{@}} variables");
      try {
        compile_query(var);
      } catch (const EvalError&) {
      }
      from = en;
    }
  };
  if (v->t == JT::Str) str(v->s);
  for (auto& e : v->a) precompile_value(e);
  for (auto& kv : v->o) {
    str(kv.first);
    precompile_value(kv.second);
  }
}
inline void precompile(const Conditions& c) {
  for (auto& e : c.list) precompile_value(e.key), precompile_value(e.value);
  for (auto& b : c.blocks) {
    for (auto& e : b.any) precompile_value(e.key), precompile_value(e.value);
    for (auto& e : b.all) precompile_value(e.key), precompile_value(e.value);
  }
}
// The background-scan / CLI JSON context: {"request": {"operation": "CREATE", "object": res}}
// and, when the resource has images, "images" (context.go:306-348 AddImageInfos: per container
// type, per container name, the ImageInfo fields with omitempty, and jsonPointer)
inline JPtr request_context(const JVal& res) {
  auto req = std::make_shared<JVal>();
  req->t = JT::Obj;
  req->o.push_back({"operation", mk_str("CREATE")});
  req->o.push_back({"object", to_ctx(res)});
  auto root = std::make_shared<JVal>();
  root->t = JT::Obj;
  root->o.push_back({"request", req});
  std::vector<img::Extracted> ims;
  try {
    ims = img::extract_images(res);
  } catch (const img::ImageError&) {  // the caller treats the resource as not evaluable
  }
  if (!ims.empty()) {
    auto all = std::make_shared<JVal>();
    all->t = JT::Obj;
    std::sort(ims.begin(), ims.end(), [](const img::Extracted& a, const img::Extracted& b) { return a.type < b.type; });
    for (auto& ex : ims) {
      auto per = std::make_shared<JVal>();
      per->t = JT::Obj;
      for (auto& kv : ex.infos) {
        const img::Info& in = kv.second;
        auto o = std::make_shared<JVal>();
        o->t = JT::Obj;
        auto put = [&](const char* k, const std::string& v, bool omitempty) {
          if (!omitempty || !v.empty()) o->o.push_back({k, mk_str(v)});
        };
        put("digest", in.digest, true);
        put("jsonPointer", in.pointer, false);
        put("name", in.name, false);
        put("path", in.path, false);
        put("reference", in.reference, true);
        put("referenceWithTag", in.reference_with_tag, true);
        put("registry", in.registry, true);
        put("tag", in.tag, true);
        per->o.push_back({kv.first, o});
      }
      all->o.push_back({ex.type, per});
    }
    root->o.push_back({"images", all});
  }
  return root;
}
// context.AddElement (context.go:280-290): element, element<nesting>, elementIndex,
// elementIndex<nesting> merged into the context (a nested element replaces `element`)
inline JPtr with_element(const JPtr& root, const JPtr& el, int64_t idx, int nesting = 0) {
  auto o = std::make_shared<JVal>(*root);
  auto put = [&](const std::string& k, const JPtr& v) {
    for (auto& kv : o->o)
      if (kv.first == k) {
        kv.second = v;
        return;
      }
    o->o.push_back({k, v});
  };
  const std::string n = std::to_string(nesting);
  put("element", el);
  put("element" + n, el);
  put("elementIndex", mk_num((double)idx));
  put("elementIndex" + n, mk_num((double)idx));
  return o;
}

}  // namespace cond
}  // namespace oracle
