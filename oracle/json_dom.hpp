// ORACLE — test infrastructure only. Never linked into the product path.
//
// Minimal JSON DOM used by the CPU restatement of the reference engine.
// It models Go's `unstructured.Unstructured` view of a resource
// (k8s.io/apimachinery util/json: whole numbers -> int64, others -> float64),
// which is what the reference engine sees after
// cmd/cli/kubectl-kyverno/resource/resource.go:36-58 (YamlToUnstructured)
// and pkg/utils/kube/unstructured.go:10-17 (BytesToUnstructured).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace oracle {

struct JVal;
using JPtr = std::shared_ptr<JVal>;

enum class JT { Null, Bool, Int, Float, Str, Arr, Obj };

struct JVal {
  JT t = JT::Null;
  bool b = false;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<JPtr> a;
  std::vector<std::pair<std::string, JPtr>> o;  // insertion order kept

  const JVal* get(const char* k) const {
    if (t != JT::Obj) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return kv.second.get();
    return nullptr;
  }
  bool is_null() const { return t == JT::Null; }
};

class JParser {
 public:
  JParser(const char* p, size_t n) : p_(p), e_(p + n) {}
  JPtr parse() {
    ws();
    JPtr v = value();
    ws();
    return v;
  }
  const char* pos() const { return p_; }
  bool at_end() {
    ws();
    return p_ >= e_;
  }

 private:
  const char* p_;
  const char* e_;
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(e_ - p_) >= n && memcmp(p_, s, n) == 0) {
      p_ += n;
      return true;
    }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e_ - p_ < 4) fail("short \\u");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = *p_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    return v;
  }
  std::string str() {
    if (*p_ != '"') fail("expected string");
    ++p_;
    std::string out;
    while (true) {
      if (p_ >= e_) fail("unterminated string");
      char c = *p_++;
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (p_ >= e_) fail("bad escape");
      char x = *p_++;
      switch (x) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  JPtr value() {
    if (p_ >= e_) fail("unexpected end");
    auto v = std::make_shared<JVal>();
    char c = *p_;
    if (c == '{') {
      ++p_;
      v->t = JT::Obj;
      ws();
      if (*p_ == '}') {
        ++p_;
        return v;
      }
      while (true) {
        ws();
        std::string k = str();
        ws();
        if (*p_ != ':') fail("expected :");
        ++p_;
        ws();
        JPtr child = value();
        // duplicate keys: last wins (encoding/json semantics)
        bool replaced = false;
        for (auto& kv : v->o)
          if (kv.first == k) {
            kv.second = child;
            replaced = true;
          }
        if (!replaced) v->o.emplace_back(std::move(k), child);
        ws();
        if (*p_ == ',') {
          ++p_;
          continue;
        }
        if (*p_ == '}') {
          ++p_;
          break;
        }
        fail("expected , or }");
      }
      return v;
    }
    if (c == '[') {
      ++p_;
      v->t = JT::Arr;
      ws();
      if (*p_ == ']') {
        ++p_;
        return v;
      }
      while (true) {
        ws();
        v->a.push_back(value());
        ws();
        if (*p_ == ',') {
          ++p_;
          continue;
        }
        if (*p_ == ']') {
          ++p_;
          break;
        }
        fail("expected , or ]");
      }
      return v;
    }
    if (c == '"') {
      v->t = JT::Str;
      v->s = str();
      return v;
    }
    if (lit("true")) {
      v->t = JT::Bool;
      v->b = true;
      return v;
    }
    if (lit("false")) {
      v->t = JT::Bool;
      v->b = false;
      return v;
    }
    if (lit("null")) return v;
    // number: int64 if it parses as an integer literal, else float64
    const char* s = p_;
    if (*p_ == '-') ++p_;
    bool isint = true;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '+' ||
                       *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') isint = false;
      ++p_;
    }
    if (p_ == s) fail("unexpected character");
    std::string num(s, p_);
    {  // RFC 8259 number grammar (encoding/json's scanner): -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
      size_t i = num[0] == '-' ? 1 : 0;
      auto digits = [&]() {
        size_t k = i;
        while (i < num.size() && num[i] >= '0' && num[i] <= '9') ++i;
        return i - k;
      };
      const size_t lead = i;
      const size_t nd = digits();
      bool ok = nd > 0 && !(nd > 1 && num[lead] == '0');
      if (ok && i < num.size() && num[i] == '.') ++i, ok = digits() > 0;
      if (ok && i < num.size() && (num[i] == 'e' || num[i] == 'E')) {
        ++i;
        if (i < num.size() && (num[i] == '+' || num[i] == '-')) ++i;
        ok = digits() > 0;
      }
      if (!ok || i != num.size()) fail("invalid number");
    }
    if (isint) {
      errno = 0;
      char* end;
      long long x = strtoll(num.c_str(), &end, 10);
      if (errno == 0 && *end == 0) {
        v->t = JT::Int;
        v->i = x;
        return v;
      }
    }
    v->t = JT::Float;
    v->f = strtod(num.c_str(), nullptr);
    return v;
  }
};

inline JPtr parse_json(const std::string& s) {
  JParser p(s.data(), s.size());
  JPtr v = p.parse();
  if (!p.at_end()) throw std::runtime_error("json: trailing data");
  return v;
}

}  // namespace oracle
