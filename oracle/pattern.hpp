// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the reference's pattern / anyPattern validation path
// (SURVEY.md §8a rows V1, V3, V5-V15), pinned by the reference's own tables
// (tests/golden/pattern_*.json, extracted by tests/golden/make_golden.py from
// pkg/engine/{validate,pattern,anchor,wildcards}/*_test.go and test/cli/test/*):
//   - pkg/engine/validate/validate.go:15-261, validate/utils.go:11-69
//   - pkg/engine/anchor/{anchor,handlers,anchormap,error,utils}.go
//   - pkg/engine/pattern/pattern.go:26-323, pkg/engine/operator/operator.go:7-61
//   - pkg/engine/wildcards/wildcards.go:60-162 (ExpandInMetadata)
//   - pkg/engine/handlers/validation/validate_resource.go:316-454 (validatePatterns)
// Third-party arithmetic restated from its published algorithm (not in the container):
//   - Go stdlib time.ParseDuration, strconv.ParseInt/ParseFloat/FormatFloat('E', -1)
//   - k8s.io/apimachinery v0.29.1 resource.ParseQuantity + Quantity.Cmp
// Deliberate, documented simplifications:
//   - anchor-error classification by message text (anchor/error.go:62-73) is applied to the
//     PatternError skip aggregate only; a plain mismatch error whose *resource value* happens
//     to contain "conditional anchor mismatch" is not reclassified;
//   - Go map iteration order (ExpandInMetadata's "first matching key") is taken as the
//     resource's document order.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "json_dom.hpp"
#include "wildcard.hpp"

namespace oracle {
namespace pat {

// ---------------------------------------------------------------------------------------
// Go strconv / time restatements
// ---------------------------------------------------------------------------------------

// strconv.ParseInt(s, 10, 64): optional sign, decimal digits only, range-checked.
inline bool go_parse_int(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (s.empty()) return false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  const uint64_t cutoff = neg ? (1ull << 63) : (1ull << 63) - 1;
  uint64_t v = 0;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;
    const uint64_t d = (uint64_t)(c - '0');
    if (v > (cutoff - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

inline bool ieq_prefix(const std::string& s, size_t at, const char* w, size_t* n) {
  size_t k = 0;
  while (w[k] && at + k < s.size() && std::tolower((unsigned char)s[at + k]) == w[k]) ++k;
  *n = k;
  return true;
}

// strconv.ParseFloat(s, 64): Go float literal syntax (decimal, or hex with a mandatory 'p'
// exponent), "inf"/"infinity"/"nan" case-insensitively; overflow to +-Inf is an error.
inline bool go_parse_float(const std::string& s, double* out) {
  if (s.empty()) return false;
  // special values (strconv/atof.go special())
  {
    size_t i = 0;
    int sign = 1;
    if (s[0] == '+' || s[0] == '-') {
      sign = s[0] == '-' ? -1 : 1;
      i = 1;
    }
    if (i < s.size() && (s[i] == 'i' || s[i] == 'I')) {
      size_t n;
      ieq_prefix(s, i, "infinity", &n);
      if (3 < n && n < 8) n = 3;
      if ((n == 3 || n == 8) && i + n == s.size()) {
        *out = sign * HUGE_VAL;
        return true;
      }
      return false;
    }
    if (i == 0 && (s[0] == 'n' || s[0] == 'N')) {
      size_t n;
      ieq_prefix(s, 0, "nan", &n);
      if (n == 3 && s.size() == 3) {
        *out = NAN;
        return true;
      }
      return false;
    }
  }
  size_t i = 0;
  if (s[i] == '+' || s[i] == '-') ++i;
  bool hex = false;
  if (i + 1 < s.size() && s[i] == '0' && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
    hex = true;
    i += 2;
  }
  bool digits = false, dot = false;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c == '.') {
      if (dot) return false;
      dot = true;
    } else if ((c >= '0' && c <= '9') || (hex && std::isxdigit((unsigned char)c))) {
      digits = true;
    } else {
      break;
    }
  }
  if (!digits) return false;
  if (i < s.size()) {
    const char e = s[i];
    if (!hex && (e == 'e' || e == 'E')) {
    } else if (hex && (e == 'p' || e == 'P')) {
    } else {
      return false;
    }
    ++i;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
    if (i >= s.size()) return false;
    for (; i < s.size(); ++i)
      if (s[i] < '0' || s[i] > '9') return false;
  } else if (hex) {
    return false;  // hex mantissa requires a 'p' exponent
  }
  const double v = strtod(s.c_str(), nullptr);
  if (std::isinf(v)) return false;  // ErrRange
  *out = v;
  return true;
}

// fmt.Sprintf("%f", v) (Go and C agree for finite values: exact, round-half-even)
inline std::string go_fmt_f(double v) {
  char buf[512];
  snprintf(buf, sizeof buf, "%f", v);
  return buf;
}

// strconv.FormatFloat(v, 'E', -1, 64): shortest round-tripping digits, "d.dddE+XX".
inline std::string go_format_E(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  char buf[64];
  int prec = 0;
  for (prec = 0; prec < 17; ++prec) {
    snprintf(buf, sizeof buf, "%.*E", prec, v);
    if (strtod(buf, nullptr) == v) break;
  }
  snprintf(buf, sizeof buf, "%.*E", prec, v);
  // C prints at least two exponent digits, as Go does; only the sign/zero forms differ
  return buf;
}

// time.ParseDuration (Go 1.21): [-+]?([0-9]*(\.[0-9]*)?[a-z]+)+ ; returns nanoseconds
inline bool go_parse_duration(const std::string& in, int64_t* out) {
  std::string s = in;
  uint64_t d = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s = s.substr(1);
  }
  if (s == "0") {
    *out = 0;
    return true;
  }
  if (s.empty()) return false;
  const uint64_t kMax = 1ull << 63;
  size_t p = 0;
  while (p < s.size()) {
    uint64_t v = 0, f = 0;
    double scale = 1;
    const char c0 = s[p];
    if (!(c0 == '.' || (c0 >= '0' && c0 <= '9'))) return false;
    const size_t p0 = p;
    for (; p < s.size() && s[p] >= '0' && s[p] <= '9'; ++p) {  // leadingInt
      if (v > kMax / 10) return false;
      v = v * 10 + (uint64_t)(s[p] - '0');
      if (v > kMax) return false;
    }
    const bool pre = p != p0;
    bool post = false;
    if (p < s.size() && s[p] == '.') {
      ++p;
      const size_t q0 = p;
      bool overflow = false;
      for (; p < s.size() && s[p] >= '0' && s[p] <= '9'; ++p) {  // leadingFraction
        if (overflow) continue;
        if (f > (kMax - 1) / 10) {
          overflow = true;
          continue;
        }
        const uint64_t y = f * 10 + (uint64_t)(s[p] - '0');
        if (y > kMax) {
          overflow = true;
          continue;
        }
        f = y;
        scale *= 10;
      }
      post = p != q0;
    }
    if (!pre && !post) return false;
    size_t u0 = p;
    while (p < s.size() && s[p] != '.' && !(s[p] >= '0' && s[p] <= '9')) ++p;
    if (p == u0) return false;  // missing unit
    const std::string u = s.substr(u0, p - u0);
    uint64_t unit;
    if (u == "ns") unit = 1;
    else if (u == "us" || u == "\xC2\xB5s" || u == "\xCE\xBCs") unit = 1000;
    else if (u == "ms") unit = 1000000;
    else if (u == "s") unit = 1000000000ull;
    else if (u == "m") unit = 60ull * 1000000000ull;
    else if (u == "h") unit = 3600ull * 1000000000ull;
    else return false;
    if (v > kMax / unit) return false;
    v *= unit;
    if (f > 0) {
      v += (uint64_t)((double)f * ((double)unit / scale));
      if (v > kMax) return false;
    }
    d += v;
    if (d > kMax) return false;
  }
  if (neg) {
    *out = (int64_t)(0 - d);
    return true;
  }
  if (d > kMax - 1) return false;
  *out = (int64_t)d;
  return true;
}

// ---------------------------------------------------------------------------------------
// apimachinery resource.Quantity: exact value as sign * M * 10^E (canonical: M has no
// trailing zeros; zero is {false, 0, 0}).
// ---------------------------------------------------------------------------------------
typedef unsigned __int128 u128;

struct Qty {
  bool neg = false;
  u128 m = 0;
  int64_t e = 0;
};

inline void qty_norm(Qty& q) {
  if (q.m == 0) {
    q.neg = false;
    q.e = 0;
    return;
  }
  while (q.m % 10 == 0) {
    q.m /= 10;
    ++q.e;
  }
}
inline int u128_digits(u128 m) {
  int d = 0;
  while (m) {
    m /= 10;
    ++d;
  }
  return d;
}
// -1 / 0 / +1
inline int qty_cmp(const Qty& a, const Qty& b) {
  const int sa = a.m == 0 ? 0 : (a.neg ? -1 : 1), sb = b.m == 0 ? 0 : (b.neg ? -1 : 1);
  if (sa != sb) return sa < sb ? -1 : 1;
  if (sa == 0) return 0;
  // compare magnitudes
  const int64_t oa = u128_digits(a.m) + a.e, ob = u128_digits(b.m) + b.e;
  int mag;
  if (oa != ob) {
    mag = oa < ob ? -1 : 1;
  } else {
    u128 ma = a.m, mb = b.m;
    int da = u128_digits(ma), db = u128_digits(mb);
    while (da < db) ma *= 10, ++da;
    while (db < da) mb *= 10, ++db;
    mag = ma == mb ? 0 : (ma < mb ? -1 : 1);
  }
  return sa > 0 ? mag : -mag;
}

// minimal arbitrary-precision unsigned integer (base 1e9 limbs, little endian) for the
// inf.Dec slow path of ParseQuantity
struct Big {
  std::vector<uint32_t> l;
  bool zero() const {
    for (auto x : l)
      if (x) return false;
    return true;
  }
  void mul_add(uint32_t m, uint32_t a) {
    uint64_t c = a;
    for (auto& x : l) {
      uint64_t t = (uint64_t)x * m + c;
      x = (uint32_t)(t % 1000000000u);
      c = t / 1000000000u;
    }
    while (c) {
      l.push_back((uint32_t)(c % 1000000000u));
      c /= 1000000000u;
    }
  }
  // divide by 10, returns remainder
  uint32_t div10() {
    uint64_t r = 0;
    for (size_t i = l.size(); i-- > 0;) {
      uint64_t cur = l[i] + r * 1000000000ull;
      l[i] = (uint32_t)(cur / 10);
      r = cur % 10;
    }
    while (!l.empty() && l.back() == 0) l.pop_back();
    return (uint32_t)r;
  }
  int digits() const {
    if (l.empty()) return 0;
    int d = 9 * (int)(l.size() - 1);
    uint32_t t = l.back();
    while (t) {
      t /= 10;
      ++d;
    }
    return d;
  }
  bool to_u128(u128* out) const {
    if (digits() > 38) return false;
    u128 v = 0;
    for (size_t i = l.size(); i-- > 0;) v = v * 1000000000u + l[i];
    *out = v;
    return true;
  }
};

// resource.ParseQuantity (apimachinery v0.29.1 quantity.go) -> exact value
inline bool go_parse_quantity(const std::string& str, Qty* out) {
  if (str.empty()) return false;
  Qty q;
  if (str == "0") {
    *out = q;
    return true;
  }
  // parseQuantityString
  bool positive = true;
  size_t pos = 0, end = str.size();
  std::string value, num, denom, suf;
  if (str[0] == '-') positive = false, ++pos;
  else if (str[0] == '+') ++pos;
  bool done = false;
  {
    size_t i = pos;
    for (;; ++i) {
      if (i >= end) {
        num = "0";
        value = num;
        done = true;
        break;
      }
      if (str[i] == '0') ++pos;
      else break;
    }
  }
  if (!done) {
    size_t i = pos;
    for (;; ++i) {
      if (i >= end) {
        num = str.substr(pos, end - pos);
        value = str.substr(0, end);
        done = true;
        break;
      }
      if (str[i] < '0' || str[i] > '9') {
        num = str.substr(pos, i - pos);
        pos = i;
        break;
      }
    }
  }
  if (!done) {
    if (num.empty()) num = "0";
    if (pos < end && str[pos] == '.') {
      ++pos;
      size_t i = pos;
      for (;; ++i) {
        if (i >= end) {
          denom = str.substr(pos, end - pos);
          value = str.substr(0, end);
          done = true;
          break;
        }
        if (str[i] < '0' || str[i] > '9') {
          denom = str.substr(pos, i - pos);
          pos = i;
          break;
        }
      }
    }
  }
  if (!done) {
    value = str.substr(0, pos);
    const size_t suffix_start = pos;
    bool fin = false;
    for (size_t i = pos;; ++i) {
      if (i >= end) {
        suf = str.substr(suffix_start);
        fin = true;
        break;
      }
      if (!strchr("eEinumkKMGTP", str[i])) {
        pos = i;
        break;
      }
    }
    if (!fin) {
      if (pos < end && (str[pos] == '-' || str[pos] == '+')) ++pos;
      for (size_t i = pos;; ++i) {
        if (i >= end) {
          suf = str.substr(suffix_start);
          fin = true;
          break;
        }
        if (str[i] < '0' || str[i] > '9') break;
      }
      if (!fin) return false;  // ErrFormatWrong
    }
  }
  // suffixer.interpret
  int32_t base = 10, exponent = 0;
  int fmt;  // 0 DecimalSI, 1 BinarySI, 2 DecimalExponent
  static const char* dec[] = {"n", "u", "m", "", "k", "M", "G", "T", "P", "E"};
  static const int32_t dexp[] = {-9, -6, -3, 0, 3, 6, 9, 12, 15, 18};
  static const char* bin[] = {"Ki", "Mi", "Gi", "Ti", "Pi", "Ei"};
  bool ok = false;
  for (int k = 0; k < 10 && !ok; ++k)
    if (suf == dec[k]) base = 10, exponent = dexp[k], fmt = 0, ok = true;
  for (int k = 0; k < 6 && !ok; ++k)
    if (suf == bin[k]) base = 2, exponent = 10 * (k + 1), fmt = 1, ok = true;
  if (!ok) {
    if (suf.size() > 1 && (suf[0] == 'E' || suf[0] == 'e')) {
      int64_t parsed;
      if (!go_parse_int(suf.substr(1), &parsed)) return false;
      base = 10, exponent = (int32_t)parsed, fmt = 2, ok = true;
    } else {
      return false;  // ErrSuffix
    }
  }
  // fast path (int64Amount)
  int32_t precision = 0, scale = 0;
  int64_t mantissa = 1;
  if (fmt == 0 || fmt == 2) {
    scale = exponent;
    precision = 18 - (int32_t)(num.size() + denom.size());
  } else {
    scale = 0;
    if (exponent >= 0 && denom.empty()) {
      mantissa = (int64_t)((uint64_t)mantissa << exponent);
      precision = 15 - (int32_t)num.size() - (int32_t)((float)exponent * 3 / 10) - 1;
    } else {
      precision = -1;
    }
  }
  if (precision >= 0) {
    scale -= (int32_t)denom.size();
    if (scale >= -9) {
      int64_t v;
      if (!go_parse_int(num + denom, &v)) return false;  // ErrNumeric
      __int128 r = (__int128)v * mantissa;
      if (r <= INT64_MAX && r >= INT64_MIN) {
        q.neg = !positive;
        q.m = (u128)(r < 0 ? -r : r);
        q.e = scale;
        qty_norm(q);
        *out = q;
        return true;
      }
    }
  }
  // inf.Dec path: exact decimal, * 10^exp or * 2^exp, round up to 1e-9, cap at MaxInt64
  Big b;
  int64_t e10 = 0;
  {
    // digits of `value` (sign, leading zeros and '.' skipped)
    bool seen_dot = false;
    for (char c : value) {
      if (c == '.') {
        seen_dot = true;
        continue;
      }
      if (c < '0' || c > '9') continue;
      b.mul_add(10, (uint32_t)(c - '0'));
      if (seen_dot) --e10;
    }
  }
  if (base == 10) {
    e10 += exponent;
  } else {
    for (int32_t k = 0; k < exponent; ++k) b.mul_add(2, 0);
  }
  if (b.zero()) {
    *out = Qty{};
    return true;
  }
  // value = b * 10^e10 ; Q = ceil(value * 1e9)
  const int64_t sh = e10 + 9;
  u128 Q = 0;
  const u128 cap = (u128)INT64_MAX * 1000000000u;
  if (sh >= 0) {
    if (b.digits() + sh > 29) {
      Q = cap + 1;  // beyond the cap for sure
    } else {
      for (int64_t k = 0; k < sh; ++k) b.mul_add(10, 0);
      b.to_u128(&Q);
    }
  } else {
    if (-sh >= b.digits() + 1) {
      Q = 1;  // nonzero below 1e-9 rounds up to 1n
    } else {
      bool rem = false;
      for (int64_t k = 0; k < -sh; ++k) rem |= b.div10() != 0;
      if (b.digits() > 29) {
        Q = cap + 1;
      } else {
        b.to_u128(&Q);
        if (rem) Q += 1;
      }
    }
  }
  if (Q > cap) Q = cap;
  q.neg = !positive;
  q.m = Q;
  q.e = -9;
  qty_norm(q);
  *out = q;
  return true;
}

// ---------------------------------------------------------------------------------------
// pattern.go leaf validation
// ---------------------------------------------------------------------------------------
enum Op { OP_EQ, OP_GE, OP_LE, OP_NE, OP_GT, OP_LT, OP_IN_RANGE, OP_NOT_IN_RANGE };

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_alpha(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
// one endpoint of operator.go:30-31: [-|\+]?\d+(?:\.\d+)?[A-Za-z]* ; returns end index or npos
inline size_t range_endpoint(const std::string& s, size_t i) {
  if (i < s.size() && (s[i] == '-' || s[i] == '|' || s[i] == '+')) ++i;
  const size_t d0 = i;
  while (i < s.size() && is_digit(s[i])) ++i;
  if (i == d0) return std::string::npos;
  if (i + 1 < s.size() && s[i] == '.' && is_digit(s[i + 1])) {
    ++i;
    while (i < s.size() && is_digit(s[i])) ++i;
  }
  while (i < s.size() && is_alpha(s[i])) ++i;
  return i;
}
// full match of ^(ep)SEP(ep)$ (backtracking over the greedy endpoint grammar)
inline bool range_split(const std::string& s, const std::string& sep, std::string* l, std::string* r) {
  // the left endpoint may end at any prefix boundary the grammar allows; try every split
  for (size_t k = 1; k + sep.size() < s.size() + 1; ++k) {
    if (s.compare(k, sep.size(), sep) != 0) continue;
    const std::string a = s.substr(0, k), b = s.substr(k + sep.size());
    auto whole = [](const std::string& x) {
      // endpoint grammar with backtracking: [-|+]? \d+ (\.\d+)? [A-Za-z]*
      size_t i = 0;
      if (i < x.size() && (x[i] == '-' || x[i] == '|' || x[i] == '+')) ++i;
      size_t d0 = i;
      while (i < x.size() && is_digit(x[i])) ++i;
      if (i == d0) return false;
      if (i < x.size() && x[i] == '.') {
        size_t j = i + 1, f0 = j;
        while (j < x.size() && is_digit(x[j])) ++j;
        if (j == f0) return false;
        i = j;
      }
      while (i < x.size() && is_alpha(x[i])) ++i;
      return i == x.size();
    };
    if (whole(a) && whole(b)) {
      *l = a;
      *r = b;
      return true;
    }
  }
  return false;
}

// operator.GetOperatorFromStringPattern
inline Op get_operator(const std::string& p) {
  if (p.size() < 2) return OP_EQ;
  if (p.compare(0, 2, ">=") == 0) return OP_GE;
  if (p.compare(0, 2, "<=") == 0) return OP_LE;
  if (p[0] == '>') return OP_GT;
  if (p[0] == '<') return OP_LT;
  if (p[0] == '!') return OP_NE;
  std::string l, r;
  if (range_split(p, "!-", &l, &r)) return OP_NOT_IN_RANGE;
  if (range_split(p, "-", &l, &r)) return OP_IN_RANGE;
  return OP_EQ;
}
inline size_t op_len(Op o) {
  switch (o) {
    case OP_GE:
    case OP_LE: return 2;
    case OP_GT:
    case OP_LT:
    case OP_NE: return 1;
    default: return 0;
  }
}

// convertNumberToString (pattern.go:307-323)
inline bool number_to_string(const JVal* v, std::string* out) {
  if (!v || v->t == JT::Null) {
    *out = "0";
    return true;
  }
  switch (v->t) {
    case JT::Str: *out = v->s; return true;
    case JT::Float: *out = go_fmt_f(v->f); return true;
    case JT::Int: *out = std::to_string(v->i); return true;
    default: return false;
  }
}

inline bool cmp_result(int c, Op op, bool* res) {
  switch (op) {
    case OP_EQ: *res = c == 0; return true;
    case OP_NE: *res = c != 0; return true;
    case OP_GT: *res = c > 0; return true;
    case OP_LT: *res = c < 0; return true;
    case OP_GE: *res = c >= 0; return true;
    case OP_LE: *res = c <= 0; return true;
    default: return false;
  }
}

inline bool compare_duration(const JVal* v, const std::string& p, Op op, bool* res) {
  int64_t pd, vd;
  std::string vs;
  if (!go_parse_duration(p, &pd)) return false;
  if (!number_to_string(v, &vs)) return false;
  if (!go_parse_duration(vs, &vd)) return false;
  return cmp_result(vd < pd ? -1 : (vd > pd ? 1 : 0), op, res);
}
inline bool compare_quantity(const JVal* v, const std::string& p, Op op, bool* res) {
  Qty pq, vq;
  std::string vs;
  if (!go_parse_quantity(p, &pq)) return false;
  if (!number_to_string(v, &vs)) return false;
  if (!go_parse_quantity(vs, &vq)) return false;
  return cmp_result(qty_cmp(vq, pq), op, res);
}
// compareString text of a value (pattern.go:270-305); false => "unexpected type"
inline bool compare_text(const JVal* v, std::string* out) {
  if (!v) return false;
  switch (v->t) {
    case JT::Float: *out = go_format_E(v->f); return true;
    case JT::Int: *out = std::to_string(v->i); return true;
    case JT::Str: *out = v->s; return true;
    case JT::Bool: *out = v->b ? "true" : "false"; return true;
    default: return false;
  }
}
inline bool compare_string(const JVal* v, const std::string& p, Op op) {
  if (op != OP_EQ && op != OP_NE) return false;
  std::string t;
  if (!compare_text(v, &t)) return false;
  const bool m = wildcard_match(p, t);
  return op == OP_NE ? !m : m;
}
inline bool validate_string(const JVal* v, const std::string& p, Op op) {
  bool r;
  if (compare_duration(v, p, op, &r)) return r;
  if (compare_quantity(v, p, op, &r)) return r;
  return compare_string(v, p, op);
}
inline std::string trim_spaces(const std::string& s) {  // strings.Trim(s, " ")
  size_t a = 0, b = s.size();
  while (a < b && s[a] == ' ') ++a;
  while (b > a && s[b - 1] == ' ') --b;
  return s.substr(a, b - a);
}
inline bool is_go_space(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r' || c == 0x85 || c == 0xA0;
}
inline std::string trim_space(const std::string& s) {  // strings.TrimSpace (ASCII + Latin-1 forms)
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\n' || s[a] == '\v' || s[a] == '\f' || s[a] == '\r')) ++a;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\n' || s[b - 1] == '\v' || s[b - 1] == '\f' ||
                   s[b - 1] == '\r'))
    --b;
  return s.substr(a, b - a);
}
inline std::vector<std::string> split_all(const std::string& s, char d) {
  std::vector<std::string> out;
  size_t a = 0;
  for (size_t i = 0; i <= s.size(); ++i)
    if (i == s.size() || s[i] == d) {
      out.push_back(s.substr(a, i - a));
      a = i + 1;
    }
  return out;
}

inline bool validate_string_pattern(const JVal* v, const std::string& pattern) {
  const Op op = get_operator(pattern);
  std::string l, r;
  if (op == OP_IN_RANGE) {
    if (!range_split(pattern, "-", &l, &r)) return false;
    return validate_string_pattern(v, ">= " + l) && validate_string_pattern(v, "<= " + r);
  }
  if (op == OP_NOT_IN_RANGE) {
    if (!range_split(pattern, "!-", &l, &r)) return false;
    return validate_string_pattern(v, "< " + l) || validate_string_pattern(v, "> " + r);
  }
  return validate_string(v, trim_space(pattern.substr(op_len(op))), op);
}
inline bool validate_string_patterns(const JVal* v, const std::string& pattern) {
  if (v && v->t == JT::Str && v->s == pattern) return true;
  for (auto& c : split_all(pattern, '|')) {
    bool all = true;
    for (auto& a : split_all(trim_spaces(c), '&'))
      if (!validate_string_pattern(v, trim_spaces(a))) {
        all = false;
        break;
      }
    if (all) return true;
  }
  return false;
}

// Go int64(float64) on amd64: out-of-range / NaN give INT64_MIN
inline int64_t go_f2i(double f) {
  if (!(f >= -9223372036854775808.0 && f < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)f;
}

// pattern.Validate (pattern.go:26-50). A null/absent value is `v == nullptr` or JT::Null.
inline bool validate_leaf(const JVal* v, const JVal& p) {
  const JT vt = v ? v->t : JT::Null;
  switch (p.t) {
    case JT::Bool: return vt == JT::Bool && v->b == p.b;
    case JT::Int:
      if (vt == JT::Int) return v->i == p.i;
      if (vt == JT::Float) return v->f == std::trunc(v->f) && go_f2i(v->f) == p.i;
      if (vt == JT::Str) {
        int64_t x;
        return go_parse_int(v->s, &x) && x == p.i;
      }
      return false;
    case JT::Float:
      if (vt == JT::Int) return p.f == std::trunc(p.f) && go_f2i(p.f) == v->i;
      if (vt == JT::Float) return v->f == p.f;
      if (vt == JT::Str) {
        double x;
        return go_parse_float(v->s, &x) && x == p.f;
      }
      return false;
    case JT::Null:
      switch (vt) {
        case JT::Float: return v->f == 0.0;
        case JT::Int: return v->i == 0;
        case JT::Str: return v->s.empty();
        case JT::Bool: return !v->b;
        case JT::Null: return true;
        default: return false;
      }
    case JT::Obj: return vt == JT::Obj;
    case JT::Str: return validate_string_patterns(v, p.s);
    case JT::Arr: return false;
  }
  return false;
}

// ---------------------------------------------------------------------------------------
// anchors (anchor/anchor.go, anchor/utils.go)
// ---------------------------------------------------------------------------------------
enum AType { A_NONE, A_COND, A_GLOBAL, A_NEG, A_ADD, A_EQ, A_EXIST };
struct Anchor {
  AType t = A_NONE;
  std::string key;
};
// regex ^([+<=X^])?\((.+)\)$ after TrimSpace ('.' excludes '\n')
inline Anchor parse_anchor(const std::string& raw) {
  Anchor a;
  const std::string s = trim_space(raw);
  if (s.size() < 3 || s.back() != ')') return a;
  size_t i = 0;
  AType t = A_COND;
  switch (s[0]) {
    case '+': t = A_ADD, i = 1; break;
    case '<': t = A_GLOBAL, i = 1; break;
    case '=': t = A_EQ, i = 1; break;
    case 'X': t = A_NEG, i = 1; break;
    case '^': t = A_EXIST, i = 1; break;
    default: break;
  }
  if (i >= s.size() || s[i] != '(') return a;
  const std::string key = s.substr(i + 1, s.size() - i - 2);
  if (key.empty() || key.find('\n') != std::string::npos) return a;
  a.t = t;
  a.key = key;
  return a;
}
inline bool is_anchor_phase(AType t) { return t == A_COND || t == A_EXIST || t == A_EQ || t == A_NEG; }
inline bool is_nested_anchor_type(AType t) { return t == A_COND || t == A_EXIST || t == A_EQ || t == A_NEG || t == A_GLOBAL; }

// ---------------------------------------------------------------------------------------
// validate.go tree walk
// ---------------------------------------------------------------------------------------
enum EKind { E_OK, E_COND, E_GLOBAL, E_NEG, E_OTHER, E_PSKIP };
struct Err {
  EKind k = E_OK;
  std::string path;  // returned element path
  bool ok() const { return k == E_OK; }
  bool skip() const { return k == E_COND || k == E_GLOBAL || k == E_PSKIP; }
  bool fail() const { return k == E_NEG; }
};
inline Err okv() { return Err{}; }
inline Err mk(EKind k, const std::string& p) {
  Err e;
  e.k = k;
  e.path = p;
  return e;
}

struct Walker {
  std::map<std::string, bool> amap;  // AnchorMap.anchorMap (keyed by the raw pattern key)

  // AnchorMap.CheckAnchorInResource
  void check_anchor_in_resource(const JVal& pmap, const JVal& rmap) {
    for (auto& kv : pmap.o) {
      Anchor a = parse_anchor(kv.first);
      if (!(a.t == A_COND || a.t == A_EXIST || a.t == A_NEG)) continue;
      auto it = amap.find(kv.first);
      if (it == amap.end()) it = amap.emplace(kv.first, false).first;
      else if (it->second) continue;
      if (rmap.get(a.key.c_str()) != nullptr || has_key(rmap, a.key)) it->second = true;
    }
  }
  static bool has_key(const JVal& m, const std::string& k) {
    for (auto& kv : m.o)
      if (kv.first == k) return true;
    return false;
  }
  bool keys_are_missing() const {
    for (auto& kv : amap)
      if (!kv.second) {
        if (parse_anchor(kv.first).t == A_NEG) continue;
        return true;
      }
    return false;
  }

  static const JVal* lookup(const JVal& m, const std::string& k) {
    for (auto& kv : m.o)
      if (kv.first == k) return kv.second.get();
    return nullptr;
  }

  // validateResourceElement (validate.go:71-114)
  Err element(const JVal* res, JVal& pat, const std::string& path) {
    switch (pat.t) {
      case JT::Obj:
        if (!res || res->t != JT::Obj) return mk(E_OTHER, path);
        check_anchor_in_resource(pat, *res);
        return map(*res, pat, path);
      case JT::Arr:
        if (!res || res->t != JT::Arr) return mk(E_OTHER, path);
        return array(*res, pat, path);
      default:
        if (res && res->t == JT::Arr) {
          for (auto& x : res->a)
            if (!validate_leaf(x.get(), pat)) return mk(E_OTHER, path);
          return okv();
        }
        if (!validate_leaf(res, pat)) return mk(E_OTHER, path);
        return okv();
    }
  }

  // anchor/handlers.go CreateElementHandler(...).Handle
  Err handle(const std::string& key, JVal& pat, const JVal& rmap, const std::string& path) {
    Anchor a = parse_anchor(key);
    switch (a.t) {
      case A_COND: {
        const std::string cur = path + a.key + "/";
        if (has_key(rmap, a.key)) {
          Err e = element(lookup(rmap, a.key), pat, cur);
          if (!e.ok()) return mk(E_COND, e.path);
          return okv();
        }
        return mk(E_COND, cur);
      }
      case A_GLOBAL: {
        const std::string cur = path + a.key + "/";
        if (has_key(rmap, a.key)) {
          Err e = element(lookup(rmap, a.key), pat, cur);
          if (!e.ok()) return mk(E_GLOBAL, e.path);
        }
        return okv();
      }
      case A_EXIST: {
        const std::string cur = path + a.key + "/";
        if (!has_key(rmap, a.key)) return okv();
        const JVal* v = lookup(rmap, a.key);
        if (!v || v->t != JT::Arr) return mk(E_OTHER, cur);
        if (pat.t != JT::Arr) return mk(E_OTHER, cur);
        Err last;
        for (auto& pm : pat.a) {
          if (pm->t != JT::Obj) return mk(E_OTHER, cur);
          // validateExistenceListResource
          bool found = false;
          for (size_t i = 0; i < v->a.size() && !found; ++i) {
            Err e = element(v->a[i].get(), *pm, cur + std::to_string(i) + "/");
            if (e.ok()) found = true;
          }
          if (!found) return mk(E_OTHER, cur);
        }
        return okv();
      }
      case A_EQ: {
        const std::string cur = path + a.key + "/";
        if (has_key(rmap, a.key)) {
          Err e = element(lookup(rmap, a.key), pat, cur);
          if (!e.ok()) return e;
        }
        return okv();
      }
      case A_NEG: {
        const std::string cur = path + a.key + "/";
        if (has_key(rmap, a.key)) return mk(E_NEG, cur);
        return okv();
      }
      default: {  // defaultHandler (also "+(...)" keys, looked up verbatim)
        const std::string cur = path + key + "/";
        const JVal* v = lookup(rmap, key);
        const bool star = pat.t == JT::Str && pat.s == "*";
        if (star) {
          if (v && v->t != JT::Null) return okv();
          return mk(E_OTHER, path);
        }
        Err e = element(v, pat, cur);
        if (!e.ok()) return e;
        return okv();
      }
    }
  }

  static bool has_nested_anchors(const JVal& p) {
    if (p.t == JT::Obj) {
      for (auto& kv : p.o)
        if (is_nested_anchor_type(parse_anchor(kv.first).t)) return true;
      for (auto& kv : p.o)
        if (has_nested_anchors(*kv.second)) return true;
      return false;
    }
    if (p.t == JT::Arr) {
      for (auto& x : p.a)
        if (has_nested_anchors(*x)) return true;
    }
    return false;
  }

  // wildcards.ExpandInMetadata (wildcards.go:83-162); mutates the pattern like the reference
  static void expand_in_metadata(JVal& pmap, const JVal& rmap) {
    JVal* pmeta = nullptr;
    for (auto& kv : pmap.o)
      if (kv.first == "metadata" || parse_anchor(kv.first).key == "metadata") {
        pmeta = kv.second.get();
        break;
      }
    if (!pmeta) return;
    const JVal* rmeta = lookup(rmap, "metadata");
    if (!rmeta || rmeta->t == JT::Null) return;
    if (pmeta->t != JT::Obj) return;  // the reference panics here (type assertion)
    for (const char* tag : {"labels", "annotations"}) {
      std::pair<std::string, JPtr>* pent = nullptr;
      for (auto& kv : pmeta->o)
        if (kv.first == tag || parse_anchor(kv.first).key == tag) {
          pent = &kv;
          break;
        }
      if (!pent || !pent->second || pent->second->t != JT::Obj) continue;
      if (rmeta->t != JT::Obj) continue;
      const JVal* rdata = nullptr;
      for (auto& kv : rmeta->o)
        if (kv.first == tag || parse_anchor(kv.first).key == tag) {
          rdata = kv.second.get();
          break;
        }
      if (!rdata || rdata->t != JT::Obj) continue;
      auto results = std::make_shared<JVal>();
      results->t = JT::Obj;
      for (auto& kv : pent->second->o) {
        std::string k = kv.first;
        if (k.find_first_of("*?") != std::string::npos) {
          Anchor a = parse_anchor(k);
          const std::string g = a.t != A_NONE ? a.key : k;
          std::string mk_ = g;
          for (auto& rk : rdata->o)  // first matching resource key (document order)
            if (rk.second && rk.second->t == JT::Str && wildcard_match(g, rk.first)) {
              mk_ = rk.first;
              break;
            }
          if (a.t != A_NONE) {
            static const char mods[] = {0, 0, '<', 'X', '+', '=', '^'};
            std::string m = a.t == A_COND ? "" : std::string(1, mods[a.t]);
            k = m + "(" + mk_ + ")";
          } else {
            k = mk_;
          }
        }
        bool dup = false;
        for (auto& rk : results->o)
          if (rk.first == k) {
            rk.second = kv.second;
            dup = true;
          }
        if (!dup) results->o.emplace_back(k, kv.second);
      }
      pent->second = results;
    }
  }

  // validateMap (validate.go:118-175)
  Err map(const JVal& rmap, JVal& pmap, const std::string& path) {
    expand_in_metadata(pmap, rmap);
    std::vector<std::string> anchors, rest;
    for (auto& kv : pmap.o) {
      if (is_anchor_phase(parse_anchor(kv.first).t)) anchors.push_back(kv.first);
      else rest.push_back(kv.first);
    }
    std::sort(anchors.begin(), anchors.end());
    int apply = 0, skips = 0;
    for (auto& k : anchors) {
      Err e = handle(k, *member(pmap, k), rmap, path);
      if (!e.ok()) {
        if (e.skip()) {
          ++skips;
          continue;
        }
        return e;
      }
      ++apply;
    }
    if (apply == 0 && skips > 0) return mk(E_PSKIP, path);
    // getSortedNestedAnchorResource (validate/utils.go:37-57)
    std::sort(rest.begin(), rest.end());
    std::vector<std::string> front, back;
    for (auto& k : rest) {
      if (parse_anchor(k).t == A_GLOBAL || has_nested_anchors(*member(pmap, k))) front.insert(front.begin(), k);
      else back.push_back(k);
    }
    for (auto* list : {&front, &back})
      for (auto& k : *list) {
        Err e = handle(k, *member(pmap, k), rmap, path);
        if (!e.ok()) return e;
      }
    return okv();
  }
  static JVal* member(JVal& m, const std::string& k) {
    JVal* out = nullptr;
    for (auto& kv : m.o)
      if (kv.first == k) out = kv.second.get();  // last duplicate wins, like a Go map decode
    return out;
  }

  // validateArray / validateArrayOfMaps (validate.go:177-261)
  Err array(const JVal& rarr, JVal& parr, const std::string& path) {
    if (parr.a.empty()) return mk(E_OTHER, path);
    JVal& p0 = *parr.a[0];
    if (p0.t == JT::Obj) {
      int apply = 0, skips = 0;
      for (size_t i = 0; i < rarr.a.size(); ++i) {
        Err e = element(rarr.a[i].get(), p0, path + std::to_string(i) + "/");
        if (!e.ok()) {
          if (e.skip()) {
            ++skips;
            continue;
          }
          return e;
        }
        ++apply;
      }
      if (apply == 0 && skips > 0) return mk(E_PSKIP, path);
      return okv();
    }
    if (p0.t != JT::Arr) return element(&rarr, p0, path);
    if (rarr.a.size() < parr.a.size()) return mk(E_OTHER, "");
    int apply = 0, skips = 0;
    for (size_t i = 0; i < parr.a.size(); ++i) {
      Err e = element(rarr.a[i].get(), *parr.a[i], path + std::to_string(i) + "/");
      if (!e.ok()) {
        if (e.skip()) {
          ++skips;
          continue;
        }
        return e;
      }
      ++apply;
    }
    if (apply == 0 && skips > 0) return mk(E_PSKIP, path);
    return okv();
  }
};

inline JPtr clone(const JVal& v) {
  auto c = std::make_shared<JVal>(v);
  for (auto& x : c->a) x = clone(*x);
  for (auto& kv : c->o) kv.second = clone(*kv.second);
  return c;
}

// validate.MatchPattern result
enum MatchKind { M_PASS, M_SKIP, M_FAIL };
struct MatchResult {
  MatchKind k = M_PASS;
  std::string path;  // PatternError.Path (FAIL with an empty path => ERROR verdict)
};
inline MatchResult match_pattern(const JVal& resource, const JVal& pattern) {
  JPtr p = clone(pattern);  // FromJSON yields a fresh pattern per evaluation
  Walker w;
  Err e = w.element(&resource, *p, "/");
  MatchResult r;
  if (e.ok()) return r;
  if (e.skip()) {
    r.k = M_SKIP;
    return r;
  }
  r.k = M_FAIL;
  if (e.fail()) {
    r.path = e.path;
    return r;
  }
  r.path = w.keys_are_missing() ? "" : e.path;
  return r;
}

// JSON decode of anyPattern through encoding/json (validate_resource.go:400-416): every
// number becomes float64.
inline void numbers_to_float(JVal& v) {
  if (v.t == JT::Int) {
    v.t = JT::Float;
    v.f = (double)v.i;
  }
  for (auto& x : v.a) numbers_to_float(*x);
  for (auto& kv : v.o) numbers_to_float(*kv.second);
}

// json.Marshal + util/json decode of a pattern (autogen SetPattern, rule.go:130-183): a whole
// float64 below 1e21 is written as an integer literal and decodes as int64 when it fits.
inline void marshal_roundtrip(JVal& v) {
  if (v.t == JT::Float && std::isfinite(v.f) && v.f == std::trunc(v.f) && std::fabs(v.f) < 1e21 &&
      v.f >= -9223372036854775808.0 && v.f < 9223372036854775808.0) {
    v.t = JT::Int;
    v.i = (int64_t)v.f;
  }
  for (auto& x : v.a) marshal_roundtrip(*x);
  for (auto& kv : v.o) marshal_roundtrip(*kv.second);
}

// any "{{" / "$(" in keys or string leaves => variable substitution (not restated here)
inline bool has_variables(const JVal& v) {
  auto bad = [](const std::string& s) {
    return s.find("{{") != std::string::npos || s.find("$(") != std::string::npos;
  };
  if (v.t == JT::Str) return bad(v.s);
  for (auto& x : v.a)
    if (has_variables(*x)) return true;
  for (auto& kv : v.o)
    if (bad(kv.first) || has_variables(*kv.second)) return true;
  return false;
}

}  // namespace pat
}  // namespace oracle
