// Host-side decoding of scalar values into the typed attributes the device leaf
// validators compare (ingestion / policy compile only; no verdict is decided here).
//
// The attributes mirror what the reference derives from a value while validating a
// pattern leaf (pkg/engine/pattern/pattern.go):
//   - strconv.ParseInt(s, 10, 64) / strconv.ParseFloat(s, 64)     (validateInt/FloatPattern)
//   - convertNumberToString (pattern.go:307-323) followed by
//       time.ParseDuration           (compareDuration, pattern.go:217-241)
//       resource.ParseQuantity       (compareQuantity, pattern.go:243-268; apimachinery v0.29.1)
//   - the compareString text: FormatFloat(v,'E',-1,64) / FormatInt / FormatBool (pattern.go:270-305)
// Quantities are reduced to an exact canonical value sign * m * 10^e (m without trailing
// zeros) so the device compares two of them with integer arithmetic only.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

namespace kpe {
namespace goval {

using u128 = unsigned __int128;

struct Quantity {
  bool neg = false;
  u128 m = 0;
  int64_t e = 0;
};

inline bool dig(char c) { return c >= '0' && c <= '9'; }

// strconv.ParseInt(s, 10, 64)
inline bool parse_int(std::string_view s, int64_t* out) {
  if (s.empty()) return false;
  const bool neg = s[0] == '-';
  if (s[0] == '-' || s[0] == '+') s.remove_prefix(1);
  if (s.empty()) return false;
  const uint64_t lim = neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull;
  uint64_t v = 0;
  for (char c : s) {
    if (!dig(c)) return false;
    const uint64_t d = (uint64_t)(c - '0');
    if (v > (lim - d) / 10) return false;
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(~v + 1) : (int64_t)v;
  return true;
}

inline bool ci_eq(std::string_view a, const char* b) {
  if (a.size() != strlen(b)) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if ((char)(a[i] | 0x20) != b[i]) return false;
  return true;
}

// strconv.ParseFloat(s, 64): Go literal grammar; overflow is an error
inline bool parse_float(std::string_view s, double* out) {
  if (s.empty()) return false;
  std::string_view body = s;
  int sign = 1;
  if (body[0] == '+' || body[0] == '-') {
    sign = body[0] == '-' ? -1 : 1;
    body.remove_prefix(1);
  }
  if (ci_eq(body, "inf") || ci_eq(body, "infinity")) {
    *out = sign * HUGE_VAL;
    return true;
  }
  if (ci_eq(s, "nan")) {
    *out = NAN;
    return true;
  }
  const bool hex = body.size() >= 2 && body[0] == '0' && (body[1] | 0x20) == 'x';
  size_t i = hex ? 2 : 0;
  int ndig = 0, ndot = 0;
  for (; i < body.size(); ++i) {
    const char c = body[i];
    if (c == '.') ++ndot;
    else if (dig(c) || (hex && isxdigit((unsigned char)c))) ++ndig;
    else break;
  }
  if (ndig == 0 || ndot > 1) return false;
  if (i < body.size()) {
    const char e = (char)(body[i] | 0x20);
    if (e != (hex ? 'p' : 'e')) return false;
    ++i;
    if (i < body.size() && (body[i] == '+' || body[i] == '-')) ++i;
    const size_t d0 = i;
    while (i < body.size() && dig(body[i])) ++i;
    if (i == d0 || i != body.size()) return false;
  } else if (hex) {
    return false;
  }
  const std::string z(s);
  const double v = strtod(z.c_str(), nullptr);
  if (std::isinf(v)) return false;
  *out = v;
  return true;
}

// time.ParseDuration -> nanoseconds
inline bool parse_duration(std::string_view s, int64_t* out) {
  bool neg = false;
  if (!s.empty() && (s[0] == '-' || s[0] == '+')) {
    neg = s[0] == '-';
    s.remove_prefix(1);
  }
  if (s == "0") {
    *out = 0;
    return true;
  }
  if (s.empty()) return false;
  constexpr uint64_t kTop = 1ull << 63;
  uint64_t total = 0;
  while (!s.empty()) {
    if (!(s[0] == '.' || dig(s[0]))) return false;
    uint64_t whole = 0, frac = 0;
    double scale = 1;
    size_t k = 0;
    for (; k < s.size() && dig(s[k]); ++k) {
      if (whole > kTop / 10) return false;
      whole = whole * 10 + (uint64_t)(s[k] - '0');
      if (whole > kTop) return false;
    }
    bool any = k > 0;
    if (k < s.size() && s[k] == '.') {
      size_t f0 = ++k;
      bool ovf = false;
      for (; k < s.size() && dig(s[k]); ++k) {
        if (ovf) continue;
        if (frac > (kTop - 1) / 10) {
          ovf = true;
          continue;
        }
        const uint64_t nf = frac * 10 + (uint64_t)(s[k] - '0');
        if (nf > kTop) {
          ovf = true;
          continue;
        }
        frac = nf;
        scale *= 10;
      }
      any = any || k > f0;
    }
    if (!any) return false;
    size_t u = k;
    while (u < s.size() && s[u] != '.' && !dig(s[u])) ++u;
    const std::string_view unit = s.substr(k, u - k);
    uint64_t mult;
    if (unit == "ns") mult = 1;
    else if (unit == "us" || unit == "\xC2\xB5s" || unit == "\xCE\xBCs") mult = 1000ull;
    else if (unit == "ms") mult = 1000000ull;
    else if (unit == "s") mult = 1000000000ull;
    else if (unit == "m") mult = 60000000000ull;
    else if (unit == "h") mult = 3600000000000ull;
    else return false;  // includes a missing unit
    if (whole > kTop / mult) return false;
    whole *= mult;
    if (frac > 0) {
      whole += (uint64_t)((double)frac * ((double)mult / scale));
      if (whole > kTop) return false;
    }
    total += whole;
    if (total > kTop) return false;
    s.remove_prefix(u);
  }
  if (!neg && total > kTop - 1) return false;
  *out = neg ? (int64_t)(~total + 1) : (int64_t)total;
  return true;
}

inline void qnorm(Quantity& q) {
  if (q.m == 0) {
    q = Quantity{};
    return;
  }
  while (q.m % 10 == 0) q.m /= 10, ++q.e;
}

// resource.ParseQuantity: returns the exact value the reference's Quantity holds
// (int64Amount fast path unrounded; inf.Dec path rounded up to 1e-9 and capped at
// 2^63-1), canonicalised.
inline bool parse_quantity(std::string_view str, Quantity* out) {
  if (str.empty()) return false;
  if (str == "0") {
    *out = Quantity{};
    return true;
  }
  // ---- lexical split: sign, integer digits (leading zeros dropped), fraction, suffix ----
  size_t p = 0;
  const bool positive = str[0] != '-';
  if (str[0] == '-' || str[0] == '+') ++p;
  size_t z = p;
  while (z < str.size() && str[z] == '0') ++z;
  std::string_view num, den, suf;
  size_t vend;  // end of the numeric part (sign + digits [. digits])
  if (z == str.size()) {
    num = "0";
    vend = str.size();
  } else {
    size_t q = z;
    while (q < str.size() && dig(str[q])) ++q;
    num = q > z ? str.substr(z, q - z) : std::string_view("0");
    vend = q;
    if (q < str.size() && str[q] == '.') {
      size_t d0 = q + 1, d = d0;
      while (d < str.size() && dig(str[d])) ++d;
      den = str.substr(d0, d - d0);
      vend = d;
    }
    if (vend < str.size()) {
      size_t s0 = vend, k = vend;
      while (k < str.size() && strchr("eEinumkKMGTP", str[k]) && str[k]) ++k;
      if (k < str.size()) {
        if (str[k] == '+' || str[k] == '-') ++k;
        while (k < str.size() && dig(str[k])) ++k;
        if (k != str.size()) return false;  // ErrFormatWrong
      }
      suf = str.substr(s0);
    }
  }
  // ---- suffix ----
  int base = 10, fmt = 0;  // fmt: 0 DecimalSI, 1 BinarySI, 2 DecimalExponent
  int32_t exp = 0;
  static const struct {
    const char* s;
    int b, e;
  } kSuf[] = {{"n", 10, -9}, {"u", 10, -6}, {"m", 10, -3}, {"", 10, 0},  {"k", 10, 3},  {"M", 10, 6},
              {"G", 10, 9},  {"T", 10, 12}, {"P", 10, 15}, {"E", 10, 18}, {"Ki", 2, 10}, {"Mi", 2, 20},
              {"Gi", 2, 30}, {"Ti", 2, 40}, {"Pi", 2, 50}, {"Ei", 2, 60}};
  bool known = false;
  for (auto& k : kSuf)
    if (suf == k.s) {
      base = k.b, exp = k.e, fmt = k.b == 2 ? 1 : 0, known = true;
      break;
    }
  if (!known) {
    int64_t x;
    if (suf.size() < 2 || (suf[0] != 'e' && suf[0] != 'E') || !parse_int(suf.substr(1), &x)) return false;
    exp = (int32_t)x, fmt = 2;
  }
  // ---- int64Amount fast path ----
  int32_t prec, scale;
  int64_t mant = 1;
  if (fmt != 1) {
    scale = exp;
    prec = 18 - (int32_t)(num.size() + den.size());
  } else {
    scale = 0;
    if (exp >= 0 && den.empty()) {
      mant = (int64_t)(1ull << exp);
      prec = 15 - (int32_t)num.size() - (int32_t)((float)exp * 3 / 10) - 1;
    } else {
      prec = -1;
    }
  }
  if (prec >= 0) {
    scale -= (int32_t)den.size();
    if (scale >= -9) {
      int64_t v;
      if (!parse_int(std::string(num) + std::string(den), &v)) return false;
      const __int128 r = (__int128)v * mant;
      if (r >= INT64_MIN && r <= INT64_MAX) {
        Quantity q;
        q.neg = !positive;
        q.m = (u128)(r < 0 ? -r : r);
        q.e = scale;
        qnorm(q);
        *out = q;
        return true;
      }
    }
  }
  // ---- inf.Dec path: exact decimal digits * 10^e10 (* 2^exp), ceil at 1e-9, cap ----
  std::vector<uint8_t> digits;  // most significant first, leading zeros dropped
  int64_t e10 = 0;
  {
    bool frac = false;
    for (size_t k = 0; k < vend; ++k) {
      const char c = str[k];
      if (c == '.') frac = true;
      if (!dig(c)) continue;
      if (frac) --e10;
      if (digits.empty() && c == '0') continue;
      digits.push_back((uint8_t)(c - '0'));
    }
  }
  if (base == 10) e10 += exp;
  // big value as base-1e9 limbs (little endian)
  std::vector<uint32_t> L;
  auto mul_add = [&](uint32_t mlt, uint32_t add) {
    uint64_t carry = add;
    for (auto& x : L) {
      const uint64_t t = (uint64_t)x * mlt + carry;
      x = (uint32_t)(t % 1000000000u);
      carry = t / 1000000000u;
    }
    if (carry) L.push_back((uint32_t)carry);
  };
  for (uint8_t d : digits) mul_add(10, d);
  if (base == 2)
    for (int32_t k = 0; k < exp; ++k) mul_add(2, 0);
  auto ndig = [&]() {
    int d = L.empty() ? 0 : 9 * (int)(L.size() - 1);
    for (uint32_t t = L.empty() ? 0 : L.back(); t; t /= 10) ++d;
    return d;
  };
  if (ndig() == 0) {
    *out = Quantity{};
    return true;
  }
  const u128 cap = (u128)INT64_MAX * 1000000000u;
  u128 Q = 0;
  const int64_t sh = e10 + 9;
  auto to128 = [&]() {
    u128 v = 0;
    for (size_t k = L.size(); k-- > 0;) v = v * 1000000000u + L[k];
    return v;
  };
  if (sh >= 0) {
    if (ndig() + sh > 29) {
      Q = cap;
    } else {
      for (int64_t k = 0; k < sh; ++k) mul_add(10, 0);
      Q = to128();
    }
  } else if (-sh > ndig()) {
    Q = 1;
  } else {
    bool rem = false;
    for (int64_t k = 0; k < -sh; ++k) {  // divide by 10
      uint64_t r = 0;
      for (size_t j = L.size(); j-- > 0;) {
        const uint64_t cur = L[j] + r * 1000000000ull;
        L[j] = (uint32_t)(cur / 10);
        r = cur % 10;
      }
      while (!L.empty() && !L.back()) L.pop_back();
      rem = rem || r;
    }
    Q = ndig() > 29 ? cap : to128() + (rem ? 1 : 0);
  }
  if (Q > cap) Q = cap;
  Quantity q;
  q.neg = !positive;
  q.m = Q;
  q.e = -9;
  qnorm(q);
  *out = q;
  return true;
}

// Comparison key of a quantity: order = number of digits of m + e, and m left-aligned to
// 38 digits (m * 10^(38 - digits) < 10^38 < 2^127). Two non-zero values of one sign then
// compare by (order, aligned m) with plain integer compares on the device.
inline void qty_key(const Quantity& q, int64_t* order, uint64_t* lo, uint64_t* hi) {
  if (q.m == 0) {
    *order = 0, *lo = 0, *hi = 0;
    return;
  }
  int d = 0;
  for (u128 t = q.m; t; t /= 10) ++d;
  u128 x = q.m;
  for (int k = d; k < 38; ++k) x *= 10;
  *order = (int64_t)d + q.e;
  *lo = (uint64_t)x, *hi = (uint64_t)(x >> 64);
}

// fmt.Sprintf("%f", v)
inline std::string fmt_f(double v) {
  char b[400];
  snprintf(b, sizeof b, "%f", v);
  return b;
}

// strconv.FormatFloat(v, 'E', -1, 64)
inline std::string fmt_E(double v) {
  char b[48];
  int p = 0;
  for (; p < 17; ++p) {
    snprintf(b, sizeof b, "%.*E", p, v);
    if (strtod(b, nullptr) == v) break;
  }
  snprintf(b, sizeof b, "%.*E", p, v);
  return b;
}

// fmt.Sprint(float64) = strconv.AppendFloat(v, 'g', -1, 64): the shortest round-trip digits,
// in %e form when the decimal exponent is < -4 or >= 6 (ftoa.go: "if precision was the
// shortest possible, use precision 6 for this decision"), e.g. 1e+06, 123456, 1.5e-05. The
// variables/operator set operators compare fmt.Sprint of JSON numbers (always float64 there).
inline std::string sprint_float(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return std::signbit(v) ? "-0" : "0";
  const std::string e = fmt_E(std::fabs(v));
  const size_t E = e.find('E');
  std::string d;
  for (size_t i = 0; i < E; ++i)
    if (dig(e[i])) d += e[i];
  const int ex = atoi(e.c_str() + E + 1), nd = (int)d.size(), dp = ex + 1;
  const std::string sign = v < 0 ? "-" : "";
  if (ex < -4 || ex >= 6) {
    std::string o = sign + d.substr(0, 1);
    if (nd > 1) o += "." + d.substr(1);
    char buf[16];
    snprintf(buf, sizeof buf, "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    return o + buf;
  }
  if (dp <= 0) return sign + "0." + std::string(-dp, '0') + d;
  if (dp >= nd) return sign + d + std::string(dp - nd, '0');
  return sign + d.substr(0, dp) + "." + d.substr(dp);
}

// operator.GetOperatorFromStringPattern(s) == InRange (pkg/engine/operator/operator.go:36-61):
// no >= <= > < ! prefix, not the NotInRange form, and
// ^([-|+]?\d+(\.\d+)?[A-Za-z]*)-([-|+]?\d+(\.\d+)?[A-Za-z]*)$
inline bool range_endpoint(std::string_view x) {
  size_t i = 0;
  auto dg = [&](size_t j) { return j < x.size() && x[j] >= '0' && x[j] <= '9'; };
  if (i < x.size() && (x[i] == '-' || x[i] == '|' || x[i] == '+')) ++i;
  if (!dg(i)) return false;
  while (dg(i)) ++i;
  if (i < x.size() && x[i] == '.') {
    if (!dg(i + 1)) return false;
    ++i;
    while (dg(i)) ++i;
  }
  while (i < x.size() && ((x[i] >= 'a' && x[i] <= 'z') || (x[i] >= 'A' && x[i] <= 'Z'))) ++i;
  return i == x.size();
}
inline bool range_split(std::string_view t, std::string_view sep, size_t* at = nullptr) {
  for (size_t k = 1; k + sep.size() <= t.size(); ++k)
    if (t.substr(k, sep.size()) == sep && range_endpoint(t.substr(0, k)) && range_endpoint(t.substr(k + sep.size()))) {
      if (at) *at = k;
      return true;
    }
  return false;
}
inline bool in_range_form(std::string_view s) {
  if (s.size() < 2) return false;
  if (s[0] == '>' || s[0] == '<' || s[0] == '!') return false;
  if (range_split(s, "!-")) return false;
  return range_split(s, "-");
}

// schema.h SC_PSIMPLE: as a pattern string (pattern.go:152-215 validateStringPatterns) s is a
// single condition equal to itself with the Equal operator: no `|` / `&` split, nothing trimmed
// (strings.Trim " ", strings.TrimSpace; a non-ASCII boundary byte is taken as possible Unicode
// space), no >= <= > < ! prefix, neither range form
inline bool pattern_simple(std::string_view s) {
  if (s.find('|') != std::string_view::npos || s.find('&') != std::string_view::npos) return false;
  if (!s.empty()) {
    auto edge = [](unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r') || c >= 0x80; };
    if (edge((unsigned char)s.front()) || edge((unsigned char)s.back())) return false;
  }
  if (s.size() >= 2 && (s[0] == '>' || s[0] == '<' || s[0] == '!')) return false;
  if (range_split(s, "!-") || range_split(s, "-")) return false;
  return true;
}

// schema.h SC_SPQ: ParseQuantity of fmt.Sprint(v) (the text the condition set operators hand
// to an InRange check) agrees with the quantity attributes computed from another text of v
inline bool sprint_qty_same(const std::string& sp, bool has_qty, bool neg, int64_t qexp, uint64_t qlo, uint64_t qhi) {
  Quantity q;
  const bool ok = parse_quantity(sp, &q);
  if (ok != has_qty) return false;
  if (!ok) return true;
  int64_t o;
  uint64_t lo, hi;
  qty_key(q, &o, &lo, &hi);
  if ((lo | hi) == 0 && (qlo | qhi) == 0) return true;
  return o == qexp && lo == qlo && hi == qhi && q.neg == neg;
}

}  // namespace goval
}  // namespace kpe
