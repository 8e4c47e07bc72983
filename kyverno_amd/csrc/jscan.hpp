// Single-pass JSON cursor used by the corpus flattener (host side).
// No DOM: the flattener walks the typed K8s schema it needs and skips the rest.
// Number classification mirrors what the reference sees after apimachinery's
// unstructured decode + MarshalJSON (whole -> int64, else float64; a float64 that
// is integral and |x| < 1e21 is re-encoded as an integer literal).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <emmintrin.h>  // SSE2 (x86-64 baseline): 16-byte scans of strings and skipped values

#include <string>
#include <string_view>

namespace kpe {

// The first byte of [p, e) that is `"` or a backslash (16 bytes per step)
inline const char* jscan_quote(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), b = _mm_set1_epi8('\\');
  while (e - p >= 16) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const int m = _mm_movemask_epi8(_mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_cmpeq_epi8(x, b)));
    if (m) return p + __builtin_ctz((unsigned)m);
    p += 16;
  }
  while (p < e && *p != '"' && *p != '\\') ++p;
  return p;
}
// The first structural byte of [p, e) for skipping a container: `"` `{` `}` `[` `]`
// ('[' | 0x20 == '{' and ']' | 0x20 == '}': two compares after an OR cover the brackets)
inline const char* jscan_struct(const char* p, const char* e) {
  const __m128i q = _mm_set1_epi8('"'), lo = _mm_set1_epi8('{'), hi = _mm_set1_epi8('}'), bit = _mm_set1_epi8(0x20);
  while (e - p >= 16) {
    const __m128i x = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
    const __m128i y = _mm_or_si128(x, bit);
    const int m = _mm_movemask_epi8(
        _mm_or_si128(_mm_cmpeq_epi8(x, q), _mm_or_si128(_mm_cmpeq_epi8(y, lo), _mm_cmpeq_epi8(y, hi))));
    if (m) return p + __builtin_ctz((unsigned)m);
    p += 16;
  }
  while (p < e && *p != '"' && *p != '{' && *p != '}' && *p != '[' && *p != ']') ++p;
  return p;
}

enum class JK : uint8_t { End, Null, Bool, Num, Str, Arr, Obj, Bad };

struct JNum {
  bool is_int = false;     // literal is an int64 integer
  int64_t i = 0;
  double f = 0;
  // integral-valued and representable as an integer literal after re-marshal
  bool integral(int64_t* out) const {
    if (is_int) {
      *out = i;
      return true;
    }
    if (!std::isfinite(f) || std::floor(f) != f || std::fabs(f) >= 1e21) return false;
    if (f < -9.2233720368547758e18 || f >= 9.2233720368547758e18) return false;
    *out = (int64_t)f;
    return true;
  }
};

class JCur {
 public:
  JCur(const char* p, const char* e) : p_(p), e_(e) {}
  bool ok() const { return ok_; }
  const char* pos() const { return p_; }

  JK peek() {
    ws();
    if (p_ >= e_) return JK::End;
    switch (*p_) {
      case '{': return JK::Obj;
      case '[': return JK::Arr;
      case '"': return JK::Str;
      case 't':
      case 'f': return JK::Bool;
      case 'n': return JK::Null;
      default:
        if (*p_ == '-' || (*p_ >= '0' && *p_ <= '9')) return JK::Num;
        return JK::Bad;
    }
  }
  // --- scalars ---
  bool null() {
    ws();
    if (e_ - p_ >= 4 && !memcmp(p_, "null", 4)) {
      p_ += 4;
      return true;
    }
    return fail();
  }
  bool boolean(bool* v) {
    ws();
    if (e_ - p_ >= 4 && !memcmp(p_, "true", 4)) {
      p_ += 4;
      *v = true;
      return true;
    }
    if (e_ - p_ >= 5 && !memcmp(p_, "false", 5)) {
      p_ += 5;
      *v = false;
      return true;
    }
    return fail();
  }
  bool number(JNum* n) {
    ws();
    const char* s = p_;
    if (p_ < e_ && *p_ == '-') ++p_;
    bool isint = true;
    const char* d0 = p_;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '+' ||
                       *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') isint = false;
      ++p_;
    }
    if (p_ == d0) return fail();
    {  // encoding/json's number grammar: -?(0|[1-9][0-9]*)(\.[0-9]+)?([eE][+-]?[0-9]+)?
      const char* q = d0;
      auto digits = [&]() {
        const char* k = q;
        while (q < p_ && *q >= '0' && *q <= '9') ++q;
        return (size_t)(q - k);
      };
      const size_t nd = digits();
      bool ok = nd > 0 && !(nd > 1 && *d0 == '0');
      if (ok && q < p_ && *q == '.') ++q, ok = digits() > 0;
      if (ok && q < p_ && (*q == 'e' || *q == 'E')) {
        ++q;
        if (q < p_ && (*q == '+' || *q == '-')) ++q;
        ok = digits() > 0;
      }
      if (!ok || q != p_) return fail();
    }
    char buf[64];
    size_t len = (size_t)(p_ - s);
    if (len >= sizeof buf) {
      n->is_int = false;
      n->f = strtod(std::string(s, len).c_str(), nullptr);
      return true;
    }
    memcpy(buf, s, len);
    buf[len] = 0;
    if (isint) {
      errno = 0;
      char* end;
      long long x = strtoll(buf, &end, 10);
      if (errno == 0 && *end == 0) {
        n->is_int = true;
        n->i = x;
        return true;
      }
    }
    n->is_int = false;
    n->f = strtod(buf, nullptr);
    return true;
  }
  // String: returns a view into the input when there are no escapes, otherwise
  // into `scratch` (decoded UTF-8).
  bool str(std::string_view* out, std::string& scratch) {
    ws();
    if (p_ >= e_ || *p_ != '"') return fail();
    ++p_;
    const char* s = p_;
    p_ = jscan_quote(p_, e_);
    if (p_ < e_ && *p_ == '"') {
      *out = std::string_view(s, (size_t)(p_ - s));
      ++p_;
      return true;
    }
    scratch.assign(s, (size_t)(p_ - s));
    while (p_ < e_) {
      char c = *p_++;
      if (c == '"') {
        *out = scratch;
        return true;
      }
      if (c != '\\') {
        scratch.push_back(c);
        continue;
      }
      if (p_ >= e_) return fail();
      char x = *p_++;
      switch (x) {
        case '"': scratch.push_back('"'); break;
        case '\\': scratch.push_back('\\'); break;
        case '/': scratch.push_back('/'); break;
        case 'b': scratch.push_back('\b'); break;
        case 'f': scratch.push_back('\f'); break;
        case 'n': scratch.push_back('\n'); break;
        case 'r': scratch.push_back('\r'); break;
        case 't': scratch.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return fail();
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            p_ += 2;
            uint32_t lo;
            if (!hex4(&lo)) return fail();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(scratch, cp);
          break;
        }
        default: return fail();
      }
    }
    return fail();
  }
  // --- containers ---
  // Usage: bool f = true; if (c.obj_begin()) while (c.obj_next(f, &key, ks)) { ...consume value... }
  bool obj_begin() {
    ws();
    if (p_ >= e_ || *p_ != '{') return fail();
    ++p_;
    return true;
  }
  bool obj_next(bool& first, std::string_view* key, std::string& scratch) {
    ws();
    if (p_ >= e_) return fail();
    if (*p_ == '}') {
      ++p_;
      return false;
    }
    if (!first) {
      if (*p_ != ',') return fail();
      ++p_;
    }
    first = false;
    if (!str(key, scratch)) return false;
    ws();
    if (p_ >= e_ || *p_ != ':') return fail();
    ++p_;
    return true;
  }
  bool arr_begin() {
    ws();
    if (p_ >= e_ || *p_ != '[') return fail();
    ++p_;
    return true;
  }
  bool arr_next(bool& first) {
    ws();
    if (p_ >= e_) return fail();
    if (*p_ == ']') {
      ++p_;
      return false;
    }
    if (!first) {
      if (*p_ != ',') return fail();
      ++p_;
    }
    first = false;
    return true;
  }

  bool skip() {
    JK k = peek();
    std::string sc;
    std::string_view sv;
    switch (k) {
      case JK::Null: return null();
      case JK::Bool: {
        bool b;
        return boolean(&b);
      }
      case JK::Num: {
        JNum n;
        return number(&n);
      }
      case JK::Str: return skip_str();
      case JK::Arr:
      case JK::Obj: {
        // bracket matching with string awareness ('[' / ']' are '{' / '}' without bit 5, and
        // only structural bytes are visited)
        int depth = 0;
        while ((p_ = jscan_struct(p_, e_)) < e_) {
          const char c = *p_;
          if (c == '"') {
            if (!skip_str()) return false;
            continue;
          }
          ++p_;
          if ((c | 0x20) == '{') ++depth;
          else if (--depth == 0) return true;
        }
        return fail();
      }
      default: return fail();
    }
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  bool fail() {
    ok_ = false;
    p_ = e_;
    return false;
  }

 private:
  const char* p_;
  const char* e_;
  bool ok_ = true;

  bool skip_str() {
    ws();
    if (p_ >= e_ || *p_ != '"') return fail();
    ++p_;
    while ((p_ = jscan_quote(p_, e_)) < e_) {
      if (*p_++ == '"') return true;
      if (p_ >= e_) return fail();  // a backslash: skip the escaped byte
      ++p_;
    }
    return fail();
  }
  bool hex4(uint32_t* v) {
    if (e_ - p_ < 4) return false;
    *v = 0;
    for (int k = 0; k < 4; ++k) {
      char c = *p_++;
      *v <<= 4;
      if (c >= '0' && c <= '9') *v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') *v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') *v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    return true;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out.push_back((char)cp);
    else if (cp < 0x800) {
      out.push_back((char)(0xC0 | (cp >> 6)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back((char)(0xE0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      out.push_back((char)(0xF0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
};

// ASCII case fold compare: `key` (any case) equals `lower` (already lower case).
inline bool keq_n(std::string_view key, const char* lower, size_t n) {
  if (key.size() != n) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = key[i];
    if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    if (c != lower[i]) return false;
  }
  return true;
}
// a literal name: the length test is inlined at the call site (most keys differ in length)
template <size_t N>
__attribute__((always_inline)) inline bool keq(std::string_view key, const char (&lower)[N]) {
  return key.size() == N - 1 && keq_n(key, lower, N - 1);
}
inline bool keq(std::string_view key, const std::string& lower) { return keq_n(key, lower.data(), lower.size()); }

}  // namespace kpe
