// Resource hashes for incremental background scans: CalculateResourceHash
// (pkg/utils/report/metadata.go:137-155) restated. The background controller compares this hash
// with the one recorded on the resource's report to decide whether the resource needs a rescan
// (pkg/controllers/report/background/controller.go:247-297, needsReconcile).
//
//   copy := resource.DeepCopy(); labels := GetLabels(); annotations := GetAnnotations()
//   RemoveNestedField(obj, "metadata"), ("status"), ("scale"), ("spec", "nodeName")
//   md5(json.Marshal([]interface{}{labels, annotations, obj})) as lower-case hex
//
// The resource goes through the unstructured decode first (k8s.io/apimachinery utiljson: a
// number literal that strconv.ParseInt accepts is an int64, every other number a float64), then
// Go 1.21 encoding/json: object keys sorted bytewise, the last of duplicate keys kept, HTML
// characters and U+2028/U+2029 escaped, control characters as \n \r \t or \u00XX, float64 in
// strconv 'f' / 'e' (exponent < -6 or >= 21) shortest form. GetLabels / GetAnnotations are
// NestedStringMap: nil (JSON null) unless metadata.<field> is a map of strings.
#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kpe.h"
#include "jscan.hpp"

namespace {

struct Node {
  enum T : uint8_t { Null, Bool, Int, Flt, Str, Arr, Obj } t = Null;
  bool b = false;
  int64_t i = 0;
  double f = 0;
  std::string s;
  std::vector<Node> a;
  std::vector<std::pair<std::string, Node>> o;  // unique keys (last wins)
  Node* get(const char* k) {
    if (t != Obj) return nullptr;
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  void erase(const char* k) {
    if (t != Obj) return;
    for (size_t j = 0; j < o.size(); ++j)
      if (o[j].first == k) {
        o.erase(o.begin() + (long)j);
        return;
      }
  }
};

bool parse(kpe::JCur& c, Node& n, int depth) {
  if (depth > 10000) return false;
  std::string sc;
  switch (c.peek()) {
    case kpe::JK::Null: n.t = Node::Null; return c.null();
    case kpe::JK::Bool: n.t = Node::Bool; return c.boolean(&n.b);
    case kpe::JK::Num: {
      kpe::JNum x;
      if (!c.number(&x)) return false;
      if (x.is_int) n.t = Node::Int, n.i = x.i;
      else n.t = Node::Flt, n.f = x.f;
      return true;
    }
    case kpe::JK::Str: {
      std::string_view v;
      if (!c.str(&v, sc)) return false;
      n.t = Node::Str, n.s.assign(v);
      return true;
    }
    case kpe::JK::Arr: {
      n.t = Node::Arr;
      if (!c.arr_begin()) return false;
      bool first = true;
      while (c.arr_next(first)) {
        n.a.emplace_back();
        if (!parse(c, n.a.back(), depth + 1)) return false;
      }
      return c.ok();
    }
    case kpe::JK::Obj: {
      n.t = Node::Obj;
      if (!c.obj_begin()) return false;
      bool first = true;
      std::string_view k;
      std::string ks;
      while (c.obj_next(first, &k, ks)) {
        std::string key(k);
        Node child;
        if (!parse(c, child, depth + 1)) return false;
        Node* prev = n.get(key.c_str());
        if (prev) *prev = std::move(child);  // a Go map decode keeps the last duplicate
        else n.o.emplace_back(std::move(key), std::move(child));
      }
      return c.ok();
    }
    default: return false;
  }
}

// encoding/json encodeState.string (Go 1.21, escapeHTML = true)
void put_str(const std::string& s, std::string& out) {
  static const char* hex = "0123456789abcdef";
  out += '"';
  const auto* p = reinterpret_cast<const unsigned char*>(s.data());
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const unsigned char b = p[i];
    if (b < 0x80) {
      if (b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&') {
        out += (char)b;
      } else if (b == '"' || b == '\\') {
        out += '\\', out += (char)b;
      } else if (b == '\n') {
        out += "\\n";
      } else if (b == '\r') {
        out += "\\r";
      } else if (b == '\t') {
        out += "\\t";
      } else {
        out += "\\u00", out += hex[b >> 4], out += hex[b & 15];
      }
      ++i;
      continue;
    }
    // one UTF-8 sequence; an invalid byte became U+FFFD when the decoder read the string
    uint32_t cp = 0;
    size_t len = 0;
    if ((b & 0xE0) == 0xC0) cp = b & 0x1F, len = 2;
    else if ((b & 0xF0) == 0xE0) cp = b & 0x0F, len = 3;
    else if ((b & 0xF8) == 0xF0) cp = b & 0x07, len = 4;
    bool ok = len && i + len <= n;
    for (size_t k = 1; ok && k < len; ++k) {
      if ((p[i + k] & 0xC0) != 0x80) ok = false;
      cp = (cp << 6) | (p[i + k] & 0x3F);
    }
    if (ok && ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)) ||
               (cp >= 0xD800 && cp < 0xE000)))
      ok = false;
    if (!ok) {
      out += "\xEF\xBF\xBD";
      ++i;
      continue;
    }
    if (cp == 0x2028 || cp == 0x2029) out += cp == 0x2028 ? "\\u2028" : "\\u2029";
    else out.append(reinterpret_cast<const char*>(p + i), len);
    i += len;
  }
  out += '"';
}

// encoding/json floatEncoder (64-bit)
void put_float(double f, std::string& out) {
  char buf[64];
  const double a = f < 0 ? -f : f;
  const bool sci = a != 0 && (a < 1e-6 || a >= 1e21);
  auto r = std::to_chars(buf, buf + sizeof buf, f, sci ? std::chars_format::scientific : std::chars_format::fixed);
  std::string s(buf, r.ptr);
  if (sci) {  // clean up e-09 to e-9
    const size_t m = s.size();
    if (m >= 4 && s[m - 4] == 'e' && s[m - 3] == '-' && s[m - 2] == '0') s.erase(m - 2, 1);
  }
  out += s;
}

void marshal(const Node& n, std::string& out) {
  switch (n.t) {
    case Node::Null: out += "null"; break;
    case Node::Bool: out += n.b ? "true" : "false"; break;
    case Node::Int: out += std::to_string(n.i); break;
    case Node::Flt: put_float(n.f, out); break;
    case Node::Str: put_str(n.s, out); break;
    case Node::Arr:
      out += '[';
      for (size_t k = 0; k < n.a.size(); ++k) {
        if (k) out += ',';
        marshal(n.a[k], out);
      }
      out += ']';
      break;
    case Node::Obj: {
      std::vector<const std::pair<std::string, Node>*> kv;
      for (auto& e : n.o) kv.push_back(&e);
      std::sort(kv.begin(), kv.end(), [](auto* x, auto* y) { return x->first < y->first; });
      out += '{';
      for (size_t k = 0; k < kv.size(); ++k) {
        if (k) out += ',';
        put_str(kv[k]->first, out);
        out += ':';
        marshal(kv[k]->second, out);
      }
      out += '}';
      break;
    }
  }
}

// RFC 1321 MD5
struct Md5 {
  uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
  void block(const uint8_t* p) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
        0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
        0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
        0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
        0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
        0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
        0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
    static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 5, 9,  14, 20, 5, 9,
                              14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              4, 11, 16, 23, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t M[16];
    for (int j = 0; j < 16; ++j)
      M[j] = (uint32_t)p[4 * j] | (uint32_t)p[4 * j + 1] << 8 | (uint32_t)p[4 * j + 2] << 16 | (uint32_t)p[4 * j + 3] << 24;
    uint32_t A = h[0], B = h[1], C = h[2], D = h[3];
    for (int j = 0; j < 64; ++j) {
      uint32_t F;
      int g;
      if (j < 16) F = (B & C) | (~B & D), g = j;
      else if (j < 32) F = (D & B) | (~D & C), g = (5 * j + 1) & 15;
      else if (j < 48) F = B ^ C ^ D, g = (3 * j + 5) & 15;
      else F = C ^ (B | ~D), g = (7 * j) & 15;
      F = F + A + K[j] + M[g];
      A = D, D = C, C = B;
      B = B + ((F << S[j]) | (F >> (32 - S[j])));
    }
    h[0] += A, h[1] += B, h[2] += C, h[3] += D;
  }
  void hex(const std::string& s, char out[33]) {
    const auto* p = reinterpret_cast<const uint8_t*>(s.data());
    const size_t n = s.size();
    size_t i = 0;
    for (; i + 64 <= n; i += 64) block(p + i);
    uint8_t tail[128] = {0};
    const size_t r = n - i;
    memcpy(tail, p + i, r);
    tail[r] = 0x80;
    const size_t tl = r + 9 <= 64 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int k = 0; k < 8; ++k) tail[tl - 8 + k] = (uint8_t)(bits >> (8 * k));
    block(tail);
    if (tl == 128) block(tail + 64);
    static const char* hx = "0123456789abcdef";
    for (int k = 0; k < 16; ++k) {
      const uint8_t byte = (uint8_t)(h[k / 4] >> (8 * (k % 4)));
      out[2 * k] = hx[byte >> 4], out[2 * k + 1] = hx[byte & 15];
    }
    out[32] = 0;
  }
};

// NestedStringMap(obj, "metadata", field): the map when every value is a string, else nil
void string_map(Node* meta, const char* field, std::string& out) {
  Node* m = meta ? meta->get(field) : nullptr;
  bool ok = m && m->t == Node::Obj;
  if (ok)
    for (auto& kv : m->o) ok = ok && kv.second.t == Node::Str;
  if (ok) marshal(*m, out);
  else out += "null";
}

bool resource_hash(const char* p, size_t n, char out[33]) {
  kpe::JCur c(p, p + n);
  Node root;
  if (!parse(c, root, 0) || root.t != Node::Obj) return false;
  c.ws();
  if (c.peek() != kpe::JK::End) return false;
  Node* meta = root.get("metadata");
  if (meta && meta->t != Node::Obj) meta = nullptr;
  std::string s = "[";
  string_map(meta, "labels", s);
  s += ',';
  string_map(meta, "annotations", s);
  s += ',';
  root.erase("metadata");
  root.erase("status");
  root.erase("scale");
  if (Node* spec = root.get("spec")) spec->erase("nodeName");
  marshal(root, s);
  s += ']';
  Md5 m;
  m.hex(s, out);
  return true;
}

}  // namespace

extern "C" kpe_status kpe_resource_hash(const char* json, size_t len, char* out33) {
  if (!json || !out33) return KPE_E_INVALID;
  return resource_hash(json, len, out33) ? KPE_OK : KPE_E_INVALID;
}

extern "C" int64_t kpe_resource_hashes(const char* ndjson, size_t len, char* out, int64_t cap_rows) {
  if (!ndjson) return -KPE_E_INVALID;
  std::vector<std::pair<const char*, size_t>> lines;
  for (size_t i = 0; i < len;) {
    size_t j = i;
    while (j < len && ndjson[j] != '\n') ++j;
    size_t a = i, b = j;
    while (a < b && (ndjson[a] == ' ' || ndjson[a] == '\t' || ndjson[a] == '\r')) ++a;
    while (b > a && (ndjson[b - 1] == ' ' || ndjson[b - 1] == '\t' || ndjson[b - 1] == '\r')) --b;
    if (b > a) lines.emplace_back(ndjson + a, b - a);
    i = j + 1;
  }
  const int64_t nl = (int64_t)lines.size();
  if (!out) return nl;
  if (cap_rows < nl) return -KPE_E_INVALID;
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int64_t r = t; r < nl; r += nt) {
        char h[33];
        if (!resource_hash(lines[r].first, lines[r].second, h)) memset(out + r * 32, '-', 32);  // no hash
        else memcpy(out + r * 32, h, 32);
      }
    });
  for (auto& x : th) x.join();
  return nl;
}
