// Image references for the `images` context (pkg/utils/image/infos.go:48-100 GetImageInfo):
// github.com/distribution/reference v0.5.0 Parse (go.mod:17) over its grammar
//   reference := name [":" tag] ["@" digest];  name := [domain-and-port "/"] remote-name
//   domain-and-port := (domain-name | "[" [a-fA-F0-9:]+ "]") [":" [0-9]+]
//   domain-name := component ("." component)*;  component := [a-zA-Z0-9] | [a-zA-Z0-9][a-zA-Z0-9-]*[a-zA-Z0-9]
//   remote-name := path-component ("/" path-component)*
//   path-component := [a-z0-9]+ (("." | "_" | "__" | "-"+) [a-z0-9]+)*
//   tag := [\w][\w.-]{0,127};  digest := [A-Za-z][A-Za-z0-9]*([-_+.][A-Za-z][A-Za-z0-9]*)* ":" [0-9A-Fa-f]{32,}
// and github.com/opencontainers/go-digest v1.0.0 Digest.Validate (go.mod:40): sha256 / sha384 /
// sha512 with exactly 64 / 96 / 128 lower-case hex digits. Hand-written (no regex): the optional
// domain is the first "/"-segment whenever it is a domain-and-port (the regexp's preferred
// alternative; when that split fails the name has no valid parse either).
#pragma once
#include <string>
#include <string_view>

namespace kpe {
namespace imageref {

struct Info {
  std::string registry, path, name, tag, digest;
};

inline bool lower_alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }
inline bool alnum(char c) { return lower_alnum(c) || (c >= 'A' && c <= 'Z'); }
inline bool word(char c) { return alnum(c) || c == '_'; }

inline bool path_component(std::string_view s) {
  size_t i = 0;
  const size_t n = s.size();
  for (;;) {
    if (i >= n || !lower_alnum(s[i])) return false;
    while (i < n && lower_alnum(s[i])) ++i;
    if (i == n) return true;
    if (s[i] == '.') {
      ++i;
    } else if (s[i] == '_') {
      ++i;
      if (i < n && s[i] == '_') ++i;
    } else if (s[i] == '-') {
      while (i < n && s[i] == '-') ++i;
    } else {
      return false;
    }
  }
}
inline bool remote_name(std::string_view s) {
  size_t a = 0;
  for (;;) {
    const size_t b = s.find('/', a);
    if (!path_component(s.substr(a, b == std::string_view::npos ? std::string_view::npos : b - a))) return false;
    if (b == std::string_view::npos) return true;
    a = b + 1;
  }
}
inline bool domain_component(std::string_view s) {
  if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-')) return false;
  return true;
}
inline bool domain_and_port(std::string_view s) {
  std::string_view host = s;
  size_t close = std::string_view::npos;
  if (!s.empty() && s[0] == '[') {
    close = s.find(']');
    if (close == std::string_view::npos || close < 2) return false;
    for (size_t i = 1; i < close; ++i) {
      const char c = s[i];
      if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F') || c == ':')) return false;
    }
    host = s.substr(0, close + 1);
  }
  const size_t colon = s.find(':', close == std::string_view::npos ? 0 : close + 1);
  if (colon != std::string_view::npos) {
    if (close == std::string_view::npos) host = s.substr(0, colon);
    else if (colon != close + 1) return false;
    std::string_view port = s.substr(colon + 1);
    if (port.empty()) return false;
    for (char c : port)
      if (c < '0' || c > '9') return false;
  } else if (close != std::string_view::npos && close + 1 != s.size()) {
    return false;
  }
  if (close != std::string_view::npos) return true;
  size_t a = 0;
  for (;;) {
    const size_t b = host.find('.', a);
    if (!domain_component(host.substr(a, b == std::string_view::npos ? std::string_view::npos : b - a))) return false;
    if (b == std::string_view::npos) return true;
    a = b + 1;
  }
}
inline bool tag_ok(std::string_view t) {
  if (t.empty() || t.size() > 128 || !word(t[0])) return false;
  for (char c : t)
    if (!(word(c) || c == '.' || c == '-')) return false;
  return true;
}
inline bool digest_grammar(std::string_view d) {
  const size_t colon = d.find(':');
  if (colon == std::string_view::npos) return false;
  std::string_view alg = d.substr(0, colon), hex = d.substr(colon + 1);
  if (hex.size() < 32) return false;
  for (char c : hex)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'))) return false;
  size_t i = 0;
  for (;;) {  // [A-Za-z][A-Za-z0-9]* components joined by [-_+.]
    if (i >= alg.size() || !((alg[i] >= 'a' && alg[i] <= 'z') || (alg[i] >= 'A' && alg[i] <= 'Z'))) return false;
    ++i;
    while (i < alg.size() && alnum(alg[i])) ++i;
    if (i == alg.size()) return true;
    if (alg[i] != '-' && alg[i] != '_' && alg[i] != '+' && alg[i] != '.') return false;
    ++i;
  }
}
inline bool digest_valid(std::string_view d) {  // go-digest Validate of an available algorithm
  const size_t colon = d.find(':');
  std::string_view alg = d.substr(0, colon), hex = d.substr(colon + 1);
  const size_t want = alg == "sha256" ? 64 : alg == "sha384" ? 96 : alg == "sha512" ? 128 : 0;
  if (!want || hex.size() != want) return false;
  for (char c : hex)
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  return true;
}
// reference.Parse; false: an error
inline bool parse(std::string_view s, std::string_view* domain, std::string_view* path, std::string_view* tag,
                  std::string_view* digest) {
  *domain = *path = *tag = *digest = std::string_view();
  std::string_view rest = s;
  const size_t at = s.find('@');
  if (at != std::string_view::npos) {
    *digest = s.substr(at + 1);
    rest = s.substr(0, at);
    if (!digest_grammar(*digest)) return false;
  }
  std::string_view name = rest, remote;
  const size_t slash = rest.find('/');
  if (slash != std::string_view::npos && domain_and_port(rest.substr(0, slash))) {
    *domain = rest.substr(0, slash);
    std::string_view rem = rest.substr(slash + 1);
    const size_t c = rem.find(':');
    remote = c == std::string_view::npos ? rem : rem.substr(0, c);
    if (c != std::string_view::npos) {
      *tag = rem.substr(c + 1);
      if (!tag_ok(*tag)) return false;
    }
    name = rest.substr(0, slash + 1 + remote.size());
  } else {
    const size_t c = rest.find(':');
    remote = c == std::string_view::npos ? rest : rest.substr(0, c);
    if (c != std::string_view::npos) {
      *tag = rest.substr(c + 1);
      if (!tag_ok(*tag)) return false;
    }
    name = remote;
  }
  if (!remote_name(remote)) return false;
  if (name.size() > 255) return false;  // ErrNameTooLong
  if (!digest->empty() && !digest_valid(*digest)) return false;
  *path = remote;
  return true;
}
// GetImageInfo with the default configuration (defaultRegistry docker.io, registry mutation on)
inline bool image_info(std::string_view image, Info* out) {
  std::string full(image);
  const size_t i = image.find('/');
  bool prefix = i == std::string_view::npos;
  if (!prefix) {
    std::string_view first = image.substr(0, i);
    bool lower = true;
    for (char c : first) lower = lower && !(c >= 'A' && c <= 'Z');
    prefix = first.find_first_of(".:") == std::string_view::npos && first != "localhost" && lower;
  }
  if (prefix) full = "docker.io/" + full;
  std::string_view d, p, t, g;
  if (!parse(full, &d, &p, &t, &g)) return false;
  out->registry.assign(d);
  out->path.assign(p);
  const size_t ls = out->path.rfind('/');
  out->name = ls == std::string::npos ? out->path : out->path.substr(ls + 1);
  out->tag.assign(t);
  out->digest.assign(g);
  if (out->tag.empty() && out->digest.empty()) out->tag = "latest";
  return true;
}

}  // namespace imageref
}  // namespace kpe
