// ORACLE — test infrastructure only. Never linked into the product path.
//
// ext/wildcard/match.go:7-9 -> github.com/IGLOU-EU/go-wildcard v1.0.3 (go.mod:8),
// absent from /root/reference. Restated published semantics: glob over runes,
// '*' = any sequence (incl. empty), '?' = exactly one rune, "" matches only "",
// "*" matches anything. Pinned by ext/wildcard/match_test.go (52 vectors) and
// ext/wildcard/utils_test.go (CheckPatterns/MatchPatterns); non-ASCII rune
// behaviour is unpinned.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace oracle {

inline std::vector<uint32_t> runes(const std::string& s) {
  std::vector<uint32_t> r;
  for (size_t i = 0; i < s.size();) {
    unsigned char c = (unsigned char)s[i];
    uint32_t cp;
    int n;
    if (c < 0x80) { cp = c; n = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; n = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; n = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; n = 4; }
    else { r.push_back(0xFFFD); ++i; continue; }
    if (i + n > s.size()) { r.push_back(0xFFFD); ++i; continue; }
    bool ok = true;
    for (int k = 1; k < n; ++k) {
      unsigned char d = (unsigned char)s[i + k];
      if ((d >> 6) != 2) { ok = false; break; }
      cp = (cp << 6) | (d & 0x3F);
    }
    if (!ok) { r.push_back(0xFFFD); ++i; continue; }
    r.push_back(cp);
    i += n;
  }
  return r;
}

// Backtracking glob (last-star restart), linear for single-star patterns.
inline bool wildcard_match(const std::string& pattern, const std::string& name) {
  if (pattern.empty()) return name.empty();
  if (pattern == "*") return true;
  std::vector<uint32_t> p = runes(pattern), s = runes(name);
  size_t pi = 0, si = 0, star = SIZE_MAX, mark = 0;
  while (si < s.size()) {
    if (pi < p.size() && (p[pi] == '?' || (p[pi] != '*' && p[pi] == s[si]))) {
      ++pi;
      ++si;
    } else if (pi < p.size() && p[pi] == '*') {
      star = pi++;
      mark = si;
    } else if (star != SIZE_MAX) {
      pi = star + 1;
      si = ++mark;
    } else {
      return false;
    }
  }
  while (pi < p.size() && p[pi] == '*') ++pi;
  return pi == p.size();
}

// ext/wildcard/utils.go:12-27
inline bool check_patterns(const std::vector<std::string>& patterns, const std::string& name) {
  for (auto& p : patterns)
    if (wildcard_match(p, name)) return true;
  return false;
}

}  // namespace oracle
