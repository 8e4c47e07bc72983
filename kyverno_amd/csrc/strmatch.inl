// go-wildcard v1.0.3 glob and k8s validation predicates over byte strings. Device code
// (included by kernels.hip inside its anonymous namespace); also compiled for the host by
// scripts/patvm_check.cpp so the pattern VM can be exercised under sanitizers.

// ---------------------------------------------------------------------------
// go-wildcard v1.0.3 over UTF-8: '*' any rune sequence, '?' exactly one rune.
__device__ __forceinline__ int rune_len(const uint8_t* s, int i, int n) {
  uint8_t c = s[i];
  int l = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
  if (i + l > n) return 1;
  for (int k = 1; k < l; ++k)
    if ((s[i + k] >> 6) != 2) return 1;  // invalid sequence: one byte = one (U+FFFD) rune
  return l;
}

__device__ bool glob(const uint8_t* p, int pn, const uint8_t* s, int sn) {
  if (pn == 0) return sn == 0;
  int pi = 0, si = 0, star = -1, mark = 0;
  while (si < sn) {
    if (pi < pn && p[pi] == '?') {
      ++pi;
      si += rune_len(s, si, sn);
    } else if (pi < pn && p[pi] == '*') {
      star = pi++;
      mark = si;
    } else if (pi < pn && p[pi] == s[si]) {
      ++pi;
      ++si;
    } else if (star >= 0) {
      pi = star + 1;
      mark += rune_len(s, mark, sn);
      si = mark;
    } else {
      return false;
    }
  }
  while (pi < pn && p[pi] == '*') ++pi;
  return pi == pn;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, const uint8_t* b, int n) {
  int i = 0;
  for (; i + 8 <= n; i += 8) {  // 8 independent byte loads per step: short dependence chains
    uint32_t d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d |= (uint32_t)(a[i + k] ^ b[i + k]);
    if (d) return false;
  }
  uint32_t d = 0;
  for (; i < n; ++i) d |= (uint32_t)(a[i] ^ b[i]);
  return d == 0;
}

// k8s.io/apimachinery v0.29.1 util/validation (IsQualifiedName / IsValidLabelValue)
__device__ __forceinline__ bool qn_char(uint8_t c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9');
}
__device__ bool name_part_ok(const uint8_t* s, int n) {
  if (n == 0 || n > 63 || !qn_char(s[0]) || !qn_char(s[n - 1])) return false;
  for (int i = 0; i < n; ++i)
    if (!(qn_char(s[i]) || s[i] == '-' || s[i] == '_' || s[i] == '.')) return false;
  return true;
}
__device__ bool dns1123_subdomain_ok(const uint8_t* s, int n) {
  if (n == 0 || n > 253) return false;
  int start = 0;
  for (int i = 0; i <= n; ++i) {
    if (i == n || s[i] == '.') {
      if (i == start) return false;
      start = i + 1;
      continue;
    }
    const uint8_t c = s[i];
    const bool an = (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9');
    if (!(an || (c == '-' && i != start && i + 1 < n && s[i + 1] != '.'))) return false;
  }
  return true;
}
__device__ bool qualified_name_ok(const uint8_t* s, int n) {
  int slash = -1;
  for (int i = 0; i < n; ++i)
    if (s[i] == '/') {
      if (slash >= 0) return false;
      slash = i;
    }
  if (slash < 0) return name_part_ok(s, n);
  return dns1123_subdomain_ok(s, slash) && name_part_ok(s + slash + 1, n - slash - 1);
}

__device__ bool pat_match(const KpePat& pt, const uint8_t* pb, const uint8_t* s, int sn) {
  const uint8_t* lit = pb + pt.off;
  const int ln = (int)pt.len;
  switch (pt.kind) {
    case PK_ANY: return true;
    case PK_EXACT: return sn == ln && bytes_eq(lit, s, ln);
    case PK_PREFIX: return sn >= ln && bytes_eq(lit, s, ln);
    case PK_SUFFIX: return sn >= ln && bytes_eq(lit, s + sn - ln, ln);
    case PK_CONTAINS:
      for (int i = 0; i + ln <= sn; ++i)
        if (bytes_eq(lit, s + i, ln)) return true;
      return false;
    case PK_QNAME: return qualified_name_ok(s, sn);
    case PK_LABVAL: return sn == 0 || name_part_ok(s, sn);
    case PK_NONEMPTY: return sn > 0;
    default: return glob(lit, ln, s, sn);
  }
}

