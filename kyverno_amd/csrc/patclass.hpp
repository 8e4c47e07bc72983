// Host-side classification of a go-wildcard pattern into a device pattern record
// (kernels_abi.h PK_*): the common shapes get literal compares, the rest the full glob.
#pragma once
#include <algorithm>
#include <string>
#include <vector>

#include "kernels_abi.h"

namespace kpe {

inline KpePat classify_pattern(const std::string& g, std::vector<uint8_t>& bytes) {
  KpePat p{PK_GLOB, (uint32_t)bytes.size(), 0, 0};
  auto put = [&](const std::string& lit) {
    p.off = (uint32_t)bytes.size();
    p.len = (uint32_t)lit.size();
    bytes.insert(bytes.end(), lit.begin(), lit.end());
  };
  size_t stars = std::count(g.begin(), g.end(), '*');
  bool q = g.find('?') != std::string::npos;
  if (g == "*") p.kind = PK_ANY;
  else if (!q && stars == 0) p.kind = PK_EXACT;
  else if (!q && stars == 1 && g.back() == '*') p.kind = PK_PREFIX;
  else if (!q && stars == 1 && g.front() == '*') p.kind = PK_SUFFIX;
  else if (!q && stars == 2 && g.size() >= 2 && g.front() == '*' && g.back() == '*') p.kind = PK_CONTAINS;
  else if (stars >= 1 && std::count(g.begin(), g.end(), '?') == 1 && stars + 1 == g.size()) p.kind = PK_NONEMPTY;
  switch (p.kind) {
    case PK_ANY: put(""); break;
    case PK_EXACT: put(g); break;
    case PK_PREFIX: put(g.substr(0, g.size() - 1)); break;
    case PK_SUFFIX: put(g.substr(1)); break;
    case PK_CONTAINS: put(g.substr(1, g.size() - 2)); break;
    default: put(g);
  }
  return p;
}

}  // namespace kpe
