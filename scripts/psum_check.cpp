// Host restatement of the per-pod PSA summary the device builds (kyverno_amd/csrc/lean.inl
// kpe_psa_dict_kernel / kpe_psa_capset_kernel / kpe_psum_kernel), for its digest test
// (tests/test_psum.py) without a GPU. Not part of libkpe:
//   scripts/build/psum_check resources.ndjson out.bin
// Flattens the resources with the product flattener and writes 2 words per row (schema.h PS_*):
// x = OR of the pod's container state bitmaps, y = capability-set bits | volume codes << 3 |
// sysctl codes << 5 | annotation codes << 8 | a container seccomp annotation not allowed << 10,
// each code taken under the PSA library's fixed sets (pss_fixed.hpp) from the list items in the
// corpus's CSR columns.
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../kyverno_amd/csrc/corpus.hpp"
#include "../kyverno_amd/csrc/pss_fixed.hpp"
#include "../kyverno_amd/csrc/schema.h"

namespace kpe {
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs);
}  // namespace kpe

using namespace kpe;

static std::vector<uint32_t> summary(const Corpus& C) {
  const int64_t n = C.n;
  std::vector<uint32_t> ps((size_t)n * 2, 0u);
  const Dict& capd = C.dict[D_CAP];
  uint64_t ok = 0, nbs = 0, all = 0;
  for (uint32_t i = 0; i < capd.size() && i < 64; ++i) {
    const std::string c(capd.at(i));
    if (pssfix::fixed_match(pssfix::kCapsBaselineOk, c)) ok |= 1ull << i;
    if (pssfix::fixed_match(pssfix::kCapNbs, c)) nbs |= 1ull << i;
    if (pssfix::fixed_match(pssfix::kCapAll, c)) all |= 1ull << i;
  }
  // kernels.hip CS_BASE / CS_DROP / CS_ADD per capability set
  std::vector<uint8_t> csb(C.capset_add.size());
  for (size_t j = 0; j < csb.size(); ++j) {
    const uint64_t ad = C.capset_add[j], dr = C.capset_drop[j];
    csb[j] = (uint8_t)(((ad & ~ok) ? 1u : 0u) | ((dr & all) ? 0u : 2u) | ((ad & ~nbs) ? 4u : 0u));
  }
  const Dict& sysd = C.dict[D_SYSCTL];
  std::vector<uint8_t> sysb(sysd.size());
  const std::vector<std::string> sv[3] = {pssfix::sysctls(0), pssfix::sysctls(1), pssfix::sysctls(2)};
  for (uint32_t i = 0; i < sysd.size(); ++i) {
    const std::string x(sysd.at(i));
    for (int v = 0; v < 3; ++v) sysb[i] |= pssfix::fixed_match(sv[v], x) ? 0u : (uint8_t)(1u << v);
  }
  const Dict &akd = C.dict[D_ANNK], &avd = C.dict[D_ANNV];
  std::vector<uint8_t> ak(akd.size()), av(avd.size());
  for (uint32_t i = 0; i < akd.size(); ++i) {
    const std::string x(akd.at(i));
    ak[i] = (pssfix::fixed_match(pssfix::kApparmorKey, x) ? 1u : 0u) |
            (pssfix::fixed_match(pssfix::kSeccompPodKey, x) ? 2u : 0u);
  }
  for (uint32_t i = 0; i < avd.size(); ++i) {
    const std::string x(avd.at(i));
    av[i] = (pssfix::fixed_match(pssfix::kApparmorOk, x) ? 1u : 0u) |
            (pssfix::fixed_match(pssfix::kSeccompAnnOk, x) ? 2u : 0u);
  }
  for (int64_t r = 0; r < n; ++r) {
    uint32_t xo = 0, co = 0, vc = 0, sc = 0, ac = 0, sa = 0;
    for (uint32_t k = C.ctr_off[r]; k < C.ctr_off[r + 1]; ++k) {
      const uint32_t x = C.crec[2 * k];
      xo |= x;
      if (x) co |= csb[CY_CAPSET(C.crec[2 * k + 1])];
      const uint32_t cs = C.c_sann[k];  // container seccomp annotation: bad unless an allowed profile
      if (cs != KPE_NO_STR && !(cs < av.size() && (av[cs] & 2u))) sa = 1u;
    }
    for (uint32_t k = C.vol_off[r]; k < C.vol_off[r + 1]; ++k) {
      const uint32_t v = C.vol_src[k];
      vc |= ((v >> VS_HOSTPATH) & 1u) | ((v & PSS_ALLOWED_VOLUMES) ? 0u : 2u);
    }
    for (uint32_t k = C.sys_off[r]; k < C.sys_off[r + 1]; ++k) sc |= C.sys_id[k] < sysb.size() ? sysb[C.sys_id[k]] : 7u;
    for (uint32_t k = C.pann_off[r]; k < C.pann_off[r + 1]; ++k) {
      const uint32_t kk = C.pann_k[k], vv = C.pann_v[k];
      const uint32_t a = kk < ak.size() ? ak[kk] : 0u, b = vv < av.size() ? av[vv] : 0u;
      ac |= ((a & 1u) && !(b & 1u) ? 1u : 0u) | ((a & 2u) && !(b & 2u) ? 2u : 0u);
    }
    ps[2 * r] = xo;
    ps[2 * r + 1] = co | (vc << 3) | (sc << 5) | (ac << 8) | (sa << 10);
  }
  return ps;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: psum_check resources.ndjson out.bin\n");
    return 2;
  }
  std::ifstream f(argv[1], std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string nd = ss.str();
  Corpus C;
  flatten_ndjson(C, nd.data(), nd.size(), nullptr, 0, false);
  const std::vector<uint32_t> ps = summary(C);
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 1;
  if (!ps.empty()) fwrite(ps.data(), 4, ps.size(), o);
  fclose(o);
  return 0;
}
