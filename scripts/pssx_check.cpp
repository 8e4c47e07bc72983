// Host build of the podSecurity exclusion pass (kyverno_amd/csrc/pssx.inl, the exact text
// kpe_pssx_kernel runs) for sanitizer runs and parity checks without a GPU:
//   scripts/build/pssx_check policies.json resources.ndjson seed.bin out.bin [exceptions.json]
// Flattens the resources, compiles the policies, evaluates the predicates the pass reads on
// the host (go-wildcard globs over the corpus dictionaries, the pbuf layout of kpe_api.cpp)
// and binds the exclusion tables the way kpe_api.cpp does, then runs pssx_eval_row over a
// verdict matrix seeded from seed.bin (N x R bytes: the plain PSS verdicts the scan kernel
// writes, i.e. the rules' verdicts without their exclusions, KPE_XFAIL_ where a podSecurity
// PolicyException matched). Writes N x R verdicts to out.bin.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#define __device__
#define __forceinline__ inline
struct uint2 {
  uint32_t x, y;
};
struct uint4 {
  uint32_t x, y, z, w;
};
inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }
inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return uint4{x, y, z, w}; }

#include "../kyverno_amd/csrc/corpus.hpp"
#include "../kyverno_amd/csrc/kernels_abi.h"
#include "../kyverno_amd/csrc/program.hpp"
#include "../kyverno_amd/csrc/schema.h"

namespace kpe {
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs);
}  // namespace kpe

// go-wildcard v1.0.3 Match over runes ('*' any run, '?' one rune): recursive, test inputs are small
static std::vector<uint32_t> runes(const std::string& x) {
  std::vector<uint32_t> r;
  for (size_t i = 0; i < x.size();) {
    const unsigned char c = (unsigned char)x[i];
    const size_t n = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 1;
    uint32_t cp = 0;
    for (size_t k = 0; k < n && i + k < x.size(); ++k) cp = cp << 8 | (unsigned char)x[i + k];
    r.push_back(cp);
    i += n;
  }
  return r;
}
static bool wmatch(const std::vector<uint32_t>& p, size_t i, const std::vector<uint32_t>& s, size_t j) {
  if (i == p.size()) return j == s.size();
  if (p[i] == '*') return wmatch(p, i + 1, s, j) || (j < s.size() && wmatch(p, i, s, j + 1));
  return j < s.size() && (p[i] == '?' || p[i] == s[j]) && wmatch(p, i + 1, s, j + 1);
}
static bool glob(const std::string& pat, const std::string& s) {
  if (pat.empty()) return s.empty();
  return pat == "*" || wmatch(runes(pat), 0, runes(s), 0);
}

namespace {
#include "../kyverno_amd/csrc/pssx.inl"
}  // namespace

static std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot read ") + p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s policies.json resources.ndjson seed.bin out.bin\n", argv[0]);
    return 2;
  }
  const std::string pj = slurp(argv[1]), nd = slurp(argv[2]), seed = slurp(argv[3]);
  const std::string xj = argc > 5 ? slurp(argv[5]) : std::string();
  kpe::Corpus C;
  kpe::flatten_ndjson(C, nd.data(), nd.size(), nullptr, 0, false);
  auto P = kpe::compile_policies(pj.data(), pj.size(), xj.empty() ? nullptr : xj.data(), xj.size(), false);
  const uint32_t R = (uint32_t)P->rules.size();
  if (seed.size() != (size_t)C.n * R) return fprintf(stderr, "seed size %zu != %lld x %u\n", seed.size(), (long long)C.n, R), 1;
  std::vector<uint8_t> verdicts(seed.begin(), seed.end());
  // predicate bitsets (every predicate global: word(id >> 5), bit id & 31)
  std::vector<uint32_t> pbuf, loc(P->preds.size());
  for (size_t p = 0; p < P->preds.size(); ++p) {
    const auto& pr = P->preds[p];
    const kpe::Dict& d = C.dict[pr.domain];
    loc[p] = (uint32_t)pbuf.size();
    pbuf.resize(pbuf.size() + ((d.size() + 63) / 64) * 2 + 2, 0);
    for (uint32_t i = 0; i < d.size(); ++i) {
      bool hit = false;
      for (auto& g : pr.globs) hit = hit || glob(g, std::string(d.at(i)));
      if (hit) pbuf[loc[p] + (i >> 5)] |= 1u << (i & 31u);
    }
  }
  auto L = [&](int32_t p) { return p < 0 ? PRED_NONE : loc[(size_t)p]; };
  std::vector<KpeXExcl> xe = P->pssx.excl;
  for (auto& x : xe) {
    x.img = (int32_t)L(x.img);
    x.pv_misc = (int32_t)L(x.pv_misc), x.pv_annv = (int32_t)L(x.pv_annv);
    x.pv_sys = (int32_t)L(x.pv_sys), x.pv_cap = (int32_t)L(x.pv_cap);
  }
  const kpe::Dict& AK = C.dict[D_ANNK];
  std::unordered_map<std::string, uint32_t> nid;
  std::vector<uint32_t> norm(AK.size() + 1, KPE_NO_STR);
  for (uint32_t i = 0; i < AK.size(); ++i) {
    std::string o;
    const std::string k(AK.at(i));
    for (size_t j = 0; j < k.size();) {
      if (k[j] >= '0' && k[j] <= '9') {
        while (j < k.size() && k[j] >= '0' && k[j] <= '9') ++j;
        o += '*';
      } else {
        o += k[j++];
      }
    }
    norm[i] = nid.emplace(o, (uint32_t)nid.size()).first->second;
  }
  std::vector<uint32_t> rf(P->pssx.rf_ann.size() + 1, KPE_NO_STR);
  for (size_t i = 0; i < P->pssx.rf_ann.size(); ++i) {
    auto it = nid.find(P->pssx.rf_ann[i]);
    if (it != nid.end()) rf[i] = it->second;
  }
  std::vector<uint32_t> capsets;
  for (size_t i = 0; i < C.capset_add.size(); ++i) {
    capsets.push_back((uint32_t)C.capset_add[i]), capsets.push_back((uint32_t)(C.capset_add[i] >> 32));
    capsets.push_back((uint32_t)C.capset_drop[i]), capsets.push_back((uint32_t)(C.capset_drop[i] >> 32));
  }
  PssxArgs a{};
  a.n = C.n, a.R = R, a.nxr = (uint32_t)P->pssx.rules.size();
  a.rules = P->pssx.rules.data(), a.excl = xe.data();
  a.rec = C.rec.data(), a.ctr_off = C.ctr_off.data(), a.vol_off = C.vol_off.data(), a.sys_off = C.sys_off.data();
  a.pann_off = C.pann_off.data(), a.crec = C.crec.data(), a.capsets = capsets.data();
  a.c_name = C.c_name.data(), a.c_image = C.c_image.data(), a.c_sann = C.c_sann.data();
  a.c_sann_key = C.c_sann_key.data(), a.c_sec_str = C.c_sec_str.data(), a.c_pm_str = C.c_pm_str.data();
  a.c_selt_str = C.c_selt_str.data(), a.c_selu_str = C.c_selu_str.data(), a.c_selr_str = C.c_selr_str.data();
  a.cport_off = C.cport_off.data(), a.cport_str = C.cport_str.data(), a.vol_src = C.vol_src.data();
  a.sys_id = C.sys_id.data(), a.pann_k = C.pann_k.data(), a.pann_v = C.pann_v.data(), a.p_cold = C.p_cold.data();
  a.misc_off = C.dict[D_MISC].off.data(), a.annv_off = C.dict[D_ANNV].off.data();
  a.sysd_off = C.dict[D_SYSCTL].off.data();
  a.ann_norm = norm.data(), a.rf_ann = rf.data();
  const int64_t kp = AK.find("seccomp.security.alpha.kubernetes.io/pod");
  const int64_t kf = AK.find("container.seccomp.security.alpha.kubernetes.io/fake");
  a.key_pod_sec = kp < 0 ? KPE_NO_STR : (uint32_t)kp;
  a.key_fake_sec = kf < 0 ? KPE_NO_STR : (uint32_t)kf;
  a.pbuf = pbuf.data();
  const int32_t* g = P->pssx_preds;
  a.pp_apparmor_key = L(g[0]), a.pp_apparmor_ok = L(g[1]), a.pp_seccomp_ok = L(g[2]);
  a.pp_caps_ok = L(g[3]), a.pp_nbs = L(g[4]), a.pp_all = L(g[5]);
  for (int v = 0; v < 3; ++v) a.pp_sysctl[v] = L(g[6 + v]);
  a.verdicts = verdicts.data();
  a.masks = nullptr;
  for (int64_t r = 0; r < a.n; ++r) pssx_eval_row(a, r);  // kpe_pssx_kernel's lane body
  FILE* f = fopen(argv[4], "wb");
  fwrite(verdicts.data(), 1, verdicts.size(), f);
  fclose(f);
  printf("%lld %u\n", (long long)C.n, R);
  return 0;
}
