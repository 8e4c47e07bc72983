// Host build of the pattern VM (kyverno_amd/csrc/patvm.inl + strmatch.inl, the exact text
// kpe_pattern_kernel runs) for sanitizer runs without a GPU:
//   make -C scripts patvm_check && scripts/build/patvm_check policies.json resources.ndjson out.bin
// Flattens the resources with document tapes, compiles the policies, binds the pattern
// program the way kpe_api.cpp does (member names -> D_KEY ids, glob names -> bitsets,
// operand records) and evaluates every pattern cell as if the rule matched. Writes the
// N x R verdict bytes (non-pattern columns 0) to out.bin.
#include <cmath>
#include <cstdint>
#include <map>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#define __device__
#define __forceinline__ inline
#define KPE_PATVM_CHECK 1
struct uint2 {
  uint32_t x, y;
};
struct uint4 {
  uint32_t x, y, z, w;
};
using std::trunc;

#include "../kyverno_amd/csrc/corpus.hpp"
#include "../kyverno_amd/csrc/kernels_abi.h"
#include "../kyverno_amd/csrc/patclass.hpp"
#include "../kyverno_amd/csrc/program.hpp"
#include "../kyverno_amd/csrc/schema.h"

namespace kpe {
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs);
}

namespace {
#include "../kyverno_amd/csrc/strmatch.inl"
#include "../kyverno_amd/csrc/patvm.inl"
}  // namespace

static std::string slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) throw std::runtime_error(std::string("cannot read ") + p);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s policies.json resources.ndjson out.bin\n", argv[0]);
    return 2;
  }
  const std::string pj = slurp(argv[1]), nd = slurp(argv[2]);
  kpe::Corpus C;
  kpe::flatten_ndjson(C, nd.data(), nd.size(), nullptr, 0, true);
  auto P = kpe::compile_policies(pj.data(), pj.size());
  const auto& PP = P->pat;
  // tape invariants: one root entry per resource; every body inside the tape
  if ((int64_t)C.doc_off.size() != C.n) return fprintf(stderr, "doc_off size\n"), 1;
  const uint64_t ndoc = C.doc.size() / 2;
  for (uint64_t i = 0; i < ndoc; ++i) {
    const uint32_t x = C.doc[2 * i], y = C.doc[2 * i + 1];
    if (DN_KIND(x) == DN_SCALAR ? y >= C.scal.size() && y != 0 && DN_KEY(x) != 0 : false) {
      fprintf(stderr, "bad scalar id at entry %llu\n", (unsigned long long)i);
      return 1;
    }
    if ((DN_KIND(x) == DN_MAP || DN_KIND(x) == DN_ARR) && (y >= ndoc || y + 1 + C.doc[2 * y] > ndoc)) {
      fprintf(stderr, "bad body at entry %llu\n", (unsigned long long)i);
      return 1;
    }
  }
  // bind: operand records, member names, glob bitsets (host copies of the device tables)
  std::vector<uint8_t> pb;
  std::vector<KpePat> pats;
  for (size_t i = 0; i < PP.operands.size(); ++i) {
    if (PP.operand_exact[i]) {
      pats.push_back({PK_EXACT, (uint32_t)pb.size(), (uint32_t)PP.operands[i].size(), 0});
      pb.insert(pb.end(), PP.operands[i].begin(), PP.operands[i].end());
    } else {
      pats.push_back(kpe::classify_pattern(PP.operands[i], pb));
    }
  }
  pb.resize(pb.size() + 17, 0);  // + slack: word-wide compares (kpe_api.cpp upload)
  std::vector<uint32_t> pbuf;
  std::vector<uint4> mem(PP.members.size() / 4);
  const auto& K = C.dict[D_KEY];
  for (size_t i = 0; i < mem.size(); ++i) {
    uint4 m{PP.members[4 * i], PP.members[4 * i + 1], PP.members[4 * i + 2], PP.members[4 * i + 3]};
    const int64_t id = K.find(PP.keys[m.y]);
    m.y = id < 0 || (m.x & PMF_VKEY) ? 0u : (uint32_t)id + 1u;
    if (m.x & PMF_GLOB) {
      const auto& pr = P->preds[m.w];
      m.w = (uint32_t)pbuf.size();
      pbuf.resize(pbuf.size() + (K.size() + 31) / 32 + 1, 0u);
      for (uint32_t s = 0; s < K.size(); ++s) {
        const auto str = K.at(s);
        bool hit = false;
        for (auto& g : pr.globs)
          hit = hit || glob(reinterpret_cast<const uint8_t*>(g.data()), (int)g.size(),
                            reinterpret_cast<const uint8_t*>(str.data()), (int)str.size());
        if (hit) pbuf[m.w + (s >> 5)] |= 1u << (s & 31u);
      }
    }
    mem[i] = m;
  }
  const uint32_t R = (uint32_t)P->rules.size();
  std::vector<uint8_t> verdicts((size_t)C.n * R + KPE_VERDICT_SLACK, 0);  // + slack: the kernel reads whole words
  for (int64_t r = 0; r < C.n; ++r)
    for (auto& pr : PP.rules) verdicts[(size_t)r * R + pr.col] = KPE_PENDING_;
  std::vector<KpeScalar> scal(C.scal);
  std::vector<uint8_t> text(C.scal_text.begin(), C.scal_text.end());
  text.resize(text.size() + 17, 0);
  PatArgs a{};
  a.n = C.n, a.R = R, a.npr = (uint32_t)PP.rules.size();
  a.doc = C.doc.data(), a.doc_off = C.doc_off.data(), a.scal = scal.data(), a.scal_text = text.data();
  a.nodes = PP.nodes.data(), a.members = mem.data(), a.lists = PP.lists.data(), a.leaves = PP.leaves.data();
  a.conds = PP.conds.data(), a.pats = pats.data(), a.pat_bytes = pb.data(), a.roots = PP.roots.data();
  a.rules = PP.rules.data(), a.pbuf = pbuf.data(), a.verdicts = verdicts.data();
  std::vector<uint32_t> col2pr(R + 4, 0u);
  for (size_t i = 0; i < PP.rules.size(); ++i)
    col2pr[PP.rules[i].col] = C2P_MAKE((uint32_t)i + 1u, PP.rules[i].flags >> PR_MEMO_SH);
  a.col2pr = col2pr.data();
  for (uint32_t k = 0; k < KPE_PAT_MEMO; ++k) a.slot_rule[k] = ~0u;  // memo slots' representative rules
  for (uint32_t i = 0; i < (uint32_t)PP.rules.size(); ++i) {
    const uint32_t sl = PP.rules[i].flags >> PR_MEMO_SH;
    if (sl < KPE_PAT_MEMO && a.slot_rule[sl] == ~0u) a.slot_rule[sl] = i;
  }
  uint32_t err = 0;
  a.nnodes = (uint32_t)PP.nodes.size(), a.nmembers = (uint32_t)mem.size(), a.nlists = (uint32_t)PP.lists.size();
  a.nleaves = (uint32_t)PP.leaves.size(), a.nconds = (uint32_t)PP.conds.size(), a.npats = (uint32_t)pats.size();
  a.nroots = (uint32_t)PP.roots.size(), a.npbuf = (uint32_t)pbuf.size(), a.nscal = scal.size();
  a.ndoc = C.doc.size() / 2, a.err = &err;
  std::vector<uint8_t> kb(K.bytes.begin(), K.bytes.end());
  kb.resize(kb.size() + 17, 0);
  a.key_bytes = kb.data(), a.key_off = K.off.data(), a.nkeyd = (uint32_t)K.size();
  // kpe_pattern_kernel's lane body: the LDS frame stack (word-planar, lane 0 of a 64-lane plane;
  // an overflow of its KPE_PAT_LDS_STACK frames re-walks on the private stack) ...
  std::vector<uint8_t> lds_v(verdicts);
  {
    std::vector<uint32_t> plane(FramesLds::kWords * FramesLds::kDepth * 64u, 0xDEADBEEFu);
    uint8_t* keep = a.verdicts;
    a.verdicts = lds_v.data();
    std::vector<uint8_t> memo(KPE_PAT_MEMO, 0xEE);  // with the shared-pattern memo (the private walk below has none)
    for (int64_t r = 0; r < a.n; ++r) pat_eval_row(a, r, FramesLds{plane.data()}, memo.data(), 1u);
    a.verdicts = keep;
  }
  // ... with undecided cells of the LDS stack deferred to the deep pass (kpe_pattern_kernel +
  // kpe_pattern_deep_kernel) ...
  std::vector<uint8_t> defer_v(verdicts);
  {
    std::vector<uint32_t> plane(FramesLds::kWords * FramesLds::kDepth * 64u, 0xDEADBEEFu);
    uint8_t* keep = a.verdicts;
    a.verdicts = defer_v.data();
    std::vector<uint8_t> memo(KPE_PAT_MEMO, 0xEE);
    for (int64_t r = 0; r < a.n; ++r) pat_eval_row<FramesLds, false, true>(a, r, FramesLds{plane.data()}, memo.data(), 1u);
    for (int64_t r = 0; r < a.n; ++r) pat_deep_row(a, r);
    a.verdicts = keep;
  }
  // ... through the leaf table (kpe_leaf_table_kernel restated: one slot per leaf without
  // variables; the LT instance when every leaf has one) ...
  std::vector<uint8_t> lt_v(verdicts);
  {
    std::vector<uint32_t> lslot(std::max<size_t>(PP.leaves.size(), 1), KPE_NO_LSLOT), slot_leaf;
    bool all = true;
    for (size_t i = 0; i < PP.leaves.size(); ++i) {
      if (PP.leaves[i].type <= PL_STR) lslot[i] = (uint32_t)slot_leaf.size(), slot_leaf.push_back((uint32_t)i);
      else if (PP.leaves[i].type != PL_NEVER) all = false;
    }
    const uint32_t words = (uint32_t)((scal.size() + 63) / 64 * 2);
    std::vector<uint32_t> ltab((size_t)std::max<size_t>(slot_leaf.size(), 1) * words + 2, 0u);
    for (size_t k = 0; k < slot_leaf.size(); ++k)
      for (uint32_t sid = 0; sid < scal.size(); ++sid) {
        uint32_t und = 0;
        if (pat_leaf_eval(a, sid, slot_leaf[k], nullptr, &und)) ltab[k * words + (sid >> 5)] |= 1u << (sid & 31u);
      }
    uint8_t* keep = a.verdicts;
    a.verdicts = lt_v.data();
    a.lslot = lslot.data(), a.ltab = ltab.data(), a.ltab_words = words;
    for (auto& m : mem)  // scalar-leaf members carry their slot, as kpe_api.cpp binds them
      if ((m.x & PMF_LEAF) && !(m.x & (PMF_GLOB | PMF_VKEY))) m.w = lslot[PP.nodes[m.z].y];
    std::vector<uint32_t> plane(FramesLds::kWords * FramesLds::kDepth * 64u, 0xDEADBEEFu);
    for (int64_t r = 0; r < a.n; ++r) {
      if (all && !slot_leaf.empty()) pat_eval_row<FramesLds, true>(a, r, FramesLds{plane.data()});
      else pat_eval_row(a, r, FramesLds{plane.data()});
    }
    a.lslot = nullptr, a.ltab = nullptr, a.ltab_words = 0;
    a.verdicts = keep;
  }
  // ... and the lane-private stack
  for (int64_t r = 0; r < a.n; ++r) pat_eval_row(a, r, FramesPriv{});
  if (lds_v != verdicts) return fprintf(stderr, "LDS frame-stack walk (with memo) differs from the private-stack walk\n"), 1;
  if (lt_v != verdicts) return fprintf(stderr, "leaf-table walk differs from the private-stack walk\n"), 1;
  if (defer_v != verdicts) return fprintf(stderr, "deferred deep walk differs from the private-stack walk\n"), 1;
  FILE* f = fopen(argv[3], "wb");
  fwrite(verdicts.data(), 1, (size_t)C.n * R, f);
  fclose(f);
  printf("%lld %u err=0x%x\n", (long long)C.n, R, err);
  if (err) return 1;
  return 0;
}
