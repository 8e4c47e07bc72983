// Host build of the condition VM (kyverno_amd/csrc/condvm.inl, the exact text kpe_cond_kernel
// runs) for sanitizer runs and parity checks without a GPU:
//   scripts/build/condvm_check policies.json resources.ndjson seed.bin out.bin
// Flattens the resources with document tapes, compiles the policies, binds the condition
// program the way kpe_api.cpp does (field names -> D_KEY ids) and runs cond_eval_row over a
// verdict matrix seeded from seed.bin (N x R bytes: what the scan kernel would have written,
// i.e. KPE_PENDING_ for matched H_COND cells, the handler verdict for other matched cells,
// KPE_NA_ for unmatched ones). Writes the resulting N x R verdict bytes to out.bin.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#define __device__
#define __forceinline__ inline
#define KPE_PATVM_CHECK 1  // pattern VM table reads bounds-flagged (foreach pattern entries)
struct uint2 {
  uint32_t x, y;
};
struct uint4 {
  uint32_t x, y, z, w;
};
using std::trunc;
inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }

#include "../kyverno_amd/csrc/corpus.hpp"
#include "../kyverno_amd/csrc/kernels_abi.h"
#include "../kyverno_amd/csrc/program.hpp"
#include "../kyverno_amd/csrc/schema.h"
#include "../kyverno_amd/csrc/patclass.hpp"

namespace kpe {
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs);
}

namespace {
#include "../kyverno_amd/csrc/strmatch.inl"
#include "../kyverno_amd/csrc/patvm.inl"
#include "../kyverno_amd/csrc/condvm.inl"
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
  kpe::Corpus C;
  kpe::flatten_ndjson(C, nd.data(), nd.size(), nullptr, 0, true);
  auto P = kpe::compile_policies(pj.data(), pj.size());
  const auto& CP = P->cond;
  const uint32_t R = (uint32_t)P->rules.size();
  if (seed.size() != (size_t)C.n * R) return fprintf(stderr, "seed size %zu != %lld x %u\n", seed.size(), (long long)C.n, R), 1;
  std::vector<uint8_t> verdicts(seed.begin(), seed.end());
  verdicts.resize(verdicts.size() + KPE_VERDICT_SLACK, 0);  // the pattern pass reads whole words
  std::vector<uint32_t> fk(CP.fields.size());
  for (size_t i = 0; i < fk.size(); ++i) {
    const int64_t id = C.dict[D_KEY].find(CP.fields[i]);
    fk[i] = id < 0 ? 0u : (uint32_t)id + 1u;
  }
  std::vector<uint8_t> text(C.scal_text.begin(), C.scal_text.end()), ctext(CP.ctext.begin(), CP.ctext.end()),
      kb(C.dict[D_KEY].bytes.begin(), C.dict[D_KEY].bytes.end());
  text.resize(text.size() + 17, 0), ctext.resize(ctext.size() + 17, 0), kb.push_back(0);
  std::vector<uint2> ops(CP.ops.size() / 2);
  for (size_t i = 0; i < ops.size(); ++i) ops[i] = uint2{CP.ops[2 * i], CP.ops[2 * i + 1]};
  CondArgs a{};
  a.n = C.n, a.R = R, a.ncr = (uint32_t)CP.rules.size();
  a.doc = C.doc.data(), a.doc_off = C.doc_off.data(), a.scal = C.scal.data(), a.scal_text = text.data();
  a.img_off = C.img_off.empty() ? nullptr : C.img_off.data();
  a.key_bytes = kb.data(), a.key_off = C.dict[D_KEY].off.data();
  a.ops = ops.data(), a.exprs = CP.exprs.data(), a.tmpls = CP.tmpls.data(), a.conds = CP.conds.data();
  a.blocks = CP.blocks.data(), a.fes = CP.fes.data(), a.rules = CP.rules.data();
  a.ctab = CP.consts.data(), a.ctext = ctext.data(), a.clist = CP.clist.data(), a.fkeys = fk.data();
  std::vector<uint2> ctp(CP.tpieces.size() / 2 + 1);
  for (size_t i = 0; i + 1 < CP.tpieces.size(); i += 2) ctp[i / 2] = uint2{CP.tpieces[i], CP.tpieces[i + 1]};
  a.tpieces = ctp.data(), a.txt = CP.tpieces.empty() ? 0u : 1u;
  // pattern program operand records (InRange values of set operators), as kpe_api.cpp binds them
  std::vector<uint8_t> pb;
  std::vector<KpePat> pp;
  for (size_t i = 0; i < P->pat.operands.size(); ++i) {
    if (P->pat.operand_exact[i]) {
      pp.push_back({PK_EXACT, (uint32_t)pb.size(), (uint32_t)P->pat.operands[i].size(), 0});
      pb.insert(pb.end(), P->pat.operands[i].begin(), P->pat.operands[i].end());
    } else {
      pp.push_back(kpe::classify_pattern(P->pat.operands[i], pb));
    }
  }
  pb.resize(pb.size() + 17, 0);
  a.leaves = P->pat.leaves.data(), a.pconds = P->pat.conds.data(), a.pats = pp.data(), a.pat_bytes = pb.data();
  a.verdicts = verdicts.data();
  // the pattern program as kpe_api.cpp binds it (members: names -> D_KEY ids, glob bitsets), for
  // foreach pattern entries and the pattern pass after the condition pass
  const auto& PP = P->pat;
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
  pbuf.push_back(0);
  std::vector<uint2> pvals((size_t)C.n * PP.vars.size() + 1);
  std::vector<uint2> tp(PP.tpieces.size() / 2 + 1);
  for (size_t i = 0; i + 1 < PP.tpieces.size(); i += 2) tp[i / 2] = uint2{PP.tpieces[i], PP.tpieces[i + 1]};
  std::vector<uint8_t> tt(PP.ttext.begin(), PP.ttext.end());
  tt.resize(tt.size() + 17, 0);
  std::vector<uint32_t> col2pr(R + 4, 0u);
  for (size_t i = 0; i < PP.rules.size(); ++i)
    col2pr[PP.rules[i].col] = C2P_MAKE((uint32_t)i + 1u, PP.rules[i].flags >> PR_MEMO_SH);
  uint32_t perr = 0;
  PatArgs pa{};
  pa.n = C.n, pa.R = R, pa.npr = (uint32_t)PP.rules.size();
  pa.doc = C.doc.data(), pa.doc_off = C.doc_off.data(), pa.scal = C.scal.data(), pa.scal_text = text.data();
  pa.nodes = PP.nodes.data(), pa.members = mem.data(), pa.lists = PP.lists.data(), pa.leaves = PP.leaves.data();
  pa.conds = PP.conds.data(), pa.pats = pp.data(), pa.pat_bytes = pb.data(), pa.roots = PP.roots.data();
  pa.rules = PP.rules.data(), pa.col2pr = col2pr.data(), pa.pbuf = pbuf.data(), pa.verdicts = verdicts.data();
  for (uint32_t k = 0; k < KPE_PAT_MEMO; ++k) pa.slot_rule[k] = ~0u;
  for (uint32_t i = 0; i < (uint32_t)PP.rules.size(); ++i) {
    const uint32_t sl = PP.rules[i].flags >> PR_MEMO_SH;
    if (sl < KPE_PAT_MEMO && pa.slot_rule[sl] == ~0u) pa.slot_rule[sl] = i;
  }
  pa.pvals = pvals.data(), pa.nvars = (uint32_t)PP.vars.size(), pa.ptmpl = tp.data(), pa.ttext = tt.data();
  pa.ctab = CP.consts.data(), pa.ctext = ctext.data();
  pa.nnodes = (uint32_t)PP.nodes.size(), pa.nmembers = (uint32_t)mem.size(), pa.nlists = (uint32_t)PP.lists.size();
  pa.nleaves = (uint32_t)PP.leaves.size(), pa.nconds = (uint32_t)PP.conds.size(), pa.npats = (uint32_t)pp.size();
  pa.nroots = (uint32_t)PP.roots.size(), pa.npbuf = (uint32_t)pbuf.size(), pa.nscal = C.scal.size();
  pa.ndoc = C.doc.size() / 2, pa.err = &perr;
  pa.key_bytes = kb.data(), pa.key_off = K.off.data(), pa.nkeyd = (uint32_t)K.size();
  a.pat = &pa, a.pvars = PP.vars.data(), a.pvals = pvals.data(), a.nvars = (uint32_t)PP.vars.size();
  std::vector<uint32_t> mtrace((size_t)C.n * CP.nmsg + 1, 0u);
  a.nmsg = CP.nmsg, a.mtrace = CP.nmsg ? mtrace.data() : nullptr;
  char nb[2][16];
  std::vector<uint8_t> txt(2 * KPE_TXT_CAP);
  for (int64_t r = 0; r < a.n; ++r) cond_eval_row<true>(a, r, nb, txt.data());  // kpe_cond_kernel's lane body
  if (!PP.rules.empty())
    for (int64_t r = 0; r < a.n; ++r) pat_eval_row(pa, r, FramesPriv{});  // then kpe_pattern_kernel's
  if (perr) return fprintf(stderr, "pattern VM bounds flags 0x%x\n", perr), 1;
  FILE* f = fopen(argv[4], "wb");
  fwrite(verdicts.data(), 1, (size_t)C.n * R, f);
  fclose(f);
  if (argc > 5) {  // condition traces, N x R words (kpe_fetch_cond_traces layout)
    std::vector<uint32_t> ct((size_t)C.n * R, 0u);
    for (const KpeCRule& cr : CP.rules)
      if (cr.mslot)
        for (int64_t r = 0; r < C.n; ++r) ct[(size_t)r * R + cr.col] = mtrace[(size_t)r * CP.nmsg + cr.mslot - 1u];
    FILE* g = fopen(argv[5], "wb");
    fwrite(ct.data(), 4, ct.size(), g);
    fclose(g);
  }
  if (argc > 6) {  // N x R x KPE_CTRACE_WORDS (kpe_fetch_cond_traces_ex layout)
    std::vector<uint32_t> cx((size_t)C.n * R * 4u, 0u);  // KPE_CTRACE_WORDS (include/kpe.h)
    for (const KpeCRule& cr : CP.rules) {
      if (!cr.mslot) continue;
      const uint32_t nw = cr.kind == CR_FOREACH ? KPE_FE_TRACE_WORDS : 1u;
      for (int64_t r = 0; r < C.n; ++r)
        for (uint32_t w = 0; w < nw; ++w)
          cx[((size_t)r * R + cr.col) * 4u + w] = mtrace[(size_t)r * CP.nmsg + cr.mslot - 1u + w];
    }
    FILE* g = fopen(argv[6], "wb");
    fwrite(cx.data(), 4, cx.size(), g);
    fclose(g);
  }
  printf("%lld %u\n", (long long)C.n, R);
  return 0;
}
