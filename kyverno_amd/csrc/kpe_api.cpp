// C-ABI implementation (include/kpe.h): device management, H2D upload of the
// columnar corpus and compiled program, evaluation launches and result fetch.
// There is no CPU evaluation path: without a usable HIP device every
// evaluation call fails with KPE_E_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <chrono>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kpe.h"
#include "corpus.hpp"
#include "kernels_abi.h"
#include "patclass.hpp"
#include "program.hpp"
#include "pss_fixed.hpp"
#include "pss_msg.hpp"

namespace kpe {
void flatten_ndjson(Corpus& C, const char* buf, size_t len, const char* nsl, size_t nsl_len, bool docs);
bool is_limit_error(const std::exception& e);
}  // namespace kpe

extern "C" hipError_t kpe_launch_pred(const PredArgs* a, uint32_t nblocks, hipStream_t s);
extern "C" hipError_t kpe_launch_pattern(const PatArgs* dargs, int64_t n, uint32_t npr, int lt, hipStream_t s);
extern "C" hipError_t kpe_launch_pattern_trace(const PatArgs* dargs, const uint64_t* cells, uint64_t n, uint32_t* out,
                                               const uint4* jobs, hipStream_t s);
extern "C" hipError_t kpe_launch_cond(const CondArgs* dargs, int64_t n, int fepat, int txt, hipStream_t s);
extern "C" hipError_t kpe_launch_fill_rows(uint8_t* verdicts, uint32_t R, const uint32_t* rows, uint32_t nrows,
                                           uint8_t value, hipStream_t s);
extern "C" hipError_t kpe_launch_prep(const ScanArgs* dargs, int pss, int narrow, size_t dyn_bytes, hipStream_t s);
extern "C" hipError_t kpe_launch_pssx(const PssxArgs* dargs, int64_t n, hipStream_t s);
extern "C" hipError_t kpe_launch_pack3(const uint8_t* v, uint64_t cells, uint32_t* out, hipStream_t s);
extern "C" hipError_t kpe_launch_apply_one(uint8_t* verdicts, uint32_t* masks, int64_t n, uint32_t R, const uint32_t* segs,
                                           uint32_t nsegs, hipStream_t s);
extern "C" hipError_t kpe_launch_scan(const ScanArgs* dargs, const ScanArgs* hargs, int64_t n, int pss, int narrow,
                                      uint32_t grid,
                                      size_t dyn_bytes, hipStream_t s);
extern "C" uint32_t kpe_scan_grid(int64_t n, int pss, int narrow, size_t dyn_bytes);
extern "C" hipError_t kpe_launch_psum(const PsumArgs* a, hipStream_t s);
extern "C" hipError_t kpe_launch_psa_codes(const PsaCodeArgs* a, hipStream_t s);
extern "C" hipError_t kpe_launch_lean6(const LeanBatchArgs* a, size_t dyn_bytes, int lc, hipStream_t s);
extern "C" hipError_t kpe_launch_selmask(const SelMaskArgs* a, hipStream_t s);
extern "C" hipError_t kpe_launch_leaf_table(const PatArgs* dargs, const uint32_t* slot_leaf, uint32_t nslots,
                                            uint64_t nscal, hipStream_t s);
extern "C" hipError_t kpe_launch_count(const uint8_t* verdicts, int64_t n, uint32_t R, unsigned long long* out,
                                       hipStream_t s);

namespace {
thread_local std::string g_err;

kpe_status fail(kpe_status s, const std::string& m) {
  g_err = m;
  return s;
}
#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail(KPE_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
  } while (0)

#define PCHK(x)                     \
  do {                              \
    hipError_t e_ = (x);            \
    if (e_ != hipSuccess) return e_; \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, std::max<size_t>(n, 16));
    if (e == hipSuccess) bytes = n;
    return e;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

template <class T>
hipError_t upload(DevBuf& b, const std::vector<T>& v, hipStream_t s) {
  hipError_t e = b.ensure(v.size() * sizeof(T) + 128);  // + slack: word-wide text compares and the pattern
                                                        // VM's 8-slot body loads read past the end
  if (e != hipSuccess) return e;
  if (!v.empty()) return hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  return hipSuccess;
}

// LDS budgets of the scan kernel's dynamic region
constexpr uint32_t kMaxLocalWords = 8192;  // 32 KiB of small-domain predicate bitsets
constexpr uint32_t kMaxDynWords = 13312;   // dynamic LDS per scan block (52 KiB)
constexpr uint32_t kMaxTerms = 1024;       // distinct match terms (term masks: 8 B x 4 waves each)
constexpr uint32_t kMaxProgLds = 4096;
constexpr uint32_t kMaxSelLds = 2048;  // label-selector requirement tables staged in LDS (8 KiB)     // filters + filter terms staged in LDS
constexpr uint32_t kMaxLocalPairs = 2048;  // domain size limit for an LDS-resident bitset
constexpr uint32_t kMaxFuseWords = 4096;   // fuse image <= 16 KiB of LDS
constexpr uint32_t kLeanBatchKinds = 4096; // kind table words a LEAN6 block stages
constexpr uint32_t kLeanCodeLds = 8192;    // code bytes a LEAN6 block stages in LDS (else read from L2)
constexpr size_t kMaxFusePairs = 1024;     // (string, pattern) pairs evaluated per block

}  // namespace

// Evaluation streams per device: a corpus binding is pinned to one of them, so the
// evaluations of independent corpora (shards, rotated batches) run concurrently and one
// launch's prologue overlaps another's tail. Setup (uploads, binds) and timed launches
// use stream 0.
constexpr int kMaxLanes = 4;
struct kpe_device {
  int ordinal = 0;
  hipStream_t stream = nullptr;  // == lanes[0]
  hipStream_t lanes[kMaxLanes] = {};
  int nlanes = 2;  // KPE_LANES (1..4) overrides
  uint32_t next_lane = 0;
  std::mutex mu;
  bool timing = false;
  struct EvPair {
    hipEvent_t a, b, c, d;
    double bytes, pbytes;
    int kind;        // scan instantiation (kpe_kernel_stats::scan_kernel)
    bool pre, post;  // a kernel ran between a and b (dictionary pass / prologue), c and d (later passes)
  };
  std::vector<EvPair> pending;
  std::vector<hipEvent_t> pool;
  uint64_t launches = 0;
  double pss_ms = 0, dict_ms = 0, pat_ms = 0, last_bytes = 0, last_pbytes = 0, sum_bytes = 0, sum_pbytes = 0;
  double pss_min = 0, pss_max = 0, pss_sq = 0;  // spread of the scan launches' durations
  int last_kind = 0;
  // knobs, read once at kpe_device_open: KPE_NO_BIND_CACHE (recompute per-binding products every
  // evaluation), KPE_PATVM_ERR (report a KPE_PATVM_CHECK build's bounds flags), KPE_LEAN6_MINW /
  // KPE_LEAN6_TPW (waves a LEAN6 launch keeps / tiles per wave, for A/B runs)
  bool no_cache = false, patvm_err = false;
  // the general scan of a podSecurity program walks each pod's lists itself; KPE_PSUM=1: it reads
  // per-pod records kpe_psum_kernel builds right before it on the second stream (round 6: C4 step
  // 0.393 ms without them against 0.416 ms with them, C3 unchanged, profiles/r06_n; round 5 kept the
  // records for their 0.92x traffic against 1.98x: profiles/r05_psA, r05_psB, r05_final5)
  bool no_psum = true;
  uint64_t lean_min_waves = 16384;  // 256 CUs x 4 SIMDs x 16 waves
  uint32_t lean_tpw = 0;
  // pinned staging for corpus uploads (two halves, double-buffered; allocated on first use): a
  // pageable hipMemcpyAsync is staged by the runtime chunk by chunk, a pinned one is one DMA
  static constexpr size_t kStageHalf = 16u << 20;
  char* stage = nullptr;
  hipEvent_t stage_ev[2] = {};
  bool stage_busy[2] = {};
  int stage_cur = 0;
  double up_alloc_s = 0, up_copy_s = 0;  // KPE_DEBUG upload breakdown (under mu)
  hipEvent_t get_ev() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
  }
};

namespace kpe {
struct DeviceProgram {
  int ordinal = -1;
  DevBuf rule_exc;  // KpeRule::exc per rule (PolicyExceptions)
  DevBuf rules, rule_lanes, narrow_rules, fmask, narrow_cls, filters, fterms, terms, kindsels, annpairs, selectors, selreqs,
      pat_bytes, pats;
  bool narrow = false;  // per-lane rule loop (kernels_abi.h NR_*)
  bool tt = false;      // + truth-table fast path
  uint32_t ncls = 0, pss_rules = 0, err_rules = 0, pat_rules = 0;
  // pattern rules: compiled trees + operand records (program.hpp PatProgram)
  DevBuf pnodes, plists, pleaves, pconds, ppats, pbytes, proots, prules;
  DevBuf plslot, pslot_leaf;  // leaf-table slot per leaf, leaf per slot (PatArgs::lslot)
  std::vector<uint32_t> lslot_h;  // host copy of plslot (bound into the scalar-leaf members' w)
  uint32_t nlslots = 0;
  bool ltab_all = false;  // every leaf has a slot or is PL_NEVER: the pattern kernel's LT instance
  DevBuf pvars, ptmpl, ttext;  // pattern variables: slots, template pieces, template texts
  DevBuf pcol2pr;  // verdict column -> pattern rule index + 1 (0: not a pattern rule)
  // condition rules: compiled programs (program.hpp CondProgram)
  DevBuf cops, cexprs, ctmpls, cconds, cblocks, cfes, crules, cconsts, ctext, cclist, ctpieces;
  DevBuf xrules;  // podSecurity rules with exclusions (program.hpp PssxProgram)
  std::vector<uint8_t> pat_bytes_h;
  std::vector<KpePat> pats_h;  // pattern k of predicate p: pats_h[pat0[p] + k]
  std::vector<uint32_t> pat0;
};

struct Binding {  // program x corpus (dictionary sizes decide predicate placement)
  const Program* prog = nullptr;
  DevBuf jobs, pbuf, verdicts, masks, counts_out;
  DevBuf apply_segs;  // ApplyOne policies' rule ranges (uint2 r0, r1)
  uint32_t napply_segs = 0;
  DevBuf dargs;        // device copy of the scan arguments (kernel reads them with scalar loads)
  DevBuf zero_page;    // 256 zero bytes (loads of columns a program does not read)
  DevBuf fuse;         // fused dictionary pass image (pairs, patterns, small dictionaries)
  uint32_t fuse_lds = 0, fuse_words = 0, npairs = 0, fuse_pats = 0, fuse_patb = 0;
  DevBuf pmembers, pargs, perr, pdeep;  // pattern rules: resolved members, PatArgs copy, check flags,
                                        // PatArgs::deep_any
  bool pargs_valid = false;
  DevBuf pvals;  // pattern variables: per-row values (kpe_cond_kernel -> kpe_pattern_kernel)
  DevBuf cfkeys, cargs;  // condition rules: resolved field names, CondArgs copy
  DevBuf mtrace;         // condition traces: N x CondProgram::nmsg words (schema.h CT_*)
  bool cargs_valid = false;
  DevBuf pimg;  // prologue image (kpe_launch_prep)
  // The large-domain predicate bitsets (pbuf) and the prologue image depend only on the
  // program and the corpus dictionaries: computed by the first evaluation of a binding and
  // kept until the binding is rebuilt (KPE_NO_BIND_CACHE=1: recomputed every evaluation).
  bool inv_ready = false;
  uint32_t pimg_words = 0, capb_lds = 0;
  size_t prep_dyn_bytes = 0;  // the prep kernel's LDS: the scan layout + the fuse area
  bool lean = false;  // LEAN scan instantiation (kind table; no check masks)
  int lean_kind = 0;  // kpe_launch_scan narrow code of the LEAN scan: 7 kpe_lean6_kernel, 2 the template
  int gen_code = 0;   // narrow code of the general scan: narrow | 4 with scan records (PSUM)
  uint32_t kt_lds = PRED_NONE, nkinds = 0;
  DevBuf xexcl, ann_norm, rf_ann, xargs;  // podSecurity exclusions: resolved excludes, key tables, PssxArgs
  bool xargs_valid = false;
  void* xmasks = nullptr;  // the masks buffer xargs points at (null: no masks)
  uint32_t xpp[9] = {}, key_pod_sec = KPE_NO_STR, key_fake_sec = KPE_NO_STR;
  ScanArgs hargs{};    // what dargs holds
  bool args_valid = false;
  DevBuf terms_r, kindsels_r, annpairs_r, selectors_r, selreqs_r, cv_classes;  // resolved tables
  // selector requirement masks (ScanArgs::selm): requirement lists per space, the tables
  DevBuf sel_rq, sel_nq, sel_km, sel_vm, sel_nsq;
  DevBuf ltab;  // leaf table (PatArgs::ltab)
  uint32_t ltab_words = 0;
  uint32_t selm = 0, sel_nrq = 0, sel_nnq = 0;
  uint64_t sm[5] = {};  // pos (EQ / In), wild, NotIn, Exists, DoesNotExist
  uint32_t pp[10] = {};  // fixed PSS predicate locations
  uint32_t wave_lds = 0, wave_words = 0, filt_lds = PRED_NONE, fterm_lds = 0, tt_lds = PRED_NONE;
  uint32_t selt_lds = PRED_NONE;  // ScanArgs::selt_lds
  uint32_t kslot_lds = PRED_NONE, nkslot_g = 0;  // ScanArgs::kslot_lds / nkslot_g
  DevBuf kslot_tab;
  size_t dyn_bytes = 0;
  uint32_t nblocks = 0, njobs = 0, blob_words = 0, scan_blocks = 0;
  uint32_t need = 0;
  double scan_bytes = 0;
  size_t cells = 0;
  int lane = -1;                  // evaluation stream (kpe_device::lanes) of this corpus
  hipStream_t last = nullptr;     // stream of the last launch (fetch orders after it)
};

struct DeviceCorpus {
  int ordinal = -1;
  DevBuf dict_bytes[KPE_NUM_DOMAINS], dict_off[KPE_NUM_DOMAINS];
  DevBuf r_gvk, r_name, r_mns, r_nsa, ann_off, ann_k, ann_v;
  DevBuf lab_off, lab_k, lab_v, r_nsl, nsl_off, nsl_k, nsl_v;
  DevBuf rec, hdr, crec, vol_src, sys_id, pann_kv, c_sann, capsets;
  DevBuf doc, doc_off, img_off, scal, scal_text;  // document tape + scalar table (pattern rules)
  DevBuf doc_perm;  // rows by descending tape size: the pattern / condition kernels' lane -> row map
  DevBuf limit_rows;                     // rows past a per-resource limit
  // cold pod columns, uploaded on the first binding of a program with podSecurity exclusions
  DevBuf ctr_off, vol_off, sys_off, pann_off, c_name, c_image, c_sann_key, c_sec_str, c_pm_str, c_selt_str, c_selu_str,
      c_selr_str, cport_off, cport_str, pann_k, pann_v, p_cold;
  bool cold = false;
  // PSA dictionary codes (kpe_psa_codes_kernel; policy-independent, per distinct string), built at
  // the first binding of a podSecurity program; psum: the general scan's per-pod records, scratch
  // rebuilt by every evaluation that reads them (kpe_psum_kernel)
  DevBuf psum, psa_codes, psa_fixed;
  PsaCodes psa_L{};
  bool codes_ready = false;
  Binding bind;
  bool has_masks = false;
};
}  // namespace kpe

struct kpe_program {
  std::unique_ptr<kpe::Program> p;
};
struct kpe_corpus {
  std::unique_ptr<kpe::Corpus> c;
  std::unique_ptr<kpe::DeviceCorpus> d;
};

extern "C" {

const char* kpe_last_error(void) { return g_err.c_str(); }
const char* kpe_version(void) { return "kpe 0.2 (gfx950)"; }

kpe_status kpe_device_open(int ordinal, kpe_device** out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) return fail(KPE_E_DEVICE, "no HIP device available");
  if (ordinal < 0 || ordinal >= n) return fail(KPE_E_DEVICE, "device ordinal out of range");
  HIPCHK(hipSetDevice(ordinal));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, ordinal));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
    return fail(KPE_E_DEVICE, std::string("kernels are built for gfx950, device is ") + prop.gcnArchName);
  auto d = new (std::nothrow) kpe_device();
  if (!d) return fail(KPE_E_DEVICE, "oom");
  d->ordinal = ordinal;
  if (const char* ev = getenv("KPE_LANES")) d->nlanes = std::max(1, std::min(kMaxLanes, atoi(ev)));
  d->no_cache = getenv("KPE_NO_BIND_CACHE") != nullptr;
  d->patvm_err = getenv("KPE_PATVM_ERR") != nullptr;
  if (const char* ev = getenv("KPE_PSUM")) d->no_psum = atoi(ev) == 0;
  if (const char* ev = getenv("KPE_LEAN6_MINW")) d->lean_min_waves = std::max(1, atoi(ev));
  if (const char* ev = getenv("KPE_LEAN6_TPW")) {
    const int t = atoi(ev);
    d->lean_tpw = t == 1 || t == 2 || t == 4 ? (uint32_t)t : 0u;
  }
  for (int k = 0; k < d->nlanes; ++k) {
    e = hipStreamCreateWithFlags(&d->lanes[k], hipStreamNonBlocking);
    if (e != hipSuccess) {
      for (int j = 0; j < k; ++j) (void)hipStreamDestroy(d->lanes[j]);
      delete d;
      return fail(KPE_E_DEVICE, hipGetErrorString(e));
    }
  }
  d->stream = d->lanes[0];
  *out = d;
  return KPE_OK;
}

void kpe_device_close(kpe_device* d) {
  if (!d) return;
  (void)hipSetDevice(d->ordinal);
  for (int k = 0; k < d->nlanes; ++k) (void)hipStreamSynchronize(d->lanes[k]);
  for (auto& p : d->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
    (void)hipEventDestroy(p.c);
    (void)hipEventDestroy(p.d);
  }
  for (auto e : d->pool) (void)hipEventDestroy(e);
  if (d->stage) {
    (void)hipHostFree(d->stage);
    for (auto e : d->stage_ev) (void)hipEventDestroy(e);
  }
  for (int k = 0; k < d->nlanes; ++k) (void)hipStreamDestroy(d->lanes[k]);
  delete d;
}

kpe_status kpe_program_compile(const char* json, size_t len, kpe_program** out) {
  return kpe_program_compile_ex(json, len, nullptr, 0, 0u, out);
}
kpe_status kpe_program_compile_ex(const char* json, size_t len, const char* exceptions, size_t exc_len, uint32_t flags,
                                  kpe_program** out) {
  try {
    auto p = kpe::compile_policies(json, len, exceptions, exc_len, (flags & KPE_COMPILE_BACKGROUND) != 0u);
    *out = new kpe_program{std::move(p)};
    return KPE_OK;
  } catch (const kpe::CompileError& e) {
    return fail(KPE_E_UNSUPPORTED, e.what());
  } catch (const std::exception& e) {
    return fail(KPE_E_INVALID, e.what());
  }
}
int kpe_program_num_rules(const kpe_program* p) { return p ? (int)p->p->rules.size() : 0; }
const char* kpe_program_rule_name(const kpe_program* p, int r) {
  if (!p || r < 0 || r >= (int)p->p->rule_names.size()) return nullptr;
  return p->p->rule_names[r].c_str();
}
int kpe_program_rule_is_pss(const kpe_program* p, int r) {
  if (!p || r < 0 || r >= (int)p->p->rules.size()) return 0;
  return p->p->rules[r].handler == H_PSS ? 1 : 0;
}
void kpe_program_free(kpe_program* p) {
  if (p) {
    for (auto* d : p->p->devs) delete d;
    delete p;
  }
}

kpe_status kpe_corpus_flatten(const char* ndjson, size_t len, const char* nsl, size_t nsl_len, kpe_corpus** out) {
  return kpe_corpus_flatten_ex(ndjson, len, nsl, nsl_len, KPE_CORPUS_DOCS, out);
}
kpe_status kpe_corpus_flatten_ex(const char* ndjson, size_t len, const char* nsl, size_t nsl_len, uint32_t flags,
                                 kpe_corpus** out) {
  auto c = std::make_unique<kpe::Corpus>();
  try {
    kpe::flatten_ndjson(*c, ndjson, len, nsl, nsl_len, (flags & KPE_CORPUS_DOCS) != 0);
  } catch (const std::exception& e) {
    return fail(kpe::is_limit_error(e) ? KPE_E_LIMIT : KPE_E_INVALID, e.what());
  }
  *out = new kpe_corpus{std::move(c), nullptr};
  return KPE_OK;
}
int64_t kpe_corpus_num_resources(const kpe_corpus* c) { return c ? c->c->n : 0; }
int64_t kpe_corpus_bytes(const kpe_corpus* c) { return c ? c->c->bytes() : 0; }

// kpe_lean6_kernel reads every column through buffer descriptors with 32-bit byte offsets
// (lean.inl: pod records, tile headers, container records and seccomp annotations, volume /
// sysctl items and the pod annotation pairs); a corpus with any of them past `lim` bytes takes the
// LEAN template instantiation, which indexes with 64-bit pointers. Offsets past a descriptor would
// read 0, i.e. silently pass an AppArmor / seccomp / sysctl check.
static constexpr uint64_t kLean6Limit = (1ull << 32) - (1ull << 20);
static bool lean6_fits(const kpe::Corpus& C, uint64_t lim) {
  const uint64_t cols[] = {
      (uint64_t)C.n * 16,                 // pod records
      ((uint64_t)C.n / 64 + 2) * 16,      // tile headers
      (uint64_t)C.c_sc.size() * 8,        // container records
      (uint64_t)C.c_sann.size() * 4,      // container seccomp annotations
      (uint64_t)C.vol_src.size() * 4,     // volume items
      (uint64_t)C.sys_id.size() * 4,      // sysctl items
      (uint64_t)C.pann_kv.size() * 4,     // pod annotation (key, value) pairs, 8 bytes each
  };
  for (uint64_t b : cols)
    if (b + 4096 > lim) return false;
  return true;
}
// Diagnostic (not in kpe.h): the LEAN instantiation a binding of c would pick under a column
// limit of `lim` bytes (0: the real limit): 7 kpe_lean6_kernel, 2 the template scan.
int kpe_debug_lean_kind(const kpe_corpus* c, uint64_t lim) {
  if (!c) return -KPE_E_INVALID;
  return lean6_fits(*c->c, lim ? lim : kLean6Limit) ? 7 : 2;
}

kpe_status kpe_corpus_row_flags(const kpe_corpus* c, uint32_t* out) {
  if (!c || !out) return fail(KPE_E_INVALID, "kpe_corpus_row_flags: null argument");
  const kpe::Corpus& C = *c->c;
  for (int64_t i = 0; i < C.n; ++i) {
    const uint32_t f = C.r_flags[i];
    out[i] = ((f & R_DECODE_ERR) ? KPE_ROW_DECODE_ERROR : 0u) | ((f & R_LIMIT) ? KPE_ROW_LIMIT : 0u) |
             ((f & R_CLASS_MASK) == R_CLASS_OTHER ? KPE_ROW_NO_SPEC : 0u) |
             ((f & R_CTX_ERR) ? KPE_ROW_CONTEXT_ERROR : 0u);
  }
  return KPE_OK;
}

uint64_t kpe_corpus_digest(const kpe_corpus* c) {
  if (!c) return 0;
  const kpe::Corpus& C = *c->c;
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&](const void* p, size_t n) {  // FNV-1a over 8-byte words, then the tail
    const uint8_t* b = static_cast<const uint8_t*>(p);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, b + i, 8);
      h = (h ^ w) * 0x100000001b3ull;
    }
    for (; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    h = (h ^ n) * 0x100000001b3ull;
  };
  auto v = [&](const auto& x) { mix(x.data(), x.size() * sizeof(x[0])); };
  mix(&C.n, sizeof(C.n));
  for (int d = 0; d < KPE_NUM_DOMAINS; ++d) v(C.dict[d].bytes), v(C.dict[d].off);
  v(C.r_flags), v(C.r_gvk), v(C.r_name), v(C.r_mns), v(C.r_nsa), v(C.r_nsl);
  v(C.lab_off), v(C.lab_k), v(C.lab_v), v(C.ann_off), v(C.ann_k), v(C.ann_v);
  v(C.p_sc), v(C.p_cold), v(C.ctr_off), v(C.vol_off), v(C.vol_src), v(C.sys_off), v(C.sys_id);
  v(C.pann_off), v(C.pann_k), v(C.pann_v), v(C.c_sc), v(C.c_add), v(C.c_drop), v(C.c_name), v(C.c_image);
  v(C.c_sann), v(C.c_sann_key), v(C.c_sec_str), v(C.c_pm_str), v(C.c_selt_str), v(C.c_selu_str), v(C.c_selr_str);
  v(C.cport_off), v(C.cport_host), v(C.cport_str), v(C.rec), v(C.hdr), v(C.crec), v(C.pann_kv);
  v(C.capset_add), v(C.capset_drop), v(C.doc), v(C.doc_off), v(C.scal_text), v(C.limit_rows);
  for (const KpeScalar& e : C.scal) mix(&e, sizeof(e));
  return h;
}
void kpe_corpus_free(kpe_corpus* c) {
  if (!c) return;
  if (c->d) (void)hipSetDevice(c->d->ordinal);
  delete c;
}

}  // extern "C"

// Copy v into b (allocated with the upload() slack) through the device's pinned staging halves:
// the CPU fills one half while the DMA drains the other. The caller synchronises the stream.
template <class T>
hipError_t upload_staged(kpe_device* dev, DevBuf& b, const std::vector<T>& v, hipStream_t s) {
  const size_t n = v.size() * sizeof(T);
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e = b.ensure(n + 128);
  const auto t1 = std::chrono::steady_clock::now();
  dev->up_alloc_s += std::chrono::duration<double>(t1 - t0).count();
  struct CopyTimer {
    double* acc;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    ~CopyTimer() { *acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count(); }
  } ct{&dev->up_copy_s};
  if (e != hipSuccess || n == 0) return e;
  if (!dev->stage) {
    e = hipHostMalloc(reinterpret_cast<void**>(&dev->stage), 2 * kpe_device::kStageHalf, hipHostMallocDefault);
    if (e != hipSuccess) {
      dev->stage = nullptr;
      return hipMemcpyAsync(b.p, v.data(), n, hipMemcpyHostToDevice, s);  // pageable copy
    }
    for (auto& ev : dev->stage_ev) (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  }
  const char* src = reinterpret_cast<const char*>(v.data());
  for (size_t off = 0; off < n;) {
    const size_t k = std::min(kpe_device::kStageHalf, n - off);
    const int h = dev->stage_cur;
    if (dev->stage_busy[h] && (e = hipEventSynchronize(dev->stage_ev[h])) != hipSuccess) return e;
    char* dst = dev->stage + (size_t)h * kpe_device::kStageHalf;
    memcpy(dst, src + off, k);
    if ((e = hipMemcpyAsync(static_cast<char*>(b.p) + off, dst, k, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(dev->stage_ev[h], s)) != hipSuccess) return e;
    dev->stage_busy[h] = true;
    dev->stage_cur ^= 1;
    off += k;
  }
  return hipSuccess;
}

extern "C" {

kpe_status kpe_corpus_upload(kpe_device* dev, kpe_corpus* cc) {
  if (!dev || !cc) return fail(KPE_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& C = *cc->c;
  cc->d = std::make_unique<kpe::DeviceCorpus>();
  auto& D = *cc->d;
  D.ordinal = dev->ordinal;
  hipStream_t s = dev->stream;
  const auto upload = [dev](DevBuf& b, const auto& v, hipStream_t st) { return upload_staged(dev, b, v, st); };
  for (int i = 0; i < KPE_NUM_DOMAINS; ++i) {
    HIPCHK(upload(D.dict_bytes[i], C.dict[i].bytes, s));
    HIPCHK(upload(D.dict_off[i], C.dict[i].off, s));
  }
  HIPCHK(upload(D.r_gvk, C.r_gvk, s));
  HIPCHK(upload(D.r_name, C.r_name, s));
  HIPCHK(upload(D.r_mns, C.r_mns, s));
  HIPCHK(upload(D.r_nsa, C.r_nsa, s));
  HIPCHK(upload(D.ann_off, C.ann_off, s));
  HIPCHK(upload(D.ann_k, C.ann_k, s));
  HIPCHK(upload(D.ann_v, C.ann_v, s));
  HIPCHK(upload(D.lab_off, C.lab_off, s));
  HIPCHK(upload(D.lab_k, C.lab_k, s));
  HIPCHK(upload(D.lab_v, C.lab_v, s));
  HIPCHK(upload(D.r_nsl, C.r_nsl, s));
  HIPCHK(upload(D.nsl_off, C.nsl_off, s));
  HIPCHK(upload(D.nsl_k, C.nsl_k, s));
  HIPCHK(upload(D.nsl_v, C.nsl_v, s));
  HIPCHK(upload(D.rec, C.rec, s));
  HIPCHK(upload(D.hdr, C.hdr, s));
  HIPCHK(upload(D.crec, C.crec, s));
  HIPCHK(upload(D.vol_src, C.vol_src, s));
  HIPCHK(upload(D.sys_id, C.sys_id, s));
  HIPCHK(upload(D.pann_kv, C.pann_kv, s));
  HIPCHK(upload(D.c_sann, C.c_sann, s));
  HIPCHK(upload(D.limit_rows, C.limit_rows, s));
  if (C.has_docs) {
    HIPCHK(upload(D.doc, C.doc, s));
    HIPCHK(upload(D.doc_off, C.doc_off, s));
    HIPCHK(upload(D.img_off, C.img_off, s));
    {  // Lanes of a wave take rows of one kind (the rules a row matches, so the rule loop's VM runs
      // are shared by the whole wave, not by the lanes of one kind among mixed Pods and
      // Deployments) and, within a kind, of similar tape size, heaviest first (a document walk's
      // length follows its size). Counting sort on (kind, 1023 - min(size, 1023)), stable.
      constexpr uint64_t kMaxSize = 1023;
      const uint64_t nd = C.doc.size() / 2;
      uint64_t nk = 1;
      for (int64_t r = 0; r < C.n; ++r) nk = std::max<uint64_t>(nk, GVK_KIND(C.r_gvk[r]) + 1);
      const uint64_t kMaxKey = nk * (kMaxSize + 1) - 1;
      std::vector<uint32_t> cnt(kMaxKey + 2, 0), perm(C.n);
      auto key = [&](int64_t r) -> uint64_t {
        const uint64_t b = C.doc_off[r], e = r + 1 < C.n ? C.doc_off[r + 1] : nd;
        return GVK_KIND(C.r_gvk[r]) * (kMaxSize + 1) + kMaxSize - std::min<uint64_t>(e > b ? e - b : 0, kMaxSize);
      };
      for (int64_t r = 0; r < C.n; ++r) ++cnt[key(r) + 1];
      for (uint64_t k = 1; k < cnt.size(); ++k) cnt[k] += cnt[k - 1];
      for (int64_t r = 0; r < C.n; ++r) perm[cnt[key(r)]++] = (uint32_t)r;
      HIPCHK(upload(D.doc_perm, perm, s));
    }
    HIPCHK(upload(D.scal, C.scal, s));
    HIPCHK(upload(D.scal_text, C.scal_text, s));
  }
  {
    std::vector<uint32_t> cs;
    for (size_t i = 0; i < C.capset_add.size(); ++i) {
      cs.push_back((uint32_t)C.capset_add[i]);
      cs.push_back((uint32_t)(C.capset_add[i] >> 32));
      cs.push_back((uint32_t)C.capset_drop[i]);
      cs.push_back((uint32_t)(C.capset_drop[i] >> 32));
    }
    HIPCHK(upload(D.capsets, cs, s));
  }
  const auto ts = std::chrono::steady_clock::now();
  HIPCHK(hipStreamSynchronize(s));
  static const bool dbg = getenv("KPE_DEBUG") != nullptr;
  if (dbg)
    fprintf(stderr, "kpe upload: alloc %.4f s, stage + enqueue %.4f s, final sync %.4f s\n", dev->up_alloc_s, dev->up_copy_s,
            std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count());
  dev->up_alloc_s = dev->up_copy_s = 0;
  return KPE_OK;
}

}  // extern "C"

namespace {

// go-wildcard pattern -> device pattern class (the literal is stored; only a
// '?' or an inner '*' needs the general backtracking matcher).

template <class T>
void append_words(std::vector<uint32_t>& img, const std::vector<T>& v, uint32_t* off) {
  static_assert(sizeof(T) % 4 == 0, "program tables are word-sized");
  *off = (uint32_t)img.size();
  const uint32_t* w = reinterpret_cast<const uint32_t*>(v.data());
  img.insert(img.end(), w, w + v.size() * sizeof(T) / 4);
}

kpe_status ensure_program(kpe_device* dev, const kpe_program* pp) {
  auto& P = *pp->p;
  if (dev->ordinal < 0 || dev->ordinal >= 16) return fail(KPE_E_DEVICE, "device ordinal past 15");
  std::lock_guard<std::mutex> plk(P.dev_mu);
  if (P.devs[dev->ordinal]) return KPE_OK;  // one copy per device: programs are shared across devices
  std::vector<uint32_t> lanes;  // rule lane records (kernels_abi.h RL_*)
  for (auto& r : P.rules) {
    if (r.match_nf > 255 || r.excl_nf > 255 || r.match_f0 > 0xFFFFFF || r.excl_f0 > 0xFFFFFF || r.cv_class > 0xFFF)
      return fail(KPE_E_LIMIT, "rule exceeds the device rule encoding (filters per block <= 255)");
    lanes.push_back(r.handler | r.cv_class << 4 | r.match_mode << 16 | r.excl_mode << 18);
    lanes.push_back(r.match_f0 | r.match_nf << 24);
    lanes.push_back(r.excl_f0 | r.excl_nf << 24);
    lanes.push_back(r.pol_term < 0 ? PRED_NONE : (uint32_t)r.pol_term);
  }
  // NARROW programs: per-rule records + per-filter term masks (kernels_abi.h NR_*)
  // Label selector terms stay on the wide path: per lane, the narrow loop walks every selector's
  // requirement records with scalar loads and is issue-bound (C4: 0.22 ms narrow, 0.19 ms wide,
  // profiles/r02_c4)
  const bool sel_terms = std::any_of(P.terms.begin(), P.terms.end(), [](const KpeTerm& t) {
    return t.type == T_SELECTOR || t.type == T_NSSELECTOR;
  });
  // (KPE_SEL_NARROW=1: selector programs on the narrow path too, for A/B runs: since the
  // requirement masks, a selector term is one mask compare per lane on either path)
  static const bool sel_narrow = [] {
    const char* e = getenv("KPE_SEL_NARROW");
    return e && atoi(e) != 0;
  }();
  const bool narrow = (!sel_terms || sel_narrow) && !P.rules.empty() && P.rules.size() <= KPE_NARROW_R &&
                      P.terms.size() <= KPE_NARROW_TERMS && P.filters.size() <= KPE_NARROW_FILTERS;
  std::vector<uint32_t> nrules, fmask;
  if (narrow) {
    for (auto& f : P.filters) {
      uint32_t m = 0;
      for (uint32_t k = 0; k < f.nt; ++k) m |= 1u << P.fterms[f.t0 + k];
      fmask.push_back(m);
    }
    uint32_t prev_policy = 0xFFFFFFFFu;
    for (auto& r : P.rules) {
      uint32_t x = r.handler | r.match_mode << 4 | r.excl_mode << 6;
      // ApplyOne runs after every evaluation kernel (kpe_apply_one_kernel), not in the scan
      if (r.policy != prev_policy) x |= NR_NEW_POLICY;
      prev_policy = r.policy;
      if (r.pol_term >= 0) x |= ((uint32_t)r.pol_term + 1u) << 16;
      nrules.push_back(x);
      nrules.push_back(r.cv_mask);
      nrules.push_back(r.match_f0 | r.match_nf << 24);
      nrules.push_back(r.excl_f0 | r.excl_nf << 24);
    }
  }
  // truth-table fast path: few terms; per PSS version set its rule mask
  const bool tt = narrow && P.terms.size() <= KPE_TT_TERMS && !P.any_const && !P.any_exc;
  std::vector<uint32_t> cls;  // (cv_mask, rule mask) pairs
  uint32_t pss_rules = 0, err_rules = 0, pat_rules = 0;
  if (tt) {
    for (size_t r = 0; r < P.rules.size(); ++r) {
      const auto& k = P.rules[r];
      if (k.handler == H_PSS) {
        pss_rules |= 1u << r;
        size_t c = 0;
        while (c < cls.size() && cls[c] != k.cv_mask) c += 2;
        if (c == cls.size()) cls.push_back(k.cv_mask), cls.push_back(0);
        cls[c + 1] |= 1u << r;
      } else if (k.handler == H_ERROR) {
        err_rules |= 1u << r;
      } else if (k.handler == H_PATTERN) {
        pat_rules |= 1u << r;
      }
    }
  }
  P.devs[dev->ordinal] = new kpe::DeviceProgram();
  auto& D = *P.devs[dev->ordinal];
  D.narrow = narrow;
  D.tt = tt;
  D.ncls = (uint32_t)cls.size() / 2;
  D.pss_rules = pss_rules;
  D.err_rules = err_rules;
  D.pat_rules = pat_rules;
  {  // pattern rules: operand records (a verbatim operand is an exact compare)
    const auto& PP = P.pat;
    std::vector<uint8_t> pb;
    std::vector<KpePat> pp;
    for (size_t i = 0; i < PP.operands.size(); ++i) {
      if (PP.operand_exact[i]) {
        pp.push_back({PK_EXACT, (uint32_t)pb.size(), (uint32_t)PP.operands[i].size(), 0});
        pb.insert(pb.end(), PP.operands[i].begin(), PP.operands[i].end());
      } else {
        pp.push_back(kpe::classify_pattern(PP.operands[i], pb));
      }
    }
    hipStream_t s0 = dev->stream;
    HIPCHK(upload(D.pnodes, PP.nodes, s0));
    HIPCHK(upload(D.plists, PP.lists, s0));
    HIPCHK(upload(D.pleaves, PP.leaves, s0));
    {  // leaf-table slots: leaves decided by the scalar alone (no variables), up to KPE_LTAB_SLOTS;
       // leaves with the same content (type, value, pattern text) share a slot
      std::vector<uint32_t> lslot(std::max<size_t>(PP.leaves.size(), 1), KPE_NO_LSLOT), slot_leaf;
      std::map<std::string, uint32_t> seen;
      bool all = true;
      for (size_t i = 0; i < PP.leaves.size(); ++i) {
        const KpeLeaf& L = PP.leaves[i];
        if (L.type == PL_NEVER) continue;
        if (L.type > PL_STR) {
          all = false;
          continue;
        }
        std::string key((const char*)&L.type, 4);
        key.append((const char*)&L.bval, 4).append((const char*)&L.ival, 8).append((const char*)&L.fval, 8);
        if (L.type == PL_STR) key += PP.operands[L.exact];
        auto it = seen.find(key);
        if (it != seen.end()) {
          lslot[i] = it->second;
        } else if (slot_leaf.size() < KPE_LTAB_SLOTS) {
          lslot[i] = (uint32_t)slot_leaf.size();
          seen.emplace(key, lslot[i]);
          slot_leaf.push_back((uint32_t)i);
        } else {
          all = false;
        }
      }
      D.nlslots = (uint32_t)slot_leaf.size();
      D.ltab_all = all && D.nlslots > 0;
      if (slot_leaf.empty()) slot_leaf.push_back(0);
      HIPCHK(upload(D.plslot, lslot, s0));
      D.lslot_h = lslot;
      HIPCHK(upload(D.pslot_leaf, slot_leaf, s0));
    }
    HIPCHK(upload(D.pconds, PP.conds, s0));
    HIPCHK(upload(D.ppats, pp, s0));
    HIPCHK(upload(D.pbytes, pb, s0));
    HIPCHK(upload(D.proots, PP.roots, s0));
    HIPCHK(upload(D.prules, PP.rules, s0));
    HIPCHK(upload(D.pvars, PP.vars, s0));
    HIPCHK(upload(D.ptmpl, PP.tpieces, s0));
    HIPCHK(upload(D.ttext, PP.ttext, s0));
    {
      std::vector<uint32_t> c2p(P.rules.size() + 4, 0u);  // + slack: the kernel reads whole words
      for (size_t i = 0; i < PP.rules.size(); ++i)
        c2p[PP.rules[i].col] = C2P_MAKE((uint32_t)i + 1u, PP.rules[i].flags >> PR_MEMO_SH);
      HIPCHK(upload(D.pcol2pr, c2p, s0));
    }
    const auto& CP = P.cond;
    HIPCHK(upload(D.cops, CP.ops, s0));
    HIPCHK(upload(D.cexprs, CP.exprs, s0));
    HIPCHK(upload(D.ctmpls, CP.tmpls, s0));
    HIPCHK(upload(D.cconds, CP.conds, s0));
    HIPCHK(upload(D.cblocks, CP.blocks, s0));
    HIPCHK(upload(D.cfes, CP.fes, s0));
    HIPCHK(upload(D.crules, CP.rules, s0));
    HIPCHK(upload(D.cconsts, CP.consts, s0));
    HIPCHK(upload(D.ctext, CP.ctext, s0));
    HIPCHK(upload(D.cclist, CP.clist, s0));
    HIPCHK(upload(D.ctpieces, CP.tpieces, s0));
    HIPCHK(upload(D.xrules, P.pssx.rules, s0));
  }
  D.ordinal = dev->ordinal;
  hipStream_t s = dev->stream;
  for (auto& pr : P.preds) {
    D.pat0.push_back((uint32_t)D.pats_h.size());
    if (pr.special == PRED_SPECIAL_QNAME)
      D.pats_h.push_back({PK_QNAME, 0, 0, 0});
    else if (pr.special == PRED_SPECIAL_LABVAL)
      D.pats_h.push_back({PK_LABVAL, 0, 0, 0});
    for (auto& g : pr.globs) D.pats_h.push_back(kpe::classify_pattern(g, D.pat_bytes_h));
  }
  HIPCHK(upload(D.rules, P.rules, s));
  HIPCHK(upload(D.rule_lanes, lanes, s));
  if (P.any_exc) {
    std::vector<uint32_t> xe;
    for (auto& r : P.rules) xe.push_back(r.exc);
    HIPCHK(upload(D.rule_exc, xe, s));
  }
  HIPCHK(upload(D.narrow_rules, nrules, s));
  HIPCHK(upload(D.fmask, fmask, s));
  HIPCHK(upload(D.narrow_cls, cls, s));
  HIPCHK(upload(D.filters, P.filters, s));
  HIPCHK(upload(D.fterms, P.fterms, s));
  HIPCHK(upload(D.terms, P.terms, s));
  HIPCHK(upload(D.kindsels, P.kindsels, s));
  HIPCHK(upload(D.annpairs, P.annpairs, s));
  HIPCHK(upload(D.selectors, P.selectors, s));
  HIPCHK(upload(D.selreqs, P.selreqs, s));
  HIPCHK(upload(D.pat_bytes, D.pat_bytes_h, s));
  HIPCHK(upload(D.pats, D.pats_h, s));
  HIPCHK(hipStreamSynchronize(s));
  return KPE_OK;
}

// Columns the compiled program reads (kernel `need` flags) and their bytes.
uint32_t need_flags(const kpe::Program& P) {
  uint32_t need = 0;
  if (P.any_pss) {
    need |= NEED_FLAGS;
    uint32_t u = P.cv_union;
    if (u & ((1u << CV_CAPS_BASELINE_1_0) | (1u << CV_CAPS_RESTRICTED_1_22) | (1u << CV_CAPS_RESTRICTED_1_25)))
      need |= NEED_CAPS;
    if (u & (1u << CV_SECCOMP_BASELINE_1_0)) need |= NEED_SANN | NEED_PANN;
    if (u & (1u << CV_APPARMOR_1_0)) need |= NEED_PANN;
    if (u & ((1u << CV_HOST_PATH_1_0) | (1u << CV_RESTRICTED_VOLUMES_1_0))) need |= NEED_VOL;
    if (u & ((1u << CV_SYSCTLS_1_0) | (1u << CV_SYSCTLS_1_27) | (1u << CV_SYSCTLS_1_29))) need |= NEED_SYS;
  }
  for (auto& r : P.rules)
    if (r.handler != H_NONE && r.handler != H_PSS) need |= NEED_FLAGS;
  for (auto& t : P.terms) {
    if (t.type == T_KINDS || t.type == T_KIND_PRED || t.type == T_NSSELECTOR) need |= NEED_GVK;
    if (t.type == T_PRED) need |= t.b == COL_NAME ? NEED_NAME : t.b == COL_MNS ? NEED_MNS : NEED_NSA;
  }
  for (auto& t : P.terms) {
    if (t.type == T_SELECTOR) need |= NEED_LAB;
    if (t.type == T_NSSELECTOR) need |= NEED_NSL;
  }
  return need;
}
// The fixed-set table of kpe_psa_codes_kernel (layout: kernels_abi.h KPE_PSF_*) from the PSA
// library's sets (pss_fixed.hpp): exact literals bucketed by byte length, then the prefix globs.
const std::vector<uint32_t>& psa_fixed_table() {
  static const std::vector<uint32_t> tab = [] {
    struct Ent {
      uint32_t set;
      bool prefix;
      std::string lit;
    };
    std::vector<Ent> ex, px;
    auto add = [&](uint32_t set, const std::vector<std::string>& globs) {
      for (const auto& g : globs) {
        const bool prefix = !g.empty() && g.back() == '*';
        (prefix ? px : ex).push_back({set, prefix, prefix ? g.substr(0, g.size() - 1) : g});
      }
    };
    namespace F = kpe::pssfix;
    add(PSF_CAPS_OK, F::kCapsBaselineOk), add(PSF_CAP_NBS, F::kCapNbs), add(PSF_CAP_ALL, F::kCapAll);
    add(PSF_SYSCTL0, F::sysctls(0)), add(PSF_SYSCTL1, F::sysctls(1)), add(PSF_SYSCTL2, F::sysctls(2));
    add(PSF_APPARMOR_KEY, F::kApparmorKey), add(PSF_SECCOMP_POD_KEY, F::kSeccompPodKey);
    add(PSF_APPARMOR_OK, F::kApparmorOk), add(PSF_SECCOMP_ANN_OK, F::kSeccompAnnOk);
    std::stable_sort(ex.begin(), ex.end(), [](const Ent& a, const Ent& b) { return a.lit.size() < b.lit.size(); });
    std::vector<uint32_t> t(KPE_PSF_ENT0, 0u);
    t[0] = (uint32_t)ex.size(), t[1] = (uint32_t)px.size();
    for (size_t e = 0; e < ex.size(); ++e) {
      const size_t len = ex[e].lit.size();
      if (len >= KPE_PSF_MAXLEN) throw std::logic_error("PSA fixed literal too long");
      uint32_t& rg = t[2 + len];
      if ((rg >> 16) == 0) rg = (uint32_t)e;  // first entry of this length
      rg = (rg & 0xFFFFu) | (uint32_t)(e + 1) << 16;
    }
    std::vector<Ent> all = ex;
    all.insert(all.end(), px.begin(), px.end());
    size_t lit = KPE_PSF_ENT0 + 2 * all.size();
    t.resize(lit, 0u);
    for (size_t e = 0; e < all.size(); ++e) {
      const std::string& L = all[e].lit;
      t[KPE_PSF_ENT0 + 2 * e] = all[e].set | (all[e].prefix ? 1u << 7 : 0u) | (uint32_t)L.size() << 8;
      t[KPE_PSF_ENT0 + 2 * e + 1] = (uint32_t)t.size();
      for (size_t k = 0; k < L.size(); k += 4) {
        uint32_t w = 0;
        for (size_t b = 0; b < 4 && k + b < L.size(); ++b) w |= (uint32_t)(uint8_t)L[k + b] << (8 * b);
        t.push_back(w);
      }
    }
    if (t.size() > 1024) throw std::logic_error("PSA fixed table past its LDS area");
    return t;
  }();
  return tab;
}
// The corpus's PSA dictionary codes (kpe_psa_codes_kernel, one launch): built on the first binding
// of a podSecurity program and again by a cold evaluation. Policy-independent, per distinct string.
kpe_status run_codes(const kpe::Corpus& C, kpe::DeviceCorpus& D, hipStream_t s) {
  const int dom[4] = {D_CAP, D_SYSCTL, D_ANNK, D_ANNV};
  PsaCodeArgs a{};
  PsaCodes& L = a.L;
  auto al = [](size_t x) { return (uint32_t)((x + 3) & ~(size_t)3); };
  L.ncapsets = (uint32_t)C.capset_add.size();
  L.nsysd = (uint32_t)C.dict[D_SYSCTL].size(), L.nannk = (uint32_t)C.dict[D_ANNK].size();
  L.nannv = (uint32_t)C.dict[D_ANNV].size();
  L.o_sys = al(L.ncapsets), L.o_annk = L.o_sys + al(L.nsysd), L.o_annv = L.o_annk + al(L.nannk);
  L.bytes = L.o_annv + al(L.nannv);
  if (!D.codes_ready) {
    HIPCHK(upload(D.psa_fixed, psa_fixed_table(), s));
    HIPCHK(D.psa_codes.ensure((size_t)L.bytes + 16));
  }
  for (int d = 0; d < 4; ++d) {
    a.dict_bytes[d] = D.dict_bytes[dom[d]].as<uint8_t>();
    a.dict_off[d] = D.dict_off[dom[d]].as<uint32_t>();
    a.dict_n[d] = C.dict[dom[d]].size();
  }
  a.capsets = D.capsets.as<uint32_t>();
  a.fixed = D.psa_fixed.as<uint32_t>();
  a.fixed_words = (uint32_t)psa_fixed_table().size();
  a.codes = D.psa_codes.as<uint8_t>();
  HIPCHK(kpe_launch_psa_codes(&a, s));
  D.psa_L = L;
  D.codes_ready = true;
  return KPE_OK;
}
// The general scan's per-pod PSA records of an uploaded corpus on stream s (kpe_launch_psum), run
// by every evaluation that reads them; summ: also the 2-word summaries (kpe_corpus_psa_summary),
// or null.
kpe_status run_psum(const kpe::Corpus& C, kpe::DeviceCorpus& D, hipStream_t s, uint32_t* summ = nullptr) {
  if (!D.codes_ready)
    if (kpe_status st = run_codes(C, D, s)) return st;
  PsumArgs a{};
  a.n = C.n;
  a.ntiles = (uint32_t)((C.n + 63) / 64);
  a.rec = D.rec.as<uint32_t>(), a.hdr = D.hdr.as<uint32_t>(), a.crec = D.crec.as<uint32_t>();
  a.vol_src = D.vol_src.as<uint32_t>(), a.sys_id = D.sys_id.as<uint32_t>(), a.pann_kv = D.pann_kv.as<uint32_t>();
  a.c_sann = D.c_sann.as<uint32_t>();
  a.codes = D.psa_codes.as<uint8_t>();
  a.L = D.psa_L;
  HIPCHK(D.psum.ensure((size_t)C.n * 12 + 16));
  a.psum = D.psum.as<uint32_t>();
  a.summ = summ;
  HIPCHK(kpe_launch_psum(&a, s));
  return KPE_OK;
}
// Algorithmic bytes of one LEAN evaluation of a shard (kpe_lean6_kernel): the pod records, the tile
// headers, the list columns the program reads, the code bytes and kind table its blocks stage
// (counted once), the verdict cells and, in the masks mode, the check masks.
double lean_bytes(const kpe::Corpus& C, const kpe::DeviceCorpus& D, uint32_t need, uint32_t R, bool masks) {
  const double n = (double)C.n;
  double b = 16.0 * n + 16.0 * (double)((C.n + 63) / 64 + 1) + 8.0 * (double)C.c_sc.size();
  if (need & NEED_SANN) b += 4.0 * (double)C.c_sc.size();
  if (need & NEED_VOL) b += 4.0 * (double)C.vol_src.size();
  if (need & NEED_SYS) b += 4.0 * (double)C.sys_id.size();
  if (need & NEED_PANN) b += 8.0 * (double)(C.pann_kv.size() / 2);
  b += (double)D.psa_L.bytes + 4.0 * (double)D.bind.nkinds;
  b += n * R * (masks ? 5.0 : 1.0);
  return b;
}
double scan_bytes(const kpe::Program& P, const kpe::Corpus& C, uint32_t need, bool masks, bool psum) {
  double b = 0;
  const double n = (double)C.n;
  if (P.any_pss && psum) {
    b += 16 * n + 12 * n;  // pod records + the scan records (each pod's failing versioned checks)
  } else if (P.any_pss) {
    b += 16 * n + 16.0 * ((C.n + 63) / 64);  // pod records + wave headers
    b += 8.0 * C.c_sc.size();               // container records
    if (need & NEED_CAPS) b += 16.0 * C.capset_add.size();
    if (need & NEED_SANN) b += 4.0 * C.c_sc.size();
    if (need & NEED_VOL) b += 4.0 * C.vol_src.size();
    if (need & NEED_SYS) b += 4.0 * C.sys_id.size();
    if (need & NEED_PANN) b += 8.0 * C.pann_kv.size() / 2;
  } else {
    if (need & NEED_GVK) b += 4 * n;
    if (need & NEED_NSA) b += 4 * n;
  }
  if (need & NEED_NAME) b += 4 * n;  // name / namespace columns read by predicate terms
  if (need & NEED_MNS) b += 4 * n;
  // label CSR / namespace-label rows read by selector terms (once per resource)
  if (need & NEED_LAB) b += 4.0 * n + 8.0 * C.lab_k.size();
  if (need & NEED_NSL) b += 4.0 * n;  // r_nsl; the namespace table itself is cache-resident
  b += n * P.rules.size() * (masks ? 5.0 : 1.0);  // verdict cells (+ check masks)
  return b;
}

// Algorithmic bytes of kpe_psum_kernel: the pod records, tile headers and the list columns the
// program reads, the code bytes, and the 12-byte records written.
double psum_bytes(const kpe::Corpus& C, const kpe::DeviceCorpus& D, uint32_t need) {
  return lean_bytes(C, D, need, 0, false) - 4.0 * (double)D.bind.nkinds + 12.0 * (double)C.n;
}

// Kind terms (T_KINDS, T_KIND_PRED) of a wide-path program as one table over the corpus's
// distinct GVKs: per GVK, bit s of its mask = kind term slot_of^-1(s) holds (CheckKind over the
// group / version / kind strings with the same go-wildcard predicates the device evaluates). The
// scan then looks the row's mask up once instead of evaluating each kind term from its selector
// records. Only for <= 64 kind terms and <= 64 distinct GVKs; tab = [GVKs ascending, padded to
// an even count][masks, 2 words each].
static void kind_table(const kpe::Program& P, const kpe::Corpus& C, std::vector<uint32_t>& tab,
                       std::vector<int32_t>& slot_of, uint32_t* ng) {
  std::vector<uint32_t> kt;
  for (size_t t = 0; t < P.terms.size(); ++t)
    if (P.terms[t].type == T_KINDS || P.terms[t].type == T_KIND_PRED) kt.push_back((uint32_t)t);
  if (kt.empty() || kt.size() > 64) return;
  auto plain = [&](int32_t p) { return p < 0 || (p < (int32_t)P.preds.size() && P.preds[p].special == PRED_SPECIAL_NONE); };
  for (uint32_t t : kt) {
    const KpeTerm& tm = P.terms[t];
    if (tm.type == T_KIND_PRED && !plain((int32_t)tm.a)) return;
    if (tm.type == T_KINDS)
      for (uint32_t k = 0; k < tm.b; ++k) {
        const KpeKindSel& ks = P.kindsels[tm.a + k];
        if (!plain(ks.pg) || !plain(ks.pv) || !plain(ks.pk)) return;
      }
  }
  std::vector<uint32_t> G;
  uint32_t last = 0xFFFFFFFFu;
  for (uint32_t g : C.r_gvk) {
    if (g == last) continue;
    last = g;
    if (std::find(G.begin(), G.end(), g) == G.end()) {
      G.push_back(g);
      if (G.size() > 64) return;
    }
  }
  if (G.empty()) return;
  std::sort(G.begin(), G.end());
  auto pred = [&](int32_t p, std::string_view s) {
    if (p < 0) return true;
    for (auto& g : P.preds[p].globs)
      if (kpe::go_wildcard(g, std::string(s))) return true;
    return false;
  };
  const uint32_t m = ((uint32_t)G.size() + 1u) & ~1u;
  tab.assign(m * 3u, 0u);
  for (size_t i = 0; i < G.size(); ++i) {
    const uint32_t g = G[i];
    tab[i] = g;
    const std::string_view kind = C.dict[D_KIND].at(GVK_KIND(g)), ver = C.dict[D_VERSION].at(GVK_VER(g)),
                           grp = C.dict[D_GROUP].at(GVK_GRP(g));
    uint64_t mask = 0;
    for (size_t s = 0; s < kt.size(); ++s) {
      const KpeTerm& tm = P.terms[kt[s]];
      bool ok = false;
      if (tm.type == T_KIND_PRED) {
        ok = pred((int32_t)tm.a, kind);
      } else {
        for (uint32_t k = 0; k < tm.b && !ok; ++k) {
          const KpeKindSel& ks = P.kindsels[tm.a + k];
          ok = ks.sub_ok && pred(ks.pg, grp) && pred(ks.pv, ver) && pred(ks.pk, kind);
        }
      }
      if (ok) mask |= 1ull << s;
    }
    tab[m + 2 * i] = (uint32_t)mask, tab[m + 2 * i + 1] = (uint32_t)(mask >> 32);
  }
  for (uint32_t i = (uint32_t)G.size(); i < m; ++i) tab[i] = 0xFFFFFFFFu;
  for (size_t s = 0; s < kt.size(); ++s) slot_of[kt[s]] = (int32_t)s;
  *ng = (uint32_t)G.size();
}

kpe_status ensure_binding(kpe_device* dev, const kpe_program* pp, kpe_corpus* cc, bool want_masks) {
  auto& P = *pp->p;
  auto& C = *cc->c;
  auto& B = cc->d->bind;
  auto& PD = *P.devs[dev->ordinal];
  size_t cells = (size_t)C.n * P.rules.size();
  if (B.prog == &P && B.cells == cells && (!want_masks || cc->d->has_masks)) return KPE_OK;
  if (B.last) HIPCHK(hipStreamSynchronize(B.last));  // no launch may still read what is rebuilt
  if (B.lane < 0) B.lane = (int)(dev->next_lane++ % (uint32_t)dev->nlanes);
  hipStream_t s = dev->stream;
  // Predicates over small dictionaries get LDS-resident bitsets ("local": every scan
  // block copies them from pbuf's blob), the rest are read from pbuf (HBM/L2). All are
  // evaluated once per binding by kpe_pred_kernel (grid x = strings / 256, y = predicate).
  // pbuf: [local bitsets (blob)][large-domain bitsets].
  // Dynamic LDS per scan block: [local bitsets][filters + filter terms][4 per-wave regions].
  const uint32_t npreds = (uint32_t)P.preds.size();
  const uint32_t nterms = (uint32_t)P.terms.size(), ncv = (uint32_t)P.cv_classes.size();
  if (nterms > kMaxTerms) return fail(KPE_E_LIMIT, "program has more than 1024 distinct match terms");
  const bool narrow = PD.narrow;
  const uint32_t wave_words = (P.any_pss ? KPE_STAGE_WORDS : 0u) +
                              (narrow ? 2 * 64 * (uint32_t)P.rules.size() / 4  // double-buffered rows
                                      : 2 * nterms + 2 * ncv + 2 * 4 * KPE_RULE_CHUNK + 64 * KPE_RULE_CHUNK / 4);
  const uint32_t prog_words = 2 * (uint32_t)P.filters.size() + (uint32_t)P.fterms.size();
  const bool stage_prog = !narrow && prog_words <= kMaxProgLds;
  // the label-selector requirement tables (sel_km, sel_vm: 4 words per label key / value id) in
  // LDS when they are small: the per-row label fold then reads LDS instead of L2
  const bool sel_lbl = std::any_of(P.terms.begin(), P.terms.end(), [](const KpeTerm& t) { return t.type == T_SELECTOR; });
  const uint64_t selt_need = 4ull * ((uint64_t)C.dict[D_LABK].size() + C.dict[D_LABV].size());
  static const bool selt_off = [] {
    const char* e = getenv("KPE_SELT");
    return e && atoi(e) == 0;
  }();
  const uint32_t selt_words = sel_lbl && !selt_off && selt_need <= kMaxSelLds ? (uint32_t)selt_need : 0u;
  static const bool kslot_off = [] {
    const char* e = getenv("KPE_KSLOT");
    return e && atoi(e) == 0;
  }();
  std::vector<uint32_t> kslot_tab;
  std::vector<int32_t> kslot_of(P.terms.size(), -1);
  uint32_t kslot_ng = 0;
  if (!narrow && !kslot_off) kind_table(P, C, kslot_tab, kslot_of, &kslot_ng);
  const uint32_t kslot_words = (uint32_t)kslot_tab.size();
  // LEAN scan candidate: prepped, NARROW truth-table program of kind-only terms (a kind table
  // replaces the per-resource term loop); confirmed below once predicate placement is known
  bool lean = narrow && PD.tt && P.any_pss &&
              C.dict[D_KIND].size() <= 4096;
  for (const auto& tm : P.terms) lean = lean && (tm.type == T_KIND_PRED || tm.type == T_FALSE);
  lean = lean && !(need_flags(P) & (NEED_NAME | NEED_MNS));  // columns a LEAN scan never loads
  const uint32_t kt_words = lean ? (C.dict[D_KIND].size() + 3) & ~3u : 0u;
  const uint32_t capb_words = P.any_pss ? ((uint32_t)C.capset_add.size() + 15) / 16 * 4 : 0u;  // 1 byte per set
  const int64_t budget =
      (int64_t)kMaxDynWords - 4 * (int64_t)wave_words - (stage_prog ? prog_words : 0) - 8 - selt_words - 4 -
      kslot_words - 2 -
      (PD.tt ? (1 << KPE_TT_TERMS) : 0) - kt_words - capb_words;
  if (budget < 0) return fail(KPE_E_LIMIT, "program does not fit the scan kernel's LDS budget");
  const uint32_t local_budget = (uint32_t)std::min<int64_t>(kMaxLocalWords, budget);
  std::vector<uint32_t> nwords(npreds);
  std::vector<char> local(npreds, 0);
  uint32_t lw = 0;
  for (uint32_t p = 0; p < npreds; ++p) {
    uint32_t n = C.dict[P.preds[p].domain].size();
    nwords[p] = ((n + 63) / 64) * 2 + 2;
    if (!P.preds[p].global_only && lw + nwords[p] <= local_budget && n <= kMaxLocalPairs) {
      local[p] = 1;
      lw += nwords[p];
    }
  }
  const uint32_t blob = std::max(4u, (lw + 3) & ~3u);
  // Fused dictionary pass: when every small-domain (local) predicate's strings and the
  // pattern bytes fit the fuse budget, the scan blocks evaluate them in their prologue
  // from a pair table; the dictionary kernel then only runs for large domains.
  size_t fuse_strings = 0, fuse_pairs = 0;
  bool fusable = lw > 0 && PD.pats_h.size() <= 4096;
  for (uint32_t p = 0; p < npreds && fusable; ++p) {
    if (!local[p]) continue;
    const auto& D0 = C.dict[P.preds[p].domain];
    const uint32_t pend = p + 1 < PD.pat0.size() ? PD.pat0[p + 1] : (uint32_t)PD.pats_h.size();
    fuse_pairs += (size_t)D0.size() * (pend - PD.pat0[p]);
    for (uint32_t i = 0; i < D0.size(); ++i)
      if (D0.off[i + 1] - D0.off[i] > 4095) fusable = false;
  }
  std::vector<bool> dom_seen(KPE_NUM_DOMAINS, false);
  for (uint32_t p = 0; p < npreds; ++p)
    if (local[p] && !dom_seen[P.preds[p].domain]) {
      dom_seen[P.preds[p].domain] = true;
      fuse_strings += C.dict[P.preds[p].domain].bytes.size();
    }
  const size_t fuse_est = 2 * fuse_pairs + 4 * PD.pats_h.size() + (PD.pat_bytes_h.size() + fuse_strings) / 4 + 16;
  const bool fused = fusable && fuse_pairs <= kMaxFusePairs && fuse_est <= kMaxFuseWords &&
                     budget - (int64_t)blob - (int64_t)fuse_est >= 0;
  // LDS layout of a scan block (words): [bitsets][truth table][kind table][capability-set bits]
  // = the prologue image [0, img_end), then [filters + filter terms][4 wave regions]; the fuse
  // area (fused dictionary pass: the prep kernel, or scans without an image) comes last.
  const uint32_t tt_words = PD.tt ? (1u << P.terms.size()) : 0u;
  const uint32_t tt_at = blob;
  const uint32_t kt_at = tt_at + ((tt_words + 3) & ~3u);
  const uint32_t capb_at = kt_at + kt_words;
  const uint32_t img_end = capb_at + capb_words;
  const uint32_t prog_at = img_end;
  const uint32_t selt_at = (prog_at + (stage_prog ? prog_words : 0) + 3) & ~3u;
  const uint32_t kslot_at = (selt_at + selt_words + 1) & ~1u;
  const uint32_t wave_at = (kslot_at + kslot_words + 1) & ~1u;
  const uint32_t scan_end = wave_at + 4 * wave_words;
  const uint32_t fuse_at = (scan_end + 3) & ~3u;
  std::vector<uint32_t> dir(npreds);
  std::vector<PredJob> jobs;
  std::vector<uint32_t> fimg;  // fuse image (words)
  std::vector<uint32_t> pairs;
  std::vector<int64_t> dom_byte(KPE_NUM_DOMAINS, -1);  // byte offset of a domain's strings in the image
  uint32_t fpats_at = 0, fpatb_at = 0, fstr_at = 0;
  if (fused) {
    fpats_at = (uint32_t)((2 * fuse_pairs + 3) & ~(size_t)3);  // 16 B aligned pattern records
    fpatb_at = fpats_at + (uint32_t)PD.pats_h.size() * 4;
    fstr_at = fpatb_at + (uint32_t)(PD.pat_bytes_h.size() + 3) / 4;
    std::vector<uint8_t> strbytes;
    for (uint32_t p = 0; p < npreds; ++p) {
      const uint32_t d = P.preds[p].domain;
      if (!local[p] || dom_byte[d] >= 0) continue;
      dom_byte[d] = (int64_t)strbytes.size();
      strbytes.insert(strbytes.end(), C.dict[d].bytes.begin(), C.dict[d].bytes.end());
    }
    fimg.assign(fstr_at + (strbytes.size() + 3) / 4, 0);
    memcpy(fimg.data() + fpats_at, PD.pats_h.data(), PD.pats_h.size() * sizeof(KpePat));
    if (!PD.pat_bytes_h.empty()) memcpy(fimg.data() + fpatb_at, PD.pat_bytes_h.data(), PD.pat_bytes_h.size());
    if (!strbytes.empty()) memcpy(fimg.data() + fstr_at, strbytes.data(), strbytes.size());
    fimg.resize((fimg.size() + 3) & ~(size_t)3, 0);
  }
  uint32_t lo = 0, go = blob, blk = 0;
  for (uint32_t p = 0; p < npreds; ++p) {
    uint32_t at;
    if (local[p]) {
      at = lo;
      lo += nwords[p];
      dir[p] = PRED_LOCAL | at;  // LDS word index (== pbuf index inside the preamble)
    } else {
      at = go;
      go += nwords[p];
      dir[p] = at;
    }
    const uint32_t d = P.preds[p].domain, n = C.dict[d].size();
    if (n) {
      const uint32_t pend = p + 1 < PD.pat0.size() ? PD.pat0[p + 1] : (uint32_t)PD.pats_h.size();
      if (fused && local[p]) {
        const uint32_t str0 = (fuse_at + fstr_at) * 4 + (uint32_t)dom_byte[d];  // LDS byte address
        for (uint32_t i = 0; i < n; ++i)
          for (uint32_t k = PD.pat0[p]; k < pend; ++k) {
            const uint32_t w = at + (i >> 5);
            pairs.push_back((str0 + C.dict[d].off[i]) | ((C.dict[d].off[i + 1] - C.dict[d].off[i]) << 20));
            pairs.push_back(k | (w << 12) | ((i & 31u) << 27));
          }
      } else {
        jobs.push_back({d, PD.pat0[p], pend - PD.pat0[p], at, 0});
        blk = std::max(blk, (n + 255) / 256);  // grid x extent (grid y = jobs)
      }
    }
  }
  auto loc = [&](int32_t p) -> uint32_t { return p < 0 ? PRED_NONE : dir[(size_t)p]; };
  std::vector<KpeTerm> terms = P.terms;
  for (auto& t : terms)
    if (t.type == T_KIND_PRED || t.type == T_PRED) t.a = loc((int32_t)t.a);
  std::vector<KpeKindSel> kindsels = P.kindsels;
  for (auto& k : kindsels) {
    k.pg = (int32_t)loc(k.pg);
    k.pv = (int32_t)loc(k.pv);
    k.pk = (int32_t)loc(k.pk);
  }
  std::vector<KpeAnnPair> annpairs = P.annpairs;
  for (auto& x : annpairs) x.pk = (int32_t)loc(x.pk), x.pv = (int32_t)loc(x.pv);
  std::vector<KpeSelector> selectors = P.selectors;
  for (auto& x : selectors) x.p_kind_ns = (int32_t)loc(x.p_kind_ns), x.p_kind_empty = (int32_t)loc(x.p_kind_empty);
  std::vector<KpeSelReq> selreqs = P.selreqs;
  for (auto& x : selreqs)
    x.pk = (int32_t)loc(x.pk), x.pv = (int32_t)loc(x.pv), x.pk_ok = (int32_t)loc(x.pk_ok), x.pv_ok = (int32_t)loc(x.pv_ok);
  {  // selector requirement masks: one bit per requirement of each space, when it fits 64
    std::vector<uint32_t> rsel, nsel, rq, nq;
    for (const auto& t : P.terms)
      if (t.type == T_SELECTOR) rsel.push_back(t.a);
      else if (t.type == T_NSSELECTOR) nsel.push_back(t.a);
    for (auto& x : selectors) x.qbit = KPE_NO_QBIT;
    auto assign = [&](const std::vector<uint32_t>& sels, std::vector<uint32_t>& bits) -> bool {
      size_t tot = 0;
      for (uint32_t si : sels) tot += selectors[si].nreq;
      if (sels.empty() || tot > 64) return false;
      for (uint32_t si : sels) {
        selectors[si].qbit = (uint32_t)bits.size();
        for (uint32_t q = 0; q < selectors[si].nreq; ++q) bits.push_back(selectors[si].req0 + q);
      }
      return true;
    };
    B.selm = (assign(rsel, rq) ? 1u : 0u) | (assign(nsel, nq) ? 2u : 0u);
    for (auto& m : B.sm) m = 0;
    for (size_t b = 0; b < rq.size(); ++b) {
      const uint32_t op = selreqs[rq[b]].op;
      const int k = op == SR_EQ || op == SR_IN ? 0 : op == SR_WILD ? 1 : op == SR_NOTIN ? 2 : op == SR_EXISTS ? 3 : 4;
      B.sm[k] |= 1ull << b;
    }
    B.sel_nrq = (uint32_t)rq.size(), B.sel_nnq = (uint32_t)nq.size();
    if (B.selm) {
      HIPCHK(upload(B.sel_rq, rq.empty() ? std::vector<uint32_t>{0} : rq, s));
      HIPCHK(upload(B.sel_nq, nq.empty() ? std::vector<uint32_t>{0} : nq, s));
      HIPCHK(B.sel_km.ensure((size_t)std::max<uint32_t>(C.dict[D_LABK].size(), 1) * 16));
      HIPCHK(B.sel_vm.ensure((size_t)std::max<uint32_t>(C.dict[D_LABV].size(), 1) * 16));
      HIPCHK(B.sel_nsq.ensure(C.nsl_off.size() * 8));
    }
  }
  // selector terms with requirement-mask bits: the binding form (T_SELQ / T_NSSELQ) the scan
  // evaluates with one mask compare (KPE_SELQ=0 keeps the selector-record form, for A/B runs)
  static const bool selq_off = [] {
    const char* e = getenv("KPE_SELQ");
    return e && atoi(e) == 0;
  }();
  if (!selq_off) {
    auto kind_id = [&](const char* k) -> uint32_t {
      const int64_t id = C.dict[D_KIND].find(k);
      return id < 0 || id >= 0xFFFF ? 0xFFFFu : (uint32_t)id;
    };
    const uint32_t ns_kid = kind_id("Namespace"), empty_kid = kind_id("");
    for (auto& t : terms) {
      if ((t.type != T_SELECTOR || !(B.selm & 1u)) && (t.type != T_NSSELECTOR || !(B.selm & 2u))) continue;
      const KpeSelector& S = selectors[t.a];
      if (S.qbit == KPE_NO_QBIT || S.qbit > 63 || S.nreq > 64) continue;
      const bool ns = t.type == T_NSSELECTOR;
      // the kind predicates of a namespaceSelector are exactly "Namespace" and "" (program.cpp)
      if (ns && (P.preds[P.selectors[t.a].p_kind_ns].globs != std::vector<std::string>{"Namespace"} ||
                 P.preds[P.selectors[t.a].p_kind_empty].globs != std::vector<std::string>{""}))
        continue;
      const uint32_t f = (S.exc ? TSQ_EXC : 0u) | (S.star_kind ? TSQ_STAR : 0u) | (S.invalid ? TSQ_INVALID : 0u);
      t.a = S.qbit | S.nreq << 8 | f << 16;
      t.b = ns ? (ns_kid | empty_kid << 16) : 0u;
      t.type = ns ? T_NSSELQ : T_SELQ;
    }
  }
  for (size_t t = 0; t < terms.size(); ++t)  // kind terms answered by the GVK table (kind_table)
    if (kslot_words && kslot_of[t] >= 0) terms[t] = KpeTerm{T_KSLOT, (uint32_t)kslot_of[t], 0u, 0u};
  HIPCHK(upload(B.terms_r, terms, s));
  HIPCHK(upload(B.kindsels_r, kindsels, s));
  HIPCHK(upload(B.annpairs_r, annpairs, s));
  HIPCHK(upload(B.selectors_r, selectors, s));
  HIPCHK(upload(B.selreqs_r, selreqs, s));
  HIPCHK(upload(B.cv_classes, P.cv_classes, s));
  const auto& ps = P.pss;
  const int32_t fixed[10] = {ps.apparmor_key, ps.apparmor_val_ok, ps.seccomp_pod_key, ps.seccomp_ann_ok,
                             ps.caps_baseline_ok, ps.cap_nbs, ps.cap_all, ps.sysctl[0], ps.sysctl[1], ps.sysctl[2]};
  for (int k = 0; k < 10; ++k) B.pp[k] = loc(fixed[k]);
  for (const auto& tm : terms) lean = lean && (tm.type != T_KIND_PRED || ((tm.a & PRED_LOCAL) && tm.a != PRED_NONE));
  if (!P.pat.rules.empty() || P.any_fe_pat) {  // pattern members: names -> D_KEY ids + 1, glob names -> bitsets
    if (!C.has_docs) return fail(KPE_E_STATE, "pattern rules need a corpus flattened with KPE_CORPUS_DOCS");
    const auto& PP = P.pat;
    std::vector<int64_t> kid(PP.keys.size());
    for (size_t i = 0; i < PP.keys.size(); ++i) kid[i] = C.dict[D_KEY].find(PP.keys[i]);
    std::vector<uint32_t> mem(PP.members);
    for (size_t i = 0; i < mem.size(); i += 4) {
      mem[i + 1] = kid[mem[i + 1]] < 0 || (mem[i] & PMF_VKEY) ? 0u : (uint32_t)kid[mem[i + 1]] + 1u;
      if (mem[i] & PMF_GLOB) mem[i + 3] = loc((int32_t)mem[i + 3]);
      else if ((mem[i] & PMF_LEAF) && !(mem[i] & PMF_VKEY))  // the leaf's table slot (schema.h PMF_LEAF)
        mem[i + 3] = PD.lslot_h.empty() ? KPE_NO_LSLOT : PD.lslot_h[PP.nodes[mem[i + 2]].y];
    }
    HIPCHK(upload(B.pmembers, mem, s));
    B.pargs_valid = false;
    B.ltab_words = (uint32_t)(((uint64_t)C.scal.size() + 63) / 64 * 2);
    if (PD.nlslots) HIPCHK(B.ltab.ensure((size_t)PD.nlslots * B.ltab_words * 4 + 16));
  }
  if (!P.cond.rules.empty()) {  // condition field names -> D_KEY ids + 1
    if (!C.has_docs) return fail(KPE_E_STATE, "condition rules need a corpus flattened with KPE_CORPUS_DOCS");
    std::vector<uint32_t> fk(P.cond.fields.size());
    for (size_t i = 0; i < fk.size(); ++i) {
      const int64_t id = C.dict[D_KEY].find(P.cond.fields[i]);
      fk[i] = id < 0 ? 0u : (uint32_t)id + 1u;
    }
    HIPCHK(upload(B.cfkeys, fk, s));
    B.cargs_valid = false;
    if (!P.pat.vars.empty()) HIPCHK(B.pvals.ensure((size_t)C.n * P.pat.vars.size() * 8 + 8));
    if (P.cond.nmsg) {
      const size_t bytes = (size_t)C.n * P.cond.nmsg * 4;
      HIPCHK(B.mtrace.ensure(bytes + 4));
      HIPCHK(hipMemsetAsync(B.mtrace.p, 0, bytes + 4, s));
    }
  }
  if (!P.pssx.rules.empty()) {  // podSecurity exclusions: cold pod columns, key tables, resolved excludes
    auto& D = *cc->d;
    if (!D.cold) {
      HIPCHK(upload(D.ctr_off, C.ctr_off, s));
      HIPCHK(upload(D.vol_off, C.vol_off, s));
      HIPCHK(upload(D.sys_off, C.sys_off, s));
      HIPCHK(upload(D.pann_off, C.pann_off, s));
      HIPCHK(upload(D.c_name, C.c_name, s));
      HIPCHK(upload(D.c_image, C.c_image, s));
      HIPCHK(upload(D.c_sann_key, C.c_sann_key, s));
      HIPCHK(upload(D.c_sec_str, C.c_sec_str, s));
      HIPCHK(upload(D.c_pm_str, C.c_pm_str, s));
      HIPCHK(upload(D.c_selt_str, C.c_selt_str, s));
      HIPCHK(upload(D.c_selu_str, C.c_selu_str, s));
      HIPCHK(upload(D.c_selr_str, C.c_selr_str, s));
      HIPCHK(upload(D.cport_off, C.cport_off, s));
      HIPCHK(upload(D.cport_str, C.cport_str, s));
      HIPCHK(upload(D.pann_k, C.pann_k, s));
      HIPCHK(upload(D.pann_v, C.pann_v, s));
      HIPCHK(upload(D.p_cold, C.p_cold, s));
      D.cold = true;
    }
    // annotation keys with digit runs replaced by "*" (parseField's regexIndex), numbered
    const kpe::Dict& AK = C.dict[D_ANNK];
    std::unordered_map<std::string, uint32_t> nid;
    auto normalise = [](std::string_view k) {
      std::string o;
      for (size_t i = 0; i < k.size();) {
        if (k[i] >= '0' && k[i] <= '9') {
          while (i < k.size() && k[i] >= '0' && k[i] <= '9') ++i;
          o += '*';
        } else {
          o += k[i++];
        }
      }
      return o;
    };
    std::vector<uint32_t> norm(std::max<uint32_t>(AK.size(), 1u), KPE_NO_STR);
    for (uint32_t i = 0; i < AK.size(); ++i) norm[i] = nid.emplace(normalise(AK.at(i)), (uint32_t)nid.size()).first->second;
    std::vector<uint32_t> rf(std::max<size_t>(P.pssx.rf_ann.size(), 1), KPE_NO_STR);
    for (size_t i = 0; i < P.pssx.rf_ann.size(); ++i) {
      auto it = nid.find(P.pssx.rf_ann[i]);
      if (it != nid.end()) rf[i] = it->second;
    }
    HIPCHK(upload(B.ann_norm, norm, s));
    HIPCHK(upload(B.rf_ann, rf, s));
    std::vector<KpeXExcl> xe = P.pssx.excl;
    for (auto& x : xe) {
      x.img = (int32_t)loc(x.img);
      x.pv_misc = (int32_t)loc(x.pv_misc), x.pv_annv = (int32_t)loc(x.pv_annv);
      x.pv_sys = (int32_t)loc(x.pv_sys), x.pv_cap = (int32_t)loc(x.pv_cap);
    }
    HIPCHK(upload(B.xexcl, xe, s));
    for (int k = 0; k < 9; ++k) B.xpp[k] = loc(P.pssx_preds[k]);
    const int64_t kp = AK.find("seccomp.security.alpha.kubernetes.io/pod");
    const int64_t kf = AK.find("container.seccomp.security.alpha.kubernetes.io/fake");
    B.key_pod_sec = kp < 0 ? KPE_NO_STR : (uint32_t)kp;
    B.key_fake_sec = kf < 0 ? KPE_NO_STR : (uint32_t)kf;
    B.xargs_valid = false;
  }
  if (fused) memcpy(fimg.data(), pairs.data(), pairs.size() * 4);
  const uint32_t fuse_words = fused ? (uint32_t)fimg.size() : 0u;
  B.tt_lds = PD.tt ? tt_at : PRED_NONE;
  B.lean = lean;
  B.kt_lds = lean ? kt_at : PRED_NONE;
  B.nkinds = lean ? C.dict[D_KIND].size() : 0u;
  B.capb_lds = capb_at;
  B.fuse_lds = fuse_at;
  B.fuse_words = fuse_words;
  B.npairs = fused ? (uint32_t)(pairs.size() / 2) : 0u;
  B.fuse_pats = fuse_at + fpats_at;
  B.fuse_patb = fuse_at + fpatb_at;
  if (fused) HIPCHK(upload(B.fuse, fimg, s));
  B.filt_lds = stage_prog ? prog_at : PRED_NONE;
  B.fterm_lds = prog_at + 2 * (uint32_t)P.filters.size();
  B.wave_lds = wave_at;
  B.selt_lds = selt_words ? selt_at : PRED_NONE;
  B.kslot_lds = kslot_words ? kslot_at : PRED_NONE;
  B.nkslot_g = kslot_ng;
  if (kslot_words) HIPCHK(upload(B.kslot_tab, kslot_tab, s));
  B.wave_words = wave_words;
  B.prep_dyn_bytes = (size_t)(fuse_at + fuse_words) * 4;
  B.pimg_words = img_end;  // prologue image: LDS [0, img_end)
  HIPCHK(B.pimg.ensure((size_t)B.pimg_words * 4 + 16));
  B.dyn_bytes = (size_t)scan_end * 4;  // scans copy the image: no fuse area
  HIPCHK(B.pbuf.ensure((size_t)go * 4 + 16));
  HIPCHK(hipMemsetAsync(B.pbuf.p, 0, (size_t)go * 4 + 16, s));
  B.blob_words = blob;
  B.njobs = (uint32_t)jobs.size();
  B.nblocks = blk;
  // LEAN evaluations run kpe_lean6_kernel (buffer loads with 32-bit byte offsets: every column it
  // reads under 4 GiB), else the template instantiation (64-bit pointers)
  B.lean_kind = !lean ? 0 : lean6_fits(C, kLean6Limit) ? 7 : 2;
  // the PSA dictionary codes of the corpus (policy-independent; per distinct string)
  if (P.any_pss && !cc->d->codes_ready)
    if (kpe_status st = run_codes(C, *cc->d, s)) return st;
  // the general scan of a podSecurity program reads per-pod PSA records (PSUM instantiation, code
  // | 4) that kpe_psum_kernel rebuilds before it every time, or (KPE_PSUM=0) walks the pods' lists
  B.gen_code = (narrow ? 1 : 0) | (P.any_pss && !dev->no_psum ? 4 : 0);
  B.scan_blocks = kpe_scan_grid(C.n, P.any_pss ? 1 : 0, lean ? B.lean_kind : B.gen_code, B.dyn_bytes);
  HIPCHK(upload(B.jobs, jobs, s));
  {  // ApplyOne policies: contiguous rule ranges in ComputeRules order
    std::vector<uint32_t> segs;
    for (size_t r = 0; r < P.rules.size();) {
      size_t e = r + 1;
      while (e < P.rules.size() && P.rules[e].policy == P.rules[r].policy) ++e;
      if (P.rules[r].apply_one && e - r > 1) segs.push_back((uint32_t)r), segs.push_back((uint32_t)e);
      r = e;
    }
    B.napply_segs = (uint32_t)(segs.size() / 2);
    if (!segs.empty()) HIPCHK(upload(B.apply_segs, segs, s));
  }
  HIPCHK(B.verdicts.ensure(std::max<size_t>(cells, 4) + KPE_VERDICT_SLACK));  // the pattern kernel's row scan
  HIPCHK(B.counts_out.ensure(std::max<size_t>(P.rules.size() * 8, 1) * 8));
  if (!B.zero_page.p) {
    HIPCHK(B.zero_page.ensure(256));
    HIPCHK(hipMemsetAsync(B.zero_page.p, 0, 256, s));
  }
  if (want_masks) {
    HIPCHK(B.masks.ensure(std::max<size_t>(cells, 1) * 4));
    cc->d->has_masks = true;
  }
  if (getenv("KPE_DEBUG")) {
    fprintf(stderr, "kpe bind: n=%lld R=%zu narrow=%d blob=%u pred_jobs=%u pred_xblocks=%u scan_blocks=%u dyn=%zu "
            "wave_words=%u npairs=%u fuse_words=%u ncapsets=%zu selm=%u (%u, %u requirement bits)\n", (long long)C.n,
            P.rules.size(), (int)narrow, blob, (unsigned)jobs.size(), blk, B.scan_blocks, B.dyn_bytes, wave_words, B.npairs,
            fuse_words, C.capset_add.size(), B.selm, B.sel_nrq, B.sel_nnq);
  }
  HIPCHK(hipStreamSynchronize(s));
  B.need = need_flags(P);
  B.args_valid = false;
  B.inv_ready = false;
  B.prog = &P;
  B.cells = cells;
  return KPE_OK;
}

kpe_status lean6_launch(kpe_device* dev, const kpe::Program& P, const kpe::DeviceProgram& PD, kpe_corpus* const* cs,
                        size_t m, bool masks, hipStream_t s, double* bytes);

kpe_status launch(kpe_device* dev, const kpe_program* pp, kpe_corpus* cc, bool masks, bool cold = false) {
  auto& P = *pp->p;
  auto& C = *cc->c;
  auto& D = *cc->d;
  auto& PD = *P.devs[dev->ordinal];
  auto& B = D.bind;
  // timed launches are serialised on stream 0 so each kernel's events measure it alone
  hipStream_t s = dev->timing || B.lane < 0 ? dev->stream : dev->lanes[B.lane];
  if (B.last && B.last != s) HIPCHK(hipStreamSynchronize(B.last));  // keep this corpus's launches ordered
  B.last = s;
  kpe_device::EvPair ev{};
  if (dev->timing) {
    ev.a = dev->get_ev();
    ev.b = dev->get_ev();
    ev.c = dev->get_ev();
    ev.d = dev->get_ev();
    HIPCHK(hipEventRecord(ev.a, s));
  }
  const size_t R = P.rules.size();
  const bool fresh = !B.inv_ready || dev->no_cache || cold;
  if (cold && P.any_pss)  // a cold evaluation rebuilds the corpus's PSA dictionary codes too
    if (kpe_status st = run_codes(C, D, s)) return st;
  const bool lean_go = B.lean && (!masks || B.lean_kind == 7);  // LEAN6 writes check masks too
  const bool six = lean_go && B.lean_kind == 7;
  const bool psum_go = P.any_pss && !lean_go && !dev->no_psum;  // the PSUM scan and its per-pod records
  if (psum_go) HIPCHK(D.psum.ensure((size_t)C.n * 12 + 16));
  if (B.nblocks && fresh) {  // dictionary pass for large-domain predicates
    PredArgs pa{};
    for (int i = 0; i < KPE_NUM_DOMAINS; ++i) {
      pa.dict_bytes[i] = D.dict_bytes[i].as<uint8_t>();
      pa.dict_off[i] = D.dict_off[i].as<uint32_t>();
      pa.dict_n[i] = C.dict[i].size();
    }
    pa.pat_bytes = PD.pat_bytes.as<uint8_t>();
    pa.pat_len = (uint32_t)PD.pat_bytes_h.size();
    pa.pats = PD.pats.as<KpePat>();
    pa.jobs = B.jobs.as<PredJob>();
    pa.njobs = B.njobs;
    pa.out = B.pbuf.as<uint32_t>();
    HIPCHK(kpe_launch_pred(&pa, B.nblocks, s));
  }
  ScanArgs sa;
  memset(&sa, 0, sizeof(sa));  // padding too: compared bytewise
  sa.n = C.n;
  sa.r_gvk = D.r_gvk.as<uint32_t>();
  sa.r_name = D.r_name.as<uint32_t>();
  sa.r_mns = D.r_mns.as<uint32_t>();
  sa.r_nsa = D.r_nsa.as<uint32_t>();
  sa.ann_off = D.ann_off.as<uint32_t>();
  sa.ann_k = D.ann_k.as<uint32_t>();
  sa.ann_v = D.ann_v.as<uint32_t>();
  sa.lab_off = D.lab_off.as<uint32_t>();
  sa.lab_k = D.lab_k.as<uint32_t>();
  sa.lab_v = D.lab_v.as<uint32_t>();
  sa.r_nsl = D.r_nsl.as<uint32_t>();
  sa.nsl_off = D.nsl_off.as<uint32_t>();
  sa.nsl_k = D.nsl_k.as<uint32_t>();
  sa.nsl_v = D.nsl_v.as<uint32_t>();
  sa.rec = D.rec.as<uint32_t>();
  sa.hdr = D.hdr.as<uint32_t>();
  sa.crec = D.crec.as<uint32_t>();
  sa.vol_src = D.vol_src.as<uint32_t>();
  sa.sys_id = D.sys_id.as<uint32_t>();
  sa.pann_kv = D.pann_kv.as<uint32_t>();
  sa.c_sann = D.c_sann.as<uint32_t>();
  sa.ntiles = (uint32_t)((C.n + 63) / 64);
  sa.zero_page = B.zero_page.as<uint32_t>();
  sa.fuse = B.fuse.as<uint32_t>();
  sa.fuse_words = B.fuse_words;
  sa.fuse_lds = B.fuse_lds;
  sa.npairs = B.npairs;
  sa.fuse_pats = B.fuse_pats;
  sa.fuse_patb = B.fuse_patb;

  sa.capsets = D.capsets.as<uint32_t>();
  sa.ncapsets = (uint32_t)C.capset_add.size();
  sa.nctr_total = (uint32_t)C.c_sc.size();
  sa.nvol_total = (uint32_t)C.vol_src.size();
  sa.nsys_total = (uint32_t)C.sys_id.size();
  sa.npann_total = (uint32_t)(C.pann_kv.size() / 2);
  sa.rules = PD.rules.as<KpeRule>();
  sa.rule_exc = P.any_exc ? PD.rule_exc.as<uint32_t>() : nullptr;
  sa.rule_lanes = PD.rule_lanes.as<uint32_t>();
  sa.narrow_rules = PD.narrow_rules.as<uint32_t>();
  sa.fmask = PD.fmask.as<uint32_t>();
  sa.nfilters = (uint32_t)P.filters.size();
  sa.tt_lds = B.tt_lds;
  sa.ncls = PD.ncls;
  sa.pss_rules = PD.pss_rules;
  sa.err_rules = PD.err_rules;
  sa.pat_rules = PD.pat_rules;
  sa.narrow_cls = PD.narrow_cls.as<uint32_t>();
  sa.nrules = (uint32_t)R;
  sa.filters = PD.filters.as<KpeFilter>();
  sa.fterms = PD.fterms.as<uint32_t>();
  sa.terms = B.terms_r.as<KpeTerm>();
  sa.kindsels = B.kindsels_r.as<KpeKindSel>();
  sa.annpairs = B.annpairs_r.as<KpeAnnPair>();
  sa.selectors = B.selectors_r.as<KpeSelector>();
  sa.selreqs = B.selreqs_r.as<KpeSelReq>();
  sa.cv_classes = B.cv_classes.as<uint32_t>();
  sa.nterms = (uint32_t)P.terms.size();
  sa.ncv = (uint32_t)P.cv_classes.size();
  sa.any_apply_one = 0u;  // ApplyOne: kpe_apply_one_kernel after every evaluation kernel
  sa.filt_lds = B.filt_lds;
  sa.fterm_lds = B.fterm_lds;
  sa.nfterms = (uint32_t)P.fterms.size();
  sa.pbuf = B.pbuf.as<uint32_t>();
  sa.blob_words = B.blob_words;
  sa.wave_lds = B.wave_lds;
  sa.wave_words = B.wave_words;
  sa.pp_apparmor_key = B.pp[0];
  sa.pp_apparmor_ok = B.pp[1];
  sa.pp_seccomp_pod_key = B.pp[2];
  sa.pp_seccomp_ann_ok = B.pp[3];
  sa.pp_caps_ok = B.pp[4];
  sa.pp_cap_nbs = B.pp[5];
  sa.pp_cap_all = B.pp[6];
  sa.pp_sysctl0 = B.pp[7];
  sa.pp_sysctl1 = B.pp[8];
  sa.pp_sysctl2 = B.pp[9];
  sa.cv_union = P.cv_union;
  sa.need = B.need;
  sa.pimg = B.pimg_words ? B.pimg.as<uint32_t>() : nullptr;
  sa.pimg_words = B.pimg_words, sa.capb_lds = B.capb_lds;
  sa.kt_lds = B.kt_lds, sa.nkinds = B.nkinds;
  sa.psum = psum_go ? D.psum.as<uint32_t>() : nullptr;
  sa.selm = B.selm;
  sa.selt_lds = PRED_NONE;
  sa.kslot_lds = B.kslot_lds, sa.nkslot_g = B.nkslot_g;
  sa.kslot_tab = B.kslot_lds != PRED_NONE ? B.kslot_tab.as<uint32_t>() : nullptr;
  if (B.selm) {
    sa.sel_km = B.sel_km.as<uint4>(), sa.sel_vm = B.sel_vm.as<uint4>(), sa.ns_q = B.sel_nsq.as<uint64_t>();
    sa.ns_none = (uint32_t)C.nsl_off.size() - 1;
    sa.nlabk = C.dict[D_LABK].size(), sa.nlabv = C.dict[D_LABV].size();
    sa.selt_lds = (B.selm & 1u) ? B.selt_lds : PRED_NONE;
    sa.sm_pos = B.sm[0], sa.sm_wild = B.sm[1], sa.sm_notin = B.sm[2], sa.sm_exists = B.sm[3], sa.sm_dne = B.sm[4];
  }
  sa.verdicts = B.verdicts.as<uint8_t>();
  sa.masks = masks ? B.masks.as<uint32_t>() : nullptr;
  if (!B.args_valid || memcmp(&sa, &B.hargs, sizeof(ScanArgs)) != 0) {  // once per binding / masks mode
    HIPCHK(B.dargs.ensure(sizeof(ScanArgs)));
    B.hargs = sa;
    HIPCHK(hipMemcpyAsync(B.dargs.p, &B.hargs, sizeof(ScanArgs), hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    B.args_valid = true;
  }
  if (sa.pimg && fresh)
    HIPCHK(kpe_launch_prep(B.dargs.as<ScanArgs>(), P.any_pss ? 1 : 0, PD.narrow ? 1 : 0, B.prep_dyn_bytes, s));
  if (B.selm && fresh) {  // selector requirement masks, from the image's and pbuf's bitsets
    SelMaskArgs ma{};
    ma.pimg = B.pimg.as<uint32_t>();
    ma.pbuf = B.pbuf.as<uint32_t>();
    ma.reqs = B.selreqs_r.as<KpeSelReq>();
    ma.rq = B.sel_rq.as<uint32_t>(), ma.nq = B.sel_nq.as<uint32_t>();
    ma.nrq = B.sel_nrq, ma.nnq = B.sel_nnq;
    ma.nlabk = C.dict[D_LABK].size(), ma.nlabv = C.dict[D_LABV].size();
    ma.nrows = (uint32_t)C.nsl_off.size() - 1;
    ma.nsl_off = D.nsl_off.as<uint32_t>(), ma.nsl_k = D.nsl_k.as<uint32_t>(), ma.nsl_v = D.nsl_v.as<uint32_t>();
    ma.km = B.sel_km.as<uint4>(), ma.vm = B.sel_vm.as<uint4>(), ma.nsq = B.sel_nsq.as<uint64_t>();
    HIPCHK(kpe_launch_selmask(&ma, s));
  }
  B.inv_ready = true;
  ev.pre = fresh;
  if (dev->timing) HIPCHK(hipEventRecord(ev.b, s));
  double lbytes = 0;
  if (six) {  // the LEAN evaluation: every pod's record and lists, one kpe_lean6_kernel launch
    kpe_corpus* one = cc;
    if (kpe_status st = lean6_launch(dev, P, PD, &one, 1, masks, s, &lbytes)) return st;
  } else {
    // the general scan of a podSecurity program reads per-pod PSA records built right here
    if (psum_go)
      if (kpe_status st = run_psum(C, D, s)) return st;
    HIPCHK(kpe_launch_scan(B.dargs.as<ScanArgs>(), &B.hargs, C.n, P.any_pss ? 1 : 0, lean_go ? B.lean_kind : B.gen_code,
                           B.scan_blocks, B.dyn_bytes, s));
  }
  if (dev->timing) HIPCHK(hipEventRecord(ev.c, s));
  auto ensure_pargs = [&]() -> hipError_t {  // the binding's PatArgs (pattern kernel, foreach patterns)
    if (!B.pargs_valid) {
      PatArgs pa{};
      pa.n = C.n;
      pa.R = (uint32_t)R;
      pa.npr = (uint32_t)P.pat.rules.size();
      pa.doc = D.doc.as<uint32_t>();
      pa.doc_off = D.doc_off.as<uint64_t>();
      pa.perm = D.doc_perm.as<uint32_t>();  // rows by kind and tape size: C3 14.0 -> 8.5 ms, C5 27.6 -> 19.4 ms
      pa.scal = D.scal.as<KpeScalar>();
      pa.scal_text = D.scal_text.as<uint8_t>();
      pa.nodes = PD.pnodes.as<KpePNode>();
      pa.members = B.pmembers.as<uint4>();
      pa.lists = PD.plists.as<uint32_t>();
      pa.leaves = PD.pleaves.as<KpeLeaf>();
      pa.conds = PD.pconds.as<KpeCond>();
      pa.pats = PD.ppats.as<KpePat>();
      pa.pat_bytes = PD.pbytes.as<uint8_t>();
      pa.roots = PD.proots.as<uint32_t>();
      pa.rules = PD.prules.as<KpePatRule>();
      pa.col2pr = PD.pcol2pr.as<uint32_t>();
      for (uint32_t k = 0; k < KPE_PAT_MEMO; ++k) pa.slot_rule[k] = ~0u;
      for (uint32_t i = 0; i < (uint32_t)P.pat.rules.size(); ++i) {
        const uint32_t sl = P.pat.rules[i].flags >> PR_MEMO_SH;
        if (sl < KPE_PAT_MEMO && pa.slot_rule[sl] == ~0u) pa.slot_rule[sl] = i;
      }
      pa.pbuf = B.pbuf.as<uint32_t>();
      pa.pvals = P.pat.vars.empty() ? nullptr : B.pvals.as<uint2>();
      pa.nvars = (uint32_t)P.pat.vars.size();
      pa.ptmpl = PD.ptmpl.as<uint2>();
      pa.ttext = PD.ttext.as<uint8_t>();
      pa.ctab = PD.cconsts.as<KpeScalar>();
      pa.ctext = PD.ctext.as<uint8_t>();
      pa.verdicts = B.verdicts.as<uint8_t>();
      pa.lslot = PD.plslot.as<uint32_t>();
      pa.ltab = PD.nlslots ? B.ltab.as<uint32_t>() : nullptr;
      pa.ltab_words = B.ltab_words;
      pa.key_bytes = D.dict_bytes[D_KEY].as<uint8_t>(), pa.key_off = D.dict_off[D_KEY].as<uint32_t>();
      pa.nkeyd = C.dict[D_KEY].size();
      pa.nnodes = (uint32_t)P.pat.nodes.size(), pa.nmembers = (uint32_t)(P.pat.members.size() / 4);
      pa.nlists = (uint32_t)P.pat.lists.size(), pa.nleaves = (uint32_t)P.pat.leaves.size();
      pa.nconds = (uint32_t)P.pat.conds.size(), pa.npats = (uint32_t)P.pat.operands.size();
      pa.nroots = (uint32_t)P.pat.roots.size(), pa.npbuf = (uint32_t)(B.pbuf.bytes / 4);
      pa.nscal = C.scal.size(), pa.ndoc = C.doc.size() / 2;
      PCHK(B.perr.ensure(4));
      PCHK(hipMemsetAsync(B.perr.p, 0, 4, s));
      pa.err = B.perr.as<uint32_t>();
      PCHK(B.pdeep.ensure(4));
      pa.deep_any = B.pdeep.as<uint32_t>();
      PCHK(B.pargs.ensure(sizeof(PatArgs)));
      PCHK(hipMemcpyAsync(B.pargs.p, &pa, sizeof(PatArgs), hipMemcpyHostToDevice, s));
      PCHK(hipStreamSynchronize(s));
      B.pargs_valid = true;
    }
    return hipSuccess;
  };
  if (fresh && PD.nlslots && (!P.pat.rules.empty() || P.any_fe_pat)) {  // the binding's leaf table
    HIPCHK(ensure_pargs());
    HIPCHK(kpe_launch_leaf_table(B.pargs.as<PatArgs>(), PD.pslot_leaf.as<uint32_t>(), PD.nlslots, C.scal.size(), s));
  }
  if (!P.cond.rules.empty()) {
    if (!B.cargs_valid) {
      CondArgs ca{};
      ca.n = C.n;
      ca.R = (uint32_t)R;
      ca.ncr = (uint32_t)P.cond.rules.size();
      ca.doc = D.doc.as<uint32_t>();
      ca.doc_off = D.doc_off.as<uint64_t>();
      ca.img_off = C.img_off.empty() ? nullptr : D.img_off.as<uint64_t>();
      ca.perm = D.doc_perm.as<uint32_t>();
      ca.scal = D.scal.as<KpeScalar>();
      ca.scal_text = D.scal_text.as<uint8_t>();
      ca.key_bytes = D.dict_bytes[D_KEY].as<uint8_t>();
      ca.key_off = D.dict_off[D_KEY].as<uint32_t>();
      ca.ops = PD.cops.as<uint2>();
      ca.exprs = PD.cexprs.as<KpeCExpr>();
      ca.tmpls = PD.ctmpls.as<KpeVTmpl>();
      ca.conds = PD.cconds.as<KpeCCond>();
      ca.blocks = PD.cblocks.as<KpeCBlock>();
      ca.fes = PD.cfes.as<KpeCForeach>();
      ca.rules = PD.crules.as<KpeCRule>();
      ca.ctab = PD.cconsts.as<KpeScalar>();
      ca.ctext = PD.ctext.as<uint8_t>();
      ca.clist = PD.cclist.as<uint32_t>();
      ca.tpieces = PD.ctpieces.as<uint2>();
      ca.txt = P.cond.tpieces.empty() ? 0u : 1u;
      ca.fkeys = B.cfkeys.as<uint32_t>();
      ca.leaves = PD.pleaves.as<KpeLeaf>();
      ca.pconds = PD.pconds.as<KpeCond>();
      ca.pats = PD.ppats.as<KpePat>();
      ca.pat_bytes = PD.pbytes.as<uint8_t>();
      if (P.any_fe_pat) {
        HIPCHK(ensure_pargs());
        ca.pat = B.pargs.as<PatArgs>();
      }
      ca.pvars = PD.pvars.as<KpePVar>();
      ca.pvals = P.pat.vars.empty() ? nullptr : B.pvals.as<uint2>();
      ca.nvars = (uint32_t)P.pat.vars.size();
      ca.verdicts = B.verdicts.as<uint8_t>();
      ca.nmsg = P.cond.nmsg;
      ca.mtrace = P.cond.nmsg ? B.mtrace.as<uint32_t>() : nullptr;
      HIPCHK(B.cargs.ensure(sizeof(CondArgs)));
      HIPCHK(hipMemcpyAsync(B.cargs.p, &ca, sizeof(CondArgs), hipMemcpyHostToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
      B.cargs_valid = true;
    }
    HIPCHK(kpe_launch_cond(B.cargs.as<CondArgs>(), C.n, P.any_fe_pat ? 1 : 0, P.cond.tpieces.empty() ? 0 : 1, s));
  }
  if (!P.pssx.rules.empty()) {
    if (!B.xargs_valid || (masks ? B.masks.p : nullptr) != B.xmasks) {
      PssxArgs xa{};
      xa.n = C.n;
      xa.R = (uint32_t)R;
      xa.nxr = (uint32_t)P.pssx.rules.size();
      xa.rules = PD.xrules.as<KpeXRule>();
      xa.excl = B.xexcl.as<KpeXExcl>();
      xa.rec = D.rec.as<uint32_t>();
      xa.ctr_off = D.ctr_off.as<uint32_t>();
      xa.vol_off = D.vol_off.as<uint32_t>();
      xa.sys_off = D.sys_off.as<uint32_t>();
      xa.pann_off = D.pann_off.as<uint32_t>();
      xa.crec = D.crec.as<uint32_t>();
      xa.capsets = D.capsets.as<uint32_t>();
      xa.c_name = D.c_name.as<uint32_t>();
      xa.c_image = D.c_image.as<uint32_t>();
      xa.c_sann = D.c_sann.as<uint32_t>();
      xa.c_sann_key = D.c_sann_key.as<uint32_t>();
      xa.c_sec_str = D.c_sec_str.as<uint32_t>();
      xa.c_pm_str = D.c_pm_str.as<uint32_t>();
      xa.c_selt_str = D.c_selt_str.as<uint32_t>();
      xa.c_selu_str = D.c_selu_str.as<uint32_t>();
      xa.c_selr_str = D.c_selr_str.as<uint32_t>();
      xa.cport_off = D.cport_off.as<uint32_t>();
      xa.cport_str = D.cport_str.as<uint32_t>();
      xa.vol_src = D.vol_src.as<uint32_t>();
      xa.sys_id = D.sys_id.as<uint32_t>();
      xa.pann_k = D.pann_k.as<uint32_t>();
      xa.pann_v = D.pann_v.as<uint32_t>();
      xa.p_cold = D.p_cold.as<uint32_t>();
      xa.misc_off = D.dict_off[D_MISC].as<uint32_t>();
      xa.annv_off = D.dict_off[D_ANNV].as<uint32_t>();
      xa.sysd_off = D.dict_off[D_SYSCTL].as<uint32_t>();
      xa.ann_norm = B.ann_norm.as<uint32_t>();
      xa.rf_ann = B.rf_ann.as<uint32_t>();
      xa.key_pod_sec = B.key_pod_sec;
      xa.key_fake_sec = B.key_fake_sec;
      xa.pbuf = B.pbuf.as<uint32_t>();
      xa.pp_apparmor_key = B.xpp[0], xa.pp_apparmor_ok = B.xpp[1], xa.pp_seccomp_ok = B.xpp[2];
      xa.pp_caps_ok = B.xpp[3], xa.pp_nbs = B.xpp[4], xa.pp_all = B.xpp[5];
      for (int v = 0; v < 3; ++v) xa.pp_sysctl[v] = B.xpp[6 + v];
      xa.verdicts = B.verdicts.as<uint8_t>();
      xa.masks = masks ? B.masks.as<uint32_t>() : nullptr;
      HIPCHK(B.xargs.ensure(sizeof(PssxArgs)));
      HIPCHK(hipMemcpyAsync(B.xargs.p, &xa, sizeof(PssxArgs), hipMemcpyHostToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
      B.xmasks = masks ? B.masks.p : nullptr;
      B.xargs_valid = true;
    }
    HIPCHK(kpe_launch_pssx(B.xargs.as<PssxArgs>(), C.n, s));
  }
  if (!P.pat.rules.empty()) {
    HIPCHK(ensure_pargs());
    HIPCHK(hipMemsetAsync(B.pdeep.p, 0, 4, s));  // PatArgs::deep_any
    HIPCHK(kpe_launch_pattern(B.pargs.as<PatArgs>(), C.n, (uint32_t)P.pat.rules.size(), PD.ltab_all ? 1 : 0, s));
    if (dev->patvm_err) {  // bounds flags of a KPE_PATVM_CHECK build (scripts/pvchk.py)
      uint32_t e = 0;
      HIPCHK(hipMemcpyAsync(&e, B.perr.p, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      fprintf(stderr, "kpe patvm err=0x%x\n", e);
    }
  }
  if (B.napply_segs)  // applyRules: One (validation.go:75-77) over the final verdicts of every kernel
    HIPCHK(kpe_launch_apply_one(B.verdicts.as<uint8_t>(), masks ? B.masks.as<uint32_t>() : nullptr, C.n, (uint32_t)R,
                                B.apply_segs.as<uint32_t>(), B.napply_segs, s));
  if (!C.limit_rows.empty())  // last: no later kernel may resolve these cells
    HIPCHK(kpe_launch_fill_rows(B.verdicts.as<uint8_t>(), (uint32_t)R, D.limit_rows.as<uint32_t>(),
                                (uint32_t)C.limit_rows.size(), KPE_UNDECIDED_, s));
  if (dev->timing) {
    HIPCHK(hipEventRecord(ev.d, s));
    ev.post = !P.cond.rules.empty() || !P.pssx.rules.empty() || !P.pat.rules.empty() || B.napply_segs || !C.limit_rows.empty();
    const bool ps = psum_go;
    ev.bytes = six ? lbytes : scan_bytes(P, C, B.need, masks, ps) + (ps ? psum_bytes(C, D, B.need) : 0.0);
    ev.pbytes = P.pat.rules.empty() ? 0.0 : (double)C.doc.size() * 4.0 + (double)C.n * (8.0 + 2.0 * (double)R);
    ev.kind = lean_go ? B.lean_kind : 1;
    dev->pending.push_back(ev);
  }
  return KPE_OK;
}

// One kpe_lean6_kernel launch over the m bound shards cs of program P on stream s (bytes: their
// algorithmic bytes). Tiles per wave: the most (up to 4) that still leaves dev->lean_min_waves
// waves; the corpora's code bytes are staged in LDS per block when they fit (LC).
kpe_status lean6_launch(kpe_device* dev, const kpe::Program& P, const kpe::DeviceProgram& PD, kpe_corpus* const* cs,
                        size_t m, bool masks, hipStream_t s, double* bytes) {
  const uint32_t R = (uint32_t)P.rules.size();
  LeanBatchArgs a;
  memset(&a, 0, sizeof(a));
  a.nshards = (uint32_t)m, a.nrules = R, a.ncls = PD.ncls, a.cv_union = P.cv_union;
  a.pss_rules = PD.pss_rules, a.err_rules = PD.err_rules, a.pat_rules = PD.pat_rules;
  a.narrow_cls = PD.narrow_cls.as<uint32_t>();
  uint64_t tiles = 0;
  uint32_t code_max = 0;
  for (size_t k = 0; k < m; ++k) {
    tiles += (uint64_t)(cs[k]->c->n + 63) / 64;
    code_max = std::max(code_max, cs[k]->d->psa_L.bytes);
  }
  const bool lc = code_max <= kLeanCodeLds;
  uint32_t tpw = lc ? 4 : 2;  // 4 tiles with global code reads would spill
  while (tpw > 1 && tiles / tpw < dev->lean_min_waves) tpw >>= 1;
  if (dev->lean_tpw) tpw = std::min(dev->lean_tpw, lc ? 4u : 2u);
  a.tpw = tpw;
  uint32_t acc = 0, kt_max = 0;
  *bytes = 0;
  for (size_t k = 0; k < m; ++k) {
    auto& C = *cs[k]->c;
    auto& D = *cs[k]->d;
    auto& B = D.bind;
    LeanShard& sh = a.sh[k];
    sh.rec = D.rec.as<uint32_t>(), sh.hdr = D.hdr.as<uint32_t>(), sh.crec = D.crec.as<uint32_t>();
    sh.vol = D.vol_src.as<uint32_t>(), sh.sys = D.sys_id.as<uint32_t>(), sh.pann = D.pann_kv.as<uint32_t>();
    sh.sann = D.c_sann.as<uint32_t>();
    sh.codes = D.psa_codes.as<uint8_t>();
    sh.kt = B.pimg.as<uint32_t>() + B.kt_lds;
    sh.verdicts = B.verdicts.as<uint8_t>();
    sh.masks = masks ? B.masks.as<uint32_t>() : nullptr;
    sh.n = (uint32_t)C.n, sh.nkinds = B.nkinds;
    sh.nctr = (uint32_t)C.c_sc.size(), sh.nvol = (uint32_t)C.vol_src.size(), sh.nsys = (uint32_t)C.sys_id.size();
    sh.npann = (uint32_t)(C.pann_kv.size() / 2);
    sh.L = D.psa_L;
    a.blk0[k] = acc;
    acc += (uint32_t)((C.n + 256 * tpw - 1) / (256 * tpw));  // 4 waves x tpw tiles of 64 pods per block
    kt_max = std::max(kt_max, B.nkinds);
    a.need |= B.need;
    *bytes += lean_bytes(C, D, B.need, R, masks);
  }
  a.blk0[m] = acc;
  a.kt_words = (kt_max + 3u) & ~3u;
  a.code_words = lc ? ((code_max + 15u) / 16u) * 4u : 0u;
  a.wave_words = ((KPE_L6_STAGE_BYTES + 64u * R + 15u) / 16u) * 4u;
  const size_t dyn = 4 * ((size_t)a.kt_words + a.code_words + 4 * (size_t)a.wave_words);
  HIPCHK(kpe_launch_lean6(&a, dyn, lc ? 1 : 0, s));
  return KPE_OK;
}

// A shard can ride in a multi-shard LEAN launch when its evaluation is that one kernel: a bound
// LEAN binding (prologue image and PSA dictionary codes built) of a program with no later
// kernels, and no rows past an encoding limit.
bool lean_batchable(const kpe_device* dev, const kpe_program* pp, const kpe_corpus* cc) {
  const auto& P = *pp->p;
  const auto& C = *cc->c;
  const auto& D = *cc->d;
  const auto& B = D.bind;
  return !dev->no_cache && B.prog == &P && B.inv_ready && B.lean && B.lean_kind == 7 && D.codes_ready && C.n > 0 &&
         B.nkinds <= kLeanBatchKinds && P.cond.rules.empty() && P.pssx.rules.empty() && P.pat.rules.empty() &&
         !B.napply_segs && C.limit_rows.empty();
}

// The shards of `run` in ceil(m / KPE_LEAN_BATCH) launches of near-equal size on the device
// stream (equal per-launch bytes, so a launch's events time the same work); clears `run`.
kpe_status launch_lean_run(kpe_device* dev, const kpe_program* pp, std::vector<kpe_corpus*>& run, bool masks) {
  if (run.empty()) return KPE_OK;
  if (run.size() == 1) {
    kpe_corpus* c = run[0];
    run.clear();
    return launch(dev, pp, c, masks);
  }
  auto& P = *pp->p;
  auto& PD = *P.devs[dev->ordinal];
  hipStream_t s = dev->stream;
  const size_t m = run.size(), nl = (m + KPE_LEAN_BATCH - 1) / KPE_LEAN_BATCH;
  for (size_t l = 0, i = 0; l < nl; ++l) {
    const size_t cnt = (m - i) / (nl - l);
    for (size_t k = 0; k < cnt; ++k) {
      auto& B = run[i + k]->d->bind;
      if (B.last && B.last != s) HIPCHK(hipStreamSynchronize(B.last));  // keep this corpus's launches ordered
      B.last = s;
    }
    kpe_device::EvPair ev{};
    if (dev->timing) {
      ev.a = dev->get_ev(), ev.b = dev->get_ev(), ev.c = dev->get_ev(), ev.d = dev->get_ev();
      HIPCHK(hipEventRecord(ev.a, s));
      HIPCHK(hipEventRecord(ev.b, s));
    }
    double bytes = 0;
    if (kpe_status st = lean6_launch(dev, P, PD, run.data() + i, cnt, masks, s, &bytes)) return st;
    i += cnt;
    if (dev->timing) {
      HIPCHK(hipEventRecord(ev.c, s));
      HIPCHK(hipEventRecord(ev.d, s));
      ev.bytes = bytes, ev.pbytes = 0, ev.kind = 9, ev.pre = ev.post = false;
      dev->pending.push_back(ev);
    }
  }
  run.clear();
  return KPE_OK;
}

kpe_status prepare(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, bool masks) {
  if (!dev || !prog || !c) return fail(KPE_E_INVALID, "null argument");
  if (!c->d || c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  HIPCHK(hipSetDevice(dev->ordinal));
  kpe_status st = ensure_program(dev, prog);
  if (st) return st;
  return ensure_binding(dev, prog, const_cast<kpe_corpus*>(c), masks);
}

}  // namespace

extern "C" {

kpe_status kpe_evaluate_async(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c) {
  if (!dev) return fail(KPE_E_INVALID, "null device");
  std::lock_guard<std::mutex> lk(dev->mu);
  kpe_status st = prepare(dev, prog, c, false);
  if (st) return st;
  return launch(dev, prog, const_cast<kpe_corpus*>(c), false);
}

kpe_status kpe_evaluate_async_ex(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, unsigned flags) {
  if (!dev) return fail(KPE_E_INVALID, "null device");
  if (flags & ~(unsigned)(KPE_EVAL_MASKS | KPE_EVAL_COLD)) return fail(KPE_E_INVALID, "unknown evaluation flags");
  std::lock_guard<std::mutex> lk(dev->mu);
  const bool masks = (flags & KPE_EVAL_MASKS) != 0;
  kpe_status st = prepare(dev, prog, c, masks);
  if (st) return st;
  return launch(dev, prog, const_cast<kpe_corpus*>(c), masks, (flags & KPE_EVAL_COLD) != 0);
}

kpe_status kpe_evaluate_batch_async(kpe_device* dev, const kpe_program* prog, const kpe_corpus* const* cs, int n,
                                    unsigned flags) {
  if (!dev || (n > 0 && !cs)) return fail(KPE_E_INVALID, "null argument");
  if (flags & ~(unsigned)(KPE_EVAL_MASKS | KPE_EVAL_COLD)) return fail(KPE_E_INVALID, "unknown evaluation flags");
  std::lock_guard<std::mutex> lk(dev->mu);
  const bool masks = (flags & KPE_EVAL_MASKS) != 0, cold = (flags & KPE_EVAL_COLD) != 0;
  // Consecutive shards whose evaluation is the LEAN evaluation alone go out as multi-shard launches
  // (kpe_lean6_kernel); any other shard is launched on its own, in order.
  std::vector<kpe_corpus*> run;
  for (int i = 0; i < n; ++i) {
    if (kpe_status st = prepare(dev, prog, cs[i], masks)) return st;
    kpe_corpus* c = const_cast<kpe_corpus*>(cs[i]);
    if (!cold && lean_batchable(dev, prog, c)) {
      run.push_back(c);
      continue;
    }
    if (kpe_status st = launch_lean_run(dev, prog, run, masks)) return st;
    if (kpe_status st = launch(dev, prog, c, masks, cold)) return st;
  }
  return launch_lean_run(dev, prog, run, masks);
}

kpe_status kpe_device_sync(kpe_device* dev) {
  if (!dev) return fail(KPE_E_INVALID, "null device");
  HIPCHK(hipSetDevice(dev->ordinal));
  for (int k = 0; k < dev->nlanes; ++k) HIPCHK(hipStreamSynchronize(dev->lanes[k]));
  return KPE_OK;
}

kpe_status kpe_corpus_psa_summary(kpe_device* dev, kpe_corpus* c, uint32_t* out) {
  if (!dev || !c || !out) return fail(KPE_E_INVALID, "null argument");
  if (!c->d || c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& D = *c->d;
  if (D.bind.last) HIPCHK(hipStreamSynchronize(D.bind.last));
  // the summary pass again, with its 2-word summaries written out (the scan records it rewrites
  // are the same)
  DevBuf summ;
  HIPCHK(summ.ensure((size_t)c->c->n * 8 + 16));
  if (kpe_status st = run_psum(*c->c, D, dev->stream, summ.as<uint32_t>())) return st;
  if (c->c->n) HIPCHK(hipMemcpyAsync(out, summ.p, (size_t)c->c->n * 8, hipMemcpyDeviceToHost, dev->stream));
  HIPCHK(hipStreamSynchronize(dev->stream));
  return KPE_OK;
}

static const uint8_t kCvCheck[KPE_NUM_CV] = KPE_CV_CHECK_TABLE;

// The scan kernel stores failing versioned checks; the public masks are per PSA check id.
static void cv_to_check_masks(uint32_t* m, size_t cells) {
  for (size_t i = 0; i < cells; ++i) {
    uint32_t f = m[i] & KPE_CVM_CHECKS, c = 0;
    while (f) {
      c |= 1u << kCvCheck[__builtin_ctz(f)];
      f &= f - 1;
    }
    m[i] = c;
  }
}

static kpe_status fetch_impl(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint8_t* verdicts,
                             uint32_t* masks, kpe_counts* counts, bool raw_cv) {
  if (!dev || !prog || !c || !c->d) return fail(KPE_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  if (B.prog != prog->p.get()) return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  size_t R = prog->p->rules.size(), cells = (size_t)c->c->n * R;
  hipStream_t s = B.last ? B.last : dev->stream;
  if (counts && R) {
    // per-rule totals from the verdict matrix (processor/result.go:34-68 counting)
    HIPCHK(kpe_launch_count(B.verdicts.as<uint8_t>(), c->c->n, (uint32_t)R, B.counts_out.as<unsigned long long>(), s));
    const unsigned long long* src = B.counts_out.as<unsigned long long>();
    std::vector<unsigned long long> h(R * 8);
    HIPCHK(hipMemcpyAsync(h.data(), src, R * 8 * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (size_t r = 0; r < R; ++r) {
      uint64_t tot = 0;
      for (int k = 1; k < 8; ++k) tot += h[r * 8 + k];
      counts[r].na = (uint64_t)c->c->n - tot;
      counts[r].pass = h[r * 8 + 1];
      counts[r].fail = h[r * 8 + 2];
      counts[r].warn = h[r * 8 + 3];
      counts[r].error = h[r * 8 + 4];
      counts[r].skip = h[r * 8 + 5];
      counts[r].undecided = h[r * 8 + 7];
    }
  }
  HIPCHK(hipStreamSynchronize(s));
  if (verdicts && cells) HIPCHK(hipMemcpy(verdicts, B.verdicts.p, cells, hipMemcpyDeviceToHost));
  if (masks && cells) {
    if (!c->d->has_masks) return fail(KPE_E_STATE, "check masks were not computed");
    HIPCHK(hipMemcpy(masks, B.masks.p, cells * 4, hipMemcpyDeviceToHost));
    if (!raw_cv) cv_to_check_masks(masks, cells);
  }
  return KPE_OK;
}

kpe_status kpe_fetch(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint8_t* verdicts,
                     uint32_t* masks, kpe_counts* counts) {
  return fetch_impl(dev, prog, c, verdicts, masks, counts, false);
}

kpe_status kpe_fetch_cv_masks(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint32_t* cv_masks) {
  if (!cv_masks) return fail(KPE_E_INVALID, "null cv_masks");
  return fetch_impl(dev, prog, c, nullptr, cv_masks, nullptr, true);
}

kpe_status kpe_evaluate(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint8_t* verdicts,
                        uint32_t* masks, kpe_counts* counts) {
  {
    if (!dev) return fail(KPE_E_INVALID, "null device");
    std::lock_guard<std::mutex> lk(dev->mu);
    kpe_status st = prepare(dev, prog, c, masks != nullptr);
    if (st) return st;
    st = launch(dev, prog, const_cast<kpe_corpus*>(c), masks != nullptr);
    if (st) return st;
  }
  return kpe_fetch(dev, prog, c, verdicts, masks, counts);
}

// ---- verdict exchange and multi-device evaluation --------------------------------------------
kpe_status kpe_device_verdicts(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, void** dptr,
                               uint64_t* bytes) {
  if (!dev || !prog || !c || !c->d || !dptr) return fail(KPE_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  if (B.prog != prog->p.get()) return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  if (c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  if (B.last) HIPCHK(hipStreamSynchronize(B.last));
  *dptr = B.verdicts.p;
  if (bytes) *bytes = (uint64_t)c->c->n * prog->p->rules.size();
  return KPE_OK;
}

uint64_t kpe_packed_words(uint64_t cells) { return (cells + 9u) / 10u; }

kpe_status kpe_pack_verdicts(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint32_t* dst_dev,
                             uint64_t words) {
  if (!dev || !prog || !c || !c->d || !dst_dev) return fail(KPE_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  if (B.prog != prog->p.get()) return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  if (c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  const uint64_t cells = (uint64_t)c->c->n * prog->p->rules.size();
  if (words < kpe_packed_words(cells)) return fail(KPE_E_INVALID, "packed buffer too small");
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, dst_dev) != hipSuccess || at.type != hipMemoryTypeDevice || at.device != dev->ordinal) {
    (void)hipGetLastError();
    return fail(KPE_E_INVALID, "dst_dev is not device memory of this device");
  }
  hipStream_t s = B.last ? B.last : dev->stream;
  HIPCHK(kpe_launch_pack3(B.verdicts.as<uint8_t>(), cells, dst_dev, s));
  HIPCHK(hipStreamSynchronize(s));
  return KPE_OK;
}

kpe_status kpe_unpack_verdicts(const uint32_t* packed, uint64_t cells, uint8_t* out) {
  if ((!packed || !out) && cells) return fail(KPE_E_INVALID, "null argument");
  for (uint64_t i = 0; i < cells; ++i) out[i] = (uint8_t)((packed[i / 10u] >> (3u * (uint32_t)(i % 10u))) & 7u);
  return KPE_OK;
}

// ---- failing paths of pattern cells (report time) ---------------------------------------------
// The foreach entry that decided a FAIL / ERROR cell from its trace words (schema.h FT_*): the
// entry index in Program::fe_reports, or -1 (no valid path)
static int64_t fe_decider(const kpe::Program& P, const kpe::RuleReport& rr, uint32_t b) {
  if (!rr.foreach || !(b & FT_VALID) || (b & FT_OVERFLOW)) return -1;
  uint32_t first = rr.fe0, count = rr.nfe;
  int64_t e = -1;
  for (uint32_t l = 0; l <= FT_DEPTH(b); ++l) {
    const uint32_t left = FT_LEFT(b, l);
    if (left == 0 || left > count) return -1;
    e = (int64_t)first + (count - left);
    if ((size_t)e >= P.fe_reports.size()) return -1;
    if (l < FT_DEPTH(b)) {
      const kpe::FeReport& f = P.fe_reports[(size_t)e];
      if (f.kind != FE_NEST) return -1;
      first = f.nested0, count = f.nnested;
    }
  }
  return e;
}

kpe_status kpe_pattern_traces(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, const uint64_t* cells,
                              uint64_t ncells, uint32_t* out) {
  if (!dev || !prog || !c || !c->d || (ncells && (!cells || !out))) return fail(KPE_E_INVALID, "null argument");
  if (!ncells) return KPE_OK;
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  const kpe::Program& P = *prog->p;
  if (B.prog != prog->p.get()) return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  if (c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  const size_t R = P.rules.size();
  const uint64_t total = (uint64_t)c->c->n * R;
  for (uint64_t i = 0; i < ncells; ++i)
    if (cells[i] >= total) return fail(KPE_E_INVALID, "cell index past the verdict matrix");
  const size_t rec = (size_t)KPE_TRACE_ROOTS * KPE_TRACE_WORDS;
  hipStream_t s = B.last ? B.last : dev->stream;
  // foreach cells decided by a pattern entry: the entry's roots on the element (the condition
  // kernel's trace words of the cell)
  std::vector<uint4> jobs;
  if (P.any_fe_pat && B.cargs_valid && P.cond.nmsg) {
    std::vector<int32_t> slot(R, -1);
    for (const KpeCRule& cr : P.cond.rules)
      if (cr.mslot && cr.kind == CR_FOREACH) slot[cr.col] = (int32_t)cr.mslot - 1;
    HIPCHK(hipStreamSynchronize(s));
    for (uint64_t i = 0; i < ncells; ++i) {
      const uint64_t row = cells[i] / R;
      const uint32_t col = (uint32_t)(cells[i] % R);
      if (slot[col] < 0) continue;
      if (jobs.empty()) jobs.assign(ncells, make_uint4(0u, 0u, 0u, 0u));
      uint32_t w[KPE_FE_TRACE_WORDS];
      HIPCHK(hipMemcpy(w, B.mtrace.as<uint32_t>() + row * P.cond.nmsg + (size_t)slot[col], sizeof w,
                       hipMemcpyDeviceToHost));
      if (FT_KIND(w[1]) != FT_PAT || w[3] == 0xFFFFFFFEu) continue;
      const int64_t e = fe_decider(P, P.reports[col], w[1]);
      if (e < 0) continue;
      const KpeCForeach& fe = P.cond.fes[(size_t)e];
      if (fe.kind != FE_PAT) continue;
      jobs[i] = make_uint4(fe.a, fe.b, w[3], 1u);
    }
  }
  if (P.pat.rules.empty() && jobs.empty()) {  // no pattern walk: every record is empty
    memset(out, 0, ncells * rec * 4);
    return KPE_OK;
  }
  if (!B.pargs_valid) return fail(KPE_E_STATE, "the binding has no completed evaluation of its pattern rules");
  void *dc = nullptr, *dout = nullptr, *dj = nullptr;
  hipError_t e = hipMalloc(&dc, ncells * 8);
  if (e == hipSuccess) e = hipMalloc(&dout, ncells * rec * 4);
  if (e == hipSuccess && !jobs.empty()) e = hipMalloc(&dj, ncells * sizeof(uint4));
  if (e == hipSuccess) e = hipMemcpyAsync(dc, cells, ncells * 8, hipMemcpyHostToDevice, s);
  if (e == hipSuccess && dj) e = hipMemcpyAsync(dj, jobs.data(), ncells * sizeof(uint4), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = kpe_launch_pattern_trace(B.pargs.as<PatArgs>(), (const uint64_t*)dc, ncells, (uint32_t*)dout,
                                 (const uint4*)dj, s);
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout, ncells * rec * 4, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (dc) (void)hipFree(dc);
  if (dout) (void)hipFree(dout);
  if (dj) (void)hipFree(dj);
  HIPCHK(e);
  return KPE_OK;
}

// ---- condition traces (report time) -----------------------------------------------------------
kpe_status kpe_fetch_cond_traces(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint64_t row0,
                                 uint64_t nrows, uint32_t* out) {
  if (!dev || !prog || !c || !c->d || (nrows && !out)) return fail(KPE_E_INVALID, "null argument");
  if (row0 > (uint64_t)c->c->n || nrows > (uint64_t)c->c->n - row0) return fail(KPE_E_INVALID, "rows past the corpus");
  if (!nrows) return KPE_OK;
  const kpe::Program& P = *prog->p;
  const size_t R = P.rules.size();
  memset(out, 0, nrows * R * 4);
  if (!P.cond.nmsg) return KPE_OK;
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  if (B.prog != prog->p.get() || !B.cargs_valid)
    return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  if (c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  const size_t m = P.cond.nmsg;
  std::vector<uint32_t> h(nrows * m);
  hipStream_t s = B.last ? B.last : dev->stream;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipMemcpy(h.data(), B.mtrace.as<uint32_t>() + row0 * m, h.size() * 4, hipMemcpyDeviceToHost));
  for (const KpeCRule& cr : P.cond.rules)
    if (cr.mslot)
      for (uint64_t i = 0; i < nrows; ++i) out[i * R + cr.col] = h[i * m + cr.mslot - 1u];
  return KPE_OK;
}

kpe_status kpe_fetch_cond_traces_ex(kpe_device* dev, const kpe_program* prog, const kpe_corpus* c, uint64_t row0,
                                    uint64_t nrows, uint32_t* out) {
  if (!dev || !prog || !c || !c->d || (nrows && !out)) return fail(KPE_E_INVALID, "null argument");
  if (row0 > (uint64_t)c->c->n || nrows > (uint64_t)c->c->n - row0) return fail(KPE_E_INVALID, "rows past the corpus");
  if (!nrows) return KPE_OK;
  const kpe::Program& P = *prog->p;
  const size_t R = P.rules.size(), W = KPE_CTRACE_WORDS;
  memset(out, 0, nrows * R * W * 4);
  if (!P.cond.nmsg) return KPE_OK;
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  auto& B = c->d->bind;
  if (B.prog != prog->p.get() || !B.cargs_valid)
    return fail(KPE_E_STATE, "no evaluation of this program on this corpus");
  if (c->d->ordinal != dev->ordinal) return fail(KPE_E_STATE, "corpus not uploaded to this device");
  const size_t m = P.cond.nmsg;
  std::vector<uint32_t> h(nrows * m);
  hipStream_t s = B.last ? B.last : dev->stream;
  HIPCHK(hipStreamSynchronize(s));
  HIPCHK(hipMemcpy(h.data(), B.mtrace.as<uint32_t>() + row0 * m, h.size() * 4, hipMemcpyDeviceToHost));
  for (const KpeCRule& cr : P.cond.rules) {
    if (!cr.mslot) continue;
    const size_t nw = cr.kind == CR_FOREACH ? KPE_FE_TRACE_WORDS : 1u;
    for (uint64_t i = 0; i < nrows; ++i)
      for (size_t w = 0; w < nw; ++w) out[(i * R + cr.col) * W + w] = h[i * m + cr.mslot - 1u + w];
  }
  return KPE_OK;
}

kpe_status kpe_evaluate_sharded(kpe_device* const* devs, kpe_corpus* const* shards, int nshards,
                                const kpe_program* prog, uint8_t* verdicts, kpe_counts* counts) {
  if (!devs || !shards || !prog || nshards <= 0) return fail(KPE_E_INVALID, "null argument");
  const size_t R = prog->p->rules.size();
  for (int i = 0; i < nshards; ++i) {  // every launch first: the devices run together
    if (!devs[i] || !shards[i]) return fail(KPE_E_INVALID, "null device or shard");
    for (int j = 0; j < i; ++j)
      if (devs[j]->ordinal == devs[i]->ordinal) return fail(KPE_E_INVALID, "one shard per device");
    if (kpe_status st = kpe_evaluate_async(devs[i], prog, shards[i])) return st;
  }
  std::vector<kpe_counts> part(counts ? R : 0);
  if (counts) memset(counts, 0, R * sizeof(kpe_counts));
  uint64_t row = 0;
  for (int i = 0; i < nshards; ++i) {
    uint8_t* v = verdicts ? verdicts + row * R : nullptr;
    if (kpe_status st = kpe_fetch(devs[i], prog, shards[i], v, nullptr, counts ? part.data() : nullptr)) return st;
    for (size_t r = 0; counts && r < R; ++r) {
      counts[r].na += part[r].na, counts[r].pass += part[r].pass, counts[r].fail += part[r].fail;
      counts[r].warn += part[r].warn, counts[r].error += part[r].error, counts[r].skip += part[r].skip;
      counts[r].undecided += part[r].undecided;
    }
    row += (uint64_t)shards[i]->c->n;
  }
  return KPE_OK;
}

static const char* const kCheckIds[KPE_NUM_CHECKS] = {
    "allowPrivilegeEscalation", "appArmorProfile", "capabilities_baseline", "capabilities_restricted",
    "hostNamespaces", "hostPathVolumes", "hostPorts", "privileged", "procMount", "restrictedVolumes",
    "runAsNonRoot", "runAsUser", "seLinuxOptions", "seccompProfile_baseline", "seccompProfile_restricted",
    "sysctls", "windowsHostProcess"};
const char* kpe_pss_check_id(int k) { return (k >= 0 && k < KPE_NUM_CHECKS) ? kCheckIds[k] : nullptr; }
int kpe_pss_num_checks(void) { return KPE_NUM_CHECKS; }
int kpe_pss_num_cv(void) { return KPE_NUM_CV; }
int kpe_pss_cv_check(int v) { return (v >= 0 && v < KPE_NUM_CV) ? (int)kCvCheck[v] : -1; }

static void json_str(std::string& o, const std::string& s) {  // encoding/json string escaping
  static const char* hx = "0123456789abcdef";
  o += '"';
  for (unsigned char ch : s) {
    if (ch == '"' || ch == '\\') {
      o += '\\';
      o += (char)ch;
    } else if (ch == '\n') {
      o += "\\n";
    } else if (ch == '\r') {
      o += "\\r";
    } else if (ch == '\t') {
      o += "\\t";
    } else if (ch < 0x20 || ch == '<' || ch == '>' || ch == '&') {
      o += "\\u00";
      o += hx[ch >> 4];
      o += hx[ch & 15];
    } else {
      o += (char)ch;
    }
  }
  o += '"';
}

// cmd/cli/kubectl-kyverno/processor/result.go:34-68 (ResultCounts.addEngineResponse): every
// response rule is counted once per validate rule of its policy with the same name; a fail is
// a warn when the policy is unscored, or with --audit-warn when its action is Audit.
kpe_status kpe_cli_summary(const kpe_program* prog, const kpe_counts* counts, int audit_warn, kpe_cli_totals* out) {
  if (!prog || !counts || !out) return fail(KPE_E_INVALID, "null argument");
  const kpe::Program& P = *prog->p;
  *out = kpe_cli_totals{};
  for (size_t r = 0; r < P.rules.size(); ++r) {
    const kpe::RuleReport& rr = P.reports[r];
    const uint64_t m = rr.name_mult;
    if (!m) continue;
    if (audit_warn && rr.overrides && rr.scored && counts[r].fail)
      return fail(KPE_E_UNSUPPORTED, "validationFailureActionOverrides with --audit-warn (per-namespace action)");
    out->pass += m * counts[r].pass;
    out->error += m * counts[r].error;
    out->skip += m * counts[r].skip;
    out->warn += m * counts[r].warn;
    if (!rr.scored || (audit_warn && rr.audit)) out->warn += m * counts[r].fail;
    else out->fail += m * counts[r].fail;
  }
  return KPE_OK;
}

// pkg/utils/report/results.go:89-156 (EngineResponseToReportResults) for one resource row,
// over every policy of the program; toPolicyResult results.go:56-71.
long kpe_report_results(const kpe_program* prog, const uint8_t* verdict_row, const uint32_t* cv_mask_row, char* buf,
                        size_t cap) {
  return kpe_report_results_msg(prog, verdict_row, cv_mask_row, nullptr, 0, buf, cap);
}

// The PatternError.Path of a trace record (validate.go: "/" then each key or index followed by
// "/"); false when the record is truncated
static bool trace_path(const kpe::Program& P, const kpe::Corpus* C, const uint32_t* t, std::string* out) {
  if (t[0] & KPE_TR_TRUNC) return false;
  const uint32_t n = t[0] & 0xFFu;
  std::string p = "/";
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t c = t[1 + i];
    if (c & KPE_TC_IDX) {
      p += std::to_string(c & ~KPE_TC_IDX);
    } else if (c & KPE_TC_KEY) {
      if (!C) return false;
      const uint32_t id = c & ~KPE_TC_KEY;
      if (id >= C->dict[D_KEY].size()) return false;
      p += std::string(C->dict[D_KEY].at(id));
    } else {
      if ((size_t)c * 4 + 1 >= P.pat.members.size()) return false;
      if (P.pat.members[(size_t)c * 4] & PMF_VKEY) return false;  // an absent substituted key: no text kept
      const uint32_t ki = P.pat.members[(size_t)c * 4 + 1];
      if (ki >= P.pat.keys.size()) return false;
      p += P.pat.keys[ki];
    }
    p += '/';
  }
  *out = std::move(p);
  return true;
}

// validate_resource.go:316-454: pattern / anyPattern messages from the cell's trace (roots in
// order) of rule `rule` with validate.message `vmsg` (substituted over the resource and, in a
// foreach, the element `el`); empty when the reference's text would need an error string the
// device does not keep (an empty-path PatternError, a skip) or a substituted message
static std::string pattern_msg(const kpe::Program& P, const kpe::Corpus* C, const std::string& rule,
                               const std::string& vmsg, bool any, uint32_t roots, uint8_t v, const uint32_t* tr,
                               const char* json, size_t json_len, const kpe::MsgElem* el) {
  auto root = [&](uint32_t k) { return tr + (size_t)k * KPE_TRACE_WORDS; };
  auto rv = [&](uint32_t k) { return (root(k)[0] & KPE_TR_VALID) ? (root(k)[0] >> 16) & 0xFFu : 0xFFu; };
  if (!any) {
    if (v != KPE_FAIL || rv(0) != KPE_FAIL) return "";
    std::string path;
    if (!trace_path(P, C, root(0), &path)) return "";
    if (vmsg.empty()) return "validation error: rule " + rule + " failed at path " + path;  // buildErrorMessage
    std::string m = vmsg;
    if (vmsg.find("{{") != std::string::npos || vmsg.find("$(") != std::string::npos) {
      // buildErrorMessage: SubstituteAll of the message (a non-string value: no text)
      bool nonstring = false;
      if (!kpe::substitute_message(vmsg, json, json_len, &m, &nonstring, nullptr, el) || nonstring) return "";
    }
    if (m.empty() || m.back() != '.') m += '.';
    return "validation error: " + m + " rule " + rule + " failed at path " + path;
  }
  if (v == KPE_PASS) {
    if (roots == 0) return vmsg;  // no pattern at all: RulePass(rule.Validation.Message)
    for (uint32_t k = 0; k < roots && k < KPE_TRACE_ROOTS; ++k) {
      if (rv(k) == KPE_PASS) return "validation rule '" + rule + "' anyPattern[" + std::to_string(k) + "] passed.";
      if (rv(k) == 0xFFu || rv(k) == KPE_UNDECIDED) return "";
    }
    return "";
  }
  if (v != KPE_FAIL || roots > KPE_TRACE_ROOTS) return "";
  std::string errs;
  for (uint32_t k = 0; k < roots; ++k) {
    const uint32_t x = rv(k);
    if (x == KPE_SKIP) continue;  // skipped patterns are not listed once one failed
    if (x != KPE_FAIL) return "";  // an empty-path failure's message is its error text
    std::string path;
    if (!trace_path(P, C, root(k), &path)) return "";
    errs += (errs.empty() ? "" : " ") + ("rule " + rule + "[" + std::to_string(k) + "] failed at path " + path);
  }
  if (errs.empty()) return "";
  if (vmsg.empty()) return "validation error: " + errs;  // buildAnyPatternErrorMessage
  if (vmsg.back() == '.') return "validation error: " + vmsg + " " + errs;
  return "validation error: " + vmsg + ". " + errs;
}
static std::string pattern_message(const kpe::Program& P, const kpe::Corpus* C, const kpe::RuleReport& rr, uint8_t v,
                                   const uint32_t* tr, const char* json, size_t json_len) {
  return pattern_msg(P, C, rr.rule, rr.vmsg, rr.any_pattern, rr.pat_roots, v, tr, json, json_len, nullptr);
}

// getDenyMessage (validate_resource.go:279-300) of a failing deny block whose condition message is
// `cm`: SubstituteAll of JoinNonEmpty(rule message, cm) over the context (the resource, and the
// foreach element `el`); on a substitution error the condition message as is; a message outside
// the restated variables: none
static std::string deny_msg(const std::string& rule, const std::string& vmsg, const std::string& cm, const char* json,
                            size_t n, const kpe::MsgElem* el) {
  if (vmsg.empty() && cm.empty()) return "validation error: rule " + rule + " failed";
  const std::string j = kpe::join_non_empty({vmsg, cm}, "; ");
  std::string out;
  bool nonstring = false, serr = false;
  if (!kpe::substitute_message(j, json, n, &out, &nonstring, &serr, el)) return serr ? cm : std::string();
  return nonstring ? "the produced message didn't resolve to a string, check your policy definition." : out;
}

// The document of tape entry e as JSON text (the foreach element: a node of the resource's
// document; Go's JSON context holds it with float64 numbers, which the renderers print alike)
static bool tape_json(const kpe::Corpus& C, uint32_t e, std::string& o, int depth = 0) {
  if ((size_t)e * 2 + 1 >= C.doc.size() || depth > 300) return false;
  const uint32_t x = C.doc[(size_t)e * 2], y = C.doc[(size_t)e * 2 + 1];
  auto str = [&](std::string_view t) {
    o += '"';
    for (unsigned char ch : t) {
      if (ch == '"' || ch == '\\') o += '\\', o += (char)ch;
      else if (ch < 0x20) {
        char b[8];
        snprintf(b, sizeof b, "\\u%04x", ch);
        o += b;
      } else o += (char)ch;
    }
    o += '"';
  };
  if (DN_KIND(x) == DN_SCALAR) {
    if (y >= C.scal.size()) return false;
    const KpeScalar& sc = C.scal[y];
    char b[40];
    switch (SC_TYPE(sc.flags)) {
      case SC_T_NULL: o += "null"; break;
      case SC_T_BOOL: o += (y == SC_TRUE_ID || (sc.flags & SC_BTRUE)) ? "true" : "false"; break;
      case SC_T_INT: o += std::to_string(sc.ival); break;
      case SC_T_FLOAT:
        snprintf(b, sizeof b, "%.17g", sc.fval);
        o += b;
        break;
      default: str(C.scal_text_of(y));
    }
    return true;
  }
  if ((size_t)y * 2 + 1 >= C.doc.size()) return false;
  const uint32_t cnt = C.doc[(size_t)y * 2];
  const bool map = DN_KIND(x) == DN_MAP;
  o += map ? '{' : '[';
  for (uint32_t k = 0; k < cnt; ++k) {
    const uint32_t m = y + 1 + k;
    if ((size_t)m * 2 >= C.doc.size()) return false;
    if (k) o += ',';
    if (map) {
      const uint32_t key = DN_KEY(C.doc[(size_t)m * 2]);
      if (key == 0 || key - 1 >= C.dict[D_KEY].size()) return false;
      str(C.dict[D_KEY].at(key - 1));
      o += ':';
    }
    if (!tape_json(C, m, o, depth + 1)) return false;
  }
  o += map ? '}' : ']';
  return true;
}
// %T of a tape entry as the JSON context holds it
static const char* tape_go_type(const kpe::Corpus& C, uint32_t e) {
  if ((size_t)e * 2 + 1 >= C.doc.size()) return nullptr;
  const uint32_t x = C.doc[(size_t)e * 2], y = C.doc[(size_t)e * 2 + 1];
  if (DN_KIND(x) == DN_MAP) return "map[string]interface {}";
  if (DN_KIND(x) == DN_ARR) return "[]interface {}";
  if (y >= C.scal.size()) return nullptr;
  switch (SC_TYPE(C.scal[y].flags)) {
    case SC_T_BOOL: return "bool";
    case SC_T_INT:
    case SC_T_FLOAT: return "float64";
    case SC_T_STR: return "string";
    default: return nullptr;
  }
}

// The message of a validate.foreach cell (validateForEach / validateElements,
// validate_resource.go:186-254) from its condition trace words `w` (schema.h FT_*) and, for an
// entry's pattern, the cell's pattern trace `ptr`
static std::string foreach_message(const kpe::Program& P, const kpe::Corpus* C, const kpe::RuleReport& rr, uint8_t v,
                                   const uint32_t* w, const uint32_t* ptr, const char* json, size_t n) {
  if (v == KPE_PASS) return "rule passed";  // :203
  if ((v != KPE_FAIL && v != KPE_ERROR) || !w) return "";
  const uint32_t b = w[1];
  const int64_t ei = fe_decider(P, rr, b);
  if (ei < 0) return "";
  const kpe::FeReport& f = P.fe_reports[(size_t)ei];
  const uint32_t depth = FT_DEPTH(b), ct = w[0] >> 16;
  kpe::MsgElem me;
  const kpe::MsgElem* el = nullptr;
  if (C && w[2] != 0xFFFFFFFFu && tape_json(*C, w[2], me.json)) {
    me.depth = (int)depth, me.index = FT_IDX(b, depth);
    el = &me;
  }
  std::string leaf, e;
  uint32_t wraps = depth + 1;  // validateElements wraps the response once per level
  switch (FT_KIND(b)) {
    case FT_SCOPE_ERR: {  // AddElementToContext (:218-221, utils/foreach.go:51-54): not wrapped at its level
      const char* t = C && w[2] != 0xFFFFFFFFu ? tape_go_type(*C, w[2]) : nullptr;
      if (!t) return "";
      leaf = std::string("failed to process foreach: cannot use elementScope=true foreach rules for elements that "
                         "are not maps, expected type=map got type=") + t;
      wraps = depth;
      break;
    }
    case FT_PRE_ERR:  // the element's preconditions (:125-128)
      if ((e = kpe::block_error_text(f.pre_json, ct, json, n, el)).empty()) return "";
      leaf = "failed to evaluate preconditions: " + e;
      break;
    case FT_DENY:
      if (CT_IS_ERR(ct)) {  // :269-271
        if ((e = kpe::block_error_text(f.deny_json, ct, json, n, el)).empty()) return "";
        leaf = "failed to check deny conditions: " + e;
      } else if ((ct & (CT_EVAL | CT_TRUE)) == (CT_EVAL | CT_TRUE)) {  // getDenyMessage over the element
        leaf = deny_msg(rr.rule, rr.vmsg, f.deny_msgs.render(CT_ANY(ct), CT_ALL(ct), true), json, n, el);
      }
      break;
    case FT_PVAR_ERR:  // substitutePatterns (:139-141)
      if ((e = kpe::doc_subst_error(f.pattern_json, json, n, el)).empty()) return "";
      leaf = "variable substitution failed: " + e;
      break;
    case FT_PAT:
      if (!f.any_bad_type.empty()) {  // deserializeAnyPattern (:347-350)
        leaf = "failed to deserialize anyPattern, expected type array: json: cannot unmarshal " + f.any_bad_type +
               " into Go value of type []interface {}";
      } else if (ptr) {
        leaf = pattern_msg(P, C, rr.rule, rr.vmsg, f.any, f.nroots, v, ptr, json, n, el);
      }
      break;
    default: break;
  }
  if (leaf.empty()) return "";
  for (uint32_t k = 0; k < wraps; ++k) leaf = "validation failure: " + leaf;
  return leaf;
}

static long report_impl(const kpe_program* prog, const kpe_corpus* corp, const uint8_t* verdict_row,
                        const uint32_t* cv_mask_row, const uint32_t* traces, const uint32_t* cond_traces,
                        const char* resource_json, size_t resource_len, char* buf, size_t cap,
                        const uint32_t* cond_traces_ex = nullptr);

static std::string deny_message(const kpe::RuleReport& rr, const std::string& cm, const char* json, size_t n) {
  return deny_msg(rr.rule, rr.deny_vmsg, cm, json, n, nullptr);
}

long kpe_report_results_ex(const kpe_report_args* a, char* buf, size_t cap) {
  if (!a) {
    fail(KPE_E_INVALID, "null argument");
    return -KPE_E_INVALID;
  }
  return report_impl(a->prog, a->corpus, a->verdict_row, a->cv_mask_row, a->pattern_traces, a->cond_traces,
                     a->resource_json, a->resource_len, buf, cap, a->cond_traces_ex);
}

long kpe_report_results_msg(const kpe_program* prog, const uint8_t* verdict_row, const uint32_t* cv_mask_row,
                            const char* resource_json, size_t resource_len, char* buf, size_t cap) {
  return report_impl(prog, nullptr, verdict_row, cv_mask_row, nullptr, nullptr, resource_json, resource_len, buf, cap);
}

long kpe_report_results_msg_tr(const kpe_program* prog, const kpe_corpus* corpus, const uint8_t* verdict_row,
                               const uint32_t* cv_mask_row, const uint32_t* traces, const char* resource_json,
                               size_t resource_len, char* buf, size_t cap) {
  return report_impl(prog, corpus, verdict_row, cv_mask_row, traces, nullptr, resource_json, resource_len, buf, cap);
}

static long report_impl(const kpe_program* prog, const kpe_corpus* corp, const uint8_t* verdict_row,
                        const uint32_t* cv_mask_row, const uint32_t* traces, const uint32_t* cond_traces,
                        const char* resource_json, size_t resource_len, char* buf, size_t cap,
                        const uint32_t* cond_traces_ex) {
  if (!prog || !verdict_row) {
    fail(KPE_E_INVALID, "null argument");
    return -KPE_E_INVALID;
  }
  // the typed pod view for podSecurity fail messages, decoded on first use
  int pod_state = 0;  // 0 not decoded, 1 ok, -1 getSpec fails
  kpe::PodView pod;
  std::string kind;
  static const char* const kResult[6] = {nullptr, "pass", "fail", "warn", "error", "skip"};
  const kpe::Program& P = *prog->p;
  std::string o = "[";
  bool first = true;
  for (size_t r = 0; r < P.rules.size(); ++r) {
    const uint8_t v = verdict_row[r];
    if (v == KPE_NA || v > KPE_SKIP) continue;  // no RuleResponse (KPE_UNDECIDED: the caller's)
    const kpe::RuleReport& rr = P.reports[r];
    const char* res = kResult[v];
    if (v == KPE_FAIL && !rr.scored) res = "warn";  // results.go:131-133
    o += first ? "{" : ",{";
    first = false;
    o += "\"source\":\"kyverno\",\"policy\":";
    json_str(o, rr.policy_key);
    // the skip's cause: preconditions false (folded at compile time, or the condition trace's
    // preconditions half) or the rule's PolicyException (after preconditions that held)
    const uint32_t* cx = (cond_traces_ex && rr.cond_slot) ? cond_traces_ex + r * (size_t)KPE_CTRACE_WORDS : nullptr;
    const uint32_t ct = cx ? cx[0] : (cond_traces && rr.cond_slot) ? cond_traces[r] : 0u;
    const uint32_t held = CT_EVAL | CT_TRUE;
    const bool pre_skip = v == KPE_SKIP && (rr.pre_const_skip || (ct & held) == CT_EVAL);
    const bool exc_skip = v == KPE_SKIP && !rr.exc_key.empty() && !pre_skip &&
                          (!rr.exc_after_pre || (ct & held) == held);
    if (resource_json) {  // RuleResponse message (validate_pss.go:85,108; validate_resource.go:339)
      std::string msg;
      const kpe::Corpus* C = corp ? corp->c.get() : nullptr;
      const uint32_t* ptr = traces ? traces + r * (size_t)(KPE_TRACE_ROOTS * KPE_TRACE_WORDS) : nullptr;
      std::string e;
      if (v == KPE_ERROR && rr.cond_slot && CT_IS_ERR(ct & 0xFFFFu)) {  // engine.go:279-281
        if (!(e = kpe::block_error_text(rr.pre_json, ct & 0xFFFFu, resource_json, resource_len, nullptr)).empty())
          msg = "failed to evaluate preconditions: " + e;
      } else if (rr.foreach) {
        msg = foreach_message(P, C, rr, v, cx, ptr, resource_json, resource_len);
      } else if (v == KPE_ERROR && rr.msg_deny && rr.cond_slot && CT_IS_ERR(ct >> 16)) {  // :269-271
        if (!(e = kpe::block_error_text(rr.deny_json, ct >> 16, resource_json, resource_len, nullptr)).empty())
          msg = "failed to check deny conditions: " + e;
      } else if (v == KPE_ERROR && !rr.any_bad_type.empty()) {  // :347-350
        msg = "failed to deserialize anyPattern, expected type array: json: cannot unmarshal " + rr.any_bad_type +
              " into Go value of type []interface {}";
      } else if (v == KPE_ERROR && rr.pat_vars &&
                 !(e = kpe::doc_subst_error(rr.pattern_json, resource_json, resource_len, nullptr)).empty()) {
        msg = "variable substitution failed: " + e;  // :139-141
      } else if (rr.pss && v == KPE_PASS) {
        msg = kpe::pss_pass_message(rr.rule);
      } else if (rr.pss && v == KPE_FAIL && !rr.pss_excl && cv_mask_row && (cv_mask_row[r] & KPE_CVM_CHECKS)) {
        if (!pod_state) pod_state = kpe::typed_pod_view(resource_json, resource_len, &pod, &kind) ? 1 : -1;
        if (pod_state > 0)
          msg = kpe::pss_fail_message(rr.rule, rr.pss_level, rr.pss_version, kind, pod, cv_mask_row[r] & KPE_CVM_CHECKS);
      } else if (rr.pss && v == KPE_FAIL && rr.pss_excl && cv_mask_row) {
        // the checks EvaluatePod's exclusions and, when it matched (KPE_CVM_XMATCH), the podSecurity
        // PolicyException's leave (validate_pss.go:76-110)
        if (!pod_state) pod_state = kpe::typed_pod_view(resource_json, resource_len, &pod, &kind) ? 1 : -1;
        const bool xm = rr.pss_has_xexcl && (cv_mask_row[r] & KPE_CVM_XMATCH);
        if (pod_state > 0)
          msg = kpe::pss_fail_message_ex(rr.rule, rr.pss_level, rr.pss_version, kind, pod, rr.pss_cv, &rr.pss_excludes,
                                         xm ? &rr.pss_xexcludes : nullptr);
      } else if (rr.pat_rule && traces && (v == KPE_FAIL || (v == KPE_PASS && rr.any_pattern))) {
        msg = pattern_message(P, corp ? corp->c.get() : nullptr, rr, v,
                              traces + r * (size_t)(KPE_TRACE_ROOTS * KPE_TRACE_WORDS), resource_json, resource_len);
      } else if (rr.msg_pattern && v == KPE_PASS) {
        msg = "validation rule '" + rr.rule + "' passed.";
      } else if (pre_skip) {  // engine.go:282-284
        msg = rr.pre_const_skip
                  ? rr.pre_skip_msg
                  : kpe::join_non_empty({"preconditions not met", rr.pre_msgs.render(CT_ANY(ct), CT_ALL(ct), false)}, "; ");
      } else if (rr.msg_deny && v == KPE_PASS) {
        msg = "validation rule '" + rr.rule + "' passed.";
      } else if (rr.msg_deny && v == KPE_FAIL) {
        const uint32_t dt = ct >> 16;
        if (!rr.cond_deny) msg = deny_message(rr, rr.deny_cm, resource_json, resource_len);
        else if ((dt & held) == held)
          msg = deny_message(rr, rr.deny_msgs.render(CT_ANY(dt), CT_ALL(dt), true), resource_json, resource_len);
      } else if (rr.msg_deny && rr.msg_pre_skip && v == KPE_SKIP && P.rules[r].exc == 0u) {
        msg = "preconditions not met";  // no exception: the skip is the preconditions'
      }
      if (exc_skip) msg = "rule skipped due to policy exception " + rr.exc_key;
      if (!msg.empty()) {
        o += ",\"message\":";
        json_str(o, msg);
      }
    }
    if (!rr.rule.empty()) {
      o += ",\"rule\":";
      json_str(o, rr.rule);
    }
    o += ",\"result\":\"";
    o += res;
    o += '"';
    if (rr.scored) o += ",\"scored\":true";
    // results.go:114-129: failing check ids (one per failing versioned check), sorted
    const uint32_t f = (rr.pss && v == KPE_FAIL && cv_mask_row) ? cv_mask_row[r] & KPE_CVM_CHECKS : 0u;
    if (f) {
      std::vector<std::string> ids;
      for (uint32_t b = f; b; b &= b - 1) ids.push_back(kCheckIds[kCvCheck[__builtin_ctz(b)]]);
      std::sort(ids.begin(), ids.end());
      std::string ctl;
      for (auto& id : ids) ctl += (ctl.empty() ? "" : ",") + id;
      o += ",\"properties\":{\"controls\":";
      json_str(o, ctl);
      o += ",\"standard\":";
      json_str(o, rr.pss_level);
      o += ",\"version\":";
      json_str(o, rr.pss_version);
      o += '}';
    }
    if (exc_skip && !rr.exc_name.empty()) {  // results.go:107-111: the exception's name
      o += ",\"properties\":{\"exception\":";
      json_str(o, rr.exc_name);
      o += '}';
    }
    if (!rr.category.empty()) {
      o += ",\"category\":";
      json_str(o, rr.category);
    }
    if (!rr.severity.empty()) {
      o += ",\"severity\":";
      json_str(o, rr.severity);
    }
    o += '}';
  }
  o += ']';
  if (buf && cap > 0) {
    const size_t n = std::min(o.size(), cap - 1);
    memcpy(buf, o.data(), n);
    buf[n] = 0;
  }
  return (long)o.size();
}

kpe_status kpe_device_set_timing(kpe_device* dev, int enabled) {
  if (!dev) return fail(KPE_E_INVALID, "null device");
  std::lock_guard<std::mutex> lk(dev->mu);
  dev->timing = enabled != 0;
  return KPE_OK;
}

kpe_status kpe_device_kernel_stats(kpe_device* dev, const kpe_program*, const kpe_corpus*, kpe_kernel_stats* out,
                                   int reset) {
  if (!dev || !out) return fail(KPE_E_INVALID, "null argument");
  std::lock_guard<std::mutex> lk(dev->mu);
  HIPCHK(hipSetDevice(dev->ordinal));
  for (int k = 0; k < dev->nlanes; ++k) HIPCHK(hipStreamSynchronize(dev->lanes[k]));
  for (auto& p : dev->pending) {
    float d1 = 0, d2 = 0, d3 = 0;
    HIPCHK(hipEventElapsedTime(&d1, p.a, p.b));
    HIPCHK(hipEventElapsedTime(&d2, p.b, p.c));
    HIPCHK(hipEventElapsedTime(&d3, p.c, p.d));
    dev->dict_ms += p.pre ? d1 : 0.0f;  // an empty event interval is not a kernel (kpe.h)
    dev->pss_ms += d2;
    dev->pss_min = dev->launches == 0 ? d2 : std::min(dev->pss_min, (double)d2);
    dev->pss_max = dev->launches == 0 ? d2 : std::max(dev->pss_max, (double)d2);
    dev->pss_sq += (double)d2 * d2;
    dev->pat_ms += p.post ? d3 : 0.0f;
    dev->last_bytes = p.bytes;
    dev->last_pbytes = p.pbytes;
    dev->sum_bytes += p.bytes;
    dev->sum_pbytes += p.post ? p.pbytes : 0.0;
    dev->last_kind = p.kind;
    dev->launches++;
    dev->pool.push_back(p.a);
    dev->pool.push_back(p.b);
    dev->pool.push_back(p.c);
    dev->pool.push_back(p.d);
  }
  dev->pending.clear();
  out->launches = dev->launches;
  out->pss_kernel_ms = dev->pss_ms;
  out->dict_kernel_ms = dev->dict_ms;
  out->scan_bytes = dev->last_bytes;
  out->pattern_kernel_ms = dev->pat_ms;
  out->pattern_bytes = dev->last_pbytes;
  out->scan_kernel = dev->last_kind;
  out->pad_ = 0;
  out->scan_bytes_sum = dev->sum_bytes;
  out->pss_kernel_ms_min = dev->pss_min, out->pss_kernel_ms_max = dev->pss_max, out->pss_kernel_ms_sq = dev->pss_sq;
  out->pattern_bytes_sum = dev->sum_pbytes;
  if (reset) {
    dev->launches = 0;
    dev->pss_ms = dev->dict_ms = dev->pat_ms = dev->sum_bytes = dev->sum_pbytes = 0;
    dev->pss_min = dev->pss_max = dev->pss_sq = 0;
  }
  return KPE_OK;
}

}  // extern "C"
