// CDNA4 (gfx950) kernels for batch policy evaluation. wave64, HBM-bound scans.
//
//  kpe_pred_kernel  — dictionary pass: every string predicate of the compiled
//                     program (OR of go-wildcard globs, ext/wildcard/match.go:7-9)
//                     evaluated once per DISTINCT string of its domain; results
//                     are bitsets (one bit per dictionary id) built with wave ballots.
//  kpe_scan_kernel  — one resource per lane: match/exclude (pkg/engine/utils/match.go:
//                     168-300) for every rule, PSS checks (PSA v0.29 policy checks via
//                     pkg/pss/evaluate.go:24-70) and the verdict cell, with ApplyOne
//                     (pkg/engine/validation.go:75-77). Containers of the block's
//                     resources are streamed cooperatively (coalesced) through LDS,
//                     so the irregular 1..64-container fan-out never diverges the
//                     HBM loads; per-rule counters are reduced with wave ballots.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "schema.h"

namespace {

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
  if (pn == 1 && p[0] == '*') return true;
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

}  // namespace

// ---------------------------------------------------------------------------
struct PredJob {
  uint32_t domain;
  uint32_t pat0, npat;      // patterns [pat0, pat0+npat) in the pattern table
  uint32_t out_word;        // first output word
  uint32_t blk0;            // first block of this job (exclusive prefix over jobs)
};

struct PredArgs {
  const uint8_t* dict_bytes[KPE_NUM_DOMAINS];
  const uint32_t* dict_off[KPE_NUM_DOMAINS];
  uint32_t dict_n[KPE_NUM_DOMAINS];
  const uint8_t* pat_bytes;
  const uint32_t* pat_off;  // pattern k = pat_bytes[pat_off[k] .. pat_off[k+1])
  const PredJob* jobs;
  uint32_t njobs;
  uint32_t* out;
};

__global__ void __launch_bounds__(256) kpe_pred_kernel(PredArgs a) {
  // job lookup: blocks are laid out job-major (uniform per block)
  uint32_t b = blockIdx.x;
  uint32_t j = 0;
  while (j + 1 < a.njobs && a.jobs[j + 1].blk0 <= b) ++j;
  const PredJob job = a.jobs[j];
  uint32_t id = (b - job.blk0) * 256u + threadIdx.x;
  uint32_t n = a.dict_n[job.domain];
  bool hit = false;
  if (id < n) {
    const uint32_t* off = a.dict_off[job.domain];
    const uint8_t* s = a.dict_bytes[job.domain] + off[id];
    int sn = (int)(off[id + 1] - off[id]);
    for (uint32_t k = 0; k < job.npat && !hit; ++k) {
      uint32_t p0 = a.pat_off[job.pat0 + k], p1 = a.pat_off[job.pat0 + k + 1];
      hit = glob(a.pat_bytes + p0, (int)(p1 - p0), s, sn);
    }
  }
  uint64_t m = __ballot(hit);
  uint32_t lane = threadIdx.x & 63u;
  uint32_t wid = id >> 6;  // 64 strings per wave => two output words
  if (lane == 0 && (uint64_t)wid * 64u < n) {
    a.out[job.out_word + 2 * wid] = (uint32_t)m;
    a.out[job.out_word + 2 * wid + 1] = (uint32_t)(m >> 32);
  }
}

// ---------------------------------------------------------------------------
struct ScanArgs {
  int64_t n;
  // resource rows
  const uint32_t* r_flags;
  const uint32_t* r_gvk;
  const uint32_t* r_name;
  const uint32_t* r_mns;
  const uint32_t* r_nsa;
  const uint32_t* ann_off;
  const uint32_t* ann_k;
  const uint32_t* ann_v;
  // pod view
  const uint32_t* p_sc;
  const uint32_t* ctr_off;
  const uint32_t* vol_off;
  const uint32_t* vol_src;
  const uint32_t* sys_off;
  const uint32_t* sys_id;
  const uint32_t* pann_off;
  const uint32_t* pann_k;
  const uint32_t* pann_v;
  // containers
  const uint32_t* c_sc;
  const uint64_t* c_add;
  const uint64_t* c_drop;
  const uint32_t* c_sann;
  // program
  const KpeRule* rules;
  uint32_t nrules;
  const KpeFilter* filters;
  const KpeTerm* terms;
  const KpeKindSel* kindsels;
  const KpeAnnPair* annpairs;
  const uint32_t* pred_bits;
  const uint32_t* pred_word;  // first word of predicate p
  int32_t pp_apparmor_key, pp_apparmor_ok, pp_seccomp_pod_key, pp_seccomp_ann_ok;
  int32_t pp_caps_ok, pp_cap_nbs, pp_cap_all, pp_sysctl0, pp_sysctl1, pp_sysctl2;
  uint32_t cv_union;
  uint32_t any_pss;
  // outputs
  uint8_t* verdicts;   // n x nrules
  uint32_t* masks;     // n x nrules or null
  unsigned long long* counts;  // nrules x 6
};

namespace {

__device__ __forceinline__ bool pbit(const ScanArgs& a, int32_t p, uint32_t id) {
  if (id == KPE_NO_STR) return false;
  return (a.pred_bits[a.pred_word[p] + (id >> 5)] >> (id & 31u)) & 1u;
}
__device__ __forceinline__ uint64_t pmask64(const ScanArgs& a, int32_t p) {  // D_CAP predicates (<= 64 ids)
  const uint32_t* w = a.pred_bits + a.pred_word[p];
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}

__device__ bool eval_filter(const ScanArgs& a, uint32_t f, int64_t r, uint32_t gvk, uint32_t flags) {
  KpeFilter fl = a.filters[f];
  for (uint32_t t = 0; t < fl.nterms; ++t) {
    KpeTerm tm = a.terms[fl.term0 + t];
    bool ok;
    switch (tm.type) {
      case T_KINDS: {
        ok = false;
        for (uint32_t s = 0; s < tm.b && !ok; ++s) {
          KpeKindSel ks = a.kindsels[tm.a + s];
          ok = ks.sub_ok && (ks.pg < 0 || pbit(a, ks.pg, GVK_GRP(gvk))) && (ks.pv < 0 || pbit(a, ks.pv, GVK_VER(gvk))) &&
               (ks.pk < 0 || pbit(a, ks.pk, GVK_KIND(gvk)));
        }
        break;
      }
      case T_PRED: {
        uint32_t id = tm.b == COL_NAME ? a.r_name[r] : (tm.b == COL_MNS ? a.r_mns[r] : a.r_nsa[r]);
        ok = pbit(a, (int32_t)tm.a, id);
        break;
      }
      case T_ANNOTATIONS: {
        ok = true;
        uint32_t lo = a.ann_off[r], hi = a.ann_off[r + 1];
        for (uint32_t pi = 0; pi < tm.b && ok; ++pi) {
          KpeAnnPair pr = a.annpairs[tm.a + pi];
          bool m = false;
          for (uint32_t j = lo; j < hi && !m; ++j) m = pbit(a, pr.pk, a.ann_k[j]) && pbit(a, pr.pv, a.ann_v[j]);
          ok = m;
        }
        break;
      }
      default: ok = false;
    }
    if (!ok) return false;
  }
  return true;
}

__device__ bool eval_block(const ScanArgs& a, uint32_t mode, uint32_t f0, uint32_t nf, int64_t r, uint32_t gvk,
                           uint32_t flags) {
  if (mode == MODE_ANY) {
    for (uint32_t f = 0; f < nf; ++f)
      if (eval_filter(a, f0 + f, r, gvk, flags)) return true;
    return false;
  }
  if (mode == MODE_ALL) {
    for (uint32_t f = 0; f < nf; ++f)
      if (!eval_filter(a, f0 + f, r, gvk, flags)) return false;
    return true;
  }
  return eval_filter(a, f0, r, gvk, flags);
}

// versioned check -> check bit
__constant__ uint8_t kCvCheck[KPE_NUM_CV] = {
    CK_APE, CK_APE, CK_APPARMOR, CK_CAPS_BASELINE, CK_CAPS_RESTRICTED, CK_CAPS_RESTRICTED, CK_HOST_NS,
    CK_HOST_PATH, CK_HOST_PORTS, CK_PRIVILEGED, CK_PROC_MOUNT, CK_RESTRICTED_VOLUMES, CK_RUN_AS_NON_ROOT,
    CK_RUN_AS_USER, CK_SELINUX, CK_SECCOMP_BASELINE, CK_SECCOMP_BASELINE, CK_SECCOMP_RESTRICTED,
    CK_SECCOMP_RESTRICTED, CK_SYSCTLS, CK_SYSCTLS, CK_SYSCTLS, CK_WIN_HOST_PROCESS};

constexpr uint32_t kBlock = 256;
constexpr uint32_t kChunk = 2048;  // containers staged per LDS pass
constexpr uint32_t kAllowedVolumes = (1u << VS_CONFIGMAP) | (1u << VS_CSI) | (1u << VS_DOWNWARDAPI) |
                                     (1u << VS_EMPTYDIR) | (1u << VS_EPHEMERAL) | (1u << VS_PVC) |
                                     (1u << VS_PROJECTED) | (1u << VS_SECRET);

__device__ __forceinline__ uint32_t container_bits(uint32_t w, uint64_t add, uint64_t drop, uint32_t sann,
                                                   uint64_t caps_ok, uint64_t nbs, uint64_t all, const ScanArgs& a) {
  uint32_t b = 0;
  bool caps = w & C_CAPS_PRESENT;
  if (FIELD(w, C_APE_SH, 2) != TRI_FALSE) b |= CB_APE;
  if (caps && (add & ~caps_ok)) b |= CB_CAPS_BASE;
  if (!caps || !(drop & all)) b |= CB_CAPS_DROP;
  if (caps && (add & ~nbs)) b |= CB_CAPS_ADD;
  if (FIELD(w, C_HOSTPORT_SH, 4)) b |= CB_HOSTPORT;
  if (FIELD(w, C_PRIV_SH, 2) == TRI_TRUE) b |= CB_PRIV;
  if (FIELD(w, C_PROCMOUNT_SH, 2) == PROCMOUNT_OTHER) b |= CB_PROCMOUNT;
  uint32_t rnr = FIELD(w, C_RNR_SH, 2);
  if (rnr == TRI_FALSE) b |= CB_RNR_FALSE;
  if (rnr == TRI_UNSET) b |= CB_RNR_UNSET;
  if (FIELD(w, C_RAU_SH, 2) == RAU_ZERO) b |= CB_RAU_ZERO;
  uint32_t sel = FIELD(w, C_SEL_SH, 3);
  if (sel != SEL_NONE && (sel == SEL_OTHER || (w & (C_SEL_USER | C_SEL_ROLE)))) b |= CB_SELINUX;
  uint32_t sec = FIELD(w, C_SECCOMP_SH, 3);
  if (sec == SECCOMP_NONE) b |= CB_SEC_UNSET;
  else if (sec != SECCOMP_RUNTIMEDEFAULT && sec != SECCOMP_LOCALHOST) b |= CB_SEC_BAD;
  if (sann != KPE_NO_STR && a.pp_seccomp_ann_ok >= 0 && !pbit(a, a.pp_seccomp_ann_ok, sann)) b |= CB_SEC_ANN;
  if (FIELD(w, C_WHP_SH, 2) == TRI_TRUE) b |= CB_WHP;
  return b;
}

// PSA versioned checks for one pod given the OR of its container bits.
__device__ uint32_t cv_fails(const ScanArgs& a, uint32_t pw, uint32_t cb, bool vol_hostpath, bool vol_restricted,
                             uint32_t sys_bad, bool apparmor_bad, bool sec_pod_ann_bad) {
  uint32_t f = 0;
  bool win = FIELD(pw, P_OS_SH, 2) == OS_WINDOWS;
  if (cb & CB_APE) f |= (1u << CV_APE_1_8) | (win ? 0u : (1u << CV_APE_1_25));
  if (apparmor_bad) f |= 1u << CV_APPARMOR_1_0;
  if (cb & CB_CAPS_BASE) f |= 1u << CV_CAPS_BASELINE_1_0;
  if (cb & (CB_CAPS_DROP | CB_CAPS_ADD)) f |= (1u << CV_CAPS_RESTRICTED_1_22) | (win ? 0u : (1u << CV_CAPS_RESTRICTED_1_25));
  if (pw & (P_HOSTNET | P_HOSTPID | P_HOSTIPC)) f |= 1u << CV_HOST_NS_1_0;
  if (vol_hostpath) f |= 1u << CV_HOST_PATH_1_0;
  if (cb & CB_HOSTPORT) f |= 1u << CV_HOST_PORTS_1_0;
  if (cb & CB_PRIV) f |= 1u << CV_PRIVILEGED_1_0;
  if (cb & CB_PROCMOUNT) f |= 1u << CV_PROC_MOUNT_1_0;
  if (vol_restricted) f |= 1u << CV_RESTRICTED_VOLUMES_1_0;
  uint32_t prnr = FIELD(pw, P_RNR_SH, 2);
  if (prnr == TRI_FALSE || (cb & CB_RNR_FALSE) || (prnr != TRI_TRUE && (cb & CB_RNR_UNSET)))
    f |= 1u << CV_RUN_AS_NON_ROOT_1_0;
  if (FIELD(pw, P_RAU_SH, 2) == RAU_ZERO || (cb & CB_RAU_ZERO)) f |= 1u << CV_RUN_AS_USER_1_23;
  uint32_t psel = FIELD(pw, P_SEL_SH, 3);
  if ((psel != SEL_NONE && (psel == SEL_OTHER || (pw & (P_SEL_USER | P_SEL_ROLE)))) || (cb & CB_SELINUX))
    f |= 1u << CV_SELINUX_1_0;
  if (sec_pod_ann_bad || (cb & CB_SEC_ANN)) f |= 1u << CV_SECCOMP_BASELINE_1_0;
  uint32_t psec = FIELD(pw, P_SECCOMP_SH, 3);
  bool psec_valid = psec == SECCOMP_RUNTIMEDEFAULT || psec == SECCOMP_LOCALHOST;
  bool psec_bad = psec != SECCOMP_NONE && !psec_valid;
  if (psec_bad || (cb & CB_SEC_BAD)) f |= 1u << CV_SECCOMP_BASELINE_1_19;
  if (psec_bad || (cb & CB_SEC_BAD) || (!psec_valid && (cb & CB_SEC_UNSET)))
    f |= (1u << CV_SECCOMP_RESTRICTED_1_19) | (win ? 0u : (1u << CV_SECCOMP_RESTRICTED_1_25));
  if (sys_bad & 1u) f |= 1u << CV_SYSCTLS_1_0;
  if (sys_bad & 2u) f |= 1u << CV_SYSCTLS_1_27;
  if (sys_bad & 4u) f |= 1u << CV_SYSCTLS_1_29;
  if (FIELD(pw, P_WHP_SH, 2) == TRI_TRUE || (cb & CB_WHP)) f |= 1u << CV_WIN_HOST_PROCESS_1_0;
  return f;
}

}  // namespace

__global__ void __launch_bounds__(kBlock) kpe_scan_kernel(ScanArgs a) {
  __shared__ uint32_t s_off[kBlock + 1];
  __shared__ uint32_t s_cb[kChunk];
  __shared__ unsigned long long s_cnt[6 * 64];

  const int64_t p0 = (int64_t)blockIdx.x * kBlock;
  const uint32_t t = threadIdx.x;
  const int64_t r = p0 + t;
  const bool live = r < a.n;
  const uint32_t np = (uint32_t)((a.n - p0) < (int64_t)kBlock ? (a.n - p0) : (int64_t)kBlock);
  const uint32_t R = a.nrules;
  const bool small_r = R <= 64;
  if (small_r)
    for (uint32_t i = t; i < 6 * R; i += kBlock) s_cnt[i] = 0;
  __syncthreads();

  uint32_t fails = 0;  // versioned-check failures of this resource
  if (a.any_pss) {
    // ---- containers: coalesced stream through LDS, OR-reduced per resource ----
    for (uint32_t i = t; i <= np; i += kBlock) s_off[i] = a.ctr_off[p0 + i];
    __syncthreads();
    const uint32_t c_begin = s_off[0], c_end = s_off[np];
    uint64_t caps_ok = a.pp_caps_ok >= 0 ? pmask64(a, a.pp_caps_ok) : 0, nbs = a.pp_cap_nbs >= 0 ? pmask64(a, a.pp_cap_nbs) : 0,
             all = a.pp_cap_all >= 0 ? pmask64(a, a.pp_cap_all) : 0;
    uint32_t cb = 0;
    const uint32_t my_lo = live ? s_off[t] : 0, my_hi = live ? s_off[t + 1] : 0;
    for (uint32_t base = c_begin; base < c_end; base += kChunk) {
      const uint32_t lim = (c_end - base) < kChunk ? (c_end - base) : kChunk;
      for (uint32_t i = t; i < lim; i += kBlock) {
        uint32_t c = base + i;
        s_cb[i] = container_bits(a.c_sc[c], a.c_add[c], a.c_drop[c], a.c_sann[c], caps_ok, nbs, all, a);
      }
      __syncthreads();
      uint32_t lo = my_lo > base ? my_lo : base, hi = my_hi < base + lim ? my_hi : base + lim;
      for (uint32_t c = lo; c < hi; ++c) cb |= s_cb[c - base];
      __syncthreads();
    }
    if (live) {
      const uint32_t pw = a.p_sc[r];
      // volumes
      bool vol_hostpath = false, vol_restricted = false;
      for (uint32_t j = a.vol_off[r], e = a.vol_off[r + 1]; j < e; ++j) {
        uint32_t s = a.vol_src[j];
        if (s & (1u << VS_HOSTPATH)) vol_hostpath = true;
        if (!(s & kAllowedVolumes)) vol_restricted = true;
      }
      // sysctls (three allow-lists: 1.0, 1.27, 1.29)
      uint32_t sys_bad = 0;
      for (uint32_t j = a.sys_off[r], e = a.sys_off[r + 1]; j < e; ++j) {
        uint32_t id = a.sys_id[j];
        if (!pbit(a, a.pp_sysctl0, id)) sys_bad |= 1u;
        if (!pbit(a, a.pp_sysctl1, id)) sys_bad |= 2u;
        if (!pbit(a, a.pp_sysctl2, id)) sys_bad |= 4u;
      }
      // pod-template annotations: AppArmor and the seccomp pod annotation
      bool apparmor_bad = false, sec_pod_ann_bad = false;
      for (uint32_t j = a.pann_off[r], e = a.pann_off[r + 1]; j < e; ++j) {
        uint32_t k = a.pann_k[j], v = a.pann_v[j];
        if (pbit(a, a.pp_apparmor_key, k) && !pbit(a, a.pp_apparmor_ok, v)) apparmor_bad = true;
        if (pbit(a, a.pp_seccomp_pod_key, k) && !pbit(a, a.pp_seccomp_ann_ok, v)) sec_pod_ann_bad = true;
      }
      fails = cv_fails(a, pw, cb, vol_hostpath, vol_restricted, sys_bad, apparmor_bad, sec_pod_ann_bad) & a.cv_union;
    }
  }

  // ---- rules: match/exclude, handler, ApplyOne, verdict cell ----
  uint32_t flags = live ? a.r_flags[r] : 0, gvk = live ? a.r_gvk[r] : 0;
  uint32_t nsa = live ? a.r_nsa[r] : KPE_NO_STR;
  bool applied = false;
  uint32_t cur_policy = 0xFFFFFFFFu;
  for (uint32_t ri = 0; ri < R; ++ri) {
    KpeRule rule = a.rules[ri];
    if (rule.policy != cur_policy) {
      cur_policy = rule.policy;
      applied = false;
    }
    uint8_t v = KPE_NA_;
    uint32_t cmask = 0;
    if (live && !(rule.apply_one && applied)) {
      bool m = rule.pol_ns_pred < 0 || pbit(a, rule.pol_ns_pred, nsa);
      m = m && eval_block(a, rule.match_mode, rule.match_f0, rule.match_nf, r, gvk, flags);
      if (m) {
        bool ex;
        if (rule.excl_mode == MODE_ANY) {
          ex = false;
          for (uint32_t f = 0; f < rule.excl_nf && !ex; ++f) ex = eval_filter(a, rule.excl_f0 + f, r, gvk, flags);
        } else if (rule.excl_mode == MODE_ALL) {
          ex = true;
          for (uint32_t f = 0; f < rule.excl_nf && ex; ++f) ex = eval_filter(a, rule.excl_f0 + f, r, gvk, flags);
        } else {
          ex = eval_filter(a, rule.excl_f0, r, gvk, flags);
        }
        m = !ex;
      }
      if (m) {
        if (rule.handler == H_PSS) {
          if ((flags & R_CLASS_MASK) == R_CLASS_OTHER || (flags & R_DECODE_ERR)) {
            v = KPE_ERROR_;
          } else {
            uint32_t f = fails & rule.cv_mask;
            v = f ? KPE_FAIL_ : KPE_PASS_;
            for (uint32_t cv = 0; cv < KPE_NUM_CV; ++cv)
              if (f & (1u << cv)) cmask |= 1u << kCvCheck[cv];
          }
        } else if (rule.handler == H_ERROR) {
          v = KPE_ERROR_;
        }
      }
      if (v == KPE_PASS_ || v == KPE_FAIL_) applied = true;
    }
    if (live) {
      a.verdicts[r * R + ri] = v;
      if (a.masks) a.masks[r * R + ri] = cmask;
    }
    if (small_r) {
      // wave-ballot histogram of this rule's verdicts
      const uint32_t lane = t & 63u;
      for (uint32_t k = 1; k < 6; ++k) {
        uint64_t b = __ballot(live && v == k);
        if (lane == 0 && b) atomicAdd(&s_cnt[ri * 6 + k], (unsigned long long)__popcll(b));
      }
    } else if (live && v != KPE_NA_) {
      atomicAdd(&a.counts[ri * 6 + v], 1ull);
    }
  }
  if (small_r) {
    __syncthreads();
    for (uint32_t i = t; i < 6 * R; i += kBlock)
      if (i % 6 != 0 && s_cnt[i]) atomicAdd(&a.counts[i], s_cnt[i]);
  }
}

// ---------------------------------------------------------------------------
// Host-side launch wrappers (called from kpe_api.cpp).
extern "C" hipError_t kpe_launch_pred(const PredArgs* a, uint32_t nblocks, hipStream_t s) {
  if (nblocks == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_pred_kernel, dim3(nblocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}
extern "C" hipError_t kpe_launch_scan(const ScanArgs* a, hipStream_t s) {
  if (a->n == 0) return hipSuccess;
  uint32_t blocks = (uint32_t)((a->n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(kpe_scan_kernel, dim3(blocks), dim3(kBlock), 0, s, *a);
  return hipGetLastError();
}
