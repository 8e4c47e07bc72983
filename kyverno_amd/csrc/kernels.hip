// CDNA4 (gfx950) kernels for batch policy evaluation. wave64, HBM-bound scans.
//
//  kpe_pred_kernel   — dictionary pass: every string predicate of the compiled
//                      program (an OR of go-wildcard globs, ext/wildcard/match.go:7-9)
//                      is evaluated once per DISTINCT string of its domain into a
//                      bitset (one wave = 64 dictionary ids, built with a ballot).
//                      Patterns are host-classified (exact / prefix / suffix /
//                      contains / general glob) so the common cases are straight
//                      byte compares without backtracking.
//  kpe_scan_kernel   — one resource per lane. Per block: (1) the compiled program,
//                      the predicate directory and the small-domain bitsets are
//                      copied into LDS; (2) the block's containers are streamed
//                      coalesced through LDS and OR-reduced per resource (the
//                      1..64-container fan-out never diverges the HBM loads);
//                      (3) PSA versioned checks (pkg/pss/evaluate.go:24-70 over the
//                      PSA v0.29 policy/check_*.go semantics); (4) match/exclude per
//                      rule (pkg/engine/utils/match.go:168-300) with ApplyOne
//                      (pkg/engine/validation.go:75-77); (5) verdict cells staged in
//                      LDS and written as coalesced dwords; per-rule counters by
//                      wave ballot into per-block partials (no atomics, no memset).
//  kpe_count_reduce  — sums the per-block counter partials (fetch time only).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels_abi.h"
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
  for (int i = 0; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
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
    default: return glob(lit, ln, s, sn);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) kpe_pred_kernel(PredArgs a) {
  uint32_t b = blockIdx.x;
  uint32_t j = 0;
  while (j + 1 < a.njobs && a.jobs[j + 1].blk0 <= b) ++j;  // uniform per block
  const PredJob job = a.jobs[j];
  const uint32_t id = (b - job.blk0) * 256u + threadIdx.x;
  const uint32_t n = a.dict_n[job.domain];
  bool hit = false;
  if (id < n) {
    const uint32_t* off = a.dict_off[job.domain];
    const uint8_t* s = a.dict_bytes[job.domain] + off[id];
    const int sn = (int)(off[id + 1] - off[id]);
    for (uint32_t k = 0; k < job.npat && !hit; ++k) hit = pat_match(a.pats[job.pat0 + k], a.pat_bytes, s, sn);
  }
  const uint64_t m = __ballot(hit);
  const uint32_t wid = id >> 6;  // 64 strings per wave => two output words
  if ((threadIdx.x & 63u) == 0 && (uint64_t)wid * 64u < n) {
    a.out[job.out_word + 2 * wid] = (uint32_t)m;
    a.out[job.out_word + 2 * wid + 1] = (uint32_t)(m >> 32);
  }
}

// one block per counter column; coalesced over blocks-of-partials
__global__ void __launch_bounds__(256) kpe_count_reduce(const uint32_t* part, uint32_t nblocks, uint32_t width,
                                                        unsigned long long* out) {
  __shared__ unsigned long long red[256];
  const uint32_t col = blockIdx.x;
  unsigned long long s = 0;
  for (uint32_t b = threadIdx.x; b < nblocks; b += 256) s += part[(size_t)b * width + col];
  red[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[col] = red[0];
}

// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kBlock = 256;
constexpr uint32_t kAllowedVolumes = (1u << VS_CONFIGMAP) | (1u << VS_CSI) | (1u << VS_DOWNWARDAPI) |
                                     (1u << VS_EMPTYDIR) | (1u << VS_EPHEMERAL) | (1u << VS_PVC) |
                                     (1u << VS_PROJECTED) | (1u << VS_SECRET);

__constant__ uint8_t kCvCheck[KPE_NUM_CV] = {
    CK_APE, CK_APE, CK_APPARMOR, CK_CAPS_BASELINE, CK_CAPS_RESTRICTED, CK_CAPS_RESTRICTED, CK_HOST_NS,
    CK_HOST_PATH, CK_HOST_PORTS, CK_PRIVILEGED, CK_PROC_MOUNT, CK_RESTRICTED_VOLUMES, CK_RUN_AS_NON_ROOT,
    CK_RUN_AS_USER, CK_SELINUX, CK_SECCOMP_BASELINE, CK_SECCOMP_BASELINE, CK_SECCOMP_RESTRICTED,
    CK_SECCOMP_RESTRICTED, CK_SYSCTLS, CK_SYSCTLS, CK_SYSCTLS, CK_WIN_HOST_PROCESS};

// PSA versioned checks for one pod given the OR of its container bits.
__device__ __forceinline__ uint32_t cv_fails(uint32_t pw, uint32_t cb, bool vol_hostpath, bool vol_restricted,
                                             uint32_t sys_bad, bool apparmor_bad, bool sec_pod_ann_bad) {
  uint32_t f = 0;
  const bool win = FIELD(pw, P_OS_SH, 2) == OS_WINDOWS;
  if (cb & CB_APE) f |= (1u << CV_APE_1_8) | (win ? 0u : (1u << CV_APE_1_25));
  if (apparmor_bad) f |= 1u << CV_APPARMOR_1_0;
  if (cb & CB_CAPS_BASE) f |= 1u << CV_CAPS_BASELINE_1_0;
  if (cb & (CB_CAPS_DROP | CB_CAPS_ADD))
    f |= (1u << CV_CAPS_RESTRICTED_1_22) | (win ? 0u : (1u << CV_CAPS_RESTRICTED_1_25));
  if (pw & (P_HOSTNET | P_HOSTPID | P_HOSTIPC)) f |= 1u << CV_HOST_NS_1_0;
  if (vol_hostpath) f |= 1u << CV_HOST_PATH_1_0;
  if (cb & CB_HOSTPORT) f |= 1u << CV_HOST_PORTS_1_0;
  if (cb & CB_PRIV) f |= 1u << CV_PRIVILEGED_1_0;
  if (cb & CB_PROCMOUNT) f |= 1u << CV_PROC_MOUNT_1_0;
  if (vol_restricted) f |= 1u << CV_RESTRICTED_VOLUMES_1_0;
  const uint32_t prnr = FIELD(pw, P_RNR_SH, 2);
  if (prnr == TRI_FALSE || (cb & CB_RNR_FALSE) || (prnr != TRI_TRUE && (cb & CB_RNR_UNSET)))
    f |= 1u << CV_RUN_AS_NON_ROOT_1_0;
  if (FIELD(pw, P_RAU_SH, 2) == RAU_ZERO || (cb & CB_RAU_ZERO)) f |= 1u << CV_RUN_AS_USER_1_23;
  const uint32_t psel = FIELD(pw, P_SEL_SH, 3);
  if ((psel != SEL_NONE && (psel == SEL_OTHER || (pw & (P_SEL_USER | P_SEL_ROLE)))) || (cb & CB_SELINUX))
    f |= 1u << CV_SELINUX_1_0;
  if (sec_pod_ann_bad || (cb & CB_SEC_ANN)) f |= 1u << CV_SECCOMP_BASELINE_1_0;
  const uint32_t psec = FIELD(pw, P_SECCOMP_SH, 3);
  const bool psec_valid = psec == SECCOMP_RUNTIMEDEFAULT || psec == SECCOMP_LOCALHOST;
  const bool psec_bad = psec != SECCOMP_NONE && !psec_valid;
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

// Capability-set violation bits (computed per block into LDS from the capset dictionary)
#define CS_BASE 1u  // add has a capability outside the baseline allow-list
#define CS_DROP 2u  // drop lacks "ALL"
#define CS_ADD 4u   // add has anything but NET_BIND_SERVICE

__device__ __forceinline__ uint32_t ctr_bits(uint32_t w, uint32_t csb) {
  uint32_t b = 0;
  const bool caps = w & C_CAPS_PRESENT;
  if (caps && (csb & CS_BASE)) b |= CB_CAPS_BASE;
  if (!caps || (csb & CS_DROP)) b |= CB_CAPS_DROP;
  if (caps && (csb & CS_ADD)) b |= CB_CAPS_ADD;
  if (FIELD(w, C_APE_SH, 2) != TRI_FALSE) b |= CB_APE;
  if (FIELD(w, C_HOSTPORT_SH, 4)) b |= CB_HOSTPORT;
  if (FIELD(w, C_PRIV_SH, 2) == TRI_TRUE) b |= CB_PRIV;
  if (FIELD(w, C_PROCMOUNT_SH, 2) == PROCMOUNT_OTHER) b |= CB_PROCMOUNT;
  const uint32_t rnr = FIELD(w, C_RNR_SH, 2);
  if (rnr == TRI_FALSE) b |= CB_RNR_FALSE;
  if (rnr == TRI_UNSET) b |= CB_RNR_UNSET;
  if (FIELD(w, C_RAU_SH, 2) == RAU_ZERO) b |= CB_RAU_ZERO;
  const uint32_t sel = FIELD(w, C_SEL_SH, 3);
  if (sel != SEL_NONE && (sel == SEL_OTHER || (w & (C_SEL_USER | C_SEL_ROLE)))) b |= CB_SELINUX;
  const uint32_t sec = FIELD(w, C_SECCOMP_SH, 3);
  if (sec == SECCOMP_NONE) b |= CB_SEC_UNSET;
  else if (sec != SECCOMP_RUNTIMEDEFAULT && sec != SECCOMP_LOCALHOST) b |= CB_SEC_BAD;
  if (FIELD(w, C_WHP_SH, 2) == TRI_TRUE) b |= CB_WHP;
  return b;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Wave-uniform table read: the address is uniform, so this is a scalar (SMEM) load
// through the constant cache — no LDS round trip and no readfirstlane to branch on it.
template <class T>
__device__ __forceinline__ T sld(const T* p, uint32_t i) {
  static_assert(sizeof(T) % 4 == 0, "word-sized tables");
  typedef __attribute__((address_space(4))) const uint32_t* cptr;
  const cptr src = (cptr)(p + i);
  T out;
  uint32_t* d = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
  for (uint32_t k = 0; k < sizeof(T) / 4; ++k) d[k] = src[k];
  return out;
}
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// Bitset word of a resolved predicate location (PRED_LOCAL | LDS index, or pbuf index).
struct Bits {
  const uint32_t* lds;
  const uint32_t* pbuf;
  __device__ __forceinline__ uint32_t word(uint32_t loc, uint32_t wi) const {
    return (loc & PRED_LOCAL) ? lds[(loc & ~PRED_LOCAL) + wi] : pbuf[loc + wi];
  }
  __device__ __forceinline__ bool bit(uint32_t loc, uint32_t id) const {
    if (id == KPE_NO_STR) return false;
    return (word(loc, id >> 5) >> (id & 31u)) & 1u;
  }
  __device__ __forceinline__ uint64_t mask64(uint32_t loc) const {  // predicate over D_CAP (<= 64 ids)
    return loc == PRED_NONE ? 0ull : ((uint64_t)word(loc, 0) | ((uint64_t)word(loc, 1) << 32));
  }
};

// Round-1 data of one 64-resource tile.
struct Tile1 {
  uint4 rec, hdr;
  uint32_t gvk, nsa, name, mns;
};

template <bool PSS>
__device__ __forceinline__ Tile1 load_tile1(const ScanArgs& a, int64_t tile, uint32_t lane) {
  Tile1 d;
  d.rec = d.hdr = make_uint4(0, 0, 0, 0);
  d.gvk = 0;
  d.nsa = d.name = d.mns = KPE_NO_STR;
  const int64_t r = tile * 64 + lane;
  const int64_t rc = r < a.n ? r : a.n - 1;  // clamped: loads are unconditional
  if (PSS) {
    d.rec = reinterpret_cast<const uint4*>(a.rec)[rc];
    // the wave header as a vector load (a scalar load would be waited on at once)
    uint32_t hv = (uint32_t)tile;
    asm volatile("" : "+v"(hv));
    d.hdr = reinterpret_cast<const uint4*>(a.hdr)[hv];
  } else {
    if (a.need & NEED_GVK) d.gvk = a.r_gvk[rc];
    if (a.need & NEED_NSA) d.nsa = a.r_nsa[rc];
  }
  if (a.need & NEED_NAME) d.name = a.r_name[rc];
  if (a.need & NEED_MNS) d.mns = a.r_mns[rc];
  return d;
}

// Persistent, wave-autonomous scan. Every wave walks 64-resource tiles
// (tile = global wave id, + total waves, ...) with the next tile's round-1 loads in
// flight while the current tile is evaluated:
//
//  round 1  pod record (dwordx4) + wave header (PSS programs) or the gvk /
//           namespace columns, plus the name columns the terms read — prefetched
//           one tile ahead;
//  round 2  (PSS) the lane's list items at header + exclusive wave scan of the
//           counts: up to 4 containers, 2 volumes, 2 annotations, 1 sysctl issued
//           together; the PSA versioned checks give a per-lane failure bitmask
//           (pkg/pss/evaluate.go:24-70 over the PSA v0.29 check semantics);
//  terms    every DISTINCT match term is evaluated once per resource and ballot-ed
//           into a 64-bit mask (LDS, per wave); so is every distinct PSS version set;
//  rules    transposed: lane j evaluates rule c0+j for all 64 resources at once with
//           64-bit mask algebra (match/exclude: pkg/engine/utils/match.go:168-300;
//           ApplyOne: pkg/engine/validation.go:75-77), then each resource lane
//           extracts its verdict bytes; cells are staged per wave and stored as
//           contiguous row segments; counts are popcounts (LDS per block).
template <bool PSS>
__global__ void __launch_bounds__(kBlock) kpe_scan_kernel(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  __shared__ __attribute__((aligned(16))) uint8_t s_capb[KPE_MAX_CAPSETS];
  __shared__ __attribute__((aligned(16))) uint32_t s_cnt[3 * KPE_LDS_R];

  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t R = a.nrules, need = a.need;
  const bool lds_cnt = R <= KPE_LDS_R;
  const bool need_caps = PSS && (need & NEED_CAPS);
  const int64_t ntiles = (a.n + 63) >> 6;
  const uint32_t W = gridDim.x * (kBlock / 64u);
  int64_t tile = (int64_t)blockIdx.x * (kBlock / 64u) + wv;

  // ---- block prologue (overlapped with the first tile's round-1 loads) ----
  Tile1 nx{};
  if (tile < ntiles) nx = load_tile1<PSS>(a, tile, lane);
  {
    const uint32_t nb4 = a.blob_words >> 2;  // >= 1
    const uint4* blob = reinterpret_cast<const uint4*>(a.pbuf);
    uint4* d4 = reinterpret_cast<uint4*>(dyn);
#pragma unroll 1
    for (uint32_t i = t; i < nb4; i += kBlock) d4[i] = blob[i];
    if (a.filt_lds != PRED_NONE) {  // program filters + filter terms for the rule lanes
      const uint32_t nw = a.fterm_lds + a.nfterms - a.filt_lds;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.filters);
#pragma unroll 1
      for (uint32_t i = t; i < nw; i += kBlock)
        dyn[a.filt_lds + i] = i < a.fterm_lds - a.filt_lds ? src[i] : a.fterms[i - (a.fterm_lds - a.filt_lds)];
    }
#pragma unroll 1
    for (uint32_t i = t; i < 3 * R && lds_cnt; i += kBlock) s_cnt[i] = 0;
  }
  __syncthreads();
  const Bits B{dyn, a.pbuf};
  if (need_caps) {  // capability-set violation bits (add/drop masks vs the fixed allow-lists)
    const uint64_t caps_ok = B.mask64(a.pp_caps_ok), nbs = B.mask64(a.pp_cap_nbs), all = B.mask64(a.pp_cap_all);
#pragma unroll 1
    for (uint32_t i = t; i < a.ncapsets; i += kBlock) {
      const uint4 c = reinterpret_cast<const uint4*>(a.capsets)[i];
      const uint64_t ad = (uint64_t)c.x | ((uint64_t)c.y << 32), dr = (uint64_t)c.z | ((uint64_t)c.w << 32);
      s_capb[i] = (uint8_t)(((ad & ~caps_ok) ? CS_BASE : 0u) | ((dr & all) ? 0u : CS_DROP) | ((ad & ~nbs) ? CS_ADD : 0u));
    }
    __syncthreads();
  }
  const KpeFilter* filt =
      a.filt_lds != PRED_NONE ? reinterpret_cast<const KpeFilter*>(dyn + a.filt_lds) : a.filters;
  const uint32_t* fterm = a.filt_lds != PRED_NONE ? dyn + a.fterm_lds : a.fterms;

  // per-wave LDS: term masks, PSS version-set masks, rule cell masks, verdict staging
  uint64_t* tmk = reinterpret_cast<uint64_t*>(dyn + a.wave_lds + wv * a.wave_words);
  uint64_t* cvm = tmk + a.nterms;
  uint64_t* rmk = cvm + a.ncv;                                       // kRC x (P, F, E)
  uint8_t* sv = reinterpret_cast<uint8_t*>(rmk + 3 * KPE_RULE_CHUNK);  // 64 x kRC bytes

  // single-chunk programs keep lane j's packed rule in registers for every tile
  uint4 myrule = make_uint4(0, 0, 0, 0);
  if (R <= KPE_RULE_CHUNK && lane < R) myrule = reinterpret_cast<const uint4*>(a.rule_lanes)[lane];

#pragma unroll 1
  for (; tile < ntiles; tile += W) {
    const Tile1 cur = nx;
    if (tile + W < ntiles) nx = load_tile1<PSS>(a, tile + W, lane);
    const int64_t r = tile * 64 + lane;
    const bool live = r < a.n;
    const int64_t rc = live ? r : a.n - 1;
    const uint4 rec = live ? cur.rec : make_uint4(0, 0, 0, 0);
    const uint4 hdr = cur.hdr;

    uint32_t fails = 0;
    if (PSS) {
      // ---- list offsets: header + exclusive wave scan of the packed counts ----
      const uint32_t z = rec.z;
      const uint32_t c01 = (z & 0xFFu) | ((z & 0xFF00u) << 8), c23 = ((z >> 16) & 0xFFu) | ((z >> 24) << 16);
      const uint32_t e01 = wave_incl_scan(c01) - c01, e23 = wave_incl_scan(c23) - c23;
      const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
      const uint32_t oc = hdr.x + (e01 & 0xFFFFu), ov = hdr.y + (e01 >> 16), os = hdr.z + (e23 & 0xFFFFu),
                     oa = hdr.w + (e23 >> 16);
      // ---- round 2: every first-pass list load issued before any is used ----
      const uint2* crec = reinterpret_cast<const uint2*>(a.crec);
      const uint2* pkv = reinterpret_cast<const uint2*>(a.pann_kv);
      const bool nvol = (need & NEED_VOL) && a.nvol_total, nsys = (need & NEED_SYS) && a.nsys_total,
                 npann = (need & NEED_PANN) && a.npann_total, nsann = (need & NEED_SANN) && a.nctr_total;
      const uint2 z2 = make_uint2(0, 0);
      uint2 k0 = z2, k1 = z2, k2 = z2, k3 = z2;
      if (a.nctr_total) {
        const uint32_t lim = a.nctr_total - 1;
        k0 = crec[min(oc, lim)];
        k1 = crec[min(oc + 1, lim)];
        k2 = crec[min(oc + 2, lim)];
        k3 = crec[min(oc + 3, lim)];
      }
      uint32_t v0 = 0, v1 = 0, sy0 = 0;
      if (nvol) {
        v0 = a.vol_src[min(ov, a.nvol_total - 1)];
        v1 = a.vol_src[min(ov + 1, a.nvol_total - 1)];
      }
      if (nsys) sy0 = a.sys_id[min(os, a.nsys_total - 1)];
      uint2 q0 = z2, q1 = z2;
      if (npann) {
        q0 = pkv[min(oa, a.npann_total - 1)];
        q1 = pkv[min(oa + 1, a.npann_total - 1)];
      }
      uint32_t sa0 = KPE_NO_STR, sa1 = KPE_NO_STR, sa2 = KPE_NO_STR, sa3 = KPE_NO_STR;
      if (nsann) {
        const uint32_t lim = a.nctr_total - 1;
        sa0 = a.c_sann[min(oc, lim)];
        sa1 = a.c_sann[min(oc + 1, lim)];
        sa2 = a.c_sann[min(oc + 2, lim)];
        sa3 = a.c_sann[min(oc + 3, lim)];
      }
      // ---- containers: violation bits OR-ed over the pod's containers ----
      auto one = [&](uint2 kk, uint32_t sann) -> uint32_t {
        uint32_t b = ctr_bits(kk.x, need_caps ? s_capb[kk.y] : 0u);
        if (nsann && sann != KPE_NO_STR && !B.bit(a.pp_seccomp_ann_ok, sann)) b |= CB_SEC_ANN;
        return b;
      };
      uint32_t cb = (nc > 0 ? one(k0, sa0) : 0u) | (nc > 1 ? one(k1, sa1) : 0u) | (nc > 2 ? one(k2, sa2) : 0u) |
                    (nc > 3 ? one(k3, sa3) : 0u);
#pragma unroll 1
      for (uint32_t k = 4; k < nc; ++k) cb |= one(crec[oc + k], nsann ? a.c_sann[oc + k] : KPE_NO_STR);
      // ---- volumes ----
      uint32_t vor = 0, vand = ~0u;  // hostPath present anywhere / some volume outside the allow-list
      auto vol = [&](uint32_t sv_) {
        vor |= sv_;
        vand &= (sv_ & kAllowedVolumes) ? ~0u : 0u;
      };
      if (nvol) {
        if (nv > 0) vol(v0);
        if (nv > 1) vol(v1);
#pragma unroll 1
        for (uint32_t k = 2; k < nv; ++k) vol(a.vol_src[ov + k]);
      }
      const bool vol_hostpath = (vor >> VS_HOSTPATH) & 1u, vol_restricted = vand == 0u;
      // ---- sysctls (allow-lists 1.0 / 1.27 / 1.29) ----
      uint32_t sys_bad = 0;
      auto sysf = [&](uint32_t id) {
        sys_bad |= (B.bit(a.pp_sysctl0, id) ? 0u : 1u) | (B.bit(a.pp_sysctl1, id) ? 0u : 2u) |
                   (B.bit(a.pp_sysctl2, id) ? 0u : 4u);
      };
      if (nsys) {
        if (ns > 0) sysf(sy0);
#pragma unroll 1
        for (uint32_t k = 1; k < ns; ++k) sysf(a.sys_id[os + k]);
      }
      // ---- pod-template annotations: AppArmor, seccomp pod annotation ----
      bool apparmor_bad = false, sec_pod_ann_bad = false;
      auto ann = [&](uint2 kv) {
        apparmor_bad |= B.bit(a.pp_apparmor_key, kv.x) && !B.bit(a.pp_apparmor_ok, kv.y);
        sec_pod_ann_bad |= B.bit(a.pp_seccomp_pod_key, kv.x) && !B.bit(a.pp_seccomp_ann_ok, kv.y);
      };
      if (npann) {
        if (na > 0) ann(q0);
        if (na > 1) ann(q1);
#pragma unroll 1
        for (uint32_t k = 2; k < na; ++k) ann(pkv[oa + k]);
      }
      if (live) fails = cv_fails(rec.x, cb, vol_hostpath, vol_restricted, sys_bad, apparmor_bad, sec_pod_ann_bad) & a.cv_union;
    }

    // ---- terms: one ballot per distinct term ----
    const uint32_t gvk = PSS ? rec.y : (live ? cur.gvk : 0u);
    const uint32_t nsa = PSS ? rec.w : (live ? cur.nsa : KPE_NO_STR);
    const uint32_t name_col = live ? cur.name : KPE_NO_STR, mns_col = live ? cur.mns : KPE_NO_STR;
#pragma unroll 1
    for (uint32_t ti = 0; ti < a.nterms; ++ti) {
      const KpeTerm tm = sld(a.terms, ti);
      bool ok = true;
      if (tm.type == T_KIND_PRED) {
        ok = B.bit(tm.a, GVK_KIND(gvk));
      } else if (tm.type == T_KINDS) {  // CheckKind: OR over kind selectors
        ok = false;
#pragma unroll 1
        for (uint32_t k = 0; k < tm.b; ++k) {
          const KpeKindSel ks = sld(a.kindsels, tm.a + k);
          ok |= ks.sub_ok && (ks.pg == PRED_NONE || B.bit(ks.pg, GVK_GRP(gvk))) &&
                (ks.pv == PRED_NONE || B.bit(ks.pv, GVK_VER(gvk))) && (ks.pk == PRED_NONE || B.bit(ks.pk, GVK_KIND(gvk)));
        }
      } else if (tm.type == T_PRED) {
        const uint32_t id = tm.b == COL_NAME ? name_col : (tm.b == COL_MNS ? mns_col : nsa);
        ok = B.bit(tm.a, id);
      } else if (tm.type == T_ANNOTATIONS) {  // CheckAnnotations: every pair matched by some annotation
        const uint32_t lo = a.ann_off[rc], hi = live ? a.ann_off[rc + 1] : lo;
#pragma unroll 1
        for (uint32_t k = 0; k < tm.b; ++k) {
          const KpeAnnPair pr = sld(a.annpairs, tm.a + k);
          bool hit = false;
#pragma unroll 1
          for (uint32_t j = lo; j < hi && !hit; ++j) hit = B.bit(pr.pk, a.ann_k[j]) && B.bit(pr.pv, a.ann_v[j]);
          ok &= hit;
        }
      } else if (tm.type == T_SELECTOR || tm.type == T_NSSELECTOR) {
        // CheckSelector (pkg/utils/match/labels.go:9-24) over the resource's labels or,
        // for namespaceSelector, its namespace's labels (utils/match.go:114-138)
        const KpeSelector S = sld(a.selectors, tm.a);
        uint32_t lo = 0, hi = 0;
        const uint32_t *K = a.lab_k, *V = a.lab_v;
        bool eval = true;
        if (tm.type == T_SELECTOR) {
          lo = a.lab_off[rc];
          hi = live ? a.lab_off[rc + 1] : lo;
        } else {
          // never for kind Namespace; skipped for an empty kind unless kinds hold "*"
          const uint32_t kid = GVK_KIND(gvk);
          const uint32_t row = a.r_nsl[rc];
          if (live && row != KPE_NO_STR) lo = a.nsl_off[row], hi = a.nsl_off[row + 1];
          K = a.nsl_k, V = a.nsl_v;
          if (B.bit(S.p_kind_ns, kid)) {
            ok = false, eval = false;
          } else if (B.bit(S.p_kind_empty, kid) && !S.star_kind) {
            ok = true, eval = false;
          } else if (S.invalid) {
            ok = false, eval = false;
          }
        }
        if (eval) {
#pragma unroll 1
          for (uint32_t qi = 0; qi < S.nreq; ++qi) {
            const KpeSelReq q = sld(a.selreqs, S.req0 + qi);
            const bool wild = q.op == SR_WILD;
            uint32_t j = lo;
#pragma unroll 1
            for (; j < hi; ++j)  // first label with a matching key (and value, for wildcards)
              if (B.bit(q.pk, K[j]) && (!wild || B.bit(q.pv, V[j]))) break;
            const bool found = j < hi;
            const uint32_t kid = found ? K[j] : KPE_NO_STR, vid = found ? V[j] : KPE_NO_STR;
            bool qok;
            switch (q.op) {
              case SR_EQ:
              case SR_IN: qok = found && B.bit(q.pv, vid); break;
              case SR_WILD: qok = found && B.bit(q.pk_ok, kid) && B.bit(q.pv_ok, vid); break;
              case SR_NOTIN: qok = !found || !B.bit(q.pv, vid); break;
              case SR_EXISTS: qok = found; break;
              default: qok = !found; break;
            }
            ok &= qok;
          }
        }
      } else {  // T_FALSE
        ok = false;
      }
      const uint64_t m = __ballot(ok);
      if (lane == 0) tmk[ti] = m;
    }
    // PSS version sets: resources failing some check of each distinct cv_mask
#pragma unroll 1
    for (uint32_t c = 0; c < a.ncv; ++c) {
      const uint64_t m = __ballot((fails & sld(a.cv_classes, c)) != 0u);
      if (lane == 0) cvm[c] = m;
    }
    const uint32_t cls = (rec.x >> PR_CLASS_SH) & R_CLASS_MASK;
    const uint64_t live_m = __ballot(live);
    const uint64_t err_m = PSS ? __ballot(live && (cls == R_CLASS_OTHER || (rec.x & PR_DECODE_ERR))) : 0ull;
    const uint32_t nrows = (uint32_t)min((int64_t)64, a.n - tile * 64);
    __builtin_amdgcn_wave_barrier();

    // ---- rules, KPE_RULE_CHUNK at a time ----
    uint64_t applied = 0;  // ApplyOne state (lane 0, rule order)
    uint32_t cur_policy = 0xFFFFFFFFu;
#pragma unroll 1
    for (uint32_t c0 = 0; c0 < R; c0 += KPE_RULE_CHUNK) {
      const uint32_t nc = min((uint32_t)KPE_RULE_CHUNK, R - c0);
      // (a) transposed: lane j evaluates rule c0 + j over the whole tile
      if (lane < nc) {
        const uint4 rl = R <= KPE_RULE_CHUNK ? myrule : reinterpret_cast<const uint4*>(a.rule_lanes)[c0 + lane];
        auto block_mask = [&](uint32_t mode, uint32_t f0, uint32_t nf) -> uint64_t {
          const bool all = mode == MODE_ALL;  // any => OR of filters, all => AND, legacy => its filter
          uint64_t acc = all ? ~0ull : 0ull;
#pragma unroll 1
          for (uint32_t f = 0; f < nf; ++f) {
            const KpeFilter fl = filt[f0 + f];
            uint64_t fm = ~0ull;  // a filter is the AND of its terms
#pragma unroll 1
            for (uint32_t k = 0; k < fl.nt; ++k) fm &= tmk[fterm[fl.t0 + k]];
            acc = all ? (acc & fm) : (acc | fm);
          }
          return acc;
        };
        const uint32_t handler = RL_HANDLER(rl.x);
        uint64_t m = live_m;
        if (rl.w != PRED_NONE) m &= tmk[rl.w];
        if (m) m &= block_mask(RL_MATCH_MODE(rl.x), RL_F0(rl.y), RL_NF(rl.y));
        if (m) m &= ~block_mask(RL_EXCL_MODE(rl.x), RL_F0(rl.z), RL_NF(rl.z));
        uint64_t pm = 0, fm = 0, em = 0;
        if (handler == H_PSS) {
          em = m & err_m;
          fm = m & ~em & cvm[RL_CV(rl.x)];
          pm = m & ~em & ~fm;
        } else if (handler == H_ERROR) {
          em = m;
        }
        rmk[lane * 3 + 0] = pm;
        rmk[lane * 3 + 1] = fm;
        rmk[lane * 3 + 2] = em;
      }
      __builtin_amdgcn_wave_barrier();
      if (a.any_apply_one) {  // ApplyOne: later rules of a policy skip resources already applied
        if (lane == 0) {
#pragma unroll 1
          for (uint32_t j = 0; j < nc; ++j) {
            const KpeRule rule = a.rules[c0 + j];
            if (rule.policy != cur_policy) {
              cur_policy = rule.policy;
              applied = 0;
            }
            uint64_t pm = rmk[j * 3], fm = rmk[j * 3 + 1], em = rmk[j * 3 + 2];
            if (rule.apply_one) {
              pm &= ~applied, fm &= ~applied, em &= ~applied;
              rmk[j * 3] = pm, rmk[j * 3 + 1] = fm, rmk[j * 3 + 2] = em;
            }
            applied |= pm | fm;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      // (b) counts: popcounts of the cell masks (rule lanes)
      if (lane < nc) {
        const uint32_t cp = (uint32_t)__popcll(rmk[lane * 3]), cf = (uint32_t)__popcll(rmk[lane * 3 + 1]),
                       ce = (uint32_t)__popcll(rmk[lane * 3 + 2]);
        const uint32_t ri = c0 + lane;
        if (lds_cnt) {
          if (cp) atomicAdd(&s_cnt[ri * 3 + 0], cp);
          if (cf) atomicAdd(&s_cnt[ri * 3 + 1], cf);
          if (ce) atomicAdd(&s_cnt[ri * 3 + 2], ce);
        } else {
          if (cp) atomicAdd(&a.counts_global[ri * 6 + KPE_PASS_], (unsigned long long)cp);
          if (cf) atomicAdd(&a.counts_global[ri * 6 + KPE_FAIL_], (unsigned long long)cf);
          if (ce) atomicAdd(&a.counts_global[ri * 6 + KPE_ERROR_], (unsigned long long)ce);
        }
      }
      // (c) verdict bytes (resource lanes)
#pragma unroll 4
      for (uint32_t j = 0; j < nc; ++j) {
        const uint64_t pm = rmk[j * 3], fm = rmk[j * 3 + 1], em = rmk[j * 3 + 2];
        const uint32_t v = ((pm >> lane) & 1u) ? KPE_PASS_ : ((fm >> lane) & 1u) ? KPE_FAIL_
                                                               : ((em >> lane) & 1u) ? KPE_ERROR_ : KPE_NA_;
        sv[lane * nc + j] = (uint8_t)v;
      }
      if (a.masks && live) {
#pragma unroll 1
        for (uint32_t j = 0; j < nc; ++j) {
          uint32_t cmask = 0;
          if ((rmk[j * 3 + 1] >> lane) & 1u) {
            const uint32_t f = fails & sld(a.rules, c0 + j).cv_mask;
#pragma unroll 1
            for (uint32_t cv = 0; cv < KPE_NUM_CV; ++cv)
              if (f & (1u << cv)) cmask |= 1u << kCvCheck[cv];
          }
          a.masks[r * R + c0 + j] = cmask;
        }
      }
      __builtin_amdgcn_wave_barrier();
      // (d) store the tile's row segments [c0, c0 + nc)
      uint8_t* base = a.verdicts + (size_t)tile * 64 * R + c0;
      if (nc == R && (R & 3u) == 0u) {  // whole rows, dword aligned: contiguous nrows x R bytes
        uint32_t* dst = reinterpret_cast<uint32_t*>(base);
        const uint32_t* src = reinterpret_cast<const uint32_t*>(sv);
#pragma unroll 1
        for (uint32_t i = lane; i < nrows * R / 4; i += 64) dst[i] = src[i];
      } else if (nc == R) {
#pragma unroll 1
        for (uint32_t i = lane; i < nrows * R; i += 64) base[i] = sv[i];
      } else {
#pragma clang loop vectorize(disable) unroll(disable)
        for (uint32_t i = lane; i < nrows * nc; i += 64) {
          const uint32_t row = i / nc, col = i - row * nc;
          base[(size_t)row * R + col] = sv[i];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }

  // ---- epilogue: per-block count partials ----
  if (lds_cnt) {
    __syncthreads();
#pragma unroll 1
    for (uint32_t i = t; i < 6 * R; i += kBlock) {
      const uint32_t ri = i / 6, k = i - ri * 6;
      const uint32_t v = k == KPE_PASS_ ? s_cnt[ri * 3] : k == KPE_FAIL_ ? s_cnt[ri * 3 + 1]
                                                          : k == KPE_ERROR_ ? s_cnt[ri * 3 + 2] : 0u;
      a.counts_part[(size_t)blockIdx.x * 6 * R + i] = v;
    }
  }
}


// ---------------------------------------------------------------------------
// Host-side launch wrappers (called from kpe_api.cpp).
extern "C" hipError_t kpe_launch_pred(const PredArgs* a, uint32_t nblocks, hipStream_t s) {
  if (nblocks == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_pred_kernel, dim3(nblocks), dim3(256), 0, s, *a);
  return hipGetLastError();
}
// Persistent grid: as many blocks as can be resident at once (occupancy x CUs),
// capped by the number of 256-resource tiles.
extern "C" uint32_t kpe_scan_grid(int64_t n, int pss, size_t dyn_bytes) {
  if (n <= 0) return 0;
  static thread_local int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per_cu = 0;
  if (pss) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kpe_scan_kernel<true>, kBlock, dyn_bytes) != hipSuccess) per_cu = 1;
  } else {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kpe_scan_kernel<false>, kBlock, dyn_bytes) != hipSuccess) per_cu = 1;
  }
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  const int64_t g = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  return (uint32_t)(g < tiles ? g : tiles);
}
extern "C" hipError_t kpe_launch_scan(const ScanArgs* a, int pss, uint32_t grid, size_t dyn_bytes, hipStream_t s) {
  if (a->n == 0 || grid == 0) return hipSuccess;
  if (pss)
    hipLaunchKernelGGL(kpe_scan_kernel<true>, dim3(grid), dim3(kBlock), dyn_bytes, s, *a);
  else
    hipLaunchKernelGGL(kpe_scan_kernel<false>, dim3(grid), dim3(kBlock), dyn_bytes, s, *a);
  return hipGetLastError();
}
extern "C" hipError_t kpe_launch_count_reduce(const uint32_t* part, uint32_t nblocks, uint32_t width,
                                              unsigned long long* out, hipStream_t s) {
  if (width == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_count_reduce, dim3(width), dim3(256), 0, s, part, nblocks, width, out);
  return hipGetLastError();
}
