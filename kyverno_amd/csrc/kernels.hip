// CDNA4 (gfx950) kernels for batch policy evaluation. wave64, HBM-bound scans.
//
//  kpe_pred_kernel   — dictionary pass: every string predicate of the compiled
//                      program (an OR of go-wildcard globs, ext/wildcard/match.go:7-9)
//                      is evaluated once per DISTINCT string of its domain into a
//                      bitset (one wave = 64 dictionary ids, built with a ballot).
//                      Each block stages its 256 strings and the pattern bytes in
//                      LDS first, so the byte-serial compares never wait on HBM/L2.
//  kpe_scan_kernel   — one resource per lane, persistent wave-autonomous 64-row
//                      tiles: (1) PSS: list offsets from a DPP wave scan, the pod's
//                      container state bitmaps OR-ed (schema.h CX_*), the PSA
//                      versioned checks decided once per pod (pkg/pss/evaluate.go:24-70
//                      over the PSA v0.29 check semantics); (2) distinct match terms once
//                      per resource; (3) rules: NARROW programs (<= 32 terms and rules)
//                      run a per-lane rule loop over term bits, WIDE programs a
//                      transposed pass (one rule per lane, 64-bit cell masks); match /
//                      exclude pkg/engine/utils/match.go:168-300, ApplyOne
//                      pkg/engine/validation.go:75-77; (4) verdict cells staged per wave
//                      in LDS and stored as contiguous row segments.
//  kpe_count_kernel  — per-rule status histogram of a verdict matrix (the CLI totals
//                      of cmd/cli/kubectl-kyverno/processor/result.go:34-68); fetch time.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>

#include <algorithm>

#include "kernels_abi.h"
#include "schema.h"

namespace {
#include "strmatch.inl"

#ifndef KPE_PSUM_LABPRE
#define KPE_PSUM_LABPRE 0  // 1: PSUM tiles carry the label bounds and namespace row (C4 0.420 / 0.427 against
                           // 0.415 / 0.416 ms, 6 spills; profiles/r06_l)
#endif
// Wave-uniform table read: the address is uniform, so this is a scalar (SMEM) load
// through the constant cache — no LDS round trip and no readfirstlane to branch on it.
#ifndef KPE_DIAG
#define KPE_DIAG 0  // diagnostic builds only (scripts/diag_scan.sh): sections of the WIDE scan left out
#endif
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

}  // namespace

#ifndef KPE_VM_ONLY
// ---------------------------------------------------------------------------
constexpr uint32_t kPredStrLds = 16384;  // staged dictionary bytes per block
constexpr uint32_t kPredPatLds = 4096;   // staged pattern bytes
constexpr uint32_t kPredPats = 64;       // staged pattern records per job

// Grid (x, y): job y (one predicate over one domain), strings [256 x, 256 x + 256).
// Every input of the block's compares is staged in LDS in one round (the job's
// pattern records and bytes, the block's strings), so no compare waits on HBM/L2.
__global__ void __launch_bounds__(256) kpe_pred_kernel(PredArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t s_str[kPredStrLds];
  __shared__ __attribute__((aligned(16))) uint8_t s_pat[kPredPatLds];
  __shared__ KpePat s_pats[kPredPats];
  const uint32_t t = threadIdx.x;
  const PredJob job = sld(a.jobs, blockIdx.y);
  const uint32_t n = a.dict_n[job.domain];
  const uint32_t id0 = blockIdx.x * 256u;
  if (id0 >= n) return;  // uniform: this job has fewer blocks than the grid's x extent
  const uint32_t* off = a.dict_off[job.domain];
  const uint8_t* bytes = a.dict_bytes[job.domain];
  const uint32_t idh = min(id0 + 256u, n);
  const uint32_t lo = off[id0], hi = off[idh];
  const uint32_t id = id0 + t;
  const uint32_t o0 = id < n ? off[id] : 0u, o1 = id < n ? off[id + 1] : 0u;
  const bool str_lds = hi - lo <= kPredStrLds;
  const bool pat_lds = a.pat_len <= kPredPatLds && job.npat <= kPredPats;
  if (str_lds)
    for (uint32_t i = t; i < hi - lo; i += 256) s_str[i] = bytes[lo + i];
  if (pat_lds) {
    for (uint32_t i = t; i < a.pat_len; i += 256) s_pat[i] = a.pat_bytes[i];
    if (t < job.npat) s_pats[t] = a.pats[job.pat0 + t];
  }
  __syncthreads();
  bool hit = false;
  if (id < n) {
    const uint8_t* s = str_lds ? s_str + (o0 - lo) : bytes + o0;
    const int sn = (int)(o1 - o0);
    if (pat_lds) {
      for (uint32_t k = 0; k < job.npat && !hit; ++k) hit = pat_match(s_pats[k], s_pat, s, sn);
    } else {
      for (uint32_t k = 0; k < job.npat && !hit; ++k) hit = pat_match(a.pats[job.pat0 + k], a.pat_bytes, s, sn);
    }
  }
  const uint64_t m = __ballot(hit);
  const uint32_t wid = id >> 6;  // 64 strings per wave => two output words
  if ((t & 63u) == 0 && (uint64_t)wid * 64u < n) {
    a.out[job.out_word + 2 * wid] = (uint32_t)m;
    a.out[job.out_word + 2 * wid + 1] = (uint32_t)(m >> 32);
  }
}

// Per-rule status histogram of a row-major N x R verdict matrix (8 slots per rule: the
// kpe_verdict codes). Each wave takes 64 rows at a time; per rule, one ballot per status,
// lane 0 accumulates in LDS; one 64-bit global add per (rule, status) and block at the end.
__global__ void __launch_bounds__(256) kpe_count_kernel(const uint8_t* v, int64_t n, uint32_t R, uint32_t r0,
                                                        uint32_t rn, unsigned long long* out) {
  extern __shared__ uint32_t hist[];  // rules [r0, r0 + rn) x 8
  const uint32_t t = threadIdx.x, lane = t & 63u;
  for (uint32_t i = t; i < rn * 8; i += 256) hist[i] = 0;
  __syncthreads();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + (t >> 6); tile * 64 < n; tile += nw) {
    const int64_t row = tile * 64 + lane;
    const bool live = row < n;
    for (uint32_t r = 0; r < rn; ++r) {
      const uint32_t c = live ? v[row * R + r0 + r] : 0u;
#pragma unroll
      for (uint32_t s = 1; s < 8; ++s) {
        const uint32_t k = (uint32_t)__popcll(__ballot(c == s));
        if (lane == 0 && k) atomicAdd(&hist[r * 8 + s], k);
      }
    }
  }
  __syncthreads();
  for (uint32_t i = t; i < rn * 8; i += 256)
    if (hist[i]) atomicAdd(&out[(size_t)r0 * 8 + i], (unsigned long long)hist[i]);
}

#endif  // !KPE_VM_ONLY

// ---------------------------------------------------------------------------
namespace {

constexpr uint32_t kBlock = 256;
// Minimum waves per SIMD the scan kernel is compiled for (register budget).
#ifndef KPE_SCAN_WAVES
#define KPE_SCAN_WAVES 6  // C4 wide scan, round 4 (profiles/r04_f): 5 / 6 / 7 waves per SIMD 0.567 / 0.553 / 0.643 ms (7: 65 VGPRs spilled)
#endif
constexpr uint32_t kAllowedVolumes = PSS_ALLOWED_VOLUMES;


// Capability-set violation bits (computed per block into LDS from the capset dictionary)
#define CS_BASE 1u  // add has a capability outside the baseline allow-list
#define CS_DROP 2u  // drop lacks "ALL" (also: no capabilities at all)
#define CS_ADD 4u   // add has anything but NET_BIND_SERVICE

// PSA versioned checks for one pod (PSA v0.29 policy/check_*.go, restated in
// oracle/pss.hpp) from the pod word and the OR of its containers' state bitmaps.
// "Containers" = initContainers + containers + ephemeralContainers.
__device__ __forceinline__ uint32_t cv_fails(uint32_t pw, uint32_t xo, uint32_t co, bool sec_ann_bad,
                                             bool vol_hostpath, bool vol_restricted, uint32_t sys_bad,
                                             bool apparmor_bad, bool sec_pod_ann_bad) {
  // Branch-free: every condition is a 0/1 value combined with & and | (no short circuit), so the
  // whole function is selects and shifts on the lane.
  auto on = [](uint32_t c, uint32_t cv) -> uint32_t { return (c ? 1u : 0u) << cv; };
  const uint32_t nwin = FIELD(pw, P_OS_SH, 2) == OS_WINDOWS ? 0u : ~0u;
  uint32_t f = 0;
  // allowPrivilegeEscalation: some container whose APE is unset (or SC nil) or true
  f |= (xo & (CX_APE_T | CX_APE_U)) ? (1u << CV_APE_1_8) | ((1u << CV_APE_1_25) & nwin) : 0u;
  f |= on(apparmor_bad, CV_APPARMOR_1_0);
  f |= on(co & CS_BASE, CV_CAPS_BASELINE_1_0);
  f |= (co & (CS_DROP | CS_ADD)) ? (1u << CV_CAPS_RESTRICTED_1_22) | ((1u << CV_CAPS_RESTRICTED_1_25) & nwin) : 0u;
  f |= on(pw & (P_HOSTNET | P_HOSTPID | P_HOSTIPC), CV_HOST_NS_1_0);
  f |= on(vol_hostpath, CV_HOST_PATH_1_0);
  f |= on(xo & CX_HOSTPORT, CV_HOST_PORTS_1_0);
  f |= on(xo & CX_PRIV_T, CV_PRIVILEGED_1_0);
  f |= on(xo & CX_PM_OTHER, CV_PROC_MOUNT_1_0);
  f |= on(vol_restricted, CV_RESTRICTED_VOLUMES_1_0);
  const uint32_t prnr = FIELD(pw, P_RNR_SH, 2);
  f |= on((uint32_t)(prnr == TRI_FALSE) | (uint32_t)((xo & CX_RNR_F) != 0u) |
              ((uint32_t)(prnr != TRI_TRUE) & (uint32_t)((xo & CX_RNR_U) != 0u)),
          CV_RUN_AS_NON_ROOT_1_0);
  f |= on((uint32_t)(FIELD(pw, P_RAU_SH, 2) == RAU_ZERO) | (uint32_t)((xo & CX_RAU_Z) != 0u), CV_RUN_AS_USER_1_23);
  const uint32_t psel = FIELD(pw, P_SEL_SH, 3);
  f |= on(((uint32_t)(psel != SEL_NONE) &
           ((uint32_t)(psel == SEL_OTHER) | (uint32_t)((pw & (P_SEL_USER | P_SEL_ROLE)) != 0u))) |
              (uint32_t)((xo & (CX_SEL_OTHER | CX_SEL_USER | CX_SEL_ROLE)) != 0u),
          CV_SELINUX_1_0);
  f |= on((uint32_t)sec_pod_ann_bad | (uint32_t)sec_ann_bad, CV_SECCOMP_BASELINE_1_0);
  // pod seccomp type: valid = RuntimeDefault | Localhost, bad = set and not valid
  const uint32_t psec = FIELD(pw, P_SECCOMP_SH, 3);
  constexpr uint32_t kSecValid = (1u << SECCOMP_RUNTIMEDEFAULT) | (1u << SECCOMP_LOCALHOST);
  constexpr uint32_t kSecBad = 0xFFu & ~kSecValid & ~(1u << SECCOMP_NONE);
  const uint32_t psec_valid = (kSecValid >> psec) & 1u, psec_bad = (kSecBad >> psec) & 1u;
  const uint32_t sec_b = psec_bad | (uint32_t)((xo & (CX_SEC_UNC | CX_SEC_OTHER)) != 0u);
  f |= on(sec_b, CV_SECCOMP_BASELINE_1_19);
  f |= (sec_b | ((psec_valid ^ 1u) & (uint32_t)((xo & CX_SEC_NONE) != 0u)))
           ? (1u << CV_SECCOMP_RESTRICTED_1_19) | ((1u << CV_SECCOMP_RESTRICTED_1_25) & nwin)
           : 0u;
  f |= on(sys_bad & 1u, CV_SYSCTLS_1_0) | on(sys_bad & 2u, CV_SYSCTLS_1_27) | on(sys_bad & 4u, CV_SYSCTLS_1_29);
  f |= on((uint32_t)(FIELD(pw, P_WHP_SH, 2) == TRI_TRUE) | (uint32_t)((xo & CX_WHP_T) != 0u), CV_WIN_HOST_PROCESS_1_0);
  return f;
}

// Inclusive wave64 prefix sum: 4 row_shr steps inside each 16-lane row, then
// row_bcast:15 / row_bcast:31 across rows (6 DPP adds, no LDS).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);
  return x;
}

// The scan's arguments live in device memory (one copy per program x corpus
// binding) and are read through the constant address space with scalar loads. The
// pointer is laundered once per tile so the loads are re-issued near their uses
// instead of being hoisted out of the tile loop (hoisted, ~60 fields exceed the
// SGPR file and spill to VGPR lanes).
typedef const __attribute__((address_space(4))) ScanArgs CArgs;
__device__ __forceinline__ CArgs* launder(const ScanArgs* p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+s"(v));
  return (CArgs*)v;
}

// Bitset word of a resolved predicate location (PRED_LOCAL | LDS index, or pbuf index).
typedef __attribute__((address_space(3))) const uint32_t* LdsPtr;
typedef __attribute__((address_space(1))) const uint32_t* GblPtr;
// Large-domain bitset words (HBM/L2): out of line, so the wait for this load sits in
// the callee and never at the join with the LDS path (where it would also wait for
// the next tile's prefetch on every call).
__device__ __noinline__ uint32_t gbl_word(GblPtr p, uint32_t i) { return p[i]; }
struct Bits {
  LdsPtr lds;
  GblPtr pbuf;
  __device__ Bits(const uint32_t* l, const uint32_t* g) : lds((LdsPtr)l), pbuf((GblPtr)g) {}
  // `loc` is wave-uniform: the branch is uniform and the reads are typed LDS / global
  // pointers, so they stay distinct instructions (a pointer select would become a flat
  // load whose wait also covers every global load in flight: the next tile's prefetch).
  __device__ __forceinline__ uint32_t word(uint32_t loc, uint32_t wi) const {
    if (loc & PRED_LOCAL) return lds[(loc & ~PRED_LOCAL) + wi];
    return gbl_word(pbuf, loc + wi);
  }
  __device__ __forceinline__ bool bit(uint32_t loc, uint32_t id) const {
    if (id == KPE_NO_STR) return false;
    return (word(loc, id >> 5) >> (id & 31u)) & 1u;
  }
  __device__ __forceinline__ uint64_t mask64(uint32_t loc) const {  // predicate over D_CAP (<= 64 ids)
    return loc == PRED_NONE ? 0ull : ((uint64_t)word(loc, 0) | ((uint64_t)word(loc, 1) << 32));
  }
};

// Data of one 64-resource tile, loaded one tile ahead of its evaluation. PSS programs
// read the pod record per lane and the tile's list items COOPERATIVELY: the tile's
// containers are crec[C0, C1) with C0/C1 from its header and the next one, so lane i
// loads items C0 + i and C0 + 64 + i (coalesced) in the same round as the pod records.
// Items past the preloaded slots (rare: > 128 containers or > 64 other items per tile)
// are loaded when the tile is evaluated.
template <bool PSS>
struct Tile;
template <>
struct Tile<true> {
  uint32_t C0, V0, S0, A0, nct, nvt, nst, nat;  // the tile's list ranges (wave-uniform)
  uint4 rec;
  uint2 c0, c1;   // containers C0 + lane, C0 + 64 + lane
  uint32_t v0, v1, s0;  // volumes V0 + lane, V0 + 64 + lane; sysctl S0 + lane
  uint2 q0;       // pod annotation A0 + lane
  uint32_t sa0, sa1;  // container seccomp annotations (NEED_SANN)
  uint32_t name, mns;
};
template <>
struct Tile<false> {
  uint32_t gvk, nsa, name, mns;
  uint32_t lo, hi;  // the resource's label bounds (lab_off), one step ahead of the label loads
  uint32_t nsl;     // its namespace's row in the namespace-label table (r_nsl)
};

// Tile header words: lane k (< 8) holds word k of hdr[tile], hdr[tile + 1]
// (C0 V0 S0 A0 C1 V1 S1 A1); read back with v_readlane into scalars.
__device__ __forceinline__ uint32_t load_hdr(CArgs& a, uint32_t tile, uint32_t lane) {
  return a.hdr[tile * 4 + (lane & 7u)];
}
__device__ __forceinline__ uint32_t hw(uint32_t h, uint32_t k) { return __builtin_amdgcn_readlane(h, k); }

template <bool PSS, bool LEAN = false, bool PSUM = false>
__device__ __forceinline__ Tile<PSS> load_tile(CArgs& a, uint32_t tile, uint32_t h, uint32_t lane);

// Pin a tile's registers here: code that uses them cannot be hoisted above this point
// (the compiler would otherwise move ALU work on a tile's loaded values above the next
// tile's load issue, or into the block prologue, and wait for the loads there).
__device__ __forceinline__ void pin(uint32_t& x) { asm volatile("" : "+v"(x)::"memory"); }
__device__ __forceinline__ void pin(uint2& x) { pin(x.x), pin(x.y); }
__device__ __forceinline__ void pin(uint4& x) { pin(x.x), pin(x.y), pin(x.z), pin(x.w); }
__device__ __forceinline__ void pin_tile(Tile<true>& d) {
  pin(d.rec), pin(d.c0), pin(d.c1), pin(d.v0), pin(d.v1), pin(d.s0), pin(d.q0), pin(d.sa0), pin(d.sa1), pin(d.name),
      pin(d.mns);
}
__device__ __forceinline__ void pin_tile(Tile<false>& d) {
  pin(d.gvk), pin(d.nsa), pin(d.name), pin(d.mns), pin(d.lo), pin(d.hi), pin(d.nsl);
}

// Every load of a tile is issued on every path (an unneeded column is read from the
// binding's zero page instead: one broadcast cache line), so the number of loads a
// prefetch puts in flight is static and the compiler can wait for an older tile with
// a counted vmcnt instead of draining the prefetch with vmcnt(0).
template <class T>
__device__ __forceinline__ const T* col(bool on, const void* p, const uint32_t* zero) {
  return reinterpret_cast<const T*>(on ? p : (const void*)zero);
}
// PSS tile. LEAN (no container seccomp annotations, names or match namespaces read): only
// the pod records and the list slots are loaded.
template <bool LEAN, bool PSUM>
__device__ __forceinline__ Tile<true> load_pss_tile(CArgs& a, uint32_t tile, uint32_t h, uint32_t lane) {
  Tile<true> d;
  const uint32_t n = (uint32_t)a.n, need = a.need;
  const uint32_t r = tile * 64 + lane;
  const uint32_t rc = r < n ? r : n - 1;  // clamped: loads are unconditional
  const uint32_t* zp = a.zero_page;
  d.C0 = hw(h, 0), d.V0 = hw(h, 1), d.S0 = hw(h, 2), d.A0 = hw(h, 3);
  d.nct = hw(h, 4) - d.C0, d.nvt = hw(h, 5) - d.V0, d.nst = hw(h, 6) - d.S0, d.nat = hw(h, 7) - d.A0;
  // item index clamped into the tile's range [b0, b0 + cnt) and the column (index 0 of
  // an empty column / of the zero page reads in-bounds garbage that is never used)
  auto at = [&](uint32_t b0, uint32_t cnt, uint32_t k, uint32_t total) {
    const uint32_t i = b0 + min(k, cnt ? cnt - 1 : 0u);
    return total ? min(i, total - 1) : 0u;
  };
  // PSUM: the corpus's scan records (ScanArgs::psum: each pod's failing versioned checks, built by
  // the summary pass) replace the lists: sa0 carries the pod's checks, nothing else is loaded
  if constexpr (PSUM) {
    d.C0 = d.V0 = d.S0 = d.A0 = d.nct = d.nvt = d.nst = d.nat = 0;
    d.rec = reinterpret_cast<const uint4*>(a.rec)[rc];
    d.sa0 = a.psum[3u * rc + 1u];
    d.c0 = d.c1 = make_uint2(0u, 0u), d.v0 = d.v1 = d.s0 = d.sa1 = 0u, d.q0 = make_uint2(0u, 0u);
    const bool on_n = need & NEED_NAME, on_m = need & NEED_MNS;
    d.name = col<uint32_t>(on_n, a.r_name, zp)[on_n ? rc : 0u];
    d.mns = col<uint32_t>(on_m, a.r_mns, zp)[on_m ? rc : 0u];
#if KPE_PSUM_LABPRE
    // the list slots the records replace carry the label bounds and the namespace row one step
    // ahead of the label loads (lab_cache)
    const bool on_l = need & NEED_LAB, on_s = need & NEED_NSL;
    const uint32_t* lo = col<uint32_t>(on_l, a.lab_off, zp) + (on_l ? rc : 0u);
    d.v0 = lo[0], d.v1 = lo[on_l ? 1u : 0u];
    d.s0 = col<uint32_t>(on_s, a.r_nsl, zp)[on_s ? rc : 0u];
#endif
    return d;
  }
  const bool on_c = a.nctr_total, on_sa = on_c && (need & NEED_SANN);
  const bool on_v = (need & NEED_VOL) && a.nvol_total, on_s = (need & NEED_SYS) && a.nsys_total;
  const bool on_q = (need & NEED_PANN) && a.npann_total;
  const uint32_t i0 = on_c ? at(d.C0, d.nct, lane, a.nctr_total) : 0u;
  const uint32_t i1 = on_c ? at(d.C0, d.nct, lane + 64, a.nctr_total) : 0u;
  d.rec = reinterpret_cast<const uint4*>(a.rec)[rc];
  d.c0 = col<uint2>(on_c, a.crec, zp)[i0];
  d.c1 = col<uint2>(on_c, a.crec, zp)[i1];
  if constexpr (!LEAN) {
    d.sa0 = col<uint32_t>(on_sa, a.c_sann, zp)[on_sa ? i0 : 0u];
    d.sa1 = col<uint32_t>(on_sa, a.c_sann, zp)[on_sa ? i1 : 0u];
  } else {
    d.sa0 = d.sa1 = KPE_NO_STR;
  }
  d.v0 = col<uint32_t>(on_v, a.vol_src, zp)[on_v ? at(d.V0, d.nvt, lane, a.nvol_total) : 0u];
  d.v1 = col<uint32_t>(on_v, a.vol_src, zp)[on_v ? at(d.V0, d.nvt, lane + 64, a.nvol_total) : 0u];
  d.s0 = col<uint32_t>(on_s, a.sys_id, zp)[on_s ? at(d.S0, d.nst, lane, a.nsys_total) : 0u];
  d.q0 = col<uint2>(on_q, a.pann_kv, zp)[on_q ? at(d.A0, d.nat, lane, a.npann_total) : 0u];
  if constexpr (!LEAN) {
    const bool on_n = need & NEED_NAME, on_m = need & NEED_MNS;
    d.name = col<uint32_t>(on_n, a.r_name, zp)[on_n ? rc : 0u];
    d.mns = col<uint32_t>(on_m, a.r_mns, zp)[on_m ? rc : 0u];
  } else {
    d.name = d.mns = KPE_NO_STR;
  }
  // no fix-ups of loaded values here (a select on a loaded register waits for the load):
  // columns that are off are masked where they are used (tile_cols, pss_tile's `nsann`)
  return d;
}

__device__ __forceinline__ Tile<false> load_match_tile(CArgs& a, uint32_t tile, uint32_t lane) {
  Tile<false> d;
  const uint32_t n = (uint32_t)a.n, need = a.need;
  const uint32_t r = tile * 64 + lane;
  const uint32_t rc = r < n ? r : n - 1;
  const uint32_t* zp = a.zero_page;
  const bool on_g = need & NEED_GVK, on_a = need & NEED_NSA, on_n = need & NEED_NAME, on_m = need & NEED_MNS;
  d.gvk = col<uint32_t>(on_g, a.r_gvk, zp)[on_g ? rc : 0u];
  d.nsa = col<uint32_t>(on_a, a.r_nsa, zp)[on_a ? rc : 0u];
  d.name = col<uint32_t>(on_n, a.r_name, zp)[on_n ? rc : 0u];
  d.mns = col<uint32_t>(on_m, a.r_mns, zp)[on_m ? rc : 0u];
  const bool on_l = need & NEED_LAB;
  const uint32_t* lo = col<uint32_t>(on_l, a.lab_off, zp) + (on_l ? rc : 0u);
  d.lo = lo[0];
  d.hi = lo[on_l ? 1u : 0u];
  const bool on_s = need & NEED_NSL;
  d.nsl = col<uint32_t>(on_s, a.r_nsl, zp)[on_s ? rc : 0u];
  return d;
}

template <bool PSS, bool LEAN, bool PSUM>
__device__ __forceinline__ Tile<PSS> load_tile(CArgs& a, uint32_t tile, uint32_t h, uint32_t lane) {
  if constexpr (PSS) return load_pss_tile<LEAN, PSUM>(a, tile, h, lane);
  else return load_match_tile(a, tile, lane);
}

// PSS part of one tile: the lane's failing versioned checks (0 for dead lanes).
// Segmented OR of the tile's list items into their pods: every list item is turned
// into its violation code by an "item lane" (item j on lane j % 64, from the tile's
// preloaded slots) and staged in the wave's LDS area; after one wave barrier each pod
// lane ORs the codes of its own items [o, o + cnt). The common path issues no memory
// operation at all (the next tile's loads stay in flight); items past the staged
// chunk (> 128 containers or > 64 other items per tile) take a rare direct-load path.
// Fixed PSA predicate locations of a LEAN scan, read once per kernel (all LDS-resident).
struct LeanPP {
  uint32_t sann_ok, aa_key, aa_ok, sp_key, sys0, sys1, sys2;
};
template <bool LEAN, bool PSUM>
__device__ __forceinline__ uint32_t pss_tile(CArgs& a, const Bits& B, const uint8_t* s_capb, const Tile<true>& d,
                                             bool live, uint32_t* stage, uint32_t lane, const LeanPP& lp) {
  if constexpr (PSUM) return live ? d.sa0 & a.cv_union : 0u;  // the scan record's checks (load_pss_tile)
  const uint32_t need = a.need;
  // LEAN: every predicate here is LDS-resident (checked by the host) and every id a real
  // dictionary id (sysctl names, annotation keys / values): a branch-free bit read
  auto pbit = [&](uint32_t loc, uint32_t id) -> uint32_t {
    if constexpr (LEAN) {
      return (B.lds[(loc & ~PRED_LOCAL) + (id >> 5)] >> (id & 31u)) & 1u;
    } else {
      return B.bit(loc, id) ? 1u : 0u;
    }
  };
  const uint32_t p_sann = LEAN ? lp.sann_ok : a.pp_seccomp_ann_ok, p_s0 = LEAN ? lp.sys0 : a.pp_sysctl0,
                 p_s1 = LEAN ? lp.sys1 : a.pp_sysctl1, p_s2 = LEAN ? lp.sys2 : a.pp_sysctl2,
                 p_aak = LEAN ? lp.aa_key : a.pp_apparmor_key, p_aao = LEAN ? lp.aa_ok : a.pp_apparmor_ok,
                 p_spk = LEAN ? lp.sp_key : a.pp_seccomp_pod_key;
  const uint32_t C0 = d.C0, V0 = d.V0, S0 = d.S0, A0 = d.A0;
  const uint32_t nct = d.nct, nvt = d.nvt, nst = d.nst, nat = d.nat;
  const bool nsann = !LEAN && (need & NEED_SANN);
  const bool nvol = (need & NEED_VOL) && nvt, nsys = (need & NEED_SYS) && nst, npann = (need & NEED_PANN) && nat;
  // ---- the pod's own item offsets: exclusive wave scans of its packed counts ----
  const uint32_t z = live ? d.rec.z : 0u;
  const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
  const uint32_t c01 = nc | (nv << 16);
  const uint32_t e01 = wave_incl_scan(c01) - c01;
  uint32_t e23 = 0;
  if (nsys || npann) {
    const uint32_t c23 = ns | (na << 16);
    e23 = wave_incl_scan(c23) - c23;
  }
  const uint32_t oc = e01 & 0xFFFFu, ov = e01 >> 16, os = e23 & 0xFFFFu, oa = e23 >> 16;
  uint2* sc = reinterpret_cast<uint2*>(stage);
  uint8_t* sbv = reinterpret_cast<uint8_t*>(stage + KPE_STAGE_CTR * 2);
  uint8_t* sbs = sbv + KPE_STAGE_VOL;
  uint8_t* sba = sbs + KPE_STAGE_SMALL;
  // item codes
  auto ctr_code = [&](uint2 e, uint32_t sa) -> uint2 {  // (state bitmap, capset bits | seccomp-annotation bit)
    uint32_t ex = s_capb[CY_CAPSET(e.y)];
    if (nsann && sa != KPE_NO_STR && !pbit(p_sann, sa)) ex |= 8u;
    return make_uint2(e.x, ex);
  };
  auto vol_code = [&](uint32_t sv) -> uint32_t {  // bit 0 hostPath, bit 1 outside the restricted allow-list
    return ((sv >> VS_HOSTPATH) & 1u) | ((sv & kAllowedVolumes) ? 0u : 2u);
  };
  auto sys_code = [&](uint32_t id) -> uint32_t {  // bit k: outside the 1.0 / 1.27 / 1.29 allow-list
    return (pbit(p_s0, id) ^ 1u) | ((pbit(p_s1, id) ^ 1u) << 1) | ((pbit(p_s2, id) ^ 1u) << 2);
  };
  auto ann_code = [&](uint2 kv) -> uint32_t {  // bit 0 AppArmor profile, bit 1 seccomp pod annotation
    return (pbit(p_aak, kv.x) & (pbit(p_aao, kv.y) ^ 1u)) | ((pbit(p_spk, kv.x) & (pbit(p_sann, kv.y) ^ 1u)) << 1);
  };
  // ---- stage the first chunk of every list from the preloaded slots ----
  if (lane < nct) sc[lane] = ctr_code(d.c0, d.sa0);
  if (lane + 64 < nct) sc[lane + 64] = ctr_code(d.c1, d.sa1);
  if (nvol && lane < nvt) sbv[lane] = (uint8_t)vol_code(d.v0);
  if (nvol && lane + 64 < nvt) sbv[lane + 64] = (uint8_t)vol_code(d.v1);
  if (nsys && lane < nst) sbs[lane] = (uint8_t)sys_code(d.s0);
  if (npann && lane < nat) sba[lane] = (uint8_t)ann_code(d.q0);
  __builtin_amdgcn_wave_barrier();
  // Each pod ORs its own staged items, four independent LDS reads per round (indices
  // clamped to the pod's last item: a repeated item does not change an OR), so a pod
  // with <= 4 items of a list pays one LDS round trip for it, not one per item.
  uint32_t xo = 0, co = 0, vcode = 0, scode = 0, acode = 0;
  {
    const uint32_t hi = min(oc + nc, (uint32_t)KPE_STAGE_CTR);
#pragma unroll 1
    for (uint32_t k = oc; k < hi; k += 4) {
      const uint2 e0 = sc[k], e1 = sc[min(k + 1, hi - 1)], e2 = sc[min(k + 2, hi - 1)], e3 = sc[min(k + 3, hi - 1)];
      xo |= e0.x | e1.x | e2.x | e3.x;
      co |= e0.y | e1.y | e2.y | e3.y;
    }
  }
  auto or_bytes = [](const uint8_t* b, uint32_t o, uint32_t cnt, uint32_t cap) -> uint32_t {
    const uint32_t hi = min(o + cnt, cap);
    uint32_t x = 0;
#pragma unroll 1
    for (uint32_t k = o; k < hi; k += 4)
      x |= (uint32_t)b[k] | b[min(k + 1, hi - 1)] | b[min(k + 2, hi - 1)] | b[min(k + 3, hi - 1)];
    return x;
  };
  if (nvol) vcode = or_bytes(sbv, ov, nv, KPE_STAGE_VOL);
  if (nsys) scode = or_bytes(sbs, os, ns, KPE_STAGE_SMALL);
  if (npann) acode = or_bytes(sba, oa, na, KPE_STAGE_SMALL);
  __builtin_amdgcn_wave_barrier();
  // ---- rare: items beyond the staged chunk, loaded directly by their pod lane ----
  if (nct > KPE_STAGE_CTR || (nvol && nvt > KPE_STAGE_VOL) || (nsys && nst > KPE_STAGE_SMALL) ||
      (npann && nat > KPE_STAGE_SMALL)) {
    const uint2* crec = reinterpret_cast<const uint2*>(a.crec);
    for (uint32_t k = max(oc, (uint32_t)KPE_STAGE_CTR); k < oc + nc; ++k) {
      const uint2 e = ctr_code(crec[C0 + k], nsann ? a.c_sann[C0 + k] : KPE_NO_STR);
      xo |= e.x;
      co |= e.y;
    }
    if (nvol)
      for (uint32_t k = max(ov, (uint32_t)KPE_STAGE_VOL); k < ov + nv; ++k) vcode |= vol_code(a.vol_src[V0 + k]);
    if (nsys)
      for (uint32_t k = max(os, (uint32_t)KPE_STAGE_SMALL); k < os + ns; ++k) scode |= sys_code(a.sys_id[S0 + k]);
    if (npann)
      for (uint32_t k = max(oa, (uint32_t)KPE_STAGE_SMALL); k < oa + na; ++k)
        acode |= ann_code(reinterpret_cast<const uint2*>(a.pann_kv)[A0 + k]);
  }
  if (!live) return 0u;
  return cv_fails(d.rec.x, xo, co & 7u, co & 8u, vcode & 1u, vcode & 2u, scode, acode & 1u, acode & 2u) & a.cv_union;
}

// Label bounds of the lane's resource and of its namespace row, and the selector requirement
// masks (ScanArgs::selm) once per tile: every selector term is then one mask test. Without masks
// (more than 64 requirements in a space) a term walks the labels per requirement.
constexpr uint32_t kLabCache = 8;
typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));  // a dword-aligned 16-byte load
struct LabCache {
  uint32_t lo, hi;    // the resource's labels
  uint32_t nlo, nhi;  // its namespace's labels (namespaceSelector), read from memory
  uint64_t selq, nsq;  // ScanArgs::selm: requirements that hold on its labels / its namespace's
  uint64_t kmask;      // T_KSLOT: the kind terms that hold for its GVK
};
// The row's kind-term mask: binary search of its GVK in the block's LDS table (ScanArgs::kslot_lds)
__device__ __forceinline__ uint64_t kslot_mask(const CArgs& a, const uint32_t* dyn, uint32_t gvk) {
  const LdsPtr g = (LdsPtr)(dyn + a.kslot_lds);
  uint32_t lo = 0, n = a.nkslot_g;
  while (n > 1u) {  // uniform trip count
    const uint32_t h = n >> 1;
    lo = g[lo + h] <= gvk ? lo + h : lo;
    n -= h;
  }
  if (g[lo] != gvk) return 0ull;
  const uint32_t m = (a.nkslot_g + 1u) & ~1u;
  return (uint64_t)g[m + 2u * lo] | (uint64_t)g[m + 2u * lo + 1u] << 32;
}

// the resource's label cache (label selectors; a namespace's labels are shared by its
// resources and stay cache-resident, so namespaceSelector terms read them from memory)
// Label-selector requirement mask of one resource (ScanArgs::selm bit 0): its labels folded in
// order. Requirement q is decided by the first label whose key matches it (and whose value
// matches too, for a wildcard matchLabels entry), as the per-requirement loop of eval_term.
__device__ __forceinline__ uint64_t sel_fold(CArgs& a, const LabCache& LC, const uint32_t* dyn) {
  uint64_t notyet = ~0ull, okacc = 0;
  const uint64_t nwild = ~a.sm_wild;
  // the requirement tables from LDS when the block staged them (ScanArgs::selt_lds), else L2;
  // the branch is uniform and each side's loads are typed, so no flat load's wait covers the
  // prefetch of the next tile
  const bool in_lds = a.selt_lds != PRED_NONE;
  const LdsPtr lt = (LdsPtr)(dyn + (in_lds ? a.selt_lds : 0u));
  auto fold = [&](uint32_t k, uint32_t v) {
    uint4 kq = make_uint4(0u, 0u, 0u, 0u), vq = make_uint4(0u, 0u, 0u, 0u);
    if (in_lds) {
      const uint32_t vi = 4u * (a.nlabk + v);
      if (k < a.nlabk) kq = make_uint4(lt[4u * k], lt[4u * k + 1u], lt[4u * k + 2u], lt[4u * k + 3u]);
      if (v < a.nlabv) vq = make_uint4(lt[vi], lt[vi + 1u], lt[vi + 2u], lt[vi + 3u]);
    } else {
      if (k < a.nlabk) kq = a.sel_km[k];
      if (v < a.nlabv) vq = a.sel_vm[v];
    }
    const uint64_t km = kq.x | (uint64_t)kq.y << 32, kok = kq.z | (uint64_t)kq.w << 32;
    const uint64_t vm = vq.x | (uint64_t)vq.y << 32, vok = vq.z | (uint64_t)vq.w << 32;
    const uint64_t f = km & (nwild | vm);  // this label is the requirement's first match
    const uint64_t val = (vm & a.sm_pos) | (kok & vok & a.sm_wild) | (~vm & a.sm_notin);
    okacc |= f & notyet & val;
    notyet &= ~f;
  };
  uint32_t k[kLabCache], v[kLabCache];  // the first labels with independent loads
#if KPE_DIAG & 16  // diagnostic build: the fold without the label loads
#pragma unroll
  for (uint32_t j = 0; j < kLabCache; ++j) k[j] = (LC.lo + j) % 37u, v[j] = (LC.hi ^ j) % 11u;
#else
  // dword-aligned 16-byte loads: the label arrays carry 128 bytes of slack past their end
  // (upload_staged), and words past the resource's labels are never folded
#pragma unroll
  for (uint32_t j = 0; j < kLabCache; j += 4u) {
    const u32x4a kk = *reinterpret_cast<const u32x4a*>(a.lab_k + LC.lo + j);
    const u32x4a vv = *reinterpret_cast<const u32x4a*>(a.lab_v + LC.lo + j);
    k[j] = kk.x, k[j + 1] = kk.y, k[j + 2] = kk.z, k[j + 3] = kk.w;
    v[j] = vv.x, v[j + 1] = vv.y, v[j + 2] = vv.z, v[j + 3] = vv.w;
  }
#endif
#if KPE_DIAG & 8  // diagnostic build: the label loads without the fold
  uint64_t acc = 0;
#pragma unroll
  for (uint32_t j = 0; j < kLabCache; ++j) acc ^= (uint64_t)k[j] << (j & 31u) ^ v[j];
#pragma unroll 1
  for (uint32_t j = LC.lo + kLabCache; j < LC.hi; ++j) acc ^= (uint64_t)a.lab_k[j] << 3 ^ a.lab_v[j];
  return acc;
#endif
#pragma unroll
  for (uint32_t j = 0; j < kLabCache; ++j)
    if (LC.lo + j < LC.hi) fold(k[j], v[j]);
#pragma unroll 1
  for (uint32_t j = LC.lo + kLabCache; j < LC.hi; ++j) fold(KPE_DIAG & 16 ? j % 37u : a.lab_k[j], KPE_DIAG & 16 ? j % 11u : a.lab_v[j]);
  const uint64_t found = ~notyet;
  return (found & okacc & (a.sm_pos | a.sm_wild)) | ((notyet | okacc) & a.sm_notin) | (found & a.sm_exists) |
         (notyet & a.sm_dne);
}

// lo / hi / nsl: the resource's lab_off bounds and r_nsl row when the tile prefetched them
// (Tile<false>, or PSUM tiles' list slots), else kNotFetched
constexpr uint32_t kNotFetched = 0xFFFFFFFEu;  // r_nsl rows and label offsets stay below it
__device__ __forceinline__ void lab_cache(CArgs& a, uint32_t rc, bool live, LabCache& LC, const uint32_t* dyn,
                                          uint32_t lo = kNotFetched, uint32_t hi = 0u, uint32_t nsl = kNotFetched) {
  if (lo == kNotFetched) {
    lo = hi = 0;
    if (a.need & NEED_LAB) lo = a.lab_off[rc], hi = a.lab_off[rc + 1];
  }
  LC.lo = lo, LC.hi = live ? hi : lo;
  LC.nlo = LC.nhi = 0;
  LC.selq = LC.nsq = 0;
  LC.kmask = 0;
  if (a.need & NEED_NSL) {  // the namespace row's bounds, once per resource instead of per term
    const uint32_t row = nsl != kNotFetched ? nsl : a.r_nsl[rc];
    if (live && row != KPE_NO_STR) LC.nlo = a.nsl_off[row], LC.nhi = a.nsl_off[row + 1];
    if (a.selm & 2u) LC.nsq = a.ns_q[live && row != KPE_NO_STR ? row : a.ns_none];
  }
#if KPE_DIAG & 4  // diagnostic build: no label fold
  LC.selq = LC.lo ^ LC.hi;
#else
  if (a.selm & 1u) LC.selq = sel_fold(a, LC, dyn);
#endif
}

// One match term for this lane's resource (utils/match.go:52-160 attributes).
__device__ __forceinline__ bool eval_term(CArgs& a, const Bits& B, const KpeTerm& tm, uint32_t gvk,
                                          uint32_t nsa, uint32_t name_col, uint32_t mns_col, uint32_t rc,
                                          bool live, const LabCache& LC) {
  bool ok = true;
  if (tm.type == T_KSLOT) {
    ok = (LC.kmask >> tm.a) & 1ull;
  } else if (tm.type == T_SELQ || tm.type == T_NSSELQ) {  // requirement-mask selectors (binding form)
    const uint32_t q = tm.a & 0xFFu, nq = (tm.a >> 8) & 0xFFu, f = tm.a >> 16;
    const uint64_t need = (nq >= 64u ? ~0ull : ((1ull << nq) - 1ull)) << q;
    if (tm.type == T_SELQ) {
      ok = (LC.selq & need) == need;
    } else {  // namespaceSelector: never for kind Namespace; skipped for an empty kind unless kinds hold "*"
      const uint32_t kid = GVK_KIND(gvk);
      if (kid == (tm.b & 0xFFFFu)) ok = (f & TSQ_EXC) != 0u;
      else if (kid == (tm.b >> 16) && (!(f & TSQ_STAR) || (f & TSQ_EXC))) ok = true;
      else ok = !(f & TSQ_INVALID) && (LC.nsq & need) == need;
    }
  } else if (tm.type == T_KIND_PRED) {
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
    const bool nssel = tm.type == T_NSSELECTOR;
    uint32_t lo = LC.lo, hi = LC.hi;
    const uint32_t *K = a.lab_k, *V = a.lab_v;
    bool eval = true;
    if (nssel) {
      // never for kind Namespace; skipped for an empty kind unless kinds hold "*"
      const uint32_t kid = GVK_KIND(gvk);
      lo = LC.nlo, hi = LC.nhi;
      K = a.nsl_k, V = a.nsl_v;
      if (B.bit(S.p_kind_ns, kid)) {
        ok = S.exc != 0u, eval = false;  // PolicyException blocks skip the check (match.go:184)
      } else if (B.bit(S.p_kind_empty, kid) && (!S.star_kind || S.exc)) {
        ok = true, eval = false;
      } else if (S.invalid) {
        ok = false, eval = false;
      }
    }
    if (eval && S.qbit != KPE_NO_QBIT) {  // requirement masks (ScanArgs::selm)
      const uint64_t need = (S.nreq >= 64u ? ~0ull : ((1ull << S.nreq) - 1ull)) << S.qbit;
      ok = ((nssel ? LC.nsq : LC.selq) & need) == need;
    } else if (eval) {
#pragma unroll 1
      for (uint32_t qi = 0; qi < S.nreq; ++qi) {
        const KpeSelReq q = sld(a.selreqs, S.req0 + qi);
        const bool wild = q.op == SR_WILD;
        // first label with a matching key (and value, for wildcards): the cached ones, then memory
        bool found = false;
        uint32_t kid = KPE_NO_STR, vid = KPE_NO_STR;
#pragma unroll 1
        for (uint32_t j = lo; !found && j < hi; ++j)
          if (B.bit(q.pk, K[j]) && (!wild || B.bit(q.pv, V[j]))) found = true, kid = K[j], vid = V[j];
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
  return ok;
}


// Store a tile's staged row segments [c0, c0 + nc) of R-byte rows.
__device__ __forceinline__ void store_rows(uint8_t* verdicts, const uint8_t* sv, uint32_t tile, uint32_t R,
                                           uint32_t c0, uint32_t nc, uint32_t nrows, uint32_t lane) {
  uint8_t* base = verdicts + (size_t)tile * (64 * R) + c0;
  if (nc == R) {  // whole rows: contiguous nrows x R bytes, dword aligned (64 R % 4 == 0)
    const uint32_t nb = nrows * R, nw = nb >> 2;
    uint32_t* dst = reinterpret_cast<uint32_t*>(base);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(sv);
    uint32_t i = lane;
#pragma unroll 1
    for (; 4u * i + 3u < nw; i += 64) {  // 16 bytes per lane and store
      const uint32_t* s4 = src + 4u * i;
      *reinterpret_cast<u32x4a*>(dst + 4u * i) = u32x4a{s4[0], s4[1], s4[2], s4[3]};
    }
#pragma unroll 1
    for (i = (nw & ~3u) + lane; i < nw; i += 64) dst[i] = src[i];
    if (lane < (nb & 3u)) base[(nw << 2) + lane] = sv[(nw << 2) + lane];
  } else if (((R | c0 | nc) & 3u) == 0u) {  // dword-aligned row segments (nc bytes of each row)
    const uint32_t* src = reinterpret_cast<const uint32_t*>(sv);
    // unit u of the chunk is row u / n, piece u % n: one division per lane, then steps of 64 units
    // (no integer division per store)
    auto walk = [&](uint32_t n, uint32_t tot, auto&& put) {
      uint32_t row = lane / n, q = lane - row * n;
      const uint32_t drow = 64u / n, dq = 64u - drow * n;
#pragma clang loop vectorize(disable) unroll(disable)
      for (uint32_t i = lane; i < tot; i += 64) {
        put(i, row, q);
        row += drow, q += dq;
        if (q >= n) q -= n, ++row;
      }
    };
    if ((nc & 15u) == 0u) {  // 16 bytes per lane and store (dword-aligned addresses)
      walk(nc >> 4, nrows * (nc >> 4), [&](uint32_t i, uint32_t row, uint32_t q) {
        const uint32_t* s4 = src + 4u * i;
        *reinterpret_cast<u32x4a*>(base + (size_t)row * R + 16u * q) = u32x4a{s4[0], s4[1], s4[2], s4[3]};
      });
    } else {
      walk(nc >> 2, nrows * (nc >> 2), [&](uint32_t i, uint32_t row, uint32_t q) {
        *reinterpret_cast<uint32_t*>(base + (size_t)row * R + 4u * q) = src[i];
      });
    }
  } else {
#pragma clang loop vectorize(disable) unroll(disable)
    for (uint32_t i = lane; i < nrows * nc; i += 64) {
      const uint32_t row = i / nc, col = i - row * nc;
      base[(size_t)row * R + col] = sv[i];
    }
  }
}

}  // namespace

// Persistent, wave-autonomous scan. Every wave walks 64-resource tiles
// (tile = global wave id, + total waves, ...); the next tile's data (pod records +
// cooperative list loads, or the match columns) is in flight while the current tile
// is evaluated, and the tile header one step further ahead.
// NARROW: terms become a per-lane bit vector and each lane runs the rule loop for
// its resource (rule records and filter masks are wave-uniform scalar loads).
// WIDE: terms are ballot-ed into per-wave 64-bit masks in LDS and lane j evaluates
// rule c0 + j for all 64 resources with 64-bit mask algebra.
// PREP (one block per evaluation): run the block prologue once and store its LDS products
// (predicate bitsets, truth table, capability-set bits) as ScanArgs::pimg; the scan blocks
// of that evaluation then copy the image instead of recomputing it.
// LEAN (PSS, NARROW, prepped, kind-only match terms, every fixed PSA predicate in LDS, no
// check masks): the rule match is one kind-table read, the PSS predicates direct LDS reads.
#ifndef KPE_LEAN_WAVES
#define KPE_LEAN_WAVES 5
#endif
template <bool PSS, bool NARROW, bool PREP, bool LEAN = false, bool PSUM = false>
__global__ void __launch_bounds__(kBlock, LEAN ? KPE_LEAN_WAVES : KPE_SCAN_WAVES)
    kpe_scan_kernel(const ScanArgs* __restrict__ ap) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  CArgs& a0 = *launder(ap);
  uint8_t* const s_capb = reinterpret_cast<uint8_t*>(dyn + a0.capb_lds);  // capability-set bits
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles;
  const uint32_t W = gridDim.x * (kBlock / 64u);
  uint32_t tile = blockIdx.x * (kBlock / 64u) + wv;

  // ---- first tile's header, the prologue's own loads, then the first tile's data; the
  // block prologue runs while the tile loads are in flight. No loaded value is touched
  // before the header is needed, so nothing waits for more than the load it uses. ----
  uint32_t h = 0;  // header words of the tile whose data is loaded next
  // unconditional, clamped (a wave without a tile re-reads the last one and never uses
  // it): the number of loads in flight is the same on every path, so waits are counted
  const uint32_t tile0 = min(tile, ntiles - 1u);
  if (PSS && !PREP && !PSUM) h = load_hdr(a0, tile0, lane);
  // capability sets (tiny dictionary) and the first slice of the LDS image, clamped and
  // unconditional (a zero page stands in for an absent table)
  const bool prepped = LEAN || (!PREP && a0.pimg != nullptr);  // the prologue image is ready in HBM
  const uint32_t ncs = a0.ncapsets;
  const bool capl = PSS && !prepped && (a0.need & NEED_CAPS) && ncs;
  const uint4 cs0 = reinterpret_cast<const uint4*>(capl ? a0.capsets : a0.zero_page)[capl ? min(t, ncs - 1u) : 0u];
  const bool fused = !prepped && a0.npairs != 0;
  const uint32_t img_n4 = (prepped ? a0.pimg_words : fused ? a0.fuse_words : a0.blob_words) >> 2;
  const uint4* img = reinterpret_cast<const uint4*>(img_n4 ? (prepped ? a0.pimg : fused ? a0.fuse : a0.pbuf)
                                                          : a0.zero_page);
  const uint4 img0 = img[img_n4 ? min(t, img_n4 - 1u) : 0u];
  // Program tables held in lanes for the whole kernel (read back with v_readlane:
  // no memory access inside the tile loop). WIDE single-chunk programs: lane j's
  // packed rule. NARROW: lane j holds rule j's record, lane f filter f's term mask,
  // lane t term t.
  uint4 myrule = make_uint4(0, 0, 0, 0);
  uint32_t fm_lane = 0, tm_type = 0, tm_a = 0, tm_b = 0;
  if (NARROW) {
    if (lane < a0.nrules) myrule = reinterpret_cast<const uint4*>(a0.narrow_rules)[lane];
    if (lane < a0.nfilters) fm_lane = a0.fmask[lane];
    if (lane < a0.nterms) {
      const KpeTerm tm = a0.terms[lane];
      tm_type = tm.type, tm_a = tm.a, tm_b = tm.b;
    }
  } else {
    if (a0.nrules <= KPE_RULE_CHUNK && lane < a0.nrules) myrule = reinterpret_cast<const uint4*>(a0.rule_lanes)[lane];
    // WIDE: term t's record in lane t as well (<= 64 terms): no scalar load per term and tile
    if (a0.nterms <= 64u && lane < a0.nterms) {
      const KpeTerm tm = a0.terms[lane];
      tm_type = tm.type, tm_a = tm.a, tm_b = tm.b;
    }
  }
  uint32_t cls_cv = 0, cls_rm = 0;  // NARROW PSS classes: (check set, rules failing on it)
  if (NARROW && a0.tt_lds != PRED_NONE && lane < a0.ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a0.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  Tile<PSS> ta{};
  if constexpr (!PREP) {
    ta = load_tile<PSS, LEAN, PSUM>(a0, tile0, h, lane);
    if (PSS) h = load_hdr(a0, min(tile + W, ntiles - 1u), lane);
  }
  {
    CArgs& a = a0;
    // prepped: the prologue image is a copy of LDS [0, pimg_words); fused dictionary pass: the
    // fuse image, and the local bitsets cleared; otherwise the small-domain predicate bitsets
    // (kpe_pred_kernel output)
    uint4* d4 = reinterpret_cast<uint4*>(dyn + (fused ? a.fuse_lds : 0u));
    if (t < img_n4) d4[t] = img0;
#pragma unroll 1
    for (uint32_t i = t + kBlock; i < img_n4; i += kBlock) d4[i] = img[i];
    if (fused) {
#pragma unroll 1
      for (uint32_t i = t; i < a.blob_words; i += kBlock) dyn[i] = 0;
    }
    if (a.kslot_lds != PRED_NONE) {  // the GVK kind-term table
      const uint32_t nw = ((a.nkslot_g + 1u) & ~1u) * 3u;
#pragma unroll 1
      for (uint32_t i = t; i < nw; i += kBlock) dyn[a.kslot_lds + i] = a.kslot_tab[i];
    }
    if (a.selt_lds != PRED_NONE) {  // label-selector requirement tables (sel_km, then sel_vm)
      uint4* d = reinterpret_cast<uint4*>(dyn + a.selt_lds);
#pragma unroll 1
      for (uint32_t i = t; i < a.nlabk + a.nlabv; i += kBlock) d[i] = i < a.nlabk ? a.sel_km[i] : a.sel_vm[i - a.nlabk];
    }
    if (!NARROW && a.filt_lds != PRED_NONE) {  // program filters + filter terms for the rule lanes
      const uint32_t nw = a.fterm_lds + a.nfterms - a.filt_lds;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.filters);
#pragma unroll 1
      for (uint32_t i = t; i < nw; i += kBlock)
        dyn[a.filt_lds + i] = i < a.fterm_lds - a.filt_lds ? src[i] : a.fterms[i - (a.fterm_lds - a.filt_lds)];
    }
  }
  __syncthreads();
  if (fused) {  // one short LDS compare per (string, pattern)
    CArgs& a = a0;
    const uint2* pairs = reinterpret_cast<const uint2*>(dyn + a.fuse_lds);
    const KpePat* pats = reinterpret_cast<const KpePat*>(dyn + a.fuse_pats);
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(dyn);
    const uint8_t* pb = lb + a.fuse_patb * 4;
#pragma unroll 1
    for (uint32_t i = t; i < a.npairs; i += kBlock) {
      const uint2 e = pairs[i];
      if (pat_match(pats[e.y & 0xFFFu], pb, lb + (e.x & 0xFFFFFu), (int)(e.x >> 20)))
        atomicOr(&dyn[(e.y >> 12) & 0x7FFFu], 1u << (e.y >> 27));
    }
    __syncthreads();
  }
  if (PSS && !prepped) {
    CArgs& a = a0;
    const Bits B{dyn, a.pbuf};
    if (a.need & NEED_CAPS) {  // capability-set violation bits (add/drop masks vs the fixed allow-lists)
      const uint64_t caps_ok = B.mask64(a.pp_caps_ok), nbs = B.mask64(a.pp_cap_nbs), all = B.mask64(a.pp_cap_all);
      auto capb = [&](uint4 c) -> uint8_t {
        const uint64_t ad = (uint64_t)c.x | ((uint64_t)c.y << 32), dr = (uint64_t)c.z | ((uint64_t)c.w << 32);
        return (uint8_t)(((ad & ~caps_ok) ? CS_BASE : 0u) | ((dr & all) ? 0u : CS_DROP) | ((ad & ~nbs) ? CS_ADD : 0u));
      };
      if (t < a.ncapsets) s_capb[t] = capb(cs0);
#pragma unroll 1
      for (uint32_t i = t + kBlock; i < a.ncapsets; i += kBlock) s_capb[i] = capb(reinterpret_cast<const uint4*>(a.capsets)[i]);
    } else {
#pragma unroll 1
      for (uint32_t i = t; i < a.ncapsets; i += kBlock) s_capb[i] = 0;
    }
    __syncthreads();
  }

  // NARROW truth table: tt[v] = rules whose match / exclude / namespaced-policy term
  // conditions hold for term vector v (pkg/engine/utils/match.go:168-300 over filters)
  if (NARROW && !prepped && a0.tt_lds != PRED_NONE) {
    const uint32_t R = a0.nrules, nv = 1u << a0.nterms;
    for (uint32_t tb = t; tb < nv; tb += kBlock) {
      uint32_t mm = 0;
      for (uint32_t ri = 0; ri < R; ++ri) {
        const uint32_t x = hw(myrule.x, ri), z = hw(myrule.z, ri), w = hw(myrule.w, ri);
        auto block = [&](uint32_t mode, uint32_t f0, uint32_t nf) -> bool {
          const bool all = mode == MODE_ALL;
          bool acc = all;
          for (uint32_t f = 0; f < nf; ++f) {
            const uint32_t fm = hw(fm_lane, f0 + f);
            const bool hit = (tb & fm) == fm;
            acc = all ? (acc && hit) : (acc || hit);
          }
          return acc;
        };
        const uint32_t pol = NR_POLTERM(x);
        bool m = pol == 0u || ((tb >> (pol - 1u)) & 1u);
        m = m && block(NR_MATCH_MODE(x), RL_F0(z), RL_NF(z));
        m = m && !block(NR_EXCL_MODE(x), RL_F0(w), RL_NF(w));
        if (m) mm |= 1u << ri;
      }
      dyn[a0.tt_lds + tb] = mm;
    }
    __syncthreads();
  }
  if constexpr (PREP) {  // store the prologue's products: LDS [0, pimg_words) with the kind table filled in
    CArgs& a = a0;
    const Bits B{dyn, a.pbuf};
    if (NARROW && a.kt_lds != PRED_NONE && a.tt_lds != PRED_NONE) {
      // kt[k]: the truth table at kind k's term vector (kind-only terms; T_FALSE: never)
#pragma unroll 1
      for (uint32_t k = t; k < a.nkinds; k += kBlock) {
        uint32_t tv = 0;
        for (uint32_t ti = 0; ti < a.nterms; ++ti)
          tv |= hw(tm_type, ti) == T_KIND_PRED && B.bit(hw(tm_a, ti), k) ? (1u << ti) : 0u;
        dyn[a.kt_lds + k] = dyn[a.tt_lds + tv];
      }
      __syncthreads();
    }
#pragma unroll 1
    for (uint32_t i = t; i < a.pimg_words; i += kBlock) a.pimg[i] = dyn[i];
    return;
  }
  LeanPP lp{};
  uint32_t kt_lds = 0;
  if constexpr (LEAN) {
    lp = LeanPP{a0.pp_seccomp_ann_ok, a0.pp_apparmor_key, a0.pp_apparmor_ok, a0.pp_seccomp_pod_key,
                a0.pp_sysctl0, a0.pp_sysctl1, a0.pp_sysctl2};
    kt_lds = a0.kt_lds;
  }
  // NARROW verdict rows are stored one tile late (double-buffered in LDS), after the
  // next tile's loads are issued, so no wait for those loads ever covers a store.
  uint32_t prev_tile = 0xFFFFFFFFu, prev_rows = 0, buf = 0;

  // Ping-pong tile buffers: the tile evaluated in one step was loaded into its own
  // registers during the previous step, and the next tile is loaded into the other
  // buffer, so no register holding an in-flight load is ever copied (a loop-carried
  // copy of a prefetched register makes the compiler wait for the prefetch at once).
  auto step = [&](Tile<PSS>& cur, Tile<PSS>& nxt) {
    CArgs& a = *launder(ap);
    const uint32_t R = a.nrules, n = (uint32_t)a.n;
    const Bits B{dyn, a.pbuf};
    // per-wave LDS: PSS list staging, then NARROW: verdict staging (64 x R bytes);
    // WIDE: term masks, PSS version-set masks, rule cell masks, verdict staging.
    uint32_t* wbase = dyn + a.wave_lds + wv * a.wave_words;
    uint32_t* stage = wbase;
    uint32_t* wrest = wbase + (PSS ? KPE_STAGE_WORDS : 0u);
    uint64_t* tmk = reinterpret_cast<uint64_t*>(wrest);
    uint64_t* cvm = tmk + a.nterms;
    uint64_t* rmk = cvm + a.ncv;  // kRC x (P, F, E, D): D = KPE_XDEFER_ cells
    uint8_t* sv = NARROW ? reinterpret_cast<uint8_t*>(wrest) + buf * 64 * R
                         : reinterpret_cast<uint8_t*>(rmk + 4 * KPE_RULE_CHUNK);
    // ---- prefetch the next tile into the other buffer, then evaluate `cur` ----
    // (unconditional, clamped: past the end it re-reads the last tile, never used)
    nxt = load_tile<PSS, LEAN, PSUM>(a, min(tile + W, ntiles - 1), h, lane);
    if (PSS && !PSUM) h = load_hdr(a, min(tile + 2 * W, ntiles - 1), lane);
    pin_tile(cur);
    const uint32_t r = tile * 64 + lane;
    const bool live = r < n;
    const uint32_t rc = live ? r : n - 1;
    uint32_t fails = 0, gvk, nsa, name_col, mns_col;
    bool err = false;
    const uint32_t need = a.need;
    if constexpr (PSS) {
      fails = pss_tile<LEAN, PSUM>(a, B, s_capb, cur, live, stage, lane, lp);
      const uint32_t cls = (cur.rec.x >> PR_CLASS_SH) & R_CLASS_MASK;
      err = live && (cls == R_CLASS_OTHER || (cur.rec.x & PR_DECODE_ERR));
      gvk = live ? cur.rec.y : 0u;
      nsa = live ? cur.rec.w : KPE_NO_STR;
    } else {
      gvk = live && (need & NEED_GVK) ? cur.gvk : 0u;
      nsa = live && (need & NEED_NSA) ? cur.nsa : KPE_NO_STR;
    }
    name_col = live && (need & NEED_NAME) ? cur.name : KPE_NO_STR;
    mns_col = live && (need & NEED_MNS) ? cur.mns : KPE_NO_STR;
    const uint32_t nrows = min(64u, n - tile * 64);
    if (NARROW && prev_tile != 0xFFFFFFFFu) {  // the previous tile's rows (other LDS buffer)
      store_rows(a.verdicts, reinterpret_cast<uint8_t*>(wrest) + (buf ^ 1u) * 64 * R, prev_tile, R, 0, R, prev_rows,
                 lane);
      prev_tile = 0xFFFFFFFFu;
    }

    if (NARROW) {
      // ---- terms -> bit vector ----
      uint32_t tb = 0;
      if constexpr (!LEAN) {
        LabCache LC;
        if constexpr (PSS && PSUM && KPE_PSUM_LABPRE) lab_cache(a, rc, live, LC, dyn, cur.v0, cur.v1, cur.s0);
        else if constexpr (PSS) lab_cache(a, rc, live, LC, dyn);
        else lab_cache(a, rc, live, LC, dyn, cur.lo, cur.hi, cur.nsl);
        if (a.kslot_lds != PRED_NONE) LC.kmask = kslot_mask(a, dyn, gvk);
#pragma unroll 1
        for (uint32_t ti = 0; ti < a.nterms; ++ti) {
          const KpeTerm tm{hw(tm_type, ti), hw(tm_a, ti), hw(tm_b, ti), 0u};
          tb |= eval_term(a, B, tm, gvk, nsa, name_col, mns_col, rc, live, LC) ? (1u << ti) : 0u;
        }
      }
      if (LEAN || (a.tt_lds != PRED_NONE && !a.masks)) {  // truth-table fast path (LEAN: the kind table)
        const uint32_t matched = !live ? 0u : LEAN ? dyn[kt_lds + GVK_KIND(gvk)] : dyn[a.tt_lds + tb];
        uint32_t failr = 0;
#pragma unroll 1
        for (uint32_t c = 0; c < a.ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
        const uint32_t E = matched & ((err ? a.pss_rules : 0u) | a.err_rules | a.pat_rules);
        const uint32_t F = (matched & a.pss_rules & failr & ~E) | (matched & a.pat_rules);  // F|E = PENDING
        const uint32_t P = matched & a.pss_rules & ~failr & ~E;
#pragma unroll 1
        for (uint32_t ri = 0; ri < R; ++ri)
          sv[lane * R + ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
        __builtin_amdgcn_wave_barrier();
        prev_tile = tile, prev_rows = nrows, buf ^= 1u;
        return;
      }
      // ---- rules, in program order, for this lane's resource ----
      bool applied = false;
#ifdef KPE_NARROW_FV
      // every filter once per lane into a bit vector (a filter holds when all of its terms hold);
      // a block is then one mask test over its filters [f0, f0 + nf)
      uint64_t fv = 0;
#pragma unroll 1
      for (uint32_t f = 0; f < a.nfilters; ++f) {
        const uint32_t fm = hw(fm_lane, f);
        fv |= (uint64_t)((tb & fm) == fm) << f;
      }
#endif
#pragma unroll 1
      for (uint32_t ri = 0; ri < R; ++ri) {
        const uint4 nr = make_uint4(hw(myrule.x, ri), hw(myrule.y, ri), hw(myrule.z, ri), hw(myrule.w, ri));
        const uint32_t x = nr.x;
        // a block is an OR (any / legacy) or AND (all) of filters; a filter holds when
        // all of its terms hold: (tb & mask) == mask
        auto block = [&](uint32_t mode, uint32_t f0, uint32_t nf) -> bool {
#ifdef KPE_NARROW_FV
          const uint64_t M = (nf >= 64u ? ~0ull : ((1ull << nf) - 1ull)) << f0;
          return mode == MODE_ALL ? (fv & M) == M : (fv & M) != 0ull;
#else
          const bool all = mode == MODE_ALL;
          bool acc = all;
#pragma unroll 1
          for (uint32_t f = 0; f < nf; ++f) {
            const uint32_t fm = hw(fm_lane, f0 + f);
            const bool h = (tb & fm) == fm;
            acc = all ? (acc && h) : (acc || h);
          }
          return acc;
#endif
        };
        const uint32_t pol = NR_POLTERM(x);
        bool m = live && (pol == 0u || ((tb >> (pol - 1u)) & 1u));
        m = m && block(NR_MATCH_MODE(x), RL_F0(nr.z), RL_NF(nr.z));
        m = m && !block(NR_EXCL_MODE(x), RL_F0(nr.w), RL_NF(nr.w));
        const uint32_t hd = NR_HANDLER(x);
        uint32_t v = KPE_NA_;
        // PolicyExceptions of the rule: their match block holds => RuleSkip before any handler
        // (XE_DEFER: the cell's verdict without the exception, flagged for kpe_cond_kernel)
        const uint32_t xe = (m && a.rule_exc) ? sld(a.rule_exc, ri) : 0u;
        const bool xm = xe && block((xe & XE_ALL) ? MODE_ALL : MODE_ANY, XE_F0(xe), XE_NF(xe));
        const bool xh = xm && !(xe & XE_DEFER);
        if (xh && !(xe & XE_PSS)) v = KPE_SKIP_;
        else if (m && hd == H_PSS)  // under a podSecurity exception kpe_pssx_kernel decides
          v = err ? KPE_ERROR_ : xh ? KPE_XFAIL_ : ((fails & nr.y) ? KPE_FAIL_ : KPE_PASS_);
        else if (m && hd == H_ERROR) v = KPE_ERROR_;
        else if (m && (hd == H_PATTERN || hd == H_COND)) v = KPE_PENDING_;
        else if (m && hd == H_CONST_SKIP) v = KPE_SKIP_;
        else if (m && hd == H_CONST_FAIL) v = KPE_FAIL_;
        else if (m && hd == H_CONST_PASS) v = KPE_PASS_;
        if (x & NR_NEW_POLICY) applied = false;
        if ((x & NR_APPLY_ONE) && applied) v = KPE_NA_;
        applied |= v == KPE_PASS_ || v == KPE_FAIL_;
        sv[lane * R + ri] = (uint8_t)(v | (xm && !xh && v != KPE_NA_ ? (uint32_t)KPE_XDEFER_ : 0u));
        if (a.masks && live) a.masks[(size_t)r * R + ri] = v == KPE_FAIL_ ? (fails & nr.y) : 0u;
      }
      __builtin_amdgcn_wave_barrier();
      prev_tile = tile, prev_rows = nrows, buf ^= 1u;
      return;
    }

    // ---- WIDE: terms, one ballot per distinct term ----
    const KpeFilter* filt =
        a.filt_lds != PRED_NONE ? reinterpret_cast<const KpeFilter*>(dyn + a.filt_lds) : a.filters;
    const uint32_t* fterm = a.filt_lds != PRED_NONE ? dyn + a.fterm_lds : a.fterms;
    LabCache LC;
    if constexpr (PSS && PSUM && KPE_PSUM_LABPRE) lab_cache(a, rc, live, LC, dyn, cur.v0, cur.v1, cur.s0);
    else if constexpr (PSS) lab_cache(a, rc, live, LC, dyn);
    else lab_cache(a, rc, live, LC, dyn, cur.lo, cur.hi, cur.nsl);
    if (a.kslot_lds != PRED_NONE) LC.kmask = kslot_mask(a, dyn, gvk);
#if KPE_DIAG & 2  // diagnostic build: no term evaluation
    if (lane < a.nterms) tmk[lane] = LC.selq ^ gvk ^ nsa;
#else
#pragma unroll 1
    for (uint32_t ti = 0; ti < a.nterms; ++ti) {
      const KpeTerm tm = a.nterms <= 64u ? KpeTerm{hw(tm_type, ti), hw(tm_a, ti), hw(tm_b, ti), 0u} : sld(a.terms, ti);
      const uint64_t m = __ballot(eval_term(a, B, tm, gvk, nsa, name_col, mns_col, rc, live, LC));
      if (lane == 0) tmk[ti] = m;
    }
#endif
    // PSS version sets: resources failing some check of each distinct cv_mask
#pragma unroll 1
    for (uint32_t c = 0; c < a.ncv; ++c) {
      const uint64_t m = __ballot((fails & sld(a.cv_classes, c)) != 0u);
      if (lane == 0) cvm[c] = m;
    }
    const uint64_t live_m = __ballot(live);
    const uint64_t err_m = __ballot(err);
    __builtin_amdgcn_wave_barrier();

#if KPE_DIAG & 1  // diagnostic build: no rule evaluation, the term masks' low bytes as verdicts
    {
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i = lane; i < nrows * R; i += 64) sv[i] = (uint8_t)(tmk[i % a.nterms] >> (i & 7u)) & 7u;
      __builtin_amdgcn_wave_barrier();
      store_rows(a.verdicts, sv, tile, R, 0, R, nrows, lane);
      __builtin_amdgcn_wave_barrier();
      return;
    }
#endif
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
        } else if (handler == H_PATTERN || handler == H_COND) {
          fm = em = m;  // both bits: KPE_PENDING_
        } else if (handler == H_CONST_SKIP) {
          pm = em = m;  // both bits: KPE_SKIP_ (no ApplyOne with constant handlers)
        } else if (handler == H_CONST_FAIL) {
          fm = m;
        } else if (handler == H_CONST_PASS) {
          pm = m;
        }
        uint64_t dm = 0;
        if (a.rule_exc && m) {  // PolicyExceptions: RuleSkip where their match block holds
          const uint32_t xe = a.rule_exc[c0 + lane];
          if (xe) {
            const uint64_t xm = m & block_mask((xe & XE_ALL) ? MODE_ALL : MODE_ANY, XE_F0(xe), XE_NF(xe));
            if (xe & XE_DEFER) dm = xm;  // kpe_cond_kernel applies it after the preconditions
            else if (xe & XE_PSS) pm |= xm & ~em, fm |= xm & ~em;  // p and f: KPE_XFAIL_ (kpe_pssx_kernel decides)
            else pm |= xm, em |= xm, fm &= ~xm;
          }
        }
        rmk[lane * 4 + 0] = pm;
        rmk[lane * 4 + 1] = fm;
        rmk[lane * 4 + 2] = em;
        rmk[lane * 4 + 3] = dm;
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
            uint64_t pm = rmk[j * 4], fm = rmk[j * 4 + 1], em = rmk[j * 4 + 2];
            if (rule.apply_one) {
              pm &= ~applied, fm &= ~applied, em &= ~applied;
              rmk[j * 4] = pm, rmk[j * 4 + 1] = fm, rmk[j * 4 + 2] = em;
            }
            applied |= pm | fm;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      // (b) verdict bytes (resource lanes): the cell's (p, f, e) bits index a nibble table --
      // NA, ERROR, FAIL, PENDING, PASS, SKIP, XFAIL, SKIP -- and four cells go to LDS as one dword
      // when the row segments are dword aligned
      constexpr uint32_t kVt = KPE_NA_ | KPE_ERROR_ << 4 | KPE_FAIL_ << 8 | KPE_PENDING_ << 12 | KPE_PASS_ << 16 |
                               KPE_SKIP_ << 20 | (uint32_t)KPE_XFAIL_ << 24 | (uint32_t)KPE_SKIP_ << 28;
      auto cell = [&](uint32_t j) -> uint32_t {
        const uint32_t idx = (uint32_t)((rmk[j * 4] >> lane) & 1u) << 2 | (uint32_t)((rmk[j * 4 + 1] >> lane) & 1u) << 1 |
                             (uint32_t)((rmk[j * 4 + 2] >> lane) & 1u);
        const uint32_t v = (kVt >> (idx << 2)) & 0xFu;
        return v | (((uint32_t)(rmk[j * 4 + 3] >> lane) & 1u) && v ? (uint32_t)KPE_XDEFER_ : 0u);
      };
      if ((nc & 3u) == 0u) {
        uint32_t* sv32 = reinterpret_cast<uint32_t*>(sv + lane * nc);
#pragma unroll 2
        for (uint32_t j = 0; j < nc; j += 4)
          sv32[j >> 2] = cell(j) | cell(j + 1) << 8 | cell(j + 2) << 16 | cell(j + 3) << 24;
      } else {
#pragma unroll 4
        for (uint32_t j = 0; j < nc; ++j) sv[lane * nc + j] = (uint8_t)cell(j);
      }
      if (a.masks && live) {
#pragma unroll 1
        for (uint32_t j = 0; j < nc; ++j) {
          const uint32_t cm = ((rmk[j * 4 + 1] >> lane) & 1u) ? (fails & sld(a.rules, c0 + j).cv_mask) : 0u;
          a.masks[(size_t)r * R + c0 + j] = cm;
        }
      }
      __builtin_amdgcn_wave_barrier();
      store_rows(a.verdicts, sv, tile, R, c0, nc, nrows, lane);
      __builtin_amdgcn_wave_barrier();
    }
    };
  Tile<PSS> tb{};
  while (tile < ntiles) {
    step(ta, tb);
    tile += W;
    if (tile >= ntiles) break;
    step(tb, ta);
    tile += W;
  }

  if (NARROW && prev_tile != 0xFFFFFFFFu) {
    CArgs& a = *launder(ap);
    const uint32_t R = a.nrules;
    const uint8_t* last = reinterpret_cast<const uint8_t*>(dyn + a.wave_lds + wv * a.wave_words +
                                                          (PSS ? KPE_STAGE_WORDS : 0u)) + (buf ^ 1u) * 64 * R;
    store_rows(a.verdicts, last, prev_tile, R, 0, R, prev_rows, lane);
  }
}


#ifndef KPE_VM_ONLY
#include "lean.inl"
#endif

// ---------------------------------------------------------------------------
// Host-side launch wrappers (called from kpe_api.cpp).
// grid: x = blocks of the largest job, y = jobs
// ===========================================================================
// Pattern rules: validate.MatchPattern over the document tape
// (pkg/engine/validate/validate.go:15-261, anchor/handlers.go:31-275, pattern/pattern.go).
// One lane per resource runs the compiled pattern (program.cpp pc::PatCompiler) against
// its document nodes; cells the scan kernel marked KPE_PENDING_ (rule matched) are
// resolved to pass / fail / error / skip. Only the class of the error a subtree returns
// and whether its path is empty decide the verdict, so that is all a subtree reports.
// The reference's recursion is an explicit per-lane frame stack (no calls, so no spilled
// call frames and no callee register budget): a frame is a map validated member by
// member, or an array validated element by element; scalar leaves resolve in place.
// ===========================================================================
namespace {
#include "patvm.inl"
}  // namespace

#ifndef KPE_SCAN_ONLY
// The VM side builds as three objects in parallel (KPE_VM_PART 1: pattern kernels, 2: condition
// kernel without the pattern VM, pssx, pack3, traces; 3: the condition kernel with it); undefined:
// all of them in one object.
#ifndef KPE_VM_PART
#define KPE_VM_PART 0
#endif
#define KPE_IN_PART(p) (KPE_VM_PART == 0 || KPE_VM_PART == (p))
// grid: 256-row blocks, one lane per row running every pattern rule
#ifndef KPE_PAT_BLOCK
#define KPE_PAT_BLOCK 128  // C5 / C3 pattern kernel (events, profiles/r03_c_ldsframes): 256 x 8 frames 20.7 / 9.2 ms,
#endif                     // 128 x 8 18.1 / 7.8, 256 x 6 17.2 / 7.0, 128 x 6 16.8 / 6.9, + 4 waves/SIMD 15.6 / 7.0
// the lane's frame stack lives in LDS (FramesLds, word-planar: conflict-free at any mix of depths)
#ifndef KPE_PAT_MINW
#define KPE_PAT_MINW 3  // the leaf-table instance takes 111 VGPRs (4 waves/SIMD, as many as the 8 LDS-bound
                        // blocks per CU hold), the one without 166; the inline map path spills at 128 (r03_e_inline)
#endif
#if KPE_IN_PART(1)
// LT: the leaf-table instance (PatVMT LT), for programs whose leaves all have table slots.
template <bool LT>
__global__ void __launch_bounds__(KPE_PAT_BLOCK, KPE_PAT_MINW) kpe_pattern_kernel(const PatArgs* __restrict__ ap) {
  constexpr uint32_t kWaveWords = FramesLds::kWords * FramesLds::kDepth * 64u;
  __shared__ uint32_t s_fs[KPE_PAT_BLOCK / 64][kWaveWords];
  __shared__ uint8_t s_memo[KPE_PAT_MEMO][KPE_PAT_BLOCK];  // byte-planar: a lane's slot s at [s][lane]
  const int64_t i = (int64_t)blockIdx.x * KPE_PAT_BLOCK + threadIdx.x;
  if (i >= ap->n) return;
  const int64_t r = ap->perm ? (int64_t)ap->perm[i] : i;
  pat_eval_row<FramesLds, LT, true>(*ap, r, FramesLds{&s_fs[threadIdx.x >> 6][threadIdx.x & 63u]},
                                    &s_memo[0][threadIdx.x], KPE_PAT_BLOCK);
}
// The cells kpe_pattern_kernel marked KPE_DEEP_ (one lane per row; rows without marks only scan),
// on a kPatStack-deep LDS frame stack (one-wave blocks: 25 KiB of LDS each).
template <bool LT>
__global__ void __launch_bounds__(64) kpe_pattern_deep_kernel(const PatArgs* __restrict__ ap) {
  __shared__ uint32_t s_fs[FramesLdsDeep::kWords * FramesLdsDeep::kDepth * 64u];
  if (ap->deep_any && *ap->deep_any == 0u) return;  // kpe_pattern_kernel marked no cell
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= ap->n) return;
  // rows through doc_perm (grouped by kind, then tape size) like the main kernel: the rows with deep
  // cells (one kind's deeper autogen patterns) fill whole waves instead of a few lanes of each
  const int64_t r = ap->perm ? (int64_t)ap->perm[i] : i;
  pat_deep_row<LT>(*ap, r, FramesLdsDeep{&s_fs[threadIdx.x]});
}

// Leaf table of a binding (PatArgs::ltab): grid y = slot, one thread per scalar of the corpus;
// a wave's 64 results are one ballot, stored as two words (ltab_words covers whole waves).
__global__ void __launch_bounds__(256) kpe_leaf_table_kernel(const PatArgs* __restrict__ ap,
                                                             const uint32_t* __restrict__ slot_leaf) {
  const PatArgs& a = *ap;
  const uint32_t sid = blockIdx.x * 256u + threadIdx.x, slot = blockIdx.y;
  uint32_t und = 0;
  const bool r = sid < a.nscal && pat_leaf_eval(a, sid, slot_leaf[slot], nullptr, &und);
  const uint64_t m = __ballot(r);
  if ((threadIdx.x & 63u) == 0u && sid < a.nscal) {
    uint32_t* w = a.ltab + (size_t)slot * a.ltab_words + (sid >> 5);
    w[0] = (uint32_t)m;
    w[1] = (uint32_t)(m >> 32);
  }
}
extern "C" hipError_t kpe_launch_leaf_table(const PatArgs* dargs, const uint32_t* slot_leaf, uint32_t nslots,
                                            uint64_t nscal, hipStream_t s) {
  if (nslots == 0 || nscal == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_leaf_table_kernel, dim3((unsigned)((nscal + 255) / 256), nslots), dim3(256), 0, s, dargs,
                     slot_leaf);
  return hipGetLastError();
}
#endif  // KPE_IN_PART(1)

// ===========================================================================
// Preconditions / deny / foreach-deny conditions (condvm.inl): one lane per resource resolves
// the cells of the rules whose conditions read the resource. Runs after the scan kernel (which
// marks H_COND cells pending and writes every other handler's verdict) and before the pattern
// kernel (a pattern cell whose preconditions hold stays pending).
// ===========================================================================
namespace {
#include "condvm.inl"
}  // namespace

// FEPAT: the instance that also holds the pattern VM, for programs with foreach pattern /
// anyPattern entries (the VM's frame stack and code stay out of the plain instance)
// Programs with partial-string variables (VT_TMPL) get 2 x KPE_TXT_CAP bytes of dynamic LDS per
// lane for the substituted key / value strings; the others launch without it.
template <bool FEPAT>
__global__ void __launch_bounds__(128) kpe_cond_kernel(const CondArgs* __restrict__ ap) {
  __shared__ char nb[128][2][16];
  extern __shared__ __attribute__((aligned(16))) uint8_t ctx[];
  const int64_t i = (int64_t)blockIdx.x * 128 + threadIdx.x;
  uint8_t* tx = ap->txt ? ctx + threadIdx.x * (2u * KPE_TXT_CAP) : nullptr;
  if (i < ap->n) cond_eval_row<FEPAT>(*ap, ap->perm ? (int64_t)ap->perm[i] : i, nb[threadIdx.x], tx);
}

#if KPE_IN_PART(3)
extern "C" hipError_t kpe_launch_cond_fepat(const CondArgs* dargs, int64_t n, int txt, hipStream_t s) {
  const size_t lds = txt ? 128u * 2u * KPE_TXT_CAP : 0u;
  hipLaunchKernelGGL(kpe_cond_kernel<true>, dim3((unsigned)((n + 127) / 128)), dim3(128), lds, s, dargs);
  return hipGetLastError();
}
#endif

#if KPE_IN_PART(2)
extern "C" hipError_t kpe_launch_cond_fepat(const CondArgs* dargs, int64_t n, int txt, hipStream_t s);
extern "C" hipError_t kpe_launch_cond(const CondArgs* dargs, int64_t n, int fepat, int txt, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (fepat) return kpe_launch_cond_fepat(dargs, n, txt, s);
  const size_t lds = txt ? 128u * 2u * KPE_TXT_CAP : 0u;
  hipLaunchKernelGGL(kpe_cond_kernel<false>, dim3((unsigned)((n + 127) / 128)), dim3(128), lds, s, dargs);
  return hipGetLastError();
}

// ===========================================================================
// podSecurity.exclude (pssx.inl): one lane per pod re-evaluates the failing cells of the
// rules with exclusions. Runs after the condition kernel (preconditions may have skipped a
// cell); reads the corpus's pod columns and the predicate bitsets in pbuf.
// ===========================================================================
namespace {
#include "pssx.inl"
}  // namespace

__global__ void __launch_bounds__(128) kpe_pssx_kernel(const PssxArgs* __restrict__ ap) {
  const int64_t r = (int64_t)blockIdx.x * 128 + threadIdx.x;
  if (r < ap->n) pssx_eval_row(*ap, r);
}

// Verdict exchange (kpe_pack_verdicts): 3-bit cells, 10 per 32-bit word, row-major. One thread
// per output word; neighbouring threads read neighbouring 10-byte runs (HBM-bound).
__global__ void __launch_bounds__(256) kpe_pack3_kernel(const uint8_t* __restrict__ v, uint64_t cells,
                                                        uint32_t* __restrict__ out, uint64_t words) {
  const uint64_t w = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (w >= words) return;
  const uint64_t c0 = w * 10u;
  uint32_t x = 0;
#pragma unroll
  for (uint32_t k = 0; k < 10u; ++k)
    if (c0 + k < cells) x |= (uint32_t)(v[c0 + k] & 7u) << (3u * k);
  out[w] = x;
}
extern "C" hipError_t kpe_launch_pack3(const uint8_t* v, uint64_t cells, uint32_t* out, hipStream_t s) {
  const uint64_t words = (cells + 9u) / 10u;
  if (!words) return hipSuccess;
  hipLaunchKernelGGL(kpe_pack3_kernel, dim3((unsigned)((words + 255u) / 256u)), dim3(256), 0, s, v, cells, out, words);
  return hipGetLastError();
}

extern "C" hipError_t kpe_launch_pssx(const PssxArgs* dargs, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_pssx_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, dargs);
  return hipGetLastError();
}

// Failing paths of listed pattern cells (kpe_pattern_traces): one lane per cell (row * R + col)
// walks each root of the cell's rule (at most KPE_TRACE_ROOTS) from the tape in HBM with the
// VM's TRACE instance, which records the path of the last failure (PatternError.Path). A cell
// with a job (jobs[i].w != 0: a validate.foreach cell that a pattern entry decided) walks the
// entry's roots [x, x + y & 0xFFFF) (PR_* flags in y >> 16) from the element node z (kNoNode: the
// resource root) instead. Report time only; the evaluation kernels never carry the tracing code.
__global__ void __launch_bounds__(128) kpe_pattern_trace_kernel(const PatArgs* __restrict__ ap,
                                                                 const uint64_t* __restrict__ cells, uint64_t n,
                                                                 uint32_t* __restrict__ out,
                                                                 const uint4* __restrict__ jobs) {
  const uint64_t i = (uint64_t)blockIdx.x * 128u + threadIdx.x;
  if (i >= n) return;
  const PatArgs& a = *ap;
  uint32_t* rec = out + i * (KPE_TRACE_ROOTS * KPE_TRACE_WORDS);
  for (uint32_t k = 0; k < KPE_TRACE_ROOTS * KPE_TRACE_WORDS; ++k) rec[k] = 0u;
  const uint64_t cell = cells[i];
  const uint64_t row = cell / a.R;
  const uint32_t col = (uint32_t)(cell - row * a.R);
  if (row >= (uint64_t)a.n) return;
  const uint4 job = jobs ? jobs[i] : make_uint4(0u, 0u, 0u, 0u);
  KpePatRule pr;
  uint32_t start = (uint32_t)a.doc_off[row];
  if (job.w) {
    pr.r0 = job.x, pr.nr = job.y & 0xFFFFu, pr.flags = job.y >> 16;
    if (job.z != kNoNode) start = job.z;
  } else {
    if (!a.col2pr || C2P_RULE(a.col2pr[col]) == 0u) return;
    pr = a.rules[C2P_RULE(a.col2pr[col]) - 1u];
  }
  PatVM vm{a, PV_DOCVIEW(a, reinterpret_cast<const uint2*>(a.doc), 0u, a.ndoc), start,
           a.pvals + (size_t)row * a.nvars, 0u};
  if (pr.flags & PR_ANY_BAD) {
    rec[0] = KPE_TR_VALID | ((uint32_t)KPE_ERROR_ << 16);
    return;
  }
  for (uint32_t k = 0; k < pr.nr && k < KPE_TRACE_ROOTS; ++k) {
    vm.tr = rec + k * KPE_TRACE_WORDS;
    const uint32_t v = pat_match_root<true>(vm, pr.r0 + k);
    vm.tr[0] = (vm.tr[0] & 0xFFFFu) | (v << 16) | KPE_TR_VALID;
  }
}

extern "C" hipError_t kpe_launch_pattern_trace(const PatArgs* dargs, const uint64_t* cells, uint64_t n, uint32_t* out,
                                               const uint4* jobs, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(kpe_pattern_trace_kernel, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, dargs, cells, n, out,
                     jobs);
  return hipGetLastError();
}

#endif  // KPE_IN_PART(2)

#if KPE_IN_PART(1)
extern "C" hipError_t kpe_launch_pattern(const PatArgs* dargs, int64_t n, uint32_t npr, int lt, hipStream_t s) {
  if (n <= 0 || npr == 0) return hipSuccess;
  // one lane per row running every pattern rule (a rows x rules grid measured no faster on C5 and
  // slower on C3's 600 rules; it also doubled the VM code the kernel holds)
  // (two or four lanes per row, each taking every 2nd / 4th pattern cell: C5 12.3 / 19.3 ms against
  // 8.5, profiles/r04_i: the lanes of a wave then walk different rules; verdicts of a 64-column
  // chunk written back once as whole words: C5 8.6 / C3 3.66 ms against 8.5 / 3.34, more spills,
  // profiles/r04_j)
  const dim3 grid((unsigned)((n + KPE_PAT_BLOCK - 1) / KPE_PAT_BLOCK));
  const dim3 rows((unsigned)((n + 63) / 64));
  if (lt) {
    hipLaunchKernelGGL(kpe_pattern_kernel<true>, grid, dim3(KPE_PAT_BLOCK), 0, s, dargs);
    hipLaunchKernelGGL(kpe_pattern_deep_kernel<true>, rows, dim3(64), 0, s, dargs);
  } else {
    hipLaunchKernelGGL(kpe_pattern_kernel<false>, grid, dim3(KPE_PAT_BLOCK), 0, s, dargs);
    hipLaunchKernelGGL(kpe_pattern_deep_kernel<false>, rows, dim3(64), 0, s, dargs);
  }
  return hipGetLastError();
}
#endif  // KPE_IN_PART(1)

#endif  // !KPE_SCAN_ONLY

#ifndef KPE_VM_ONLY
extern "C" hipError_t kpe_launch_pred(const PredArgs* a, uint32_t xblocks, hipStream_t s) {
  if (xblocks == 0 || a->njobs == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_pred_kernel, dim3(xblocks, a->njobs), dim3(256), 0, s, *a);
  return hipGetLastError();
}

namespace {
typedef void (*ScanFn)(const ScanArgs*);
// narrow codes: 0 wide, 1 narrow, 2 the LEAN instantiation, | 4: PSUM (scan records, no lists)
ScanFn scan_fn(int pss, int narrow) {
  if (pss && narrow == 2) return kpe_scan_kernel<true, true, false, true>;
  if (pss && (narrow & 4))
    return (narrow & 1) ? kpe_scan_kernel<true, true, false, false, true> : kpe_scan_kernel<true, false, false, false, true>;
  if (pss) return narrow ? kpe_scan_kernel<true, true, false> : kpe_scan_kernel<true, false, false>;
  return narrow ? kpe_scan_kernel<false, true, false> : kpe_scan_kernel<false, false, false>;
}
ScanFn prep_fn(int pss, int narrow) {
  if (pss) return narrow ? kpe_scan_kernel<true, true, true> : kpe_scan_kernel<true, false, true>;
  return narrow ? kpe_scan_kernel<false, true, true> : kpe_scan_kernel<false, false, true>;
}
}  // namespace

// Scan grid: persistent, as many blocks as can be resident at once (occupancy x CUs), capped by
// the number of 256-resource tiles. (The LEAN evaluation, kpe_lean6_kernel, sizes its own grid.)
extern "C" uint32_t kpe_scan_grid(int64_t n, int pss, int narrow, size_t dyn_bytes) {
  if (n <= 0 || (pss && narrow == 7)) return 0;
  static thread_local int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, scan_fn(pss, narrow), kBlock, dyn_bytes) != hipSuccess)
    per_cu = 1;
  const int64_t tiles = (n + kBlock - 1) / kBlock;
  const int64_t g = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
  return (uint32_t)(g < tiles ? g : tiles);
}
// `dargs` is the device copy of the arguments; `n` its row count.
extern "C" hipError_t kpe_launch_scan(const ScanArgs* dargs, const ScanArgs* hargs, int64_t n, int pss, int narrow,
                                      uint32_t grid, size_t dyn_bytes, hipStream_t s) {
  if (n == 0 || grid == 0) return hipSuccess;
  (void)hargs;
  hipLaunchKernelGGL(scan_fn(pss, narrow), dim3(grid), dim3(kBlock), dyn_bytes, s, dargs);
  return hipGetLastError();
}
// ---- selector requirement masks (ScanArgs::selm), once per binding ----------------------------
__device__ __forceinline__ bool sm_bit(const SelMaskArgs& a, uint32_t loc, uint32_t id) {
  if (loc == PRED_NONE || id == KPE_NO_STR) return false;
  const uint32_t w = (loc & PRED_LOCAL) ? a.pimg[(loc & ~PRED_LOCAL) + (id >> 5)] : a.pbuf[loc + (id >> 5)];
  return (w >> (id & 31u)) & 1u;
}
// grid y = 0: label keys (sel_km), 1: label values (sel_vm), 2: namespace rows (ns_q; row nrows:
// no namespace row, i.e. no labels). The namespace rows run eval_term's requirement loop.
__global__ void __launch_bounds__(256) kpe_selmask_kernel(SelMaskArgs a) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (blockIdx.y == 0) {
    if (i >= a.nlabk) return;
    uint64_t km = 0, kok = 0;
    for (uint32_t b = 0; b < a.nrq; ++b) {
      const KpeSelReq q = a.reqs[a.rq[b]];
      km |= sm_bit(a, (uint32_t)q.pk, i) ? 1ull << b : 0ull;
      kok |= q.op == SR_WILD && sm_bit(a, (uint32_t)q.pk_ok, i) ? 1ull << b : 0ull;
    }
    a.km[i] = make_uint4((uint32_t)km, (uint32_t)(km >> 32), (uint32_t)kok, (uint32_t)(kok >> 32));
  } else if (blockIdx.y == 1) {
    if (i >= a.nlabv) return;
    uint64_t vm = 0, vok = 0;
    for (uint32_t b = 0; b < a.nrq; ++b) {
      const KpeSelReq q = a.reqs[a.rq[b]];
      const bool has_pv = q.op == SR_EQ || q.op == SR_IN || q.op == SR_NOTIN || q.op == SR_WILD;
      vm |= has_pv && sm_bit(a, (uint32_t)q.pv, i) ? 1ull << b : 0ull;
      vok |= q.op == SR_WILD && sm_bit(a, (uint32_t)q.pv_ok, i) ? 1ull << b : 0ull;
    }
    a.vm[i] = make_uint4((uint32_t)vm, (uint32_t)(vm >> 32), (uint32_t)vok, (uint32_t)(vok >> 32));
  } else {
    if (i > a.nrows) return;
    const uint32_t lo = i < a.nrows ? a.nsl_off[i] : 0u, hi = i < a.nrows ? a.nsl_off[i + 1] : 0u;
    uint64_t okm = 0;
    for (uint32_t b = 0; b < a.nnq; ++b) {
      const KpeSelReq q = a.reqs[a.nq[b]];
      const bool wild = q.op == SR_WILD;
      bool found = false;
      uint32_t kid = KPE_NO_STR, vid = KPE_NO_STR;
      for (uint32_t j = lo; !found && j < hi; ++j)
        if (sm_bit(a, (uint32_t)q.pk, a.nsl_k[j]) && (!wild || sm_bit(a, (uint32_t)q.pv, a.nsl_v[j])))
          found = true, kid = a.nsl_k[j], vid = a.nsl_v[j];
      bool qok;
      switch (q.op) {
        case SR_EQ:
        case SR_IN: qok = found && sm_bit(a, (uint32_t)q.pv, vid); break;
        case SR_WILD: qok = found && sm_bit(a, (uint32_t)q.pk_ok, kid) && sm_bit(a, (uint32_t)q.pv_ok, vid); break;
        case SR_NOTIN: qok = !found || !sm_bit(a, (uint32_t)q.pv, vid); break;
        case SR_EXISTS: qok = found; break;
        default: qok = !found; break;
      }
      okm |= qok ? 1ull << b : 0ull;
    }
    a.nsq[i] = okm;
  }
}
extern "C" hipError_t kpe_launch_selmask(const SelMaskArgs* a, hipStream_t s) {
  const uint32_t m = std::max(std::max(a->nlabk, a->nlabv), a->nrows + 1);
  hipLaunchKernelGGL(kpe_selmask_kernel, dim3((m + 255u) / 256u, 3), dim3(256), 0, s, *a);
  return hipGetLastError();
}
// The LEAN evaluation of one or more bound shards of one program in one grid (lean.inl).
// tpw: tiles per wave (1, 2 or 4; 4 only with the code bytes in LDS, lc).
extern "C" hipError_t kpe_launch_lean6(const LeanBatchArgs* a, size_t dyn_bytes, int lc, hipStream_t s) {
  const uint32_t grid = a->blk0[a->nshards];
  if (a->nshards == 0 || grid == 0) return hipSuccess;
  const dim3 g(grid), b(kLB);
  if (a->tpw == 4 && lc) hipLaunchKernelGGL((kpe_lean6_kernel<4, true>), g, b, dyn_bytes, s, *a);
  else if (a->tpw == 2 && lc) hipLaunchKernelGGL((kpe_lean6_kernel<2, true>), g, b, dyn_bytes, s, *a);
  else if (a->tpw == 1 && lc) hipLaunchKernelGGL((kpe_lean6_kernel<1, true>), g, b, dyn_bytes, s, *a);
  else if (a->tpw == 2) hipLaunchKernelGGL((kpe_lean6_kernel<2, false>), g, b, dyn_bytes, s, *a);
  else if (a->tpw == 1) hipLaunchKernelGGL((kpe_lean6_kernel<1, false>), g, b, dyn_bytes, s, *a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}
// The PSA dictionary codes of a corpus (lean.inl), one launch.
extern "C" hipError_t kpe_launch_psa_codes(const PsaCodeArgs* a, hipStream_t s) {
  uint32_t m = a->L.ncapsets;
  for (int d = 1; d < 4; ++d) m = std::max(m, a->dict_n[d]);
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_psa_codes_kernel, dim3((m + 255u) / 256u, 4), dim3(256), 0, s, *a);
  return hipGetLastError();
}
// The general scan's per-pod PSA records (lean.inl), one wave per 64-pod tile.
extern "C" hipError_t kpe_launch_psum(const PsumArgs* a, hipStream_t s) {
  if (a->n <= 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_psum_kernel, dim3((a->ntiles + 3u) / 4u), dim3(256), 0, s, *a);
  return hipGetLastError();
}
// One block: the evaluation's prologue image (ScanArgs::pimg).
extern "C" hipError_t kpe_launch_prep(const ScanArgs* dargs, int pss, int narrow, size_t dyn_bytes, hipStream_t s) {
  hipLaunchKernelGGL(prep_fn(pss, narrow), dim3(1), dim3(kBlock), dyn_bytes, s, dargs);
  return hipGetLastError();
}
// Rows past a per-resource encoding limit (Corpus::limit_rows): every cell undecided.
__global__ void __launch_bounds__(256) kpe_fill_rows_kernel(uint8_t* verdicts, uint32_t R, const uint32_t* rows,
                                                            uint32_t nrows, uint8_t value) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (uint64_t)nrows * R) verdicts[(size_t)rows[i / R] * R + i % R] = value;
}
extern "C" hipError_t kpe_launch_fill_rows(uint8_t* verdicts, uint32_t R, const uint32_t* rows, uint32_t nrows,
                                           uint8_t value, hipStream_t s) {
  const uint64_t cells = (uint64_t)nrows * R;
  if (cells == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_fill_rows_kernel, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, s, verdicts, R, rows,
                     nrows, value);
  return hipGetLastError();
}
// applyRules: One (pkg/engine/validation.go:75-77: stop after the first rule whose response is
// pass or fail, RulesAppliedCount) over the final verdicts: cells after an applied rule of the
// policy give no response; after an undecided cell they are undecided (unless unmatched).
__global__ void __launch_bounds__(256) kpe_apply_one_kernel(uint8_t* verdicts, uint32_t* masks, uint32_t n, uint32_t R,
                                                            const uint2* segs, uint32_t nsegs) {
  const uint32_t r = blockIdx.x * 256u + threadIdx.x;
  if (r >= n) return;
  uint8_t* row = verdicts + (size_t)r * R;
#pragma unroll 1
  for (uint32_t s = 0; s < nsegs; ++s) {
    const uint2 sg = segs[s];
    uint32_t state = 0;  // 0 open, 1 applied, 2 an earlier cell undecided
#pragma unroll 1
    for (uint32_t i = sg.x; i < sg.y; ++i) {
      const uint32_t v = row[i];
      if (state == 1u) {
        if (v != KPE_NA_) {
          row[i] = KPE_NA_;
          if (masks) masks[(size_t)r * R + i] = 0u;
        }
      } else if (state == 2u) {
        if (v != KPE_NA_) row[i] = KPE_UNDECIDED_;
      } else if (v == KPE_PASS_ || v == KPE_FAIL_) {
        state = 1u;
      } else if (v == KPE_UNDECIDED_) {
        state = 2u;
      }
    }
  }
}
extern "C" hipError_t kpe_launch_apply_one(uint8_t* verdicts, uint32_t* masks, int64_t n, uint32_t R, const uint32_t* segs,
                                           uint32_t nsegs, hipStream_t s) {
  if (n <= 0 || nsegs == 0) return hipSuccess;
  hipLaunchKernelGGL(kpe_apply_one_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, verdicts, masks,
                     (uint32_t)n, R, reinterpret_cast<const uint2*>(segs), nsegs);
  return hipGetLastError();
}
extern "C" hipError_t kpe_launch_count(const uint8_t* verdicts, int64_t n, uint32_t R, unsigned long long* out,
                                       hipStream_t s) {
  if (R == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(out, 0, (size_t)R * 8 * 8, s);
  if (e != hipSuccess || n == 0) return e;
  const int64_t waves = (n + 63) / 64;
  const uint32_t grid = (uint32_t)std::min<int64_t>((waves + 3) / 4, 1024);
  for (uint32_t r0 = 0; r0 < R; r0 += 1536) {  // <= 48 KiB of LDS histogram per launch
    const uint32_t rn = std::min<uint32_t>(1536, R - r0);
    hipLaunchKernelGGL(kpe_count_kernel, dim3(grid), dim3(256), (size_t)rn * 8 * 4, s, verdicts, n, R, r0, rn, out);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
#endif  // !KPE_VM_ONLY
