// LEAN evaluation of kind-matched PSS programs (C2: restricted:latest and its autogen columns), the
// PSA dictionary codes it reads, and the general scan's per-pod PSA records. Same verdicts as
// kpe_scan_kernel<PSS, NARROW> (the reference path: pkg/engine/engine.go:87-101 validate ->
// validatePssHandler.Process, validate_pss.go:64-110, pkg/pss/evaluate.go:24-70).
//
// Every PSA check of the v0.29 library is "some container / list item of the pod is in state s"
// for fixed, policy-independent sets s (pss_fixed.hpp). A pod's checks are therefore decided from
// the OR of its containers' state bitmaps and of its list items' codes under those sets. The codes
// belong to the corpus's dictionaries (one byte per distinct capability set, sysctl name and
// annotation key / value: kpe_psa_codes_kernel, once per corpus, like the interned ids
// themselves); everything per pod is read and decided by every evaluation (kpe_lean6_kernel).
// Included by kernels.hip (uses its anonymous-namespace helpers).

typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint32_t bload1(Rsrc r, uint32_t off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
__device__ __forceinline__ uint2 bload2(Rsrc r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_uint2(v[0], v[1]);
}
__device__ __forceinline__ uint4 bload4(Rsrc r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// The kernel arguments, read from the kernarg segment through a laundered pointer (one hop less
// than a device copy before the first load).
__device__ __forceinline__ const __attribute__((address_space(4))) void* kargs() {
  uint64_t v = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(v));
  return (const __attribute__((address_space(4))) void*)v;
}

#ifndef KPE_LEAN6_WAVES
#define KPE_LEAN6_WAVES 6
#endif
constexpr uint32_t kLB = 256;
// XCD-aware block order: the dispatcher deals workgroups round-robin to the 8 XCDs (block b on
// XCD b % 8), so block b takes the (b / 8)-th block of XCD b % 8's contiguous share of the tiles:
// neighbouring tiles (whose list items share cache lines) stay on one XCD's L2.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u;
  return x * q + min(x, r) + (b >> 3);
}

// ---- PSA dictionary codes (once per corpus) -----------------------------------------------------
// Four bytes of s from p on (any alignment): two aligned dword loads and a shift. Dictionary
// buffers carry 128 bytes of slack past their end (kpe_api.cpp upload).
__device__ __forceinline__ uint32_t ld4u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint64_t v = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  return (uint32_t)(v >> ((a & 3u) * 8u));
}
// Set-hit word of string s (n bytes): bit k = s matches a glob of fixed set k. Exact entries are
// bucketed by length, so a string is compared only with the literals of its own length, then with
// the few prefix entries; literals are compared four bytes per step from the LDS-staged table
// (layout in kernels_abi.h).
__device__ __forceinline__ uint32_t psa_sets(const uint32_t* fx, const uint8_t* s, uint32_t n) {
  auto eq = [&](uint32_t e, uint32_t len) -> bool {
    const uint32_t lit = fx[KPE_PSF_ENT0 + 2u * e + 1u];
    for (uint32_t i = 0; i < len; i += 4u) {
      const uint32_t m = len - i >= 4u ? ~0u : (1u << (8u * (len - i))) - 1u;
      if ((ld4u(s + i) ^ fx[lit + (i >> 2)]) & m) return false;
    }
    return true;
  };
  uint32_t hit = 0;
  if (n < KPE_PSF_MAXLEN) {
    const uint32_t rg = fx[2u + n];
    for (uint32_t e = rg & 0xFFFFu; e < (rg >> 16); ++e)
      if (eq(e, n)) hit |= 1u << (fx[KPE_PSF_ENT0 + 2u * e] & 0x7Fu);
  }
  const uint32_t E = fx[0], X = fx[1];
  for (uint32_t e = E; e < E + X; ++e) {
    const uint32_t h = fx[KPE_PSF_ENT0 + 2u * e], len = h >> 8;
    if (n >= len && eq(e, len)) hit |= 1u << (h & 0x7Fu);
  }
  return hit;
}
#define KPE_PSF_LDS_WORDS 1024u
// One launch: grid y = 0 capability sets (each block first codes the capability names, ids < 64),
// 1 sysctls, 2 annotation keys, 3 annotation values (PSD_*); one thread per entry.
__global__ void __launch_bounds__(256) kpe_psa_codes_kernel(PsaCodeArgs a) {
  __shared__ uint32_t fx[KPE_PSF_LDS_WORDS];
  __shared__ uint32_t s_m[6];
  const uint32_t t = threadIdx.x, y = blockIdx.y;
  for (uint32_t i = t; i < a.fixed_words; i += 256u) fx[i] = a.fixed[i];
  if (t < 6) s_m[t] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * 256u + t;
  if (y == 0) {
    const uint32_t ncap = min(a.dict_n[PSD_CAP], 64u);
    if (t < ncap) {
      const uint32_t o0 = a.dict_off[PSD_CAP][t], o1 = a.dict_off[PSD_CAP][t + 1];
      const uint32_t h = psa_sets(fx, a.dict_bytes[PSD_CAP] + o0, o1 - o0);
      const uint32_t c = ((h >> PSF_CAPS_OK) & 1u) | (((h >> PSF_CAP_NBS) & 1u) << 1) | (((h >> PSF_CAP_ALL) & 1u) << 2);
      for (uint32_t k = 0; k < 3; ++k)
        if ((c >> k) & 1u) atomicOr(&s_m[2 * k + (t >> 5)], 1u << (t & 31u));
    }
    __syncthreads();
    if (i >= a.L.ncapsets) return;
    const uint64_t ok = s_m[0] | (uint64_t)s_m[1] << 32, nbs = s_m[2] | (uint64_t)s_m[3] << 32,
                   all = s_m[4] | (uint64_t)s_m[5] << 32;
    const uint4 cs = reinterpret_cast<const uint4*>(a.capsets)[i];
    const uint64_t ad = cs.x | (uint64_t)cs.y << 32, dr = cs.z | (uint64_t)cs.w << 32;
    a.codes[i] = (uint8_t)(((ad & ~ok) ? CS_BASE : 0u) | ((dr & all) ? 0u : CS_DROP) | ((ad & ~nbs) ? CS_ADD : 0u));
    return;
  }
  if (i >= a.dict_n[y]) return;
  const uint32_t o0 = a.dict_off[y][i], o1 = a.dict_off[y][i + 1];
  const uint32_t h = psa_sets(fx, a.dict_bytes[y] + o0, o1 - o0);
  uint32_t c, at;
  if (y == PSD_SYSCTL) {
    c = (((h >> PSF_SYSCTL0) & 1u) ^ 1u) | ((((h >> PSF_SYSCTL1) & 1u) ^ 1u) << 1) | ((((h >> PSF_SYSCTL2) & 1u) ^ 1u) << 2);
    at = a.L.o_sys;
  } else if (y == PSD_ANNK) {
    c = ((h >> PSF_APPARMOR_KEY) & 1u) | (((h >> PSF_SECCOMP_POD_KEY) & 1u) << 1);
    at = a.L.o_annk;
  } else {
    c = ((h >> PSF_APPARMOR_OK) & 1u) | (((h >> PSF_SECCOMP_ANN_OK) & 1u) << 1);
    at = a.L.o_annv;
  }
  a.codes[at + i] = (uint8_t)c;
}

// Code of one list item from the corpus's code bytes (`cb`: LDS or global), shared by the LEAN
// evaluation and the general scan's per-pod records. Branch-free: every code byte is read at an
// index clamped into the code table (the part's pad byte stands in for an id past the part) and
// the result selected afterwards, so no lane waits on a divergent load.
struct PsaCoder {
  const PsaCodes& L;
  // capability-set code of a container record (0 for an empty slot: no state bits)
  template <class CB>
  __device__ __forceinline__ uint32_t cap(const CB& cb, uint2 e) const {
    const uint32_t c = cb(CY_CAPSET(e.y)) & 7u;  // a real record's set id is < ncapsets; a zero slot reads set 0
    return e.x ? c : 0u;
  }
  // a container's seccomp annotation value (check_seccompProfile v1.0): 1 when set and not allowed
  template <class CB>
  __device__ __forceinline__ uint32_t sann(const CB& cb, uint32_t cs) const {
    const uint32_t v = cb(L.o_annv + min(cs, L.nannv));
    const uint32_t ok = cs < L.nannv ? (v >> 1) & 1u : 0u;
    return cs == KPE_NO_STR ? 0u : ok ^ 1u;
  }
  template <class CB>
  __device__ __forceinline__ uint32_t sys(const CB& cb, uint32_t id) const {
    const uint32_t v = cb(L.o_sys + min(id, L.nsysd));
    return id < L.nsysd ? v : 7u;
  }
  template <class CB>
  __device__ __forceinline__ uint32_t ann(const CB& cb, uint2 q) const {
    const uint32_t k = cb(L.o_annk + min(q.x, L.nannk)), v = cb(L.o_annv + min(q.y, L.nannv));
    const uint32_t ka = q.x < L.nannk ? k : 0u, va = q.y < L.nannv ? v : 0u;
    return ka & ~va & 3u;  // bit 0 AppArmor key with a disallowed profile, bit 1 pod seccomp key likewise
  }
};
__device__ __forceinline__ uint32_t vol_code(uint32_t v) {
  return ((v >> VS_HOSTPATH) & 1u) | ((v & kAllowedVolumes) ? 0u : 2u);
}

// ---- kpe_psum_kernel: the general scan's per-pod PSA records ----------------------------------
// One wave per 64-pod tile: list offsets from the tile header plus a wave scan of the pod
// records' packed counts, then each lane ORs its own pod's items. Out: {pod word, failing
// versioned checks, kind id << 16} per pod and, when asked (PsumArgs::summ), the summary {OR of
// container states, list codes} (schema.h PS_*). Launched by every evaluation of a podSecurity
// program that takes the general scan, right before it.
__global__ void __launch_bounds__(256) kpe_psum_kernel(PsumArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t tile = blockIdx.x * 4u + (threadIdx.x >> 6);
  if (tile >= a.ntiles) return;
  const uint32_t r = tile * 64u + lane;
  const bool live = r < (uint32_t)a.n;
  const uint32_t h = a.hdr[tile * 4u + (lane & 3u)];
  const uint4 rc = live ? reinterpret_cast<const uint4*>(a.rec)[r] : make_uint4(0u, 0u, 0u, 0u);
  const uint32_t z = rc.z;
  const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
  const uint32_t c01 = nc | (nv << 16), c23 = ns | (na << 16);
  const uint32_t e01 = wave_incl_scan(c01) - c01, e23 = wave_incl_scan(c23) - c23;
  const uint32_t oc = hw(h, 0) + (e01 & 0xFFFFu), ov = hw(h, 1) + (e01 >> 16), os = hw(h, 2) + (e23 & 0xFFFFu),
                 oa = hw(h, 3) + (e23 >> 16);
  if (!live) return;
  const PsaCoder K{a.L};
  const uint8_t* codes = a.codes;
  auto cb = [&](uint32_t i) -> uint32_t { return codes[i]; };
  uint32_t xo = 0, co = 0, vc = 0, sc = 0, ac = 0, sa = 0;
  const uint2* crec = reinterpret_cast<const uint2*>(a.crec);
  for (uint32_t k = 0; k < nc; ++k) {
    const uint2 e = crec[oc + k];
    xo |= e.x;
    co |= K.cap(cb, e);
    sa |= K.sann(cb, a.c_sann[oc + k]);
  }
  for (uint32_t k = 0; k < nv; ++k) vc |= vol_code(a.vol_src[ov + k]);
  for (uint32_t k = 0; k < ns; ++k) sc |= K.sys(cb, a.sys_id[os + k]);
  const uint2* kv = reinterpret_cast<const uint2*>(a.pann_kv);
  for (uint32_t k = 0; k < na; ++k) ac |= K.ann(cb, kv[oa + k]);
  const uint32_t y = co | (vc << 3) | (sc << 5) | (ac << 8) | (sa << 10);
  uint32_t* o = a.psum + 3u * r;
  o[0] = rc.x;
  o[1] = cv_fails(rc.x, xo, PS_CAPS(y), PS_SECANN(y), PS_VOL(y) & 1u, PS_VOL(y) & 2u, PS_SYS(y), PS_ANN(y) & 1u,
                  PS_ANN(y) & 2u);
  o[2] = GVK_KIND(rc.y) << 16;
  if (a.summ) a.summ[2u * r] = xo, a.summ[2u * r + 1u] = y;
}

// ---- kpe_lean6_kernel: the LEAN evaluation, one or many shards per launch ----------------------
// A wave evaluates T consecutive 64-pod tiles of its block's shard (blocks find their shard by a
// scalar binary search over LeanBatchArgs::blk0). Two dependent memory steps per wave:
//   1. the T + 1 tile headers (one dword per lane) and the T tiles' pod records (16 B per lane);
//   2. every tile's list items, cooperatively and coalesced: lane i loads container i and 64 + i
//      of the tile (crec, and c_sann when a v1.0 seccomp check runs), volumes i and 64 + i,
//      sysctl i and annotation i, from the tile's first item (header) on.
// Then per tile: lane i codes its staged items (capability-set / sysctl / annotation codes from
// the corpus's code bytes, LDS-staged per block when they fit: LC) into the wave's LDS stage, each
// pod ORs its own items from there (its offsets: one wave scan of the packed list counts), pods
// with more items than the clamped reads cover (or items past the stage) loop over the rest, the
// PSA checks are decided (cv_fails), masked by the program's version classes and the kind table,
// and the tile's rows are stored as dwords through LDS (with the failing versioned checks per
// cell in the masks mode).
typedef const __attribute__((address_space(4))) LeanBatchArgs CBArgs;
typedef const __attribute__((address_space(4))) LeanShard CShard;
struct L6Items {
  uint2 c0, c1, q0;
  uint32_t v0, v1, s0, a0, a1;
};
template <int T, bool LC>
__global__ void __launch_bounds__(kLB, KPE_LEAN6_WAVES) kpe_lean6_kernel(LeanBatchArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  CBArgs& a = *(CBArgs*)kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t gb = xcd_block(blockIdx.x, gridDim.x);
  uint32_t lo = 0, hi = a.nshards;  // blk0[lo] <= gb < blk0[hi]
  while (hi - lo > 1u) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a.blk0[mid] <= gb) lo = mid;
    else hi = mid;
  }
  CShard& S = a.sh[lo];
  const uint32_t n = S.n, ntiles = (n + 63u) >> 6;
  const uint32_t tile0 = ((gb - a.blk0[lo]) * 4u + wv) * (uint32_t)T;
  const uint32_t need = a.need;
  // columns a program does not read get zero-length descriptors: their loads return 0 and move
  // no data (so do loads past a column's end)
  const Rsrc REC = make_rsrc(S.rec, n * 16u), HDR = make_rsrc(S.hdr, (ntiles + 1u) * 16u);
  const Rsrc CREC = make_rsrc(S.crec, S.nctr * 8u);
  const Rsrc SAN = make_rsrc(S.sann, (need & NEED_SANN) ? S.nctr * 4u : 0u);
  const Rsrc VOL = make_rsrc(S.vol, (need & NEED_VOL) ? S.nvol * 4u : 0u);
  const Rsrc SYS = make_rsrc(S.sys, (need & NEED_SYS) ? S.nsys * 4u : 0u);
  const Rsrc ANN = make_rsrc(S.pann, (need & NEED_PANN) ? S.npann * 8u : 0u);
  // ---- step 1: headers (lane k: word k of hdr[tile0 + k / 4]; past the sentinel: 0), records
  const uint32_t hall = bload1(HDR, (tile0 * 4u + min(lane, 4u * T + 3u)) * 4u);
  uint4 rec[T];
#pragma unroll
  for (int j = 0; j < T; ++j) rec[j] = bload4(REC, ((tile0 + j) * 64u + lane) * 16u);  // past n: zeros
  // the block's kind table and (LC) code bytes, for the LDS below
  const uint32_t nk = S.nkinds;
  const uint32_t k0 = t < nk ? S.kt[t] : 0u;
  const uint32_t ncw = LC ? (S.L.bytes + 3u) >> 2 : 0u;
  const uint32_t* gcw = reinterpret_cast<const uint32_t*>(S.codes);
  const uint32_t cw0 = LC && t < ncw ? gcw[t] : 0u;
  // ---- step 2: the list items of every tile
  L6Items it[T];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    if (tile0 + j >= ntiles) break;
    const uint32_t C0 = hw(hall, 4u * j), V0 = hw(hall, 4u * j + 1u), S0 = hw(hall, 4u * j + 2u),
                   A0 = hw(hall, 4u * j + 3u);
    it[j].c0 = bload2(CREC, (C0 + lane) * 8u);
    it[j].c1 = bload2(CREC, (C0 + 64u + lane) * 8u);
    it[j].a0 = bload1(SAN, (C0 + lane) * 4u);
    it[j].a1 = bload1(SAN, (C0 + 64u + lane) * 4u);
    it[j].v0 = bload1(VOL, (V0 + lane) * 4u);
    it[j].v1 = bload1(VOL, (V0 + 64u + lane) * 4u);
    it[j].s0 = bload1(SYS, (S0 + lane) * 4u);
    it[j].q0 = bload2(ANN, (A0 + lane) * 8u);
  }
  if (t < nk) dyn[t] = k0;
#pragma unroll 1
  for (uint32_t i = t + kLB; i < nk; i += kLB) dyn[i] = S.kt[i];
  uint32_t* const cl = dyn + a.kt_words;
  if (LC) {
    if (t < ncw) cl[t] = cw0;
#pragma unroll 1
    for (uint32_t i = t + kLB; i < ncw; i += kLB) cl[i] = gcw[i];
  }
  uint32_t cls_cv = 0, cls_rm = 0;
  const uint32_t ncls = a.ncls;
  if (lane < ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  __syncthreads();
  const uint8_t* const lcodes = reinterpret_cast<const uint8_t*>(cl);
  const uint8_t* const gcodes = S.codes;
  auto cb = [&](uint32_t i) -> uint32_t { return LC ? (uint32_t)lcodes[i] : (uint32_t)gcodes[i]; };
  PsaCodes L;
  L.ncapsets = S.L.ncapsets, L.nsysd = S.L.nsysd, L.nannk = S.L.nannk, L.nannv = S.L.nannv;
  L.o_sys = S.L.o_sys, L.o_annk = S.L.o_annk, L.o_annv = S.L.o_annv, L.bytes = S.L.bytes;
  const PsaCoder K{L};
  const bool nsann = need & NEED_SANN, nvol = need & NEED_VOL, nsys = need & NEED_SYS, npann = need & NEED_PANN;
  auto ctr_code = [&](uint2 e, uint32_t cs) -> uint2 {  // a real container record always has state bits
    const uint32_t sa = nsann ? K.sann(cb, cs) << 3 : 0u;
    return make_uint2(e.x, K.cap(cb, e) | (e.x ? sa : 0u));
  };
  const uint32_t R = a.nrules, cv_union = a.cv_union, pss_rules = a.pss_rules;
  const uint32_t ep_rules = a.err_rules | a.pat_rules, pat_rules = a.pat_rules;
  uint8_t* const stg = reinterpret_cast<uint8_t*>(cl + a.code_words + wv * a.wave_words);
  uint2* const sc = reinterpret_cast<uint2*>(stg);
  uint8_t* const sbv = stg + 8u * KPE_L6_CTR;
  uint8_t* const sbs = sbv + KPE_L6_VOL;
  uint8_t* const sba = sbs + KPE_L6_SMALL;
  uint8_t* const sv = sba + KPE_L6_SMALL;  // the tile's verdict rows (64 x R bytes)
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t tile = tile0 + j;
    if (tile >= ntiles) break;
    const L6Items& d = it[j];
    const uint32_t C0 = hw(hall, 4u * j), V0 = hw(hall, 4u * j + 1u), S0 = hw(hall, 4u * j + 2u),
                   A0 = hw(hall, 4u * j + 3u);
    const uint32_t nct = hw(hall, 4u * j + 4u) - C0, nvt = hw(hall, 4u * j + 5u) - V0,
                   nst = hw(hall, 4u * j + 6u) - S0, nat = hw(hall, 4u * j + 7u) - A0;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    // the pod's item offsets: exclusive wave scans of its packed counts
    const uint32_t z = rec[j].z;  // 0 for rows past n
    const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
    uint32_t oc, ov, os, oa;
    if ((nct | nvt | nst | nat) < 256u) {  // one scan of the four packed byte counts (no carries)
      const uint32_t e = wave_incl_scan(z) - z;
      oc = e & 0xFFu, ov = (e >> 8) & 0xFFu, os = (e >> 16) & 0xFFu, oa = e >> 24;
    } else {
      const uint32_t c01 = nc | (nv << 16), c23 = ns | (na << 16);
      const uint32_t e01 = wave_incl_scan(c01) - c01, e23 = wave_incl_scan(c23) - c23;
      oc = e01 & 0xFFFFu, ov = e01 >> 16, os = e23 & 0xFFFFu, oa = e23 >> 16;
    }
    // stage the codes of the loaded slots (slots past the tile's items hold codes of the next
    // tile's items, or of zeros past a column's end, that no pod reads)
    __builtin_amdgcn_wave_barrier();  // the previous tile's stage reads are done
    sc[lane] = ctr_code(d.c0, d.a0);
    sc[lane + 64u] = ctr_code(d.c1, d.a1);
    if (nvol) sbv[lane] = (uint8_t)vol_code(d.v0), sbv[lane + 64u] = (uint8_t)vol_code(d.v1);
    if (nsys && nst) sbs[lane] = (uint8_t)K.sys(cb, d.s0);
    if (npann && nat) sba[lane] = (uint8_t)K.ann(cb, d.q0);
    __builtin_amdgcn_wave_barrier();
    // each pod ORs its first items with clamped reads (a repeated item does not change an OR)
    uint32_t xo, co, vcode = 0, scode = 0, acode = 0;
    {
      const uint32_t last = min(oc + (nc ? nc - 1u : 0u), KPE_L6_CTR - 1u);
      const uint2 e0 = sc[min(oc, last)], e1 = sc[min(oc + 1u, last)], e2 = sc[min(oc + 2u, last)],
                  e3 = sc[min(oc + 3u, last)];
      const uint32_t m = nc ? ~0u : 0u;
      xo = (e0.x | e1.x | e2.x | e3.x) & m;
      co = (e0.y | e1.y | e2.y | e3.y) & m;
    }
    if (nvol) {
      const uint32_t last = min(ov + (nv ? nv - 1u : 0u), KPE_L6_VOL - 1u);
      const uint32_t x = (uint32_t)sbv[min(ov, last)] | sbv[min(ov + 1u, last)] | sbv[min(ov + 2u, last)] |
                         sbv[min(ov + 3u, last)];
      vcode = nv ? x : 0u;
    }
    if (nsys && nst) {
      const uint32_t last = min(os + (ns ? ns - 1u : 0u), KPE_L6_SMALL - 1u);
      const uint32_t x = (uint32_t)sbs[min(os, last)] | sbs[min(os + 1u, last)];
      scode = ns ? x : 0u;
    }
    if (npann && nat) {
      const uint32_t last = min(oa + (na ? na - 1u : 0u), KPE_L6_SMALL - 1u);
      const uint32_t x = (uint32_t)sba[min(oa, last)] | sba[min(oa + 1u, last)];
      acode = na ? x : 0u;
    }
    // pods with more items than that, or items past the stage: recomputed over all their items
    // (staged ones from LDS, the rest loaded)
    const bool tile_over = nct > KPE_L6_CTR || (nvol && nvt > KPE_L6_VOL) || (nsys && nst > KPE_L6_SMALL) ||
                           (npann && nat > KPE_L6_SMALL);
    const bool more_c = nc > 4u, more_v = nvol && nv > 4u, more_s = nsys && ns > 2u, more_a = npann && na > 2u;
    if (tile_over || __builtin_amdgcn_ballot_w64(more_c || more_v || more_s || more_a)) {
      if (more_c || oc + nc > KPE_L6_CTR) {
        xo = co = 0;
        for (uint32_t k = oc; k < oc + nc; ++k) {
          const uint2 e = k < KPE_L6_CTR ? sc[k]
                                         : ctr_code(bload2(CREC, (C0 + k) * 8u), nsann ? bload1(SAN, (C0 + k) * 4u) : 0u);
          xo |= e.x, co |= e.y;
        }
      }
      if (nvol && (more_v || ov + nv > KPE_L6_VOL)) {
        vcode = 0;
        for (uint32_t k = ov; k < ov + nv; ++k)
          vcode |= k < KPE_L6_VOL ? (uint32_t)sbv[k] : vol_code(bload1(VOL, (V0 + k) * 4u));
      }
      if (nsys && (more_s || os + ns > KPE_L6_SMALL)) {
        scode = 0;
        for (uint32_t k = os; k < os + ns; ++k)
          scode |= k < KPE_L6_SMALL ? (uint32_t)sbs[k] : K.sys(cb, bload1(SYS, (S0 + k) * 4u));
      }
      if (npann && (more_a || oa + na > KPE_L6_SMALL)) {
        acode = 0;
        for (uint32_t k = oa; k < oa + na; ++k)
          acode |= k < KPE_L6_SMALL ? (uint32_t)sba[k] : K.ann(cb, bload2(ANN, (A0 + k) * 8u));
      }
    }
    // ---- the PSA checks, the rule match (kind table) and the verdict bytes ----
    const uint32_t pw = rec[j].x;
    const uint32_t fails =
        cv_fails(pw, xo, co & 7u, (co >> 3) & 1u, vcode & 1u, vcode & 2u, scode, acode & 1u, acode & 2u) & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t kind = GVK_KIND(rec[j].y);
    const uint32_t matched = live && kind < nk ? dyn[kind] : 0u;
    uint32_t failr = 0;
    if (ncls <= 4u) {  // the usual few version classes: no loop
#pragma unroll
      for (uint32_t c = 0; c < 4u; ++c)
        failr |= (c < ncls && (fails & hw(cls_cv, c))) ? hw(cls_rm, c) : 0u;
    } else {
#pragma unroll 1
      for (uint32_t c = 0; c < ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
    }
    const uint32_t E = matched & ((err ? pss_rules : 0u) | ep_rules);
    const uint32_t F = (matched & pss_rules & failr & ~E) | (matched & pat_rules);  // F|E = PENDING
    const uint32_t P = matched & pss_rules & ~failr & ~E;
    if (R <= 4u) {  // (C2: R = 3) the row's bytes without a loop
#pragma unroll
      for (uint32_t ri = 0; ri < 4u; ++ri)
        if (ri < R)
          sv[lane * R + ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
    } else {
#pragma unroll 1
      for (uint32_t ri = 0; ri < R; ++ri)
        sv[lane * R + ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
    }
    if (S.masks && live) {
      uint32_t* mrow = S.masks + (size_t)r * R;
      const uint32_t fm = F & pss_rules;
#pragma unroll 1
      for (uint32_t ri = 0; ri < R; ++ri) {
        uint32_t cv = 0;
        for (uint32_t c = 0; c < ncls; ++c) cv = ((hw(cls_rm, c) >> ri) & 1u) ? hw(cls_cv, c) : cv;
        mrow[ri] = ((fm >> ri) & 1u) ? (fails & cv) : 0u;
      }
    }
    __builtin_amdgcn_wave_barrier();
    store_rows(S.verdicts, sv, tile, R, 0, R, min(64u, n - tile * 64u), lane);
  }
}
