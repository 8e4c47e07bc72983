// LEAN scan of kind-matched PSS programs (C2: restricted:latest and its autogen columns), and the
// per-pod PSA summary it reads. Same verdicts as kpe_scan_kernel<PSS, NARROW> (the reference path:
// pkg/engine/engine.go:87-101 validate -> validatePssHandler.Process, validate_pss.go:64-110,
// pkg/pss/evaluate.go:24-70).
//
// Every PSA check of the v0.29 library is "some container / list item of the pod is in state s"
// for fixed, policy-independent sets s (pss_fixed.hpp), so a pod reduces to one summary: the OR
// of its container state bitmaps and of its list items' codes under those sets. The summary is
// built on the device once per corpus (kpe_psa_dict_kernel -> kpe_psa_capset_kernel ->
// kpe_psum_kernel, at the first binding of a LEAN program and again on a cold evaluation), as a
// 12-byte scan record per pod: the pod word and kind id of the pod record beside the pod's
// failing versioned checks (cv_fails of the summary: also policy-independent). An evaluation then
// reads 12 bytes per pod and masks the checks with the program's version classes.
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
__device__ __forceinline__ uint3 bload3(Rsrc r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b96(r, off, 0, 0);
  return make_uint3(v[0], v[1], v[2]);
}
__device__ __forceinline__ uint4 bload4(Rsrc r, uint32_t off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// The arguments are passed by value (read from the kernarg segment: one hop less than a device
// copy before the first load).
__device__ __forceinline__ CArgs* kargs() {
  uint64_t v = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(v));
  return (CArgs*)v;
}

#ifndef KPE_LEAN2_WAVES
#define KPE_LEAN2_WAVES 6
#endif
constexpr uint32_t kLB = 256;
// XCD-aware block order: the dispatcher deals workgroups round-robin to the 8 XCDs (block b on
// XCD b % 8), so block b takes the (b / 8)-th block of XCD b % 8's contiguous share of the tiles:
// neighbouring tiles (whose record lines share L2 sectors) stay on one XCD's L2.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u;
  return x * q + min(x, r) + (b >> 3);
}

// ---- the per-pod PSA summary ---------------------------------------------------------------
// Fixed-set table (PsumArgs::fixed, built on the host from pss_fixed.hpp): entries of
// [set | prefix << 7 | len << 8] then the literal, padded to 4 bytes. A prefix entry is a literal
// followed by one trailing '*' (go-wildcard: a byte-prefix match, pss_fixed.hpp fixed_match).
__device__ __forceinline__ uint32_t psa_sets(const uint8_t* tab, uint32_t tab_len, const uint8_t* s, uint32_t n) {
  uint32_t hit = 0;
  for (uint32_t o = 0; o + 4u <= tab_len;) {
    const uint32_t h = *reinterpret_cast<const uint32_t*>(tab + o);
    const uint32_t set = h & 0x7Fu, prefix = (h >> 7) & 1u, len = h >> 8;
    const uint8_t* lit = tab + o + 4u;
    if (prefix ? n >= len : n == len) {
      bool eq = true;
      for (uint32_t i = 0; i < len && eq; ++i) eq = s[i] == lit[i];
      if (eq) hit |= 1u << set;
    }
    o += 4u + ((len + 3u) & ~3u);
  }
  return hit;
}

// Code byte of every string of the four dictionaries the summary reads (grid y = PSD_*):
//   capabilities: bit 0 baseline-allowed, bit 1 NET_BIND_SERVICE, bit 2 "ALL";
//   sysctls: bit v = outside version v's allowed set (check_sysctls.go v1.0 / v1.27 / v1.29);
//   annotation keys: bit 0 AppArmor container key, bit 1 pod seccomp key;
//   annotation values: bit 0 allowed AppArmor profile, bit 1 allowed seccomp profile.
__global__ void __launch_bounds__(256) kpe_psa_dict_kernel(PsumArgs a) {
  const uint32_t d = blockIdx.y;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= a.dict_n[d]) return;
  const uint32_t* off = a.dict_off[d];
  const uint32_t o0 = off[i], o1 = off[i + 1];
  const uint32_t h = psa_sets(a.fixed, a.fixed_len, a.dict_bytes[d] + o0, o1 - o0);
  uint32_t c = 0;
  if (d == PSD_CAP) {
    c = ((h >> PSF_CAPS_OK) & 1u) | (((h >> PSF_CAP_NBS) & 1u) << 1) | (((h >> PSF_CAP_ALL) & 1u) << 2);
  } else if (d == PSD_SYSCTL) {
    c = (((h >> PSF_SYSCTL0) & 1u) ^ 1u) | ((((h >> PSF_SYSCTL1) & 1u) ^ 1u) << 1) | ((((h >> PSF_SYSCTL2) & 1u) ^ 1u) << 2);
  } else if (d == PSD_ANNK) {
    c = ((h >> PSF_APPARMOR_KEY) & 1u) | (((h >> PSF_SECCOMP_POD_KEY) & 1u) << 1);
  } else {
    c = ((h >> PSF_APPARMOR_OK) & 1u) | (((h >> PSF_SECCOMP_ANN_OK) & 1u) << 1);
  }
  a.codes[d][i] = (uint8_t)c;
}

// Capability-set code byte (CS_* of kernels.hip) of every (add, drop) pair of the corpus's
// capability-set dictionary, from the capability codes (capability ids < 64: a 65th name is a
// per-resource limit).
__global__ void __launch_bounds__(256) kpe_psa_capset_kernel(PsumArgs a) {
  __shared__ uint32_t s_m[6];
  const uint32_t t = threadIdx.x;
  if (t < 6) s_m[t] = 0;
  __syncthreads();
  const uint32_t ncap = min(a.dict_n[PSD_CAP], 64u);
  if (t < ncap) {
    const uint32_t c = a.codes[PSD_CAP][t];
    for (uint32_t k = 0; k < 3; ++k)
      if ((c >> k) & 1u) atomicOr(&s_m[2 * k + (t >> 5)], 1u << (t & 31u));
  }
  __syncthreads();
  const uint64_t ok = s_m[0] | (uint64_t)s_m[1] << 32, nbs = s_m[2] | (uint64_t)s_m[3] << 32,
                 all = s_m[4] | (uint64_t)s_m[5] << 32;
  const uint32_t j = blockIdx.x * 256u + t;
  if (j >= a.ncapsets) return;
  const uint4 cs = reinterpret_cast<const uint4*>(a.capsets)[j];
  const uint64_t ad = cs.x | (uint64_t)cs.y << 32, dr = cs.z | (uint64_t)cs.w << 32;
  a.csb[j] = (uint8_t)(((ad & ~ok) ? CS_BASE : 0u) | ((dr & all) ? 0u : CS_DROP) | ((ad & ~nbs) ? CS_ADD : 0u));
}

// One wave per 64-pod tile: list offsets from the tile header plus a wave scan of the pod
// records' packed counts, then each lane ORs its own pod's items (schema.h PS_* layout). Out: the
// pod's LEAN scan record {pod word, failing versioned checks, kind id << 16} and, when asked
// (PsumArgs::summ), the summary itself {OR of container states, list codes} (schema.h PS_*).
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
  uint32_t xo = 0, co = 0, vc = 0, sc = 0, ac = 0, sa = 0;
  const uint2* crec = reinterpret_cast<const uint2*>(a.crec);
  const uint32_t nsv = a.dict_n[PSD_ANNV];
  for (uint32_t k = 0; k < nc; ++k) {
    const uint2 e = crec[oc + k];
    xo |= e.x;
    if (e.x) co |= a.csb[CY_CAPSET(e.y)];  // a real container record always has state bits
    const uint32_t cs = a.c_sann[oc + k];  // the container's seccomp annotation value (v1.0 check)
    if (cs != KPE_NO_STR) sa |= (cs < nsv ? ((uint32_t)a.codes[PSD_ANNV][cs] >> 1) & 1u : 0u) ^ 1u;
  }
  for (uint32_t k = 0; k < nv; ++k) {
    const uint32_t v = a.vol_src[ov + k];
    vc |= ((v >> VS_HOSTPATH) & 1u) | ((v & kAllowedVolumes) ? 0u : 2u);
  }
  const uint32_t nsys = a.dict_n[PSD_SYSCTL], nak = a.dict_n[PSD_ANNK], nav = a.dict_n[PSD_ANNV];
  for (uint32_t k = 0; k < ns; ++k) {
    const uint32_t id = a.sys_id[os + k];
    sc |= id < nsys ? (uint32_t)a.codes[PSD_SYSCTL][id] : 7u;
  }
  const uint2* kv = reinterpret_cast<const uint2*>(a.pann_kv);
  for (uint32_t k = 0; k < na; ++k) {
    const uint2 q = kv[oa + k];
    const uint32_t ka = q.x < nak ? (uint32_t)a.codes[PSD_ANNK][q.x] : 0u;
    const uint32_t va = q.y < nav ? (uint32_t)a.codes[PSD_ANNV][q.y] : 0u;
    ac |= ((ka & 1u) && !(va & 1u) ? 1u : 0u) | ((ka & 2u) && !(va & 2u) ? 2u : 0u);
  }
  const uint32_t y = co | (vc << 3) | (sc << 5) | (ac << 8) | (sa << 10);
  uint32_t* o = a.psum + 3u * r;
  o[0] = rc.x;
  o[1] = cv_fails(rc.x, xo, PS_CAPS(y), PS_SECANN(y), PS_VOL(y) & 1u, PS_VOL(y) & 2u, PS_SYS(y), PS_ANN(y) & 1u,
                  PS_ANN(y) & 2u);
  o[2] = GVK_KIND(rc.y) << 16;
  if (a.summ) a.summ[2u * r] = xo, a.summ[2u * r + 1u] = y;
}

// ---- kpe_lean5_kernel: the 12-byte scan records only ------------------------------------
// A wave loads one 12-byte record per pod (768 contiguous bytes) in one memory step and
// evaluates with no staging, scans or list loops: the failing checks of the program's classes, the kind
// table, the rows stored as dwords through LDS and, when asked, the check masks.
__global__ void __launch_bounds__(kLB, KPE_LEAN2_WAVES) kpe_lean5_kernel(ScanArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  CArgs& a0 = *kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles, n = (uint32_t)a0.n;
  const uint32_t tile = xcd_block(blockIdx.x, gridDim.x) * (kLB / 64u) + wv;
  const Rsrc PS = make_rsrc(a0.psum, n * 12u);
  const uint32_t r = tile * 64u + lane;
  const uint3 sr = bload3(PS, r * 12u);
  // the kind table and the class table of the prologue image (a few hundred words)
  const uint32_t img_n4 = a0.pimg_words >> 2;
  const uint4* img = reinterpret_cast<const uint4*>(a0.pimg);
  const uint4 img0 = img[min(t, img_n4 - 1u)];
  uint32_t cls_cv = 0, cls_rm = 0;
  if (lane < a0.ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a0.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  {
    uint4* d4 = reinterpret_cast<uint4*>(dyn);
    if (t < img_n4) d4[t] = img0;
#pragma unroll 1
    for (uint32_t i = t + kLB; i < img_n4; i += kLB) d4[i] = img[i];
  }
  __syncthreads();
  if (tile >= ntiles) return;
  const uint32_t R = a0.nrules, cv_union = a0.cv_union, pss_rules = a0.pss_rules, ncls = a0.ncls;
  const uint32_t ep_rules = a0.err_rules | a0.pat_rules, pat_rules = a0.pat_rules;
  uint8_t* sv = reinterpret_cast<uint8_t*>(dyn + a0.wave_lds + wv * a0.wave_words + KPE_STAGE_WORDS);
  const bool live = r < n;
  const uint32_t pw = sr.x, y = sr.z;
  const uint32_t fails = sr.y & cv_union;
  const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
  const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
  const uint32_t matched = dyn[a0.kt_lds + (y >> 16)];
  uint32_t failr;
  if (ncls == 1u) {
    failr = (fails & hw(cls_cv, 0)) ? hw(cls_rm, 0) : 0u;
  } else {
    failr = 0;
#pragma unroll 1
    for (uint32_t c = 0; c < ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
  }
  const uint32_t E = matched & ((err ? pss_rules : 0u) | ep_rules);
  const uint32_t F = (matched & pss_rules & failr & ~E) | (matched & pat_rules);
  const uint32_t P = matched & pss_rules & ~failr & ~E;
#pragma unroll 1
  for (uint32_t ri = 0; ri < R; ++ri)
    sv[lane * R + ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
  if (a0.masks && live) {
    uint32_t* mrow = a0.masks + (size_t)r * R;
    const uint32_t fm = F & pss_rules;
#pragma unroll 1
    for (uint32_t ri = 0; ri < R; ++ri) {
      uint32_t cv = 0;
      for (uint32_t c = 0; c < ncls; ++c) cv = ((hw(cls_rm, c) >> ri) & 1u) ? hw(cls_cv, c) : cv;
      mrow[ri] = ((fm >> ri) & 1u) ? (fails & cv) : 0u;
    }
  }
  __builtin_amdgcn_wave_barrier();
  store_rows(a0.verdicts, sv, tile, R, 0, R, min(64u, n - tile * 64u), lane);
}

typedef const __attribute__((address_space(4))) LeanBatchArgs CBArgs;
// ---- kpe_lean5_batch_kernel: many shards in one launch ---------------------------------------
// The same per-pod evaluation as kpe_lean5_kernel over up to KPE_LEAN_BATCH bound shards of one
// program (each with its own corpus dictionaries, hence its own kind table): the shards' blocks
// are one grid, so a batch of K steps costs one launch and one ramp instead of K. Every block
// finds its shard by a scalar binary search over LeanBatchArgs::blk0 (kernel arguments) and
// stages only that shard's kind table in LDS. A wave takes T tiles of its block's 4T (tiles
// b*4T + 4i + wave): the T record loads are issued together, then the tiles are evaluated and
// stored one by one. One tile per wave leaves a streaming launch bound by the wave launch rate
// (20 shards, 312k waves: 2.9 TB/s).
template <int T>
__global__ void __launch_bounds__(kLB, KPE_LEAN2_WAVES) kpe_lean5_batch_kernel(LeanBatchArgs) {
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
  const __attribute__((address_space(4))) LeanShard& S = a.sh[lo];
  const uint32_t n = S.n, tile0 = (gb - a.blk0[lo]) * (4u * T) + wv;
  const Rsrc PS = make_rsrc(S.psum, n * 12u);
  uint3 sr[T];
#pragma unroll
  for (int i = 0; i < T; ++i) sr[i] = bload3(PS, ((tile0 + 4u * i) * 64u + lane) * 12u);  // past n: zeros
  const uint32_t nk = S.nkinds;
  const uint32_t k0 = t < nk ? S.kt[t] : 0u;
  uint32_t cls_cv = 0, cls_rm = 0;
  const uint32_t ncls = a.ncls;
  if (lane < ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  if (t < nk) dyn[t] = k0;
#pragma unroll 1
  for (uint32_t i = t + kLB; i < nk; i += kLB) dyn[i] = S.kt[i];
  __syncthreads();
  const uint32_t R = a.nrules, cv_union = a.cv_union, pss_rules = a.pss_rules;
  const uint32_t ep_rules = a.err_rules | a.pat_rules, pat_rules = a.pat_rules;
  uint8_t* sv = reinterpret_cast<uint8_t*>(dyn + a.kt_words) + wv * 64u * R;
#pragma unroll
  for (int i = 0; i < T; ++i) {
    const uint32_t tile = tile0 + 4u * i;
    if (tile * 64u >= n) break;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    const uint32_t pw = sr[i].x, y = sr[i].z;
    const uint32_t fails = sr[i].y & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t kind = y >> 16;
    const uint32_t matched = live && kind < nk ? dyn[kind] : 0u;
    uint32_t failr = 0;
#pragma unroll 1
    for (uint32_t c = 0; c < ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
    const uint32_t E = matched & ((err ? pss_rules : 0u) | ep_rules);
    const uint32_t F = (matched & pss_rules & failr & ~E) | (matched & pat_rules);
    const uint32_t P = matched & pss_rules & ~failr & ~E;
    __builtin_amdgcn_wave_barrier();  // the previous tile's rows are out of the staging area
#pragma unroll 1
    for (uint32_t ri = 0; ri < R; ++ri)
      sv[lane * R + ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
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
