// LEAN scan (kpe_lean_kernel): the resource scan of a PSS program whose match terms are all
// kind predicates, with the prologue image ready in HBM and no check masks (C2: restricted:latest
// and its autogen columns). Same verdicts as kpe_scan_kernel<PSS, NARROW> (the reference path:
// pkg/engine/engine.go:87-101 validate -> validatePssHandler.Process, validate_pss.go:64-110,
// pkg/pss/evaluate.go:24-70), restructured for instruction count:
//  * every column is read through a raw buffer descriptor: 32-bit byte offsets, and loads past
//    a column's end return 0 (hardware range check) instead of being clamped per lane, so a
//    tile's loads cost one address op each;
//  * a pod ORs its first few staged list items with fixed clamped LDS reads (no loop); a loop
//    runs only for the items past them, when some pod of the wave has more;
//  * the matched-rule mask is one kind-table read, the fixed PSA predicates direct LDS reads.
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

struct LeanCols {
  Rsrc rec, hdr, crec, vol, sys, ann;
};
struct LeanTile {
  uint32_t h;   // header words of the tile and the next (lane k < 8: word k)
  uint32_t hn;  // header of the tile this buffer loads next (three steps later)
  uint4 rec;
  uint2 c0, c1, q0;
  uint32_t v0, v1, s0;
};
__device__ __forceinline__ void pin_lean(LeanTile& d) {
  pin(d.h), pin(d.rec), pin(d.c0), pin(d.c1), pin(d.q0), pin(d.v0), pin(d.v1), pin(d.s0);
}
// header words of tiles `tile` and `tile + 1` (lane k < 8: word k)
__device__ __forceinline__ uint32_t lean_hdr(const LeanCols& L, uint32_t tile, uint32_t lane) {
  return bload1(L.hdr, (tile * 4u + (lane & 7u)) * 4u);
}
// A tile's loads: pod records per lane, list items cooperatively (lane i: items base + i and
// base + 64 + i). Items past the tile's range belong to the next tiles or read 0 past the
// column's end; they are never used.
__device__ __forceinline__ LeanTile lean_load(const LeanCols& L, uint32_t tile, uint32_t h, uint32_t lane) {
  LeanTile d;
  const uint32_t C0 = hw(h, 0), V0 = hw(h, 1), S0 = hw(h, 2), A0 = hw(h, 3);
  d.h = h;
  d.rec = bload4(L.rec, (tile * 64u + lane) * 16u);
  d.c0 = bload2(L.crec, (C0 + lane) * 8u);
  d.c1 = bload2(L.crec, (C0 + 64u + lane) * 8u);
  d.v0 = bload1(L.vol, (V0 + lane) * 4u);
  d.v1 = bload1(L.vol, (V0 + 64u + lane) * 4u);
  d.s0 = bload1(L.sys, (S0 + lane) * 4u);
  d.q0 = bload2(L.ann, (A0 + lane) * 8u);
  return d;
}

#ifndef KPE_LEAN2_WAVES
#define KPE_LEAN2_WAVES 6
#endif
// The arguments are passed by value (read from the kernarg segment: one hop less than a device
// copy before the first header load); re-read through a laundered pointer per tile.
__device__ __forceinline__ CArgs* kargs() {
  uint64_t v = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(v));
  return (CArgs*)v;
}
__global__ void __launch_bounds__(kBlock, KPE_LEAN2_WAVES) kpe_lean_kernel(ScanArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  if (KPE_DIAG & DIAG_EMPTY) return;
  CArgs& a0 = *kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles, n = (uint32_t)a0.n;
  const uint32_t W = gridDim.x * (kBlock / 64u);
  uint32_t tile = blockIdx.x * (kBlock / 64u) + wv;
  const uint32_t need = a0.need;
  // columns a program does not read get zero-length descriptors: their loads return 0
  LeanCols L;
  L.rec = make_rsrc(a0.rec, n * 16u);
  L.hdr = make_rsrc(a0.hdr, (ntiles + 1u) * 16u);
  L.crec = make_rsrc(a0.crec, a0.nctr_total * 8u);
  L.vol = make_rsrc(a0.vol_src, (need & NEED_VOL) ? a0.nvol_total * 4u : 0u);
  L.sys = make_rsrc(a0.sys_id, (need & NEED_SYS) ? a0.nsys_total * 4u : 0u);
  L.ann = make_rsrc(a0.pann_kv, (need & NEED_PANN) ? a0.npann_total * 8u : 0u);
  const bool nvol = need & NEED_VOL, nsys = need & NEED_SYS, npann = need & NEED_PANN;

  // ---- Loads run two tiles ahead of the evaluation: step s evaluates tile s while the items
  // of tiles s + 1 and s + 2 and the header of tile s + 3 are in flight. Issue order per step:
  // header s + 3, then items s + 2 (which wait for header s + 2, issued one step earlier before
  // items s + 1), so the only wait of a step leaves items s + 1, s + 2 and header s + 3 in flight.
  // Prologue: headers 0, 1, 2; the image; items 0 and 1.
  const uint32_t h0 = lean_hdr(L, tile, lane);
  const uint32_t h1 = lean_hdr(L, tile + W, lane);
  const uint32_t h2 = lean_hdr(L, tile + 2u * W, lane);
  const uint32_t img_n4 = a0.pimg_words >> 2;
  const uint4* img = reinterpret_cast<const uint4*>(a0.pimg);
  const uint4 img0 = img[min(t, img_n4 - 1u)];
  uint32_t cls_cv = 0, cls_rm = 0;  // (check set, rules failing on it) per PSS version class
  if (lane < a0.ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a0.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  LeanTile ta = lean_load(L, tile, h0, lane);
  LeanTile tb = lean_load(L, tile + W, h1, lane);
  LeanTile tc{};
  tc.hn = h2;
  {
    uint4* d4 = reinterpret_cast<uint4*>(dyn);
    if (t < img_n4) d4[t] = img0;
#pragma unroll 1
    for (uint32_t i = t + kBlock; i < img_n4; i += kBlock) d4[i] = img[i];
  }
  __syncthreads();
  if (KPE_DIAG & DIAG_NOLOOP) {
    if (tile < ntiles && lane == 0) a0.verdicts[tile] = (uint8_t)(dyn[0] + ta.rec.x + tb.rec.x);
    return;
  }
  const uint8_t* s_capb = reinterpret_cast<const uint8_t*>(dyn + a0.capb_lds);
  const LdsPtr lds = (LdsPtr)dyn;
  const uint32_t p_sann = a0.pp_seccomp_ann_ok & ~PRED_LOCAL, p_aak = a0.pp_apparmor_key & ~PRED_LOCAL,
                 p_aao = a0.pp_apparmor_ok & ~PRED_LOCAL, p_spk = a0.pp_seccomp_pod_key & ~PRED_LOCAL,
                 p_s0 = a0.pp_sysctl0 & ~PRED_LOCAL, p_s1 = a0.pp_sysctl1 & ~PRED_LOCAL,
                 p_s2 = a0.pp_sysctl2 & ~PRED_LOCAL;
  auto pbit = [&](uint32_t loc, uint32_t id) -> uint32_t { return (lds[loc + (id >> 5)] >> (id & 31u)) & 1u; };
  const uint32_t kt = a0.kt_lds;

  // per-kernel constants (scalar registers)
  const uint32_t R = a0.nrules, cv_union = a0.cv_union, pss_rules = a0.pss_rules, ncls = a0.ncls;
  const uint32_t ep_rules = a0.err_rules | a0.pat_rules, pat_rules = a0.pat_rules;
  uint8_t* const verdicts = a0.verdicts;
  uint32_t* const stage = dyn + a0.wave_lds + wv * a0.wave_words;
  const uint32_t cls_cv0 = hw(cls_cv, 0), cls_rm0 = hw(cls_rm, 0);
  auto step = [&](LeanTile& cur, LeanTile& far) {
    // header of tile s + 3 (into this buffer, which loads that tile two steps from now), then
    // the items of tile s + 2 into the buffer tile s - 1 used (its header arrived a step ago);
    // no register holding an in-flight load is ever copied
    cur.hn = lean_hdr(L, tile + 3u * W, lane);
    far = lean_load(L, tile + 2u * W, far.hn, lane);
    pin_lean(cur);
    const uint32_t C0 = hw(cur.h, 0), V0 = hw(cur.h, 1), S0 = hw(cur.h, 2), A0 = hw(cur.h, 3);
    const uint32_t nct = hw(cur.h, 4) - C0, nvt = hw(cur.h, 5) - V0, nst = hw(cur.h, 6) - S0,
                   nat = hw(cur.h, 7) - A0;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    if (KPE_DIAG & DIAG_NOPSS) {  // loads consumed, no PSS evaluation
      if (live)
        verdicts[(size_t)r * R] =
            (uint8_t)(cur.rec.x ^ cur.rec.z ^ cur.c0.x ^ cur.c1.y ^ cur.v0 ^ cur.v1 ^ cur.s0 ^ cur.q0.x ^ nct);
      return;
    }
    // ---- the pod's item offsets: exclusive wave scans of its packed counts ----
    const uint32_t z = cur.rec.z;  // 0 for rows past n (range-checked load)
    const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
    const uint32_t c01 = nc | (nv << 16);
    const uint32_t e01 = wave_incl_scan(c01) - c01;
    uint32_t e23 = 0;
    if (nst | nat) {
      const uint32_t c23 = ns | (na << 16);
      e23 = wave_incl_scan(c23) - c23;
    }
    const uint32_t oc = e01 & 0xFFFFu, ov = e01 >> 16, os = e23 & 0xFFFFu, oa = e23 >> 16;
    uint2* sc = reinterpret_cast<uint2*>(stage);
    uint8_t* sbv = reinterpret_cast<uint8_t*>(stage + KPE_STAGE_CTR * 2);
    uint8_t* sbs = sbv + KPE_STAGE_VOL;
    uint8_t* sba = sbs + KPE_STAGE_SMALL;
    auto ctr_code = [&](uint2 e) { return make_uint2(e.x, (uint32_t)s_capb[CY_CAPSET(e.y)]); };
    auto vol_code = [&](uint32_t sv0) -> uint32_t { return ((sv0 >> VS_HOSTPATH) & 1u) | ((sv0 & kAllowedVolumes) ? 0u : 2u); };
    auto sys_code = [&](uint32_t id) -> uint32_t {
      return (pbit(p_s0, id) ^ 1u) | ((pbit(p_s1, id) ^ 1u) << 1) | ((pbit(p_s2, id) ^ 1u) << 2);
    };
    auto ann_code = [&](uint2 kv) -> uint32_t {
      return (pbit(p_aak, kv.x) & (pbit(p_aao, kv.y) ^ 1u)) | ((pbit(p_spk, kv.x) & (pbit(p_sann, kv.y) ^ 1u)) << 1);
    };
    // ---- stage the tile's item codes, unconditionally: slots past the tile's items hold codes
    // of the next tile's items (or of zeros past a column's end) that no pod reads ----
    sc[lane] = ctr_code(cur.c0);
    sc[lane + 64u] = ctr_code(cur.c1);
    if (nvol) sbv[lane] = (uint8_t)vol_code(cur.v0), sbv[lane + 64u] = (uint8_t)vol_code(cur.v1);
    if (nsys && nst) sbs[lane] = (uint8_t)sys_code(cur.s0);
    if (npann && nat) sba[lane] = (uint8_t)ann_code(cur.q0);
    __builtin_amdgcn_wave_barrier();
    // ---- each pod ORs its first items with fixed clamped reads (a repeated item does not
    // change an OR); pods without items of a list mask the read off ----
    uint32_t xo, co, vcode = 0, scode = 0, acode = 0;
    {
      const uint32_t last = min(oc + (nc ? nc - 1u : 0u), KPE_STAGE_CTR - 1u);
      const uint2 e0 = sc[min(oc, last)], e1 = sc[min(oc + 1u, last)], e2 = sc[min(oc + 2u, last)],
                  e3 = sc[min(oc + 3u, last)];
      const uint32_t m = nc ? ~0u : 0u;
      xo = (e0.x | e1.x | e2.x | e3.x) & m;
      co = (e0.y | e1.y | e2.y | e3.y) & m;
    }
    if (nvol) {
      const uint32_t last = min(ov + (nv ? nv - 1u : 0u), KPE_STAGE_VOL - 1u);
      const uint32_t x = (uint32_t)sbv[min(ov, last)] | sbv[min(ov + 1u, last)] | sbv[min(ov + 2u, last)] |
                         sbv[min(ov + 3u, last)];
      vcode = nv ? x : 0u;
    }
    if (nsys && nst) {
      const uint32_t last = min(os + (ns ? ns - 1u : 0u), KPE_STAGE_SMALL - 1u);
      const uint32_t x = (uint32_t)sbs[min(os, last)] | sbs[min(os + 1u, last)];
      scode = ns ? x : 0u;
    }
    if (npann && nat) {
      const uint32_t last = min(oa + (na ? na - 1u : 0u), KPE_STAGE_SMALL - 1u);
      const uint32_t x = (uint32_t)sba[min(oa, last)] | sba[min(oa + 1u, last)];
      acode = na ? x : 0u;
    }
    // ---- pods with more items than that, or a tile whose items overflow the staging area:
    // recomputed over all their items (staged ones from LDS, the rest loaded) ----
    const bool tile_over = nct > KPE_STAGE_CTR || (nvol && nvt > KPE_STAGE_VOL) || (nsys && nst > KPE_STAGE_SMALL) ||
                           (npann && nat > KPE_STAGE_SMALL);
    const bool more_c = nc > 4u, more_v = nvol && nv > 4u, more_s = nsys && ns > 2u, more_a = npann && na > 2u;
    if (tile_over || __builtin_amdgcn_ballot_w64(more_c || more_v || more_s || more_a)) {
      if (more_c || (tile_over && oc + nc > KPE_STAGE_CTR)) {
        xo = co = 0;
        for (uint32_t k = oc; k < oc + nc; ++k) {
          const uint2 e = k < KPE_STAGE_CTR ? sc[k] : ctr_code(bload2(L.crec, (C0 + k) * 8u));
          xo |= e.x, co |= e.y;
        }
      }
      if (nvol && (more_v || (tile_over && ov + nv > KPE_STAGE_VOL))) {
        vcode = 0;
        for (uint32_t k = ov; k < ov + nv; ++k)
          vcode |= k < KPE_STAGE_VOL ? (uint32_t)sbv[k] : vol_code(bload1(L.vol, (V0 + k) * 4u));
      }
      if (nsys && (more_s || (tile_over && os + ns > KPE_STAGE_SMALL))) {
        scode = 0;
        for (uint32_t k = os; k < os + ns; ++k)
          scode |= k < KPE_STAGE_SMALL ? (uint32_t)sbs[k] : sys_code(bload1(L.sys, (S0 + k) * 4u));
      }
      if (npann && (more_a || (tile_over && oa + na > KPE_STAGE_SMALL))) {
        acode = 0;
        for (uint32_t k = oa; k < oa + na; ++k)
          acode |= k < KPE_STAGE_SMALL ? (uint32_t)sba[k] : ann_code(bload2(L.ann, (A0 + k) * 8u));
      }
    }
    __builtin_amdgcn_wave_barrier();
    // ---- PSA checks, rule match (kind table), verdict bytes stored straight from the lane ----
    const uint32_t pw = cur.rec.x;
    const uint32_t fails = cv_fails(pw, xo, co & 7u, false, vcode & 1u, vcode & 2u, scode, acode & 1u, acode & 2u) & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t matched = dyn[kt + GVK_KIND(cur.rec.y)];
    uint32_t failr;
    if (ncls == 1u) {
      failr = (fails & cls_cv0) ? cls_rm0 : 0u;
    } else {
      failr = 0;
#pragma unroll 1
      for (uint32_t c = 0; c < ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
    }
    const uint32_t E = matched & ((err ? pss_rules : 0u) | ep_rules);
    const uint32_t F = (matched & pss_rules & failr & ~E) | (matched & pat_rules);  // F|E = PENDING
    const uint32_t P = matched & pss_rules & ~failr & ~E;
    if (live && !(KPE_DIAG & DIAG_NOSTORE)) {
      uint8_t* row = verdicts + (size_t)r * R;
#pragma unroll 1
      for (uint32_t ri = 0; ri < R; ++ri)
        row[ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
    }
    __builtin_amdgcn_wave_barrier();
  };
  while (tile < ntiles) {  // three rotating buffers: (evaluate, load two ahead)
    step(ta, tc);
    tile += W;
    if (tile >= ntiles) break;
    step(tb, ta);
    tile += W;
    if (tile >= ntiles) break;
    step(tc, tb);
    tile += W;
  }
}

// ---- kpe_lean3_kernel: the same scan, non-persistent, every load of a wave issued up front ----
// Each wave evaluates KPE_LEAN_T consecutive tiles. One load brings the header words of all of
// them (lane k < 4T + 4: word k of tile t0 + k / 4), the pod records are issued before that
// header arrives and the list items of all T tiles right after it, so a wave has one dependent
// load step (header -> items) and then only evaluation; tile j waits for its own loads alone.
// The grid covers the tiles (no persistent loop): the dispatcher starts a wave as soon as an
// earlier one retires, which keeps every CU's memory pipeline full across waves.
#ifndef KPE_LEAN_T
#define KPE_LEAN_T 1
#endif
struct LeanItems {
  uint4 rec;
  uint2 c0, c1, q0;
  uint32_t v0, v1, s0;
};
#ifndef KPE_LEAN3_BLOCK
#define KPE_LEAN3_BLOCK 256
#endif
#ifndef KPE_LEAN3_XCD
#define KPE_LEAN3_XCD 1
#endif
#ifndef KPE_LEAN3_DIRECT
#define KPE_LEAN3_DIRECT 1  // per-lane list loads (1) or cooperative loads staged through LDS (0)
#endif
constexpr uint32_t kLB = KPE_LEAN3_BLOCK;
// XCD-aware block order: the dispatcher deals workgroups round-robin to the 8 XCDs (block b on
// XCD b % 8), so block b takes the (b / 8)-th block of XCD b % 8's contiguous share of the tiles.
// A tile's list loads run past its end into the next tile's items, and the header of the next
// tile is read too: with neighbouring tiles on one XCD those reads hit the L2 that loads them.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
  if (!KPE_LEAN3_XCD) return b;
  const uint32_t q = nb >> 3, r = nb & 7u, x = b & 7u;
  return x * q + min(x, r) + (b >> 3);
}
__global__ void __launch_bounds__(kLB, KPE_LEAN2_WAVES) kpe_lean3_kernel(ScanArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  if (KPE_DIAG & DIAG_EMPTY) return;
  CArgs& a0 = *kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles, n = (uint32_t)a0.n;
  const uint32_t t0 = (xcd_block(blockIdx.x, gridDim.x) * (kLB / 64u) + wv) * KPE_LEAN_T;
  const uint32_t need = a0.need;
  LeanCols L;
  L.rec = make_rsrc(a0.rec, n * 16u);
  L.hdr = make_rsrc(a0.hdr, (ntiles + 1u) * 16u);
  L.crec = make_rsrc(a0.crec, a0.nctr_total * 8u);
  L.vol = make_rsrc(a0.vol_src, (need & NEED_VOL) ? a0.nvol_total * 4u : 0u);
  L.sys = make_rsrc(a0.sys_id, (need & NEED_SYS) ? a0.nsys_total * 4u : 0u);
  L.ann = make_rsrc(a0.pann_kv, (need & NEED_PANN) ? a0.npann_total * 8u : 0u);
  const bool nvol = need & NEED_VOL, nsys = need & NEED_SYS, npann = need & NEED_PANN;

  // header words of tiles t0 .. t0 + T (past the last header: 0), image, pod records, items
  const uint32_t hall = bload1(L.hdr, (t0 * 4u + min(lane, 4u * KPE_LEAN_T + 3u)) * 4u);
  const uint32_t img_n4 = a0.pimg_words >> 2;
  const uint4* img = reinterpret_cast<const uint4*>(a0.pimg);
  const uint4 img0 = img[min(t, img_n4 - 1u)];
  uint32_t cls_cv = 0, cls_rm = 0;
  if (lane < a0.ncls) {
    const uint2 c = reinterpret_cast<const uint2*>(a0.narrow_cls)[lane];
    cls_cv = c.x, cls_rm = c.y;
  }
  LeanItems it[KPE_LEAN_T];
#pragma unroll
  for (uint32_t j = 0; j < KPE_LEAN_T; ++j) it[j].rec = bload4(L.rec, ((t0 + j) * 64u + lane) * 16u);
#pragma unroll
  for (uint32_t j = 0; j < KPE_LEAN_T && !KPE_LEAN3_DIRECT; ++j) {
    const uint32_t C0 = hw(hall, 4u * j), V0 = hw(hall, 4u * j + 1u), S0 = hw(hall, 4u * j + 2u),
                   A0 = hw(hall, 4u * j + 3u);
    it[j].c0 = bload2(L.crec, (C0 + lane) * 8u);
    it[j].c1 = bload2(L.crec, (C0 + 64u + lane) * 8u);
    it[j].v0 = bload1(L.vol, (V0 + lane) * 4u);
    it[j].v1 = bload1(L.vol, (V0 + 64u + lane) * 4u);
    it[j].s0 = bload1(L.sys, (S0 + lane) * 4u);
    it[j].q0 = bload2(L.ann, (A0 + lane) * 8u);
  }
  {
    uint4* d4 = reinterpret_cast<uint4*>(dyn);
    if (t < img_n4) d4[t] = img0;
#pragma unroll 1
    for (uint32_t i = t + kLB; i < img_n4; i += kLB) d4[i] = img[i];
  }
  __syncthreads();
  if (KPE_DIAG & DIAG_NOLOOP) {
    if (t0 < ntiles && lane == 0) a0.verdicts[t0] = (uint8_t)(dyn[0] + it[0].rec.x + it[0].c0.x);
    return;
  }
  const uint8_t* s_capb = reinterpret_cast<const uint8_t*>(dyn + a0.capb_lds);
  const LdsPtr lds = (LdsPtr)dyn;
  const uint32_t p_sann = a0.pp_seccomp_ann_ok & ~PRED_LOCAL, p_aak = a0.pp_apparmor_key & ~PRED_LOCAL,
                 p_aao = a0.pp_apparmor_ok & ~PRED_LOCAL, p_spk = a0.pp_seccomp_pod_key & ~PRED_LOCAL,
                 p_s0 = a0.pp_sysctl0 & ~PRED_LOCAL, p_s1 = a0.pp_sysctl1 & ~PRED_LOCAL,
                 p_s2 = a0.pp_sysctl2 & ~PRED_LOCAL;
  auto pbit = [&](uint32_t loc, uint32_t id) -> uint32_t { return (lds[loc + (id >> 5)] >> (id & 31u)) & 1u; };
  const uint32_t kt = a0.kt_lds;
  const uint32_t R = a0.nrules, cv_union = a0.cv_union, pss_rules = a0.pss_rules, ncls = a0.ncls;
  const uint32_t ep_rules = a0.err_rules | a0.pat_rules, pat_rules = a0.pat_rules;
  uint8_t* const verdicts = a0.verdicts;
  uint32_t* const stage = dyn + a0.wave_lds + wv * a0.wave_words;
  const uint32_t cls_cv0 = hw(cls_cv, 0), cls_rm0 = hw(cls_rm, 0);
#if KPE_LEAN3_DIRECT
  // Phase 1 for every tile of the wave: the scan of the pod records' packed counts, then every
  // tile's list loads at once, so the wave has two dependent memory steps in all (records /
  // headers, then items) whatever KPE_LEAN_T is; phase 2 (below) evaluates the tiles in turn.
  struct DItems {
    uint32_t oc, ov, os, oa;
    uint2 e0, e1, e2, e3, q0, q1;
    uint32_t w0, w1, s0, s1;
  };
  DItems di[KPE_LEAN_T];
  constexpr uint32_t kOOB = 0xFFFFFFF0u;
#pragma unroll
  for (uint32_t j = 0; j < KPE_LEAN_T; ++j) {
    DItems& d = di[j];
    const uint32_t C0 = hw(hall, 4u * j), V0 = hw(hall, 4u * j + 1u), S0 = hw(hall, 4u * j + 2u),
                   A0 = hw(hall, 4u * j + 3u);
    const uint32_t nct = hw(hall, 4u * j + 4u) - C0, nvt = hw(hall, 4u * j + 5u) - V0,
                   nst = hw(hall, 4u * j + 6u) - S0, nat = hw(hall, 4u * j + 7u) - A0;
    const uint32_t z = it[j].rec.z;
    const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
    if ((nct | nvt | nst | nat) < 256u) {  // one scan of the four packed byte counts (no carries)
      const uint32_t e = wave_incl_scan(z) - z;
      d.oc = e & 0xFFu, d.ov = (e >> 8) & 0xFFu, d.os = (e >> 16) & 0xFFu, d.oa = e >> 24;
    } else {
      const uint32_t c01 = nc | (nv << 16), c23 = ns | (na << 16);
      const uint32_t e01 = wave_incl_scan(c01) - c01, e23 = wave_incl_scan(c23) - c23;
      d.oc = e01 & 0xFFFFu, d.ov = e01 >> 16, d.os = e23 & 0xFFFFu, d.oa = e23 >> 16;
    }
    const uint32_t cb = (C0 + d.oc) * 8u, vb = (V0 + d.ov) * 4u, sb = (S0 + d.os) * 4u, ab = (A0 + d.oa) * 8u;
    d.e0 = bload2(L.crec, nc > 0u ? cb : kOOB), d.e1 = bload2(L.crec, nc > 1u ? cb + 8u : kOOB);
    d.e2 = bload2(L.crec, nc > 2u ? cb + 16u : kOOB), d.e3 = bload2(L.crec, nc > 3u ? cb + 24u : kOOB);
    d.w0 = nvol ? bload1(L.vol, nv > 0u ? vb : kOOB) : 0u, d.w1 = nvol ? bload1(L.vol, nv > 1u ? vb + 4u : kOOB) : 0u;
    d.s0 = d.s1 = 0u, d.q0 = d.q1 = make_uint2(0u, 0u);
    if (nsys && nst) d.s0 = bload1(L.sys, ns > 0u ? sb : kOOB), d.s1 = bload1(L.sys, ns > 1u ? sb + 4u : kOOB);
    if (npann && nat) d.q0 = bload2(L.ann, na > 0u ? ab : kOOB), d.q1 = bload2(L.ann, na > 1u ? ab + 8u : kOOB);
  }
#endif
#pragma unroll
  for (uint32_t j = 0; j < KPE_LEAN_T; ++j) {
    const uint32_t tile = t0 + j;
    if (tile >= ntiles) break;
    const LeanItems& cur = it[j];
    const uint32_t C0 = hw(hall, 4u * j), V0 = hw(hall, 4u * j + 1u), S0 = hw(hall, 4u * j + 2u),
                   A0 = hw(hall, 4u * j + 3u);
    const uint32_t nct = hw(hall, 4u * j + 4u) - C0, nvt = hw(hall, 4u * j + 5u) - V0,
                   nst = hw(hall, 4u * j + 6u) - S0, nat = hw(hall, 4u * j + 7u) - A0;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    if (KPE_DIAG & DIAG_NOPSS) {
      if (live)
        verdicts[(size_t)r * R] =
            (uint8_t)(cur.rec.x ^ cur.rec.z ^ cur.c0.x ^ cur.c1.y ^ cur.v0 ^ cur.v1 ^ cur.s0 ^ cur.q0.x ^ nct);
      continue;
    }
    const uint32_t z = cur.rec.z;
    const uint32_t nc = PRC_CTR(z), nv = PRC_VOL(z), ns = PRC_SYS(z), na = PRC_PANN(z);
#if KPE_LEAN3_DIRECT
    const uint32_t oc = di[j].oc, ov = di[j].ov, os = di[j].os, oa = di[j].oa;
#else
    uint32_t oc, ov, os, oa;
    if ((nct | nvt | nst | nat) < 256u) {  // one scan of the four packed byte counts (no carries)
      const uint32_t e = wave_incl_scan(z) - z;
      oc = e & 0xFFu, ov = (e >> 8) & 0xFFu, os = (e >> 16) & 0xFFu, oa = e >> 24;
    } else {
      const uint32_t c01 = nc | (nv << 16), c23 = ns | (na << 16);
      const uint32_t e01 = wave_incl_scan(c01) - c01, e23 = wave_incl_scan(c23) - c23;
      oc = e01 & 0xFFFFu, ov = e01 >> 16, os = e23 & 0xFFFFu, oa = e23 >> 16;
    }
#endif
#if KPE_LEAN3_DIRECT
    // Each lane reads its own pod's list items (its offsets from the scan): the first four
    // containers, two volumes and (when the tile has any) two sysctls / annotations are issued
    // together; an item past the pod's count reads past the column's end and returns 0. Pods
    // with more items take a loop. No staging area, no wave barrier, no capacity limit.
    (void)nvt;
    const uint32_t cb = (C0 + oc) * 8u, vb = (V0 + ov) * 4u, sb = (S0 + os) * 4u, ab = (A0 + oa) * 8u;
    const uint2 e0 = di[j].e0, e1 = di[j].e1, e2 = di[j].e2, e3 = di[j].e3, q0 = di[j].q0, q1 = di[j].q1;
    const uint32_t w0 = di[j].w0, w1 = di[j].w1, s0 = di[j].s0, s1 = di[j].s1;
    auto vol_code = [&](uint32_t sv0) -> uint32_t { return ((sv0 >> VS_HOSTPATH) & 1u) | ((sv0 & kAllowedVolumes) ? 0u : 2u); };
    auto sys_code = [&](uint32_t id) -> uint32_t {
      return (pbit(p_s0, id) ^ 1u) | ((pbit(p_s1, id) ^ 1u) << 1) | ((pbit(p_s2, id) ^ 1u) << 2);
    };
    auto ann_code = [&](uint2 kv) -> uint32_t {
      return (pbit(p_aak, kv.x) & (pbit(p_aao, kv.y) ^ 1u)) | ((pbit(p_spk, kv.x) & (pbit(p_sann, kv.y) ^ 1u)) << 1);
    };
    // a real container record always has state bits (every field state is one-hot)
    auto cap = [&](uint2 e) -> uint32_t { return e.x ? (uint32_t)s_capb[CY_CAPSET(e.y)] : 0u; };
    uint32_t xo = e0.x | e1.x | e2.x | e3.x;
    uint32_t co = cap(e0) | cap(e1) | cap(e2) | cap(e3);
    uint32_t vcode = 0, scode = 0, acode = 0;
    if (nvol) vcode = (nv > 0u ? vol_code(w0) : 0u) | (nv > 1u ? vol_code(w1) : 0u);
    if (nsys && nst) scode = (ns > 0u ? sys_code(s0) : 0u) | (ns > 1u ? sys_code(s1) : 0u);
    if (npann && nat) acode = (na > 0u ? ann_code(q0) : 0u) | (na > 1u ? ann_code(q1) : 0u);
    if (__builtin_amdgcn_ballot_w64(nc > 4u || (nvol && nv > 2u) || (nsys && ns > 2u) || (npann && na > 2u))) {
      for (uint32_t k = 4; k < nc; ++k) {
        const uint2 e = bload2(L.crec, cb + 8u * k);
        xo |= e.x, co |= cap(e);
      }
      if (nvol)
        for (uint32_t k = 2; k < nv; ++k) vcode |= vol_code(bload1(L.vol, vb + 4u * k));
      if (nsys)
        for (uint32_t k = 2; k < ns; ++k) scode |= sys_code(bload1(L.sys, sb + 4u * k));
      if (npann)
        for (uint32_t k = 2; k < na; ++k) acode |= ann_code(bload2(L.ann, ab + 8u * k));
    }
#else
    uint2* sc = reinterpret_cast<uint2*>(stage);
    uint8_t* sbv = reinterpret_cast<uint8_t*>(stage + KPE_STAGE_CTR * 2);
    uint8_t* sbs = sbv + KPE_STAGE_VOL;
    uint8_t* sba = sbs + KPE_STAGE_SMALL;
    auto ctr_code = [&](uint2 e) { return make_uint2(e.x, (uint32_t)s_capb[CY_CAPSET(e.y)]); };
    auto vol_code = [&](uint32_t sv0) -> uint32_t { return ((sv0 >> VS_HOSTPATH) & 1u) | ((sv0 & kAllowedVolumes) ? 0u : 2u); };
    auto sys_code = [&](uint32_t id) -> uint32_t {
      return (pbit(p_s0, id) ^ 1u) | ((pbit(p_s1, id) ^ 1u) << 1) | ((pbit(p_s2, id) ^ 1u) << 2);
    };
    auto ann_code = [&](uint2 kv) -> uint32_t {
      return (pbit(p_aak, kv.x) & (pbit(p_aao, kv.y) ^ 1u)) | ((pbit(p_spk, kv.x) & (pbit(p_sann, kv.y) ^ 1u)) << 1);
    };
    if (KPE_DIAG & DIAG_NOSTAGE) {  // diagnostic: no staging, no per-pod OR
      const uint32_t fails = (KPE_DIAG & DIAG_NOCV)
                                 ? (cur.rec.x ^ cur.c0.x ^ cur.v0 ^ cur.s0 ^ cur.q0.x ^ oc)
                                 : cv_fails(cur.rec.x, cur.c0.x | cur.c1.x, (cur.c0.y | cur.c1.y) & 7u, false, cur.v0 & 1u,
                                            cur.v1 & 2u, cur.s0 & 7u, cur.q0.x & 1u, cur.q0.y & 2u) & cv_union;
      const uint32_t matched = dyn[kt + GVK_KIND(cur.rec.y)];
      const uint32_t failr = (fails & cls_cv0) ? cls_rm0 : 0u;
      const uint32_t F = matched & failr, P = matched & ~failr;
      if (live) {
        uint8_t* row = verdicts + (size_t)r * R;
#pragma unroll 1
        for (uint32_t ri = 0; ri < R; ++ri) row[ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1));
      }
      continue;
    }
    sc[lane] = ctr_code(cur.c0);
    sc[lane + 64u] = ctr_code(cur.c1);
    if (nvol) sbv[lane] = (uint8_t)vol_code(cur.v0), sbv[lane + 64u] = (uint8_t)vol_code(cur.v1);
    if (nsys && nst) sbs[lane] = (uint8_t)sys_code(cur.s0);
    if (npann && nat) sba[lane] = (uint8_t)ann_code(cur.q0);
    __builtin_amdgcn_wave_barrier();
    uint32_t xo, co, vcode = 0, scode = 0, acode = 0;
    {
      const uint32_t last = min(oc + (nc ? nc - 1u : 0u), KPE_STAGE_CTR - 1u);
      const uint2 e0 = sc[min(oc, last)], e1 = sc[min(oc + 1u, last)], e2 = sc[min(oc + 2u, last)],
                  e3 = sc[min(oc + 3u, last)];
      const uint32_t m = nc ? ~0u : 0u;
      xo = (e0.x | e1.x | e2.x | e3.x) & m;
      co = (e0.y | e1.y | e2.y | e3.y) & m;
    }
    if (nvol) {
      const uint32_t last = min(ov + (nv ? nv - 1u : 0u), KPE_STAGE_VOL - 1u);
      const uint32_t x = (uint32_t)sbv[min(ov, last)] | sbv[min(ov + 1u, last)] | sbv[min(ov + 2u, last)] |
                         sbv[min(ov + 3u, last)];
      vcode = nv ? x : 0u;
    }
    if (nsys && nst) {
      const uint32_t last = min(os + (ns ? ns - 1u : 0u), KPE_STAGE_SMALL - 1u);
      const uint32_t x = (uint32_t)sbs[min(os, last)] | sbs[min(os + 1u, last)];
      scode = ns ? x : 0u;
    }
    if (npann && nat) {
      const uint32_t last = min(oa + (na ? na - 1u : 0u), KPE_STAGE_SMALL - 1u);
      const uint32_t x = (uint32_t)sba[min(oa, last)] | sba[min(oa + 1u, last)];
      acode = na ? x : 0u;
    }
    const bool tile_over = nct > KPE_STAGE_CTR || (nvol && nvt > KPE_STAGE_VOL) || (nsys && nst > KPE_STAGE_SMALL) ||
                           (npann && nat > KPE_STAGE_SMALL);
    const bool more_c = nc > 4u, more_v = nvol && nv > 4u, more_s = nsys && ns > 2u, more_a = npann && na > 2u;
    if (tile_over || __builtin_amdgcn_ballot_w64(more_c || more_v || more_s || more_a)) {
      if (more_c || (tile_over && oc + nc > KPE_STAGE_CTR)) {
        xo = co = 0;
        for (uint32_t k = oc; k < oc + nc; ++k) {
          const uint2 e = k < KPE_STAGE_CTR ? sc[k] : ctr_code(bload2(L.crec, (C0 + k) * 8u));
          xo |= e.x, co |= e.y;
        }
      }
      if (nvol && (more_v || (tile_over && ov + nv > KPE_STAGE_VOL))) {
        vcode = 0;
        for (uint32_t k = ov; k < ov + nv; ++k)
          vcode |= k < KPE_STAGE_VOL ? (uint32_t)sbv[k] : vol_code(bload1(L.vol, (V0 + k) * 4u));
      }
      if (nsys && (more_s || (tile_over && os + ns > KPE_STAGE_SMALL))) {
        scode = 0;
        for (uint32_t k = os; k < os + ns; ++k)
          scode |= k < KPE_STAGE_SMALL ? (uint32_t)sbs[k] : sys_code(bload1(L.sys, (S0 + k) * 4u));
      }
      if (npann && (more_a || (tile_over && oa + na > KPE_STAGE_SMALL))) {
        acode = 0;
        for (uint32_t k = oa; k < oa + na; ++k)
          acode |= k < KPE_STAGE_SMALL ? (uint32_t)sba[k] : ann_code(bload2(L.ann, (A0 + k) * 8u));
      }
    }
    __builtin_amdgcn_wave_barrier();
#endif
    const uint32_t pw = cur.rec.x;
    const uint32_t fails = (KPE_DIAG & DIAG_NOCV)
                               ? (pw ^ xo ^ co ^ vcode ^ scode ^ acode)
                               : cv_fails(pw, xo, co & 7u, false, vcode & 1u, vcode & 2u, scode, acode & 1u, acode & 2u) & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t matched = dyn[kt + GVK_KIND(cur.rec.y)];
    uint32_t failr;
    if (ncls == 1u) {
      failr = (fails & cls_cv0) ? cls_rm0 : 0u;
    } else {
      failr = 0;
#pragma unroll 1
      for (uint32_t c = 0; c < ncls; ++c) failr |= (fails & hw(cls_cv, c)) ? hw(cls_rm, c) : 0u;
    }
    const uint32_t E = matched & ((err ? pss_rules : 0u) | ep_rules);
    const uint32_t F = (matched & pss_rules & failr & ~E) | (matched & pat_rules);
    const uint32_t P = matched & pss_rules & ~failr & ~E;
    if (live && !(KPE_DIAG & DIAG_NOSTORE)) {
      uint8_t* row = verdicts + (size_t)r * R;
#pragma unroll 1
      for (uint32_t ri = 0; ri < R; ++ri)
        row[ri] = (uint8_t)(((P >> ri) & 1u) | (((F >> ri) & 1u) << 1) | (((E >> ri) & 1u) << 2));
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ---- kpe_lean4_kernel: one memory step per wave -------------------------------------------
// kpe_lean3_kernel's waves wait on two dependent HBM round trips (pod records and tile header,
// then the list items at header offsets), and 1M pods are ~2 generations of resident waves, so
// the latency chain, not bandwidth, sets its time. Here every list is also laid out in tile
// slabs (DeviceCorpus::slab_*: tile t's first K items at [t * K, (t + 1) * K), zero padded; K
// per list from the corpus's per-tile counts), so the wave issues the pod records, the tile
// header and its slab loads together: one round trip. The items are staged in LDS, a pod ORs its
// range of slots, and only items past a tile's K (rare: K covers >= 99.5% of the tiles) are
// loaded from the CSR columns at header offsets afterwards.
struct Lean4Loads {
  uint32_t hall;
  uint4 rec;
  uint2 c0, c1, q0;
  uint32_t v0, v1, s0;
};
template <int T>
__global__ void __launch_bounds__(kLB, KPE_LEAN2_WAVES) kpe_lean4_kernel(ScanArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  if (KPE_DIAG & DIAG_EMPTY) return;
  CArgs& a0 = *kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles, n = (uint32_t)a0.n;
  const uint32_t tile0 = (xcd_block(blockIdx.x, gridDim.x) * (kLB / 64u) + wv) * (uint32_t)T;
  const uint32_t need = a0.need;
  const bool nvol = need & NEED_VOL, nsys = need & NEED_SYS, npann = need & NEED_PANN;
  const uint32_t kc = a0.kc, kv = nvol ? a0.kv : 0u, ks = nsys ? a0.ks : 0u, ka = npann ? a0.ka : 0u;
  LeanCols L;
  L.rec = make_rsrc(a0.rec, n * 16u);
  L.hdr = make_rsrc(a0.hdr, (ntiles + 1u) * 16u);
  L.crec = make_rsrc(a0.crec, a0.nctr_total * 8u);
  L.vol = make_rsrc(a0.vol_src, nvol ? a0.nvol_total * 4u : 0u);
  L.sys = make_rsrc(a0.sys_id, nsys ? a0.nsys_total * 4u : 0u);
  L.ann = make_rsrc(a0.pann_kv, npann ? a0.npann_total * 8u : 0u);
  const Rsrc SC = make_rsrc(a0.slab_c, ntiles * kc * 8u), SV = make_rsrc(a0.slab_v, ntiles * kv * 4u),
             SS = make_rsrc(a0.slab_s, ntiles * ks * 4u), SA = make_rsrc(a0.slab_a, ntiles * ka * 8u);
  constexpr uint32_t kOOB = 0xFFFFFFF0u;  // a range-checked load of 0

  // ---- the one memory step: header words of this tile and the next, pod record, slab slots
  // lane and lane + 64 of each list (slots past K read 0), the prologue image ----
  Lean4Loads ld[T];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t tile = tile0 + (uint32_t)j;
    Lean4Loads& d = ld[j];
    d.hall = bload1(L.hdr, (tile * 4u + min(lane, 7u)) * 4u);
    d.rec = bload4(L.rec, (tile * 64u + lane) * 16u);
    d.c0 = bload2(SC, lane < kc ? (tile * kc + lane) * 8u : kOOB);
    d.c1 = bload2(SC, lane + 64u < kc ? (tile * kc + 64u + lane) * 8u : kOOB);
    d.v0 = bload1(SV, lane < kv ? (tile * kv + lane) * 4u : kOOB);
    d.v1 = bload1(SV, lane + 64u < kv ? (tile * kv + 64u + lane) * 4u : kOOB);
    d.s0 = bload1(SS, lane < ks ? (tile * ks + lane) * 4u : kOOB);
    d.q0 = bload2(SA, lane < ka ? (tile * ka + lane) * 8u : kOOB);
  }
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
  if (KPE_DIAG & DIAG_NOLOOP) {  // loads and image only: every loaded value consumed
    uint32_t x = dyn[0];
#pragma unroll
    for (int j = 0; j < T; ++j)
      x += ld[j].hall + ld[j].rec.x + ld[j].rec.z + ld[j].c0.x + ld[j].c1.y + ld[j].v0 + ld[j].v1 + ld[j].s0 + ld[j].q0.x;
    if (tile0 < ntiles) a0.verdicts[(size_t)tile0 * 64u + lane] = (uint8_t)x;
    return;
  }
  const uint8_t* s_capb = reinterpret_cast<const uint8_t*>(dyn + a0.capb_lds);
  const LdsPtr lds = (LdsPtr)dyn;
  const uint32_t p_sann = a0.pp_seccomp_ann_ok & ~PRED_LOCAL, p_aak = a0.pp_apparmor_key & ~PRED_LOCAL,
                 p_aao = a0.pp_apparmor_ok & ~PRED_LOCAL, p_spk = a0.pp_seccomp_pod_key & ~PRED_LOCAL,
                 p_s0 = a0.pp_sysctl0 & ~PRED_LOCAL, p_s1 = a0.pp_sysctl1 & ~PRED_LOCAL,
                 p_s2 = a0.pp_sysctl2 & ~PRED_LOCAL;
  auto pbit = [&](uint32_t loc, uint32_t id) -> uint32_t { return (lds[loc + (id >> 5)] >> (id & 31u)) & 1u; };
  const uint32_t R = a0.nrules, cv_union = a0.cv_union, pss_rules = a0.pss_rules, ncls = a0.ncls;
  const uint32_t ep_rules = a0.err_rules | a0.pat_rules, pat_rules = a0.pat_rules;
  uint32_t* const stage = dyn + a0.wave_lds + wv * a0.wave_words;
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t tile = tile0 + (uint32_t)j;
    if (tile >= ntiles) break;
    const uint32_t hall = ld[j].hall;
    const uint4 rec = ld[j].rec;
    const uint2 c0 = ld[j].c0, c1 = ld[j].c1, q0 = ld[j].q0;
    const uint32_t v0 = ld[j].v0, v1 = ld[j].v1, s0 = ld[j].s0;
    const uint32_t C0 = hw(hall, 0), V0 = hw(hall, 1), S0 = hw(hall, 2), A0 = hw(hall, 3);
    const uint32_t nct = hw(hall, 4) - C0, nvt = hw(hall, 5) - V0, nst = hw(hall, 6) - S0, nat = hw(hall, 7) - A0;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    // ---- the pod's slots: exclusive wave scans of its packed counts ----
    const uint32_t z = rec.z;  // 0 for rows past n (range-checked load)
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
    // ---- stage the slab slots' codes (slots past the tile's items hold padding no pod reads) ----
    uint2* sc = reinterpret_cast<uint2*>(stage);
    uint8_t* sbv = reinterpret_cast<uint8_t*>(stage + KPE_STAGE_CTR * 2);
    uint8_t* sbs = sbv + KPE_STAGE_VOL;
    uint8_t* sba = sbs + KPE_STAGE_SMALL;
    auto ctr_code = [&](uint2 e) { return make_uint2(e.x, e.x ? (uint32_t)s_capb[CY_CAPSET(e.y)] : 0u); };
    auto vol_code = [&](uint32_t sv0) -> uint32_t { return ((sv0 >> VS_HOSTPATH) & 1u) | ((sv0 & kAllowedVolumes) ? 0u : 2u); };
    auto sys_code = [&](uint32_t id) -> uint32_t {
      return (pbit(p_s0, id) ^ 1u) | ((pbit(p_s1, id) ^ 1u) << 1) | ((pbit(p_s2, id) ^ 1u) << 2);
    };
    auto ann_code = [&](uint2 kv2) -> uint32_t {
      return (pbit(p_aak, kv2.x) & (pbit(p_aao, kv2.y) ^ 1u)) | ((pbit(p_spk, kv2.x) & (pbit(p_sann, kv2.y) ^ 1u)) << 1);
    };
    sc[lane] = ctr_code(c0);
    sc[lane + 64u] = ctr_code(c1);
    if (nvol) sbv[lane] = (uint8_t)vol_code(v0), sbv[lane + 64u] = (uint8_t)vol_code(v1);
    if (nsys && nst) sbs[lane] = (uint8_t)sys_code(s0);
    if (npann && nat) sba[lane] = (uint8_t)ann_code(q0);
    __builtin_amdgcn_wave_barrier();
    // ---- each pod ORs its first slots with fixed clamped reads (a repeated slot does not change
    // an OR); pods without items of a list mask the read off ----
    uint32_t xo, co, vcode = 0, scode = 0, acode = 0;
    {
      const uint32_t last = min(oc + (nc ? nc - 1u : 0u), kc - 1u);
      const uint2 e0 = sc[min(oc, last)], e1 = sc[min(oc + 1u, last)], e2 = sc[min(oc + 2u, last)],
                  e3 = sc[min(oc + 3u, last)];
      const uint32_t m = (nc && oc < kc) ? ~0u : 0u;
      xo = (e0.x | e1.x | e2.x | e3.x) & m;
      co = (e0.y | e1.y | e2.y | e3.y) & m;
    }
    if (nvol) {
      const uint32_t last = min(ov + (nv ? nv - 1u : 0u), kv - 1u);
      const uint32_t x = (uint32_t)sbv[min(ov, last)] | sbv[min(ov + 1u, last)] | sbv[min(ov + 2u, last)] |
                         sbv[min(ov + 3u, last)];
      vcode = (nv && ov < kv) ? x : 0u;
    }
    if (nsys && nst) {
      const uint32_t last = min(os + (ns ? ns - 1u : 0u), ks - 1u);
      const uint32_t x = (uint32_t)sbs[min(os, last)] | sbs[min(os + 1u, last)];
      scode = (ns && os < ks) ? x : 0u;
    }
    if (npann && nat) {
      const uint32_t last = min(oa + (na ? na - 1u : 0u), ka - 1u);
      const uint32_t x = (uint32_t)sba[min(oa, last)] | sba[min(oa + 1u, last)];
      acode = (na && oa < ka) ? x : 0u;
    }
    // ---- pods with more items than the fixed reads cover, or whose items run past the tile's
    // slab: recomputed over all their items (slab slots from LDS, the rest from the CSR columns) ----
    const bool over = nct > kc || (nvol && nvt > kv) || (nsys && nst > ks) || (npann && nat > ka);
    const bool more_c = nc > 4u, more_v = nvol && nv > 4u, more_s = nsys && ns > 2u, more_a = npann && na > 2u;
    if (over || __builtin_amdgcn_ballot_w64(more_c || more_v || more_s || more_a)) {
      if (more_c || oc + nc > kc) {
        xo = co = 0;
        for (uint32_t k = oc; k < oc + nc; ++k) {
          const uint2 e = k < kc ? sc[k] : ctr_code(bload2(L.crec, (C0 + k) * 8u));
          xo |= e.x, co |= e.y;
        }
      }
      if (nvol && (more_v || ov + nv > kv)) {
        vcode = 0;
        for (uint32_t k = ov; k < ov + nv; ++k) vcode |= k < kv ? (uint32_t)sbv[k] : vol_code(bload1(L.vol, (V0 + k) * 4u));
      }
      if (nsys && (more_s || os + ns > ks)) {
        scode = 0;
        for (uint32_t k = os; k < os + ns; ++k) scode |= k < ks ? (uint32_t)sbs[k] : sys_code(bload1(L.sys, (S0 + k) * 4u));
      }
      if (npann && (more_a || oa + na > ka)) {
        acode = 0;
        for (uint32_t k = oa; k < oa + na; ++k)
          acode |= k < ka ? (uint32_t)sba[k] : ann_code(bload2(L.ann, (A0 + k) * 8u));
      }
    }
    // ---- PSA checks, rule match (kind table), verdict bytes stored straight from the lane ----
    const uint32_t pw = rec.x;
    const uint32_t fails = cv_fails(pw, xo, co & 7u, false, vcode & 1u, vcode & 2u, scode, acode & 1u, acode & 2u) & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t matched = dyn[a0.kt_lds + GVK_KIND(rec.y)];
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
    // verdict bytes: the wave's rows staged in LDS (row-major, R bytes per lane) and stored as
    // dwords, 64 R contiguous bytes per tile; check masks (FAIL cells of PSS rules) per lane
    uint8_t* sv = reinterpret_cast<uint8_t*>(stage + KPE_STAGE_WORDS);
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
    if (!(KPE_DIAG & DIAG_NOSTORE)) store_rows(a0.verdicts, sv, tile, R, 0, R, min(64u, n - tile * 64u), lane);
    __builtin_amdgcn_wave_barrier();  // the next tile reuses the staging area
  }
}

// ---- kpe_lean5_kernel: pod records and PSA summaries only --------------------------------
// The corpus's per-pod PSA summary (Corpus::psum, schema.h PS_*: the OR of the container state
// bitmaps and of the list items' codes under the PSA library's fixed sets, built once at
// flatten) stands in for the container / volume / sysctl / annotation lists, so a wave loads
// one 16-byte record and one 8-byte summary per pod in one memory step and evaluates with no
// staging, scans or list loops: the versioned checks (cv_fails), the kind table, the rows
// stored as dwords through LDS and, when asked, the check masks.
template <int T>
__global__ void __launch_bounds__(kLB, KPE_LEAN2_WAVES) kpe_lean5_kernel(ScanArgs) {
  extern __shared__ __attribute__((aligned(16))) uint32_t dyn[];
  if (KPE_DIAG & DIAG_EMPTY) return;
  CArgs& a0 = *kargs();
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint32_t ntiles = a0.ntiles, n = (uint32_t)a0.n;
  const uint32_t tile0 = (xcd_block(blockIdx.x, gridDim.x) * (kLB / 64u) + wv) * (uint32_t)T;
  const Rsrc RC = make_rsrc(a0.rec, n * 16u), PS = make_rsrc(a0.psum, n * 8u);
  uint4 rec[T];
  uint2 sum[T];
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t r = (tile0 + (uint32_t)j) * 64u + lane;
    rec[j] = bload4(RC, r * 16u);
    sum[j] = bload2(PS, r * 8u);
  }
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
  if (KPE_DIAG & DIAG_NOLOOP) {
    uint32_t x = dyn[0];
#pragma unroll
    for (int j = 0; j < T; ++j) x += rec[j].x + rec[j].y + sum[j].x + sum[j].y;
    if (tile0 < ntiles) a0.verdicts[(size_t)tile0 * 64u + lane] = (uint8_t)x;
    return;
  }
  const uint32_t R = a0.nrules, cv_union = a0.cv_union, pss_rules = a0.pss_rules, ncls = a0.ncls;
  const uint32_t ep_rules = a0.err_rules | a0.pat_rules, pat_rules = a0.pat_rules;
  uint8_t* sv = reinterpret_cast<uint8_t*>(dyn + a0.wave_lds + wv * a0.wave_words + KPE_STAGE_WORDS);
#pragma unroll
  for (int j = 0; j < T; ++j) {
    const uint32_t tile = tile0 + (uint32_t)j;
    if (tile >= ntiles) break;
    const uint32_t r = tile * 64u + lane;
    const bool live = r < n;
    const uint32_t pw = rec[j].x, y = sum[j].y;
    const uint32_t fails = cv_fails(pw, sum[j].x, PS_CAPS(y), false, PS_VOL(y) & 1u, PS_VOL(y) & 2u, PS_SYS(y),
                                    PS_ANN(y) & 1u, PS_ANN(y) & 2u) & cv_union;
    const uint32_t cls = (pw >> PR_CLASS_SH) & R_CLASS_MASK;
    const bool err = cls == R_CLASS_OTHER || (pw & PR_DECODE_ERR);
    const uint32_t matched = dyn[a0.kt_lds + GVK_KIND(rec[j].y)];
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
    if (!(KPE_DIAG & DIAG_NOSTORE)) store_rows(a0.verdicts, sv, tile, R, 0, R, min(64u, n - tile * 64u), lane);
    __builtin_amdgcn_wave_barrier();
  }
}
