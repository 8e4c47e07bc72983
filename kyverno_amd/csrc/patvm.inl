// Pattern VM: validate.MatchPattern over the document tape (see kernels.hip). Device code
// included inside kernels.hip's anonymous namespace; scripts/patvm_check.cpp compiles the
// same text for the host (sanitizers, no GPU).
constexpr uint32_t PE_OK = 0, PE_SKIP = 1, PE_NEG = 2, PE_OTHER = 3, PE_OTHER_NOPATH = 4, PE_PUSHED = 8,
                   PE_NONE = 9;
constexpr uint32_t kNoNode = 0xFFFFFFFFu;
#ifndef KPE_PAT_STACK
#define KPE_PAT_STACK 14
#endif
constexpr int kPatStack = KPE_PAT_STACK;  // frames of one lane; deeper walks give KPE_UNDECIDED
constexpr uint32_t PF_MAP = 0, PF_AMAPS = 1, PF_APOS = 2;
#ifndef KPE_PAT_LCACHE
#define KPE_PAT_LCACHE 0  // member lookups a lane remembers across the rules of its row (0: off; 4 entries
                          // measured C5 9.25 / C3 3.06 ms against 6.15 / 2.08: 135 VGPRs, one wave per
                          // SIMD fewer, profiles/r06_h)
#endif
#ifndef KPE_PAT_FLAT
#define KPE_PAT_FLAT 2  // maps of inline depth <= this resolve in their BEGIN step (0: all through frames;
                        // C5 / C3 ms, profiles/r03_e_inline: 0 14.2 / 5.3, 1 12.9 / 5.6, 2 at 4 waves 15.1 / 7.1
                        // (spills), 2 at 3 waves 13.0 / 5.2, 3 15.3 / 8.0)
#endif

// The tape as the VM reads it: entry i (an absolute tape index) is p[i - base] (a staged copy of a
// tape range, or the tape itself with base 0). Round 3 measured a kernel that staged batches of
// rows' tape segments in LDS and ran one lane per cell: C5 55-120 ms against the lane-per-row
// kernel's 15.6 (profiles/r03_b_ldstape, r03_d_tapeframes), so every walk now reads the tape in
// HBM; the view stays for the host check builds' bounded copies.
struct DocView {
  const uint2* p;
  uint32_t base;
#if defined(KPE_PATVM_CHECK) && KPE_PATVM_CHECK
  uint64_t lim;  // entries present at p (host check builds: an index outside flags bit 12)
  uint32_t* err;
  __device__ __forceinline__ uint2 operator[](uint64_t i) const {
    if (i < base || i - base >= lim) {
      *err |= 1u << 12;
      return p[0];
    }
    return p[i - base];
  }
#else
  __device__ __forceinline__ uint2 operator[](uint64_t i) const { return p[(uint32_t)i - base]; }
#endif
};
#if defined(KPE_PATVM_CHECK) && KPE_PATVM_CHECK
#define PV_DOCVIEW(a, ptr, b, n) DocView{(ptr), (b), (n), (a).err}
#else
#define PV_DOCVIEW(a, ptr, b, n) DocView{(ptr), (b)}
#endif

// Bounds-checked table reads in KPE_PATVM_CHECK builds (scripts/patvm_check.cpp, the
// libkpe_pvchk.so diagnostic): an out-of-range index reads element 0 instead and sets
// bit `code` of *a.err, so a bad index shows up as a flag, never as a fault.
#if defined(KPE_PATVM_CHECK) && KPE_PATVM_CHECK
__device__ __forceinline__ uint32_t pv_fail(const PatArgs& a, uint32_t code) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(a.err, 1u << code);
#else
  *a.err |= 1u << code;
#endif
  return 0u;
}
#define PV(i, n, code) ((uint64_t)(i) < (uint64_t)(n) ? (i) : pv_fail(a, code))
#define PVD(i) ((uint64_t)(i) < a.ndoc ? (i) : pv_fail(a, 9))
#else
#define PV(i, n, code) (i)
#define PVD(i) (i)
#endif

// Program tables (nodes, members, lists, leaves, string conditions, operand records): the lanes
// of a wave walk the same rule's pattern in step, so an index is usually the same in every active
// lane; then the record is read with a scalar load through the constant cache instead of a vector
// load through L1 / L2 (the tables are read-only while the kernel runs).
template <class T>
__device__ __forceinline__ T pu_load(const T* p, uint32_t i) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t u = __builtin_amdgcn_readfirstlane(i);
  if (__ballot(i != u) == 0ull) return sld(p, u);
#endif
  return p[i];
}
#if defined(KPE_PATVM_CHECK) && KPE_PATVM_CHECK
#define PU(tbl, i, n, code) ((tbl)[PV(i, n, code)])
#else
#define PU(tbl, i, n, code) pu_load((tbl), (uint32_t)(i))
#endif

// children of container entry e: entries [first, end) of its body
#define PV_KIDS(e, first, end)                   \
  const uint32_t first##_b = doc[PVD(e)].y;      \
  const uint32_t first = first##_b + 1u;         \
  const uint32_t end = first + doc[PVD(first##_b)].x

// member named key1 (the flattener keeps only the last of duplicate names, as a Go map
// decode does); kNoNode if absent
__device__ __forceinline__ uint32_t pat_lookup(const PatArgs& a, DocView doc, uint32_t m, uint32_t key1) {
  if (key1 == 0u) return kNoNode;
  PV_KIDS(m, c, end);
  uint32_t i = c;
  for (; i + 4u <= end; i += 4u) {  // four independent entry loads per step
    const uint2 n0 = doc[PVD(i)], n1 = doc[PVD(i + 1u)], n2 = doc[PVD(i + 2u)], n3 = doc[PVD(i + 3u)];
    if (DN_KEY(n0.x) == key1) return i;
    if (DN_KEY(n1.x) == key1) return i + 1u;
    if (DN_KEY(n2.x) == key1) return i + 2u;
    if (DN_KEY(n3.x) == key1) return i + 3u;
  }
  for (; i < end; ++i)
    if (DN_KEY(doc[PVD(i)].x) == key1) return i;
  return kNoNode;
}
// ExpandInMetadata: first string member whose name matches the glob (bitset over D_KEY)
__device__ __forceinline__ uint32_t pat_lookup_glob(const PatArgs& a, DocView doc, uint32_t m, uint32_t loc) {
  PV_KIDS(m, c0, end);
  for (uint32_t c = c0; c < end; ++c) {
    const uint2 n = doc[PVD(c)];
    const uint32_t k1 = DN_KEY(n.x);
    if (k1 && DN_KIND(n.x) == DN_SCALAR && SC_TYPE(a.scal[PV(n.y, a.nscal, 7)].flags) == SC_T_STR &&
        ((a.pbuf[PV(loc + ((k1 - 1u) >> 5), a.npbuf, 10)] >> ((k1 - 1u) & 31u)) & 1u))
      return c;
  }
  return kNoNode;
}

// Eight bytes at any address of a device text buffer (pattern bytes, scalar texts): two aligned
// 8-byte loads and a funnel shift instead of eight byte loads (buffers carry 16 bytes of slack,
// kpe_api.cpp upload; the bytes past a string are masked off by the caller)
__device__ __forceinline__ uint64_t ld8u(const uint8_t* p) {
  const uintptr_t x = reinterpret_cast<uintptr_t>(p);
  const uint64_t* w = reinterpret_cast<const uint64_t*>(x & ~(uintptr_t)7);
  const uint32_t sh = (uint32_t)(x & 7u) * 8u;
  const uint64_t lo = w[0];
  return sh ? (lo >> sh) | (w[1] << (64u - sh)) : lo;
}
__device__ __forceinline__ bool bytes_eq_w(const uint8_t* a, const uint8_t* b, int n) {
  for (int i = 0; i < n; i += 8) {
    uint64_t d = ld8u(a + i) ^ ld8u(b + i);
    if (n - i < 8) d &= (1ull << (8u * (uint32_t)(n - i))) - 1ull;
    if (d) return false;
  }
  return true;
}
// compareString / exact-equality match: literal classes inline, contains / glob out of line
__device__ __forceinline__ bool pv_match(const KpePat pt, const uint8_t* pb, const uint8_t* s, int sn) {
  const uint8_t* lit = pb + pt.off;
  const int ln = (int)pt.len;
  switch (pt.kind) {
    case PK_ANY: return true;
    case PK_NONEMPTY: return sn > 0;
    case PK_EXACT: return sn == ln && bytes_eq_w(lit, s, ln);
    case PK_PREFIX: return sn >= ln && bytes_eq_w(lit, s, ln);
    case PK_SUFFIX: return sn >= ln && bytes_eq_w(lit, s + sn - ln, ln);
    default: return pat_match(pt, pb, s, sn);
  }
}

// Quantity.Cmp on comparison keys (goval::qty_key): sign, order, 38-digit aligned mantissa
__device__ __forceinline__ int qcmp(bool vneg, int64_t vo, uint64_t vlo, uint64_t vhi, bool pneg, int64_t po,
                                    uint64_t plo, uint64_t phi) {
  const int sv = (vlo | vhi) ? (vneg ? -1 : 1) : 0, sp = (plo | phi) ? (pneg ? -1 : 1) : 0;
  if (sv != sp) return sv < sp ? -1 : 1;
  if (sv == 0) return 0;
  int mag;
  if (vo != po) mag = vo < po ? -1 : 1;
  else if (vhi != phi) mag = vhi < phi ? -1 : 1;
  else mag = vlo == plo ? 0 : (vlo < plo ? -1 : 1);
  return sv * mag;
}
__device__ __forceinline__ bool op_holds(uint32_t op, int c) {
  switch (op) {
    case PC_EQ: return c == 0;
    case PC_NE: return c != 0;
    case PC_GT: return c > 0;
    case PC_LT: return c < 0;
    case PC_GE: return c >= 0;
    default: return c <= 0;  // PC_LE
  }
}
// validateString (pattern.go:201-305): duration, then quantity, then wildcard string compare
__device__ __forceinline__ bool pat_cond(const PatArgs& a, const KpeScalar* v, uint32_t vf, const KpeCond* cd) {
  const uint32_t cop = cd->op, op = PC_OP(cop);
  if ((cop & PC_DUR) && (vf & SC_DUR)) {
    const int64_t x = v->dur, y = cd->dur;
    return op_holds(op, x < y ? -1 : (x > y ? 1 : 0));
  }
  if ((cop & PC_QTY) && (vf & SC_QTY))
    return op_holds(op, qcmp(vf & SC_QNEG, v->qexp, v->qlo, v->qhi, cop & PC_QNEG, cd->qexp, cd->qlo, cd->qhi));
  if (op != PC_EQ && op != PC_NE) return false;
  if (!(vf & SC_TEXT)) return false;
  const bool m = pv_match(PU(a.pats, cd->pat, a.npats, 6), a.pat_bytes, a.scal_text + v->text_off, (int)v->text_len);
  return op == PC_NE ? !m : m;
}
__device__ __forceinline__ int64_t go_f2i(double f) {
  return (f >= -9223372036854775808.0 && f < 9223372036854775808.0) ? (int64_t)f : INT64_MIN;
}
// ---- pattern variables (substitutePatterns, validate_resource.go:456-476) ----------------
// A resolved variable of the row: its scalar record and text base (PVK_NUM: null record)
__device__ __forceinline__ const KpeScalar* pv_scalar(const PatArgs& a, uint2 x, const uint8_t** tb) {
  if (x.x == PVK_SCAL) {
    *tb = a.scal_text;
    return a.scal + PV(x.y, a.nscal, 7);
  }
  *tb = a.ctext;
  return a.ctab + x.y;
}
struct TPiece {
  const uint8_t* p;  // null: the decimal digits of `num` (an elementIndex)
  int n;
  uint32_t num;
};
constexpr int kTPieces = 8;  // program.cpp var_leaf bound
// The template's pieces after substitution (substituteVarInPattern: a string as is, a number /
// bool / null json.Marshal-ed; kpe_cond_kernel already made other values undecided). Returns
// the total length.
__device__ __forceinline__ int tmpl_pieces(const PatArgs& a, const KpeLeaf* L, const uint2* pv, TPiece* pc) {
  int total = 0;
  for (uint32_t k = 0; k < L->nc && k < (uint32_t)kTPieces; ++k) {
    const uint2 t = a.ptmpl[L->c0 + k];
    TPiece q;
    if ((t.x & 1u) == PT_TEXT) {  // PT_TEXT | len << 1
      q = TPiece{a.ttext + t.y, (int)(t.x >> 1), 0u};
    } else {
      const uint2 x = pv[t.y];
      if (x.x == PVK_NULL) {
        q = TPiece{reinterpret_cast<const uint8_t*>("null"), 4, 0u};
      } else if (x.x == PVK_NUM) {  // json.Marshal of a float64 index: its decimal digits
        int d = 1;
        for (uint32_t y = x.y; y >= 10u; y /= 10u) ++d;
        q = TPiece{nullptr, d, x.y};
      } else {
        const uint8_t* tb;
        const KpeScalar* s = pv_scalar(a, x, &tb);
        const uint32_t ty = SC_TYPE(s->flags);
        // floats: the fmt.Sprint text after the compareString text (no exponent: checked)
        q = ty == SC_T_FLOAT ? TPiece{tb + s->text_off + s->text_len, (int)s->sp_len, 0u}
                             : TPiece{tb + s->text_off, (int)s->text_len, 0u};
      }
    }
    pc[k] = q;
    total += q.n;
  }
  return total;
}
__device__ __forceinline__ uint8_t tp_at(const TPiece* pc, int np, int i) {
  for (int k = 0; k < np; ++k) {
    if (i < pc[k].n) {
      if (pc[k].p) return pc[k].p[i];
      uint32_t x = pc[k].num;
      for (int j = pc[k].n - 1; j > i; --j) x /= 10u;
      return (uint8_t)('0' + x % 10u);
    }
    i -= pc[k].n;
  }
  return 0;
}
// go-wildcard glob of the template's bytes [pb, pe) against s (strmatch.inl glob)
__device__ __forceinline__ bool tp_glob(const TPiece* pc, int np, int pb, int pe, const uint8_t* s, int sn) {
  if (pe == pb) return sn == 0;
  int pi = pb, si = 0, star = -1, mark = 0;
  while (si < sn) {
    const uint8_t c = pi < pe ? tp_at(pc, np, pi) : 0;
    if (pi < pe && c == '?') {
      ++pi;
      si += rune_len(s, si, sn);
    } else if (pi < pe && c == '*') {
      star = pi++;
      mark = si;
    } else if (pi < pe && c == s[si]) {
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
  while (pi < pe && tp_at(pc, np, pi) == '*') ++pi;
  return pi == pe;
}
// The resolved leaf equals the string "*" (the default handler's presence check)
__device__ __forceinline__ bool pat_var_star(const PatArgs& a, uint32_t li, const uint2* pv) {
  const KpeLeaf Lv = PU(a.leaves, li, a.nleaves, 4);
  const KpeLeaf* L = &Lv;
  if (L->type == PL_VAR) {
    const uint2 x = pv[L->c0];
    if (x.x != PVK_SCAL && x.x != PVK_CONST) return false;
    const uint8_t* tb;
    const KpeScalar* s = pv_scalar(a, x, &tb);
    return SC_TYPE(s->flags) == SC_T_STR && s->text_len == 1u && tb[s->text_off] == '*';
  }
  if (L->type != PL_TMPL) return false;
  TPiece pc[kTPieces];
  const int np = (int)(L->nc < (uint32_t)kTPieces ? L->nc : (uint32_t)kTPieces);
  return tmpl_pieces(a, L, pv, pc) == 1 && tp_at(pc, np, 0) == '*';
}

// PMF_VKEY: the member of resource map m named by the row's substituted key template (leaf li),
// kNoNode if absent. *und is set where the device does not follow the reference: a substituted
// key that parses as an anchor (anchor.Parse: TrimSpace, then `^([+<=X^])?\((.+)\)$`), that
// equals another key of the map (a rename onto it, traverse.go:108-114, depends on Go's map
// order), that holds a glob under ExpandInMetadata, or (ORDER: the failure-path walk) that sorts
// to another place among the map's plain keys than the compiled walk order gives it. An anchored
// key (bval bit 2: the template is the whole written key, "=(" + key + ")", pad[2] = the anchor
// text's lengths before | after the key) keeps its anchor, needs a non-empty key, and its place
// among the map's anchors is checked in every walk; the member is looked up by the key inside.
template <bool ORDER>
__device__ __forceinline__ uint32_t pat_lookup_vkey(const PatArgs& a, DocView doc, uint32_t m, uint32_t li,
                                                    const uint2* pv, uint32_t* und) {
  const KpeLeaf L = PU(a.leaves, li, a.nleaves, 4);
  TPiece pc[kTPieces];
  int np = 1, n;
  if (L.type == PL_VAR) {  // a string (kpe_cond_kernel: PVF_KEY)
    const uint8_t* tb;
    const KpeScalar* s = pv_scalar(a, pv[L.c0], &tb);
    pc[0] = TPiece{tb + s->text_off, (int)s->text_len, 0u};
    n = (int)s->text_len;
  } else {
    np = (int)(L.nc < (uint32_t)kTPieces ? L.nc : (uint32_t)kTPieces);
    n = tmpl_pieces(a, &L, pv, pc);
  }
  const bool anc = (L.bval & 4u) != 0u;
  const int pre = anc ? (int)(L.pad[2] & 0xFFFFu) : 0, kn = anc ? n - pre - (int)(L.pad[2] >> 16) : n;
  if (anc) {
    if (kn < 1) {  // "=()" is no anchor (`.+`): a plain key the device does not track
      *und = 1u;
      return kNoNode;
    }
  } else {  // anchor.Parse of the substituted key
    int b = 0, e = n;
    auto ws = [](uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); };
    while (b < e && ws(tp_at(pc, np, b))) ++b;
    while (e > b && ws(tp_at(pc, np, e - 1))) --e;
    if (e - b >= 3 && tp_at(pc, np, e - 1) == ')') {
      const uint8_t c0 = tp_at(pc, np, b);
      const bool mod = c0 == '+' || c0 == '<' || c0 == '=' || c0 == 'X' || c0 == '^';
      if (c0 == '(' || (mod && e - b >= 4 && tp_at(pc, np, b + 1) == '(')) {
        *und = 1u;
        return kNoNode;
      }
    }
  }
  if (ORDER && (L.bval & 2u)) {  // the map has other keys with variables: their walk order is not kept
    *und = 1u;
    return kNoNode;
  }
  if (L.bval & 1u) {  // ExpandInMetadata target: a substituted glob would be expanded
    for (int i = 0; i < n; ++i) {
      const uint8_t c = tp_at(pc, np, i);
      if (c == '*' || c == '?') {
        *und = 1u;
        return kNoNode;
      }
    }
  }
  // Go string order of the substituted text [o, o + len) against t: -1 / 0 / 1
  auto cmp = [&](int o, int len, const uint8_t* t, int tn) -> int {
    for (int i = 0; i < len && i < tn; ++i) {
      const uint8_t x = tp_at(pc, np, o + i);
      if (x != t[i]) return x < t[i] ? -1 : 1;
    }
    return len == tn ? 0 : (len < tn ? -1 : 1);
  };
  const uint8_t* sib = a.ttext + L.pad[0];
  const uint32_t nsib = L.pad[1] & 0xFFFFu, at = L.pad[1] >> 16;
  for (uint32_t k = 0; k < nsib; ++k) {
    const int tn = (int)sib[0] | (int)sib[1] << 8;
    const int c = cmp(0, n, sib + 2, tn);
    if (c == 0 || ((ORDER || anc) && (k < at ? c < 0 : c > 0))) {
      *und = 1u;
      return kNoNode;
    }
    sib += 2 + tn;
  }
  PV_KIDS(m, c0, end);
  for (uint32_t c = c0; c < end; ++c) {
    const uint32_t k1 = DN_KEY(doc[PVD(c)].x);
    if (!k1 || k1 > a.nkeyd) continue;
    const uint32_t o0 = a.key_off[k1 - 1u], o1 = a.key_off[k1];
    if ((int)(o1 - o0) == kn && cmp(pre, kn, a.key_bytes + o0, kn) == 0) return c;
  }
  return kNoNode;
}

__device__ __forceinline__ bool leaf_float(const KpeScalar* v, uint32_t vf, double pf) {  // validateFloatPattern
  const uint32_t t = SC_TYPE(vf);
  if (t == SC_T_INT) return pf == trunc(pf) && go_f2i(pf) == v->ival;
  if (t == SC_T_FLOAT) return v->fval == pf;
  if (t == SC_T_STR) return (vf & SC_PFLOAT) && v->fval == pf;
  return false;
}
__device__ __forceinline__ bool leaf_nil(const KpeScalar* v, uint32_t vf) {  // validateNilPattern
  switch (SC_TYPE(vf)) {
    case SC_T_NULL: return true;
    case SC_T_BOOL: return !(vf & SC_BTRUE);
    case SC_T_INT: return v->ival == 0;
    case SC_T_FLOAT: return v->fval == 0.0;
    default: return v->text_len == 0u;
  }
}

// pattern.Validate (pattern.go:26-50) of scalar `sid` (kNoNode: a map / list value); pv: the
// row's resolved pattern variables; *und set where the device leaves the cell undecided
__device__ __forceinline__ bool pat_leaf_eval(const PatArgs& a, uint32_t sid, uint32_t li, const uint2* pv,
                                              uint32_t* und) {
  if (sid == kNoNode) return false;  // no scalar validator accepts a map / list
  const KpeLeaf Lv = PU(a.leaves, li, a.nleaves, 4);
  const KpeLeaf* L = &Lv;
  const KpeScalar* v = a.scal + PV(sid, a.nscal, 7);
  const uint32_t vf = v->flags, t = SC_TYPE(vf);
  if (L->type == PL_VAR) {  // the variable's typed value is the pattern (context numbers: float64)
    const uint2 x = pv[L->c0];
    if (x.x == PVK_NULL) return leaf_nil(v, vf);
    if (x.x == PVK_NUM) return leaf_float(v, vf, (double)x.y);
    const uint8_t* tb;
    const KpeScalar* S = pv_scalar(a, x, &tb);
    switch (SC_TYPE(S->flags)) {
      case SC_T_NULL: return leaf_nil(v, vf);
      case SC_T_BOOL: return t == SC_T_BOOL && ((vf & SC_BTRUE) != 0u) == ((S->flags & SC_BTRUE) != 0u);
      case SC_T_INT: return leaf_float(v, vf, (double)S->ival);
      case SC_T_FLOAT: return leaf_float(v, vf, S->fval);
      default: {  // a plain string pattern (SC_PSIMPLE): value == pattern, then validateString Equal
        const uint8_t* p = tb + S->text_off;
        const int pn = (int)S->text_len;
        if (t == SC_T_STR && (int)v->text_len == pn && bytes_eq_w(a.scal_text + v->text_off, p, pn)) return true;
        if ((S->flags & SC_DUR) && (vf & SC_DUR)) return v->dur == S->dur;
        if ((S->flags & SC_QTY) && (vf & SC_QTY))
          return qcmp(vf & SC_QNEG, v->qexp, v->qlo, v->qhi, S->flags & SC_QNEG, S->qexp, S->qlo, S->qhi) == 0;
        if (!(vf & SC_TEXT)) return false;
        return glob(p, pn, a.scal_text + v->text_off, (int)v->text_len);
      }
    }
  }
  if (L->type == PL_TMPL) {  // a string with variables spliced in
    TPiece pc[kTPieces];
    const int np = (int)(L->nc < (uint32_t)kTPieces ? L->nc : (uint32_t)kTPieces);
    const int n = tmpl_pieces(a, L, pv, pc);
    if (t == SC_T_STR && (int)v->text_len == n) {  // value == pattern
      const uint8_t* s = a.scal_text + v->text_off;
      bool eq = true;
      for (int i = 0; i < n && eq; ++i) eq = tp_at(pc, np, i) == s[i];
      if (eq) return true;
    }
    for (int i = 0; i < n; ++i) {  // `|` / `&` splits: not restated on the device
      const uint8_t c = tp_at(pc, np, i);
      if (c == '|' || c == '&') {
        *und = 1u;
        return false;
      }
    }
    int b = 0, e = n;  // strings.Trim(" ") and TrimSpace (ASCII; a non-ASCII edge: undecided)
    auto ws = [](uint8_t c) { return c == ' ' || (c >= '\t' && c <= '\r'); };
    while (b < e && ws(tp_at(pc, np, b))) ++b;
    while (e > b && ws(tp_at(pc, np, e - 1))) --e;
    if (b < e) {
      const uint8_t c0 = tp_at(pc, np, b), c1 = tp_at(pc, np, e - 1);
      // an operator prefix, a duration / quantity / range operand, or a non-ASCII edge
      if (c0 >= 0x80 || c1 >= 0x80 || (e - b >= 2 && (c0 == '<' || c0 == '>' || c0 == '!')) || c0 == '+' ||
          c0 == '-' || c0 == '.' || (c0 >= '0' && c0 <= '9')) {
        *und = 1u;
        return false;
      }
    }
    if (!(vf & SC_TEXT)) return false;  // compareString of nil
    return tp_glob(pc, np, b, e, a.scal_text + v->text_off, (int)v->text_len);
  }
  switch (L->type) {
    case PL_BOOL: return t == SC_T_BOOL && ((vf & SC_BTRUE) != 0u) == (L->bval != 0u);
    case PL_INT:
      if (t == SC_T_INT) return v->ival == L->ival;
      if (t == SC_T_FLOAT) return v->fval == trunc(v->fval) && go_f2i(v->fval) == L->ival;
      if (t == SC_T_STR) return (vf & SC_PINT) && v->ival == L->ival;
      return false;
    case PL_FLOAT:
      if (t == SC_T_INT) return L->fval == trunc(L->fval) && go_f2i(L->fval) == v->ival;
      if (t == SC_T_FLOAT) return v->fval == L->fval;
      if (t == SC_T_STR) return (vf & SC_PFLOAT) && v->fval == L->fval;
      return false;
    case PL_NIL:
      switch (t) {
        case SC_T_NULL: return true;
        case SC_T_BOOL: return !(vf & SC_BTRUE);
        case SC_T_INT: return v->ival == 0;
        case SC_T_FLOAT: return v->fval == 0.0;
        default: return v->text_len == 0u;
      }
    case PL_STR: {
      if (t == SC_T_STR && pv_match(PU(a.pats, L->exact, a.npats, 6), a.pat_bytes, a.scal_text + v->text_off, (int)v->text_len))
        return true;  // value == pattern
      bool group = true;  // OR over `|` alternatives of an AND over their `&` terms
      const uint32_t c0 = L->c0, ce = c0 + L->nc;
      for (uint32_t i = c0; i < ce; ++i) {
        const KpeCond cdv = PU(a.conds, i, a.nconds, 5);
        const KpeCond* cd = &cdv;
        const uint32_t cop = cd->op;
        if ((cop & PC_NEWGROUP) && i != c0) {
          if (group) return true;
          group = true;
        }
        bool r = group && pat_cond(a, v, vf, cd);
        if (cop & PC_OR2) {  // NotInRange: `< lo` OR `> hi`
          ++i;
          const KpeCond cd2 = PU(a.conds, i, a.nconds, 5);
          r = group && (r || pat_cond(a, v, vf, &cd2));
        }
        group = group && r;
      }
      return group;
    }
    default: return false;
  }
}
// pat_leaf_eval through the binding's leaf table where the leaf has a slot: one bit load
// instead of the scalar record, its text and the comparison. LT: the program's every leaf has a
// slot or is PL_NEVER (no variables), so the instance holds no comparison code at all.
template <bool LT = false>
__device__ __forceinline__ bool pat_leaf(const PatArgs& a, uint32_t sid, uint32_t li, const uint2* pv, uint32_t* und) {
  if (sid == kNoNode) return false;
  if (LT) {
    const uint32_t slot = PU(a.lslot, li, a.nleaves, 4);
    return slot != KPE_NO_LSLOT && ((a.ltab[(size_t)slot * a.ltab_words + (sid >> 5)] >> (sid & 31u)) & 1u);
  }
  if (a.ltab) {
    const uint32_t slot = PU(a.lslot, li, a.nleaves, 4);
    if (slot != KPE_NO_LSLOT) return (a.ltab[(size_t)slot * a.ltab_words + (sid >> 5)] >> (sid & 31u)) & 1u;
  }
  return pat_leaf_eval(a, sid, li, pv, und);
}

// pat_leaf of a scalar-leaf member m (leaf li): its bound table slot (m.w) instead of lslot[li]
template <bool LT = false>
__device__ __forceinline__ bool pat_leaf_mem(const PatArgs& a, uint32_t sid, const uint4& m, uint32_t li,
                                             const uint2* pv, uint32_t* und) {
  if (m.x & (PMF_GLOB | PMF_VKEY)) return pat_leaf<LT>(a, sid, li, pv, und);
  if (sid == kNoNode) return false;
  if (LT) return m.w != KPE_NO_LSLOT && ((a.ltab[(size_t)m.w * a.ltab_words + (sid >> 5)] >> (sid & 31u)) & 1u);
  if (a.ltab && m.w != KPE_NO_LSLOT) return (a.ltab[(size_t)m.w * a.ltab_words + (sid >> 5)] >> (sid & 31u)) & 1u;
  return pat_leaf_eval(a, sid, li, pv, und);
}

// scalar id of node c (kNoNode for maps / lists); an absent member is null
__device__ __forceinline__ uint32_t node_sid(const PatArgs& a, DocView doc, uint32_t c) {
  if (c == kNoNode) return SC_NULL_ID;
  const uint2 n = doc[PVD(c)];
  return DN_KIND(n.x) == DN_SCALAR ? n.y : kNoNode;
}

struct PFrame {
  uint32_t kind_k;  // PF_* | index << 2 (MAP: member k, APOS: pattern element j)
  uint32_t r, pi;   // resource node, pattern node
  uint32_t cnt;     // MAP: applied | skips << 16; arrays: applied
  uint32_t cur;     // arrays: element cursor; MAP existence search: element cursor
  uint32_t x;       // arrays: skips; MAP existence search: pattern element j + 1 (0 = idle)
  uint32_t c;       // MAP existence search: the resource list node
};

// The VM is one loop over three states, so every piece of the walk exists once in the
// kernel: BEGIN evaluates an element against a pattern node (a leaf resolves at once, a
// map / array pushes a frame), STEP advances the top frame (it either asks for a BEGIN of
// the next child or completes), RET hands a completed verdict to the frame below. Lanes of
// a wave in different states then run each state's code once per iteration instead of
// every inlined copy. Nothing is called: a callee would reach the lane's private frame
// stack through a generic pointer, and flat accesses into the private aperture fault.
constexpr uint32_t VM_BEGIN = 0, VM_STEP = 1, VM_RET = 2;

// A lane's frame stack. FramesPriv: a lane-private array (scratch memory). FramesLds: LDS,
// word-planar (word w of frame i of the lane at b[(w * kDepth + i) * 64], b already offset by
// the lane's index in its wave), so 64 lanes at any mix of depths hit 64 distinct banks and a
// frame access costs an LDS round trip instead of a scratch one (scratch spills of 20 waves per
// CU do not fit the L1 / L2 and wait on the Infinity Cache).
struct FramesPriv {
  static constexpr int kDepth = kPatStack;
  PFrame st[kPatStack];
  __device__ __forceinline__ PFrame get(int i) const { return st[i]; }
  __device__ __forceinline__ void put(int i, const PFrame& f) { st[i] = f; }
};
#ifndef KPE_PAT_LDS_STACK
#define KPE_PAT_LDS_STACK 5  // deeper walks: kpe_pattern_deep_kernel. 4 / 5 / 6 frames, C5 9.0 / 7.0 / 7.6 ms, C3 3.1 / 3.2 / 3.5 ms (profiles/r04_n)
#endif
template <int D>
struct FramesLdsD {
  static constexpr int kDepth = D;
  static constexpr uint32_t kWords = 7u;  // PFrame
  uint32_t* b;
  __device__ __forceinline__ PFrame get(int i) const {
    const uint32_t* q = b + (uint32_t)i * 64u;
    constexpr uint32_t W = (uint32_t)kDepth * 64u;
    return PFrame{q[0], q[W], q[2 * W], q[3 * W], q[4 * W], q[5 * W], q[6 * W]};
  }
  __device__ __forceinline__ void put(int i, const PFrame& f) {
    uint32_t* q = b + (uint32_t)i * 64u;
    constexpr uint32_t W = (uint32_t)kDepth * 64u;
    q[0] = f.kind_k, q[W] = f.r, q[2 * W] = f.pi, q[3 * W] = f.cnt, q[4 * W] = f.cur, q[5 * W] = f.x, q[6 * W] = f.c;
  }
};
using FramesLds = FramesLdsD<KPE_PAT_LDS_STACK>;   // kpe_pattern_kernel
using FramesLdsDeep = FramesLdsD<kPatStack>;       // kpe_pattern_deep_kernel

template <class FS, bool LT = false>
struct PatVMT {
  const PatArgs& a;
  DocView doc;   // the whole tape (absolute entry indices)
  uint32_t root;      // this resource's root entry (or a foreach element's entry)
  const uint2* pv;    // the row's resolved pattern variables
  uint32_t und;       // a leaf the device does not decide was reached
  uint32_t reg, val;  // AnchorMap: slots registered / present in the resource
  int sp;
  FS fs;
  uint32_t* tr;  // TRACE walks: the path record of the last failure (KPE_TRACE_WORDS words)
#if KPE_PAT_LCACHE
  // The lane's last KPE_PAT_LCACHE plain member lookups (tape entry, key) -> member entry: the
  // rules of a row walk the same spine (root -> spec -> containers) one after another, and each
  // lookup there is a chain of dependent body loads. Tape entries are absolute, so entries of an
  // earlier row never match a later one; the aggregate initialisers of the VM leave the entries
  // zero, and key 0 (a name absent from the corpus) is never cached.
  uint32_t lcm[KPE_PAT_LCACHE], lck[KPE_PAT_LCACHE], lcr[KPE_PAT_LCACHE];
  uint32_t lcn;
  __device__ __forceinline__ uint32_t mlookup(uint32_t m, uint32_t key1) {
    if (key1 == 0u) return kNoNode;
#pragma unroll
    for (int i = 0; i < KPE_PAT_LCACHE; ++i)
      if (lcm[i] == m && lck[i] == key1) return lcr[i];
    const uint32_t c = pat_lookup(a, doc, m, key1);
    const uint32_t at = lcn % (uint32_t)KPE_PAT_LCACHE;
#pragma unroll
    for (int i = 0; i < KPE_PAT_LCACHE; ++i)
      if (at == (uint32_t)i) lcm[i] = m, lck[i] = key1, lcr[i] = c;
    ++lcn;
    return c;
  }
#else
  __device__ __forceinline__ uint32_t mlookup(uint32_t m, uint32_t key1) { return pat_lookup(a, doc, m, key1); }
#endif

  // ---- failing paths (TRACE walks only; kpe_pattern_trace_kernel) ----
  // PatternError.Path (validate.go:31-56): the reference returns the path of the element where
  // the failure was found; a failure a condition / global anchor or an existence search
  // absorbs is followed by further walking, so the last failure recorded is the one that
  // reaches the root. A component is a pattern member (the key the handler appends:
  // anchor.Key() or the raw key), an ExpandInMetadata key (the matched resource member's
  // name) or an array index.
  __device__ __forceinline__ uint32_t mcomp(uint32_t r, uint32_t mi) {
    const uint4 m = PU(a.members, mi, a.nmembers, 2);
    if (m.x & (PMF_GLOB | PMF_VKEY)) {  // the resource member's name (a VKEY member found by it)
      const uint32_t c = lookup<true>(m, r);
      if (c != kNoNode) return KPE_TC_KEY | (DN_KEY(doc[PVD(c)].x) - 1u);
    }
    return mi;  // an absent VKEY member: the host renders no path for it
  }
  // the resource member a pattern member names (kNoNode: absent); TRACE: failure-path walks
  template <bool TRACE>
  __device__ __forceinline__ uint32_t lookup(const uint4& m, uint32_t r) {
    if (m.x & PMF_GLOB) return pat_lookup_glob(a, doc, r, m.w);
    if (m.x & PMF_VKEY) return pat_lookup_vkey<TRACE>(a, doc, r, m.w, pv, &und);
    return TRACE ? pat_lookup(a, doc, r, m.y) : mlookup(r, m.y);
  }
  __device__ __forceinline__ void tput(uint32_t& n, uint32_t c) {
    if (n < KPE_TRACE_WORDS - 1u) tr[1u + n] = c;
    ++n;
  }
  // the path of frames [0, nf) (each frame's current child) followed by `extra` (~0u: none)
  __device__ __forceinline__ void snap(int nf, uint32_t extra) {
    uint32_t n = 0;
    for (int i = 0; i < nf; ++i) {
      const PFrame F = fs.get(PV(i, FS::kDepth, 11));
      const uint32_t kind = F.kind_k & 3u;
      if (kind == PF_MAP) {
        tput(n, mcomp(F.r, PU(a.nodes, F.pi, a.nnodes, 1).y + (F.kind_k >> 2)));
        if (F.x) tput(n, KPE_TC_IDX | (F.cur - (doc[PVD(F.c)].y + 1u)));  // existence search element
      } else if (kind == PF_AMAPS) {
        tput(n, KPE_TC_IDX | (F.cur - (doc[PVD(F.r)].y + 1u)));
      } else {
        tput(n, KPE_TC_IDX | (F.kind_k >> 2));
      }
    }
    if (extra != ~0u) tput(n, extra);
    tr[0] = (tr[0] & 0xFFFF0000u) | (n < KPE_TRACE_WORDS ? n : (KPE_TRACE_WORDS - 1u) | KPE_TR_TRUNC);
  }

  // validateMap (validate.go:118-175) of a map of inline depth <= D (schema.h PNF_FLAT) against the
  // resource map whose body is at tape index b: the body (at most 8 entries) is read once into
  // registers, every member's handler (anchor/handlers.go) resolves against it in the member order
  // the STEP state uses, and a map-valued member recurses. PE_NONE: some body on the way holds
  // more than 8 entries, and the frame path validates the whole map (what the attempt set in the
  // AnchorMap and `und` the frame walk sets again: it visits the same maps and leaves first).
  template <int D>
  __device__ __forceinline__ uint32_t flat_map(uint32_t b, const KpePNode pn) {
    // the body header and its first 8 entry slots in one round of independent loads (the tape
    // carries slack past its last body, kpe_api.cpp upload), then the slots past the count cleared
    uint2 e[8];
#if defined(KPE_PATVM_CHECK) && KPE_PATVM_CHECK
    const uint32_t cnt = doc[PVD(b)].x;
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) e[j] = j < cnt ? doc[PVD(b + 1u + j)] : uint2{0u, 0u};
#else
    const uint32_t cnt = doc[b].x;
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) e[j] = doc[b + 1u + j];
#pragma unroll
    for (uint32_t j = 0; j < 8u; ++j) e[j] = j < cnt ? e[j] : uint2{0u, 0u};
#endif
    if (cnt > 8u) return PE_NONE;
    // the entry named key1 (key ids are >= 1; padding entries carry key 0): index j, or 8
    auto find = [&](uint32_t key1) -> uint32_t {
      uint32_t f = 8u;
#pragma unroll
      for (uint32_t j = 0; j < 8u; ++j) f = (key1 != 0u && DN_KEY(e[j].x) == key1) ? j : f;
      return f;
    };
    auto entry = [&](uint32_t j) -> uint2 {
      uint2 x{0u, 0u};
#pragma unroll
      for (uint32_t q = 0; q < 8u; ++q) x = q == j ? e[q] : x;
      return x;
    };
    const uint32_t m0 = pn.y, nanch = pn.z & 0xFFFFu, nmem = pn.z >> 16;
    for (uint32_t k = 0; k < nmem; ++k) {  // AnchorMap.CheckAnchorInResource (anchormap.go:33-48)
      const uint4 m = PU(a.members, m0 + k, a.nmembers, 2);
      if (m.x & PMF_SLOT) {
        const uint32_t bit = 1u << PM_SLOT(m.x);
        reg |= bit;
        if (find(m.y) < 8u) val |= bit;
      }
    }
    uint32_t applied = 0, skips = 0;
    for (uint32_t k = 0;; ++k) {
      if (k == nanch && applied == 0u && skips > 0u) return PE_SKIP;  // every anchor skipped
      if (k == nmem) return PE_OK;
      const uint4 m = PU(a.members, m0 + k, a.nmembers, 2);
      const uint32_t h = PM_HANDLER(m.x), j = find(m.y);
      const uint2 x = entry(j);
      uint32_t ek;
      if (h == PM_NEG) {
        ek = j < 8u ? PE_NEG : PE_OK;
      } else if (j == 8u && h != PM_DEFAULT) {
        ek = h == PM_COND ? PE_SKIP : PE_OK;  // absent: condition skips, =() <() ^() hold
      } else if ((m.x & PMF_STAR) ||
                 ((!LT && (m.x & PMF_VSTAR)) && pat_var_star(a, PU(a.nodes, m.z, a.nnodes, 1).y, pv))) {
        ek = (j < 8u && (DN_KIND(x.x) != DN_SCALAR || x.y != SC_NULL_ID)) ? PE_OK : PE_OTHER;
      } else {
        const KpePNode vn = PU(a.nodes, m.z, a.nnodes, 1);
        uint32_t v1;
        if (!(m.x & PMF_LEAF)) {  // a map value: validateResourceElement needs a map
          if (D <= 1) return PE_NONE;  // not reached: the compiler bounds the depth
          if (j == 8u || DN_KIND(x.x) != DN_MAP) {
            v1 = PE_OTHER;
          } else {
            v1 = flat_map<(D > 1 ? D - 1 : 1)>(x.y, vn);
            if (v1 == PE_NONE) return PE_NONE;
          }
        } else if (j < 8u && DN_KIND(x.x) == DN_ARR) {  // a scalar leaf against a list: every element
          const uint32_t l0 = x.y + 1u, le = l0 + doc[PVD(x.y)].x;
          v1 = PE_OK;
          for (uint32_t c = l0; c < le && v1 == PE_OK; ++c)
            if (!pat_leaf<LT>(a, node_sid(a, doc, c), vn.y, pv, &und)) v1 = PE_OTHER;
        } else {
          const uint32_t sid = j == 8u ? SC_NULL_ID : (DN_KIND(x.x) == DN_SCALAR ? x.y : kNoNode);
          v1 = pat_leaf_mem<LT>(a, sid, m, vn.y, pv, &und) ? PE_OK : PE_OTHER;
        }
        ek = (h == PM_COND || h == PM_GLOBAL) ? (v1 == PE_OK ? PE_OK : PE_SKIP) : v1;
      }
      if (k < nanch) {
        if (ek == PE_SKIP) ++skips;
        else if (ek != PE_OK) return ek;
        else ++applied;
      } else if (ek != PE_OK) {
        return ek;
      }
    }
  }

  // validate.MatchPattern (validate.go:31-56) of pattern root node `root_pi`
  template <bool TRACE>
  __device__ __forceinline__ uint32_t run(uint32_t root_pi) {
    sp = -1, reg = 0u, val = 0u;
    uint32_t state = VM_BEGIN, br = root, bpi = root_pi, v = PE_NONE;
    for (;;) {
      if (state == VM_BEGIN) {
        // ---- validateResourceElement (validate.go:71-114) ----
        const KpePNode pn = PU(a.nodes, bpi, a.nnodes, 1);
        const uint32_t rk = br == kNoNode ? 0xFFu : DN_KIND(doc[PVD(br)].x);
        state = VM_RET;
        if (pn.kind == PN_LEAF && rk != DN_ARR) {
          v = pat_leaf<LT>(a, node_sid(a, doc, br), pn.y, pv, &und) ? PE_OK : PE_OTHER;
        } else if (pn.kind == PN_LEAF || pn.kind == PN_ARR_LEAF) {  // scalar pattern vs a list
          if (rk != DN_ARR) {
            v = PE_OTHER;
          } else {
            PV_KIDS(br, c0, end);
            v = PE_OK;
            for (uint32_t c = c0; c < end && v == PE_OK; ++c)
              if (!pat_leaf<LT>(a, node_sid(a, doc, c), pn.y, pv, &und)) v = PE_OTHER;
          }
        } else if (pn.kind == PN_MAP) {
          const uint32_t pw = pn.w & PNW_DEPTH;
          if (rk != DN_MAP) {
            v = PE_OTHER;
          } else if (!TRACE && (pn.w & PNW_CHAIN) && !(pw && pw <= (uint32_t)KPE_PAT_FLAT)) {
            // one plain member: its value's verdict is the map's (no frame; TRACE walks keep the
            // frame for the member's path component)
            const uint4 m = PU(a.members, pn.y, a.nmembers, 2);
            br = mlookup(br, m.y), bpi = m.z, state = VM_BEGIN;
            continue;
          } else if (KPE_PAT_FLAT && !TRACE && pw && pw <= (uint32_t)KPE_PAT_FLAT &&
                     (v = flat_map<KPE_PAT_FLAT>(doc[PVD(br)].y, pn)) != PE_NONE) {
            // resolved from the body in registers
          } else {
            const uint32_t nmem = pn.z >> 16;
            for (uint32_t k = 0; k < nmem; ++k) {  // AnchorMap.CheckAnchorInResource (anchormap.go:33-48)
              const uint4 m = PU(a.members, pn.y + k, a.nmembers, 2);
              if (m.x & PMF_XSLOT) und = 1u;
              if (m.x & PMF_SLOT) {
                const uint32_t bit = 1u << PM_SLOT(m.x);
                reg |= bit;  // a glob key counts under its expansion (ExpandInMetadata ran first)
                if (lookup<TRACE>(m, br) != kNoNode) val |= bit;
              }
            }
            v = push(PF_MAP, br, bpi, 0u);
          }
        } else if (rk != DN_ARR || pn.kind == PN_ARR_EMPTY) {
          v = PE_OTHER;  // a list pattern needs a list; [] is "pattern Array empty"
        } else {
          PV_KIDS(br, c0, end);
          if (pn.kind == PN_ARR_POS && end - c0 < pn.z) v = PE_OTHER_NOPATH;  // length mismatch: no path
          else v = push(pn.kind == PN_ARR_POS ? PF_APOS : PF_AMAPS, br, bpi, c0);
        }
        if (TRACE && v == PE_OTHER) snap(sp + 1, ~0u);  // validateResourceElement returns its path
        if (v == PE_PUSHED) state = VM_STEP, v = PE_NONE;
        continue;
      }
      if (state == VM_RET) {
        if (sp < 0) return v;
        state = VM_STEP;  // deliver v to the frame below
        continue;
      }
      // ---- VM_STEP: advance the top frame with child verdict v (PE_NONE: none pending) ----
      PFrame F = fs.get(PV(sp, FS::kDepth, 11));
      const KpePNode pn = PU(a.nodes, F.pi, a.nnodes, 1);
      if ((F.kind_k & 3u) == PF_MAP) {
        // validateMap (validate.go:118-175) + anchor/handlers.go
        const uint32_t m0 = pn.y, nanch = pn.z & 0xFFFFu, nmem = pn.z >> 16;
        uint32_t k = F.kind_k >> 2, applied = F.cnt & 0xFFFFu, skips = F.cnt >> 16;
        uint32_t e = PE_NONE;
        bool begin_child = false;
        if (v != PE_NONE) {  // the child BEGIN of member k finished with v
          const uint32_t h = PM_HANDLER(PU(a.members, m0 + k, a.nmembers, 2).x);
          if (F.x) {  // existence search: element F.cur against pattern element F.x - 1
            if (v == PE_OK) F.x += 1u, F.cur = doc[PVD(F.c)].y + 1u;
            else F.cur += 1u;
          } else {
            e = (h == PM_COND || h == PM_GLOBAL) ? (v == PE_OK ? PE_OK : PE_SKIP) : v;
          }
        }
        for (;;) {
          if (e == PE_NONE && F.x) {  // existence anchor: each pattern map needs one matching element
            const KpePNode xl = PU(a.nodes, PU(a.members, m0 + k, a.nmembers, 2).z, a.nnodes, 1);
            PV_KIDS(F.c, c0, end);
            (void)c0;
            if (F.x - 1u >= xl.z) {
              e = PE_OK, F.x = 0u;
            } else {
              const uint32_t pj = PU(a.lists, xl.y + F.x - 1u, a.nlists, 3);
              if (PU(a.nodes, pj, a.nnodes, 1).kind == PN_BAD || F.cur >= end) {
                e = PE_OTHER, F.x = 0u;
                if (TRACE) snap(sp, mcomp(F.r, m0 + k));  // existence: the anchor key's path
              } else {
                br = F.cur, bpi = pj, begin_child = true;
                break;
              }
            }
          }
          if (e == PE_NONE) {  // start member k
            if (k == nanch && applied == 0u && skips > 0u) {  // every anchor skipped
              e = PE_SKIP;
              k = nmem + 1u;  // completes below
            } else if (k == nmem) {
              e = PE_OK;
              k = nmem + 1u;
            } else {
              const uint4 m = PU(a.members, m0 + k, a.nmembers, 2);
              const uint32_t h = PM_HANDLER(m.x);
              const uint32_t c = lookup<TRACE>(m, F.r);
              if (h == PM_NEG) {
                e = c == kNoNode ? PE_OK : PE_NEG;
                if (TRACE && e == PE_NEG) snap(sp, mcomp(F.r, m0 + k));
              } else if (c == kNoNode && h != PM_DEFAULT) {
                e = h == PM_COND ? PE_SKIP : PE_OK;  // absent: condition skips, =() <() ^() hold
              } else if ((m.x & PMF_STAR) ||
                         ((!LT && (m.x & PMF_VSTAR)) && pat_var_star(a, PU(a.nodes, m.z, a.nnodes, 1).y, pv))) {
                e = (c != kNoNode && node_sid(a, doc, c) != SC_NULL_ID) ? PE_OK : PE_OTHER;
                if (TRACE && e == PE_OTHER) snap(sp, ~0u);  // "*": the map's own path (handlers.go:124-140)
              } else if (h == PM_EXIST) {
                if (DN_KIND(doc[PVD(c)].x) != DN_ARR || PU(a.nodes, m.z, a.nnodes, 1).kind != PN_EXLIST) {
                  e = PE_OTHER;  // existence anchor on a non-list value / non-list pattern
                  if (TRACE) snap(sp, mcomp(F.r, m0 + k));
                } else {
                  F.x = 1u, F.cur = doc[PVD(c)].y + 1u, F.c = c;
                  continue;  // search
                }
              } else if ((m.x & PMF_LEAF) && (c == kNoNode || DN_KIND(doc[PVD(c)].x) != DN_ARR)) {
                // a scalar pattern against a scalar / absent value resolves in place: BEGIN's
                // pattern.Validate and RET's anchor mapping without the two VM round trips
                const uint32_t li = PU(a.nodes, m.z, a.nnodes, 1).y;
                const uint32_t v1 = pat_leaf_mem<LT>(a, node_sid(a, doc, c), m, li, pv, &und) ? PE_OK : PE_OTHER;
                if (TRACE && v1 == PE_OTHER) snap(sp, mcomp(F.r, m0 + k));
                e = (h == PM_COND || h == PM_GLOBAL) ? (v1 == PE_OK ? PE_OK : PE_SKIP) : v1;
              } else {
                br = c, bpi = m.z, begin_child = true;
                break;
              }
            }
          }
          if (k > nmem) break;  // the map itself completed with e
          // member k's verdict e
          if (k < nanch) {
            if (e == PE_SKIP) ++skips;
            else if (e != PE_OK) break;
            else ++applied;
          } else if (e != PE_OK) {
            break;
          }
          ++k, e = PE_NONE;
        }
        if (begin_child) {
          F.kind_k = PF_MAP | (k << 2), F.cnt = applied | (skips << 16);
          fs.put(sp, F);
          state = VM_BEGIN, v = PE_NONE;
        } else {
          --sp;
          state = VM_RET, v = e;
        }
        continue;
      }
      // validateArrayOfMaps / positional validateArray (validate.go:177-261)
      {
        const bool pos = (F.kind_k & 3u) == PF_APOS;
        PV_KIDS(F.r, c0, end);
        (void)c0;
        uint32_t applied = F.cnt, skips = F.x, j = F.kind_k >> 2, cur = F.cur;
        uint32_t e = PE_NONE;
        if (v != PE_NONE) {  // element `cur` finished
          if (v == PE_SKIP) ++skips;
          else if (v != PE_OK) e = v;
          else ++applied;
          cur += 1u, ++j;
        }
        if (e == PE_NONE && (pos ? j >= pn.z : cur >= end)) e = (applied == 0u && skips > 0u) ? PE_SKIP : PE_OK;
        if (e != PE_NONE) {
          --sp;
          state = VM_RET, v = e;
        } else {
          F.kind_k = (F.kind_k & 3u) | (j << 2), F.cnt = applied, F.x = skips, F.cur = cur;
          fs.put(sp, F);
          br = cur, bpi = pos ? PU(a.lists, pn.y + j, a.nlists, 3) : pn.y;
          state = VM_BEGIN, v = PE_NONE;
        }
      }
    }
  }

  __device__ __forceinline__ uint32_t push(uint32_t kind, uint32_t r, uint32_t pi, uint32_t cur) {
    if (sp + 1 >= FS::kDepth) {  // a resource as deep as a pattern nested past the lane's frame
      und = 1u;                 // stack: the cell is KPE_UNDECIDED (the caller decides)
      return PE_OTHER;
    }
    ++sp;
    fs.put(PV(sp, FS::kDepth, 11), PFrame{kind, r, pi, 0u, cur, 0u, 0u});
    return PE_PUSHED;
  }
};

// verdict of one pattern: pass / skip / fail, or error when the PatternError path is empty
using PatVM = PatVMT<FramesPriv>;

template <bool TRACE = false, class VM>
__device__ __forceinline__ uint32_t pat_match_root(VM& vm, uint32_t root) {
  const PatArgs& a = vm.a;
  vm.und = 0u;
  const uint32_t e = vm.template run<TRACE>(a.roots[PV(2 * root, a.nroots, 8)]);
  if (vm.und) return KPE_UNDECIDED_;
  if (e == PE_OK) return KPE_PASS_;
  if (e == PE_SKIP) return KPE_SKIP_;
  if (e == PE_NEG) return KPE_FAIL_;
  if (e == PE_OTHER_NOPATH || (vm.reg & ~vm.val)) return KPE_ERROR_;  // AnchorMap.KeysAreMissing
  return KPE_FAIL_;
}

// One KPE_PENDING_ pattern cell (row r, column col) of pattern rule `pi` (col2pr - 1):
// validate_resource.go:316-398: one pattern, or anyPattern's first pass / skip / fail
template <class VM>
__device__ __forceinline__ uint32_t pat_eval_cell(VM& vm, uint32_t pi) {
  const PatArgs& a = vm.a;
  const KpePatRule pr = a.rules[pi];
  if (pr.flags & PR_ANY_BAD) return KPE_ERROR_;  // anyPattern is not a list
  const bool any = (pr.flags & PR_ANY) != 0u;
  uint32_t fails = 0, skips = 0, last = KPE_PASS_;
  bool passed = false, undec = false;
  for (uint32_t k = 0; k < pr.nr && !passed && !undec; ++k) {
    last = pat_match_root(vm, pr.r0 + k);
    if (last == KPE_PASS_) passed = true;
    else if (last == KPE_SKIP_) ++skips;
    else if (last == KPE_UNDECIDED_) undec = true;
    else ++fails;  // anyPattern: an empty-path error counts as a failure
  }
  return undec ? KPE_UNDECIDED_ : !any ? last : passed ? KPE_PASS_ : (fails ? KPE_FAIL_ : (skips ? KPE_SKIP_ : KPE_PASS_));
}

// kpe_pattern_kernel's body for resource r: resolve the row's KPE_PENDING_ pattern cells.
// The pattern roots of every rule run through one VM call site (a plain pattern is one root),
// so the kernel holds a single copy of the VM: its code stays within the instruction cache.
// Rules that carry the same pattern share a memo slot (PR_MEMO_SH): the row's first pending cell
// of the slot is evaluated and the others take its verdict from `memo` (LDS bytes, slot s at
// memo[s * memo_stride]; null: no memo).
// DEFER: a cell that comes back undecided from a shallow (LDS) stack is marked KPE_DEEP_ for
// kpe_pattern_deep_kernel instead of being re-walked here (the kernel then holds one copy of the
// VM, not two).
template <class FS, bool LT = false, bool DEFER = false>
__device__ __forceinline__ void pat_eval_row(const PatArgs& a, int64_t r, FS fs, uint8_t* memo = nullptr,
                                             uint32_t memo_stride = 0) {
  uint32_t memo_ok = 0;  // slots holding this row's verdict
  PatVMT<FS, LT> vm{a, PV_DOCVIEW(a, reinterpret_cast<const uint2*>(a.doc), 0u, a.ndoc), (uint32_t)a.doc_off[r],
                a.pvals + (size_t)r * a.nvars, 0u, 0u, 0u, -1, fs, nullptr};
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  // The row's cells are scanned 64 columns at a time: the 17 aligned words that cover them are
  // loaded together (one memory round trip per 64 columns instead of one per 4) and reduced to a
  // mask of the KPE_PENDING_ cells, whose rules then run in column order, so the lanes of a wave
  // run the VM for the same pattern rule together.
  const uint64_t start = (uint64_t)r * a.R;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(a.verdicts);
  // the pending cells of the row's 64 columns from c00
  // (a rolling pair of words, not a 17-word array: an array here is put in scratch memory)
  auto pending = [&](uint32_t c00) -> uint64_t {
    const uint64_t p0 = start + c00;
    const uint32_t sh = (uint32_t)(p0 & 3u);
    const uint32_t* wp = words + (p0 >> 2);  // the buffer carries slack past the matrix
    uint64_t pend = 0;
    uint32_t lo = wp[0];
#pragma unroll
    for (uint32_t j = 0; j < 16u; ++j) {
      const uint32_t hi = wp[j + 1u];
      uint32_t x = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh)) : lo;  // cells 4j .. 4j + 3
      lo = hi;
      const uint32_t t = x ^ 0x06060606u;  // KPE_PENDING_ cells -> 0
      // exact zero-byte test (no borrow between bytes): bit 8q + 7 set iff byte q was pending
      const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
      pend |= (uint64_t)(((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4u * j);
    }
    if (a.R - c00 < 64u) pend &= (1ull << (a.R - c00)) - 1ull;  // past the row
    return pend;
  };
  // Memo slots first, in slot order: each lane evaluates the slots its pending cells need, so the
  // lanes of a wave that need slot s walk its pattern together (in column order, a lane whose first
  // cell of slot s comes later than its neighbours' walked it alone: C3's rows differ in which
  // rules their names and namespaces select). The cells then take their slot's verdict.
  if (memo && KPE_PAT_SLOT_ORDER) {
    uint32_t need = 0;
    for (uint32_t c00 = 0; c00 < a.R; c00 += 64u) {
      uint64_t pend = pending(c00);
      while (pend) {
        const uint32_t cq = c00 + (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1ull;
        const uint32_t e = a.col2pr ? a.col2pr[cq] : 0u;
        const uint32_t slot = C2P_SLOT(e);
        if (C2P_RULE(e) != 0u && slot < KPE_PAT_MEMO) need |= 1u << slot;
      }
    }
#pragma unroll 1
    for (uint32_t s = 0; s < KPE_PAT_MEMO; ++s) {
      if (!((need >> s) & 1u)) continue;
      uint32_t v = pat_eval_cell(vm, a.slot_rule[s]);
      if (FS::kDepth < kPatStack && v == KPE_UNDECIDED_) {
        if constexpr (DEFER) {
          v = KPE_DEEP_;  // every cell of the slot goes to kpe_pattern_deep_kernel
        if (a.deep_any) a.deep_any[0] = 1u;
        } else {
          PatVMT<FramesPriv, LT> deep{a, vm.doc, vm.root, vm.pv, 0u};
          v = pat_eval_cell(deep, a.slot_rule[s]);
        }
      }
      memo[s * memo_stride] = (uint8_t)v;
    }
    memo_ok = need;
  }
  for (uint32_t c00 = 0; c00 < a.R; c00 += 64u) {
    uint64_t pend = pending(c00);
    while (pend) {
      const uint32_t q = (uint32_t)__builtin_ctzll(pend);
      pend &= pend - 1ull;
      const uint32_t cq = c00 + q;
      const uint32_t e = a.col2pr ? a.col2pr[cq] : 0u;
      const uint32_t pi = C2P_RULE(e);
      if (pi == 0u) continue;
      const uint32_t slot = memo ? C2P_SLOT(e) : PR_NO_MEMO;
      if (slot < KPE_PAT_MEMO && ((memo_ok >> slot) & 1u)) {
        row[cq] = memo[slot * memo_stride];
        continue;
      }
      uint32_t v = pat_eval_cell(vm, pi - 1u);
      if (FS::kDepth < kPatStack && v == KPE_UNDECIDED_) {
        // a shallow (LDS) stack may have overflowed: the lane-private kPatStack-deep one decides
        if constexpr (DEFER) {
          row[cq] = (uint8_t)KPE_DEEP_;
          if (a.deep_any) a.deep_any[0] = 1u;
          continue;
        } else {
          PatVMT<FramesPriv, LT> deep{a, vm.doc, vm.root, vm.pv, 0u};
          v = pat_eval_cell(deep, pi - 1u);
        }
      }
      row[cq] = (uint8_t)v;
      if (slot < KPE_PAT_MEMO) memo[slot * memo_stride] = (uint8_t)v, memo_ok |= 1u << slot;
    }
  }
}

// kpe_pattern_deep_kernel's body for row r: its KPE_DEEP_ cells walked again on a kPatStack-deep
// frame stack (the kernel's LDS one; the host check's private one): walks deeper than the main
// kernel's LDS stack, and cells undecided for other reasons, which come back undecided again.
template <bool LT = false, class FS = FramesPriv>
__device__ __forceinline__ void pat_deep_row(const PatArgs& a, int64_t r, FS fs = FS{}) {
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  const uint64_t start = (uint64_t)r * a.R;
  const uint32_t* words = reinterpret_cast<const uint32_t*>(a.verdicts);
  for (uint32_t c00 = 0; c00 < a.R; c00 += 64u) {
    const uint64_t p0 = start + c00;
    const uint32_t sh = (uint32_t)(p0 & 3u);
    const uint32_t* wp = words + (p0 >> 2);
    uint64_t mark = 0;
    uint32_t lo = wp[0];
#pragma unroll
    for (uint32_t j = 0; j < 16u; ++j) {
      const uint32_t hi = wp[j + 1u];
      const uint32_t x = sh ? (uint32_t)((((uint64_t)hi << 32) | lo) >> (8u * sh)) : lo;
      lo = hi;
      const uint32_t t = x ^ 0x26262626u;  // KPE_DEEP_ cells -> 0
      const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
      mark |= (uint64_t)(((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4u * j);
    }
    if (a.R - c00 < 64u) mark &= (1ull << (a.R - c00)) - 1ull;
    if (!mark) continue;
    PatVMT<FS, LT> vm{a, PV_DOCVIEW(a, reinterpret_cast<const uint2*>(a.doc), 0u, a.ndoc), (uint32_t)a.doc_off[r],
                      a.pvals + (size_t)r * a.nvars, 0u, 0u, 0u, -1, fs, nullptr};
    while (mark) {
      const uint32_t q = (uint32_t)__builtin_ctzll(mark);
      mark &= mark - 1ull;
      const uint32_t cq = c00 + q;
      const uint32_t pi = a.col2pr ? C2P_RULE(a.col2pr[cq]) : 0u;
      row[cq] = (uint8_t)(pi ? pat_eval_cell(vm, pi - 1u) : KPE_UNDECIDED_);
    }
  }
}
