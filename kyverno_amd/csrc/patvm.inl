// Pattern VM: validate.MatchPattern over the document tape (see kernels.hip). Device code
// included inside kernels.hip's anonymous namespace; scripts/patvm_check.cpp compiles the
// same text for the host (sanitizers, no GPU).
constexpr uint32_t PE_OK = 0, PE_SKIP = 1, PE_NEG = 2, PE_OTHER = 3, PE_OTHER_NOPATH = 4, PE_PUSHED = 8,
                   PE_NONE = 9;
constexpr uint32_t kNoNode = 0xFFFFFFFFu;
constexpr int kPatStack = 14;  // program.cpp kMaxDepth (12) + root + 1
constexpr uint32_t PF_MAP = 0, PF_AMAPS = 1, PF_APOS = 2;

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
#define PVD(i) ((uint64_t)(doc - reinterpret_cast<const uint2*>(a.doc)) + (uint64_t)(i) < a.ndoc ? (i) : pv_fail(a, 9))
#else
#define PV(i, n, code) (i)
#define PVD(i) (i)
#endif

__device__ __forceinline__ uint32_t nd_skip(uint2 n) { return 1u + (DN_KIND(n.x) != DN_SCALAR ? n.y : 0u); }

// member named key1 (the flattener keeps only the last of duplicate names, as a Go map
// decode does); kNoNode if absent
__device__ __forceinline__ uint32_t pat_lookup(const PatArgs& a, const uint2* doc, uint32_t m, uint32_t key1) {
  if (key1 == 0u) return kNoNode;
  const uint32_t end = m + 1u + doc[PVD(m)].y;
  for (uint32_t c = m + 1u; c < end;) {
    const uint2 n = doc[PVD(c)];
    if (DN_KEY(n.x) == key1) return c;
    c += nd_skip(n);
  }
  return kNoNode;
}
// ExpandInMetadata: first string member whose name matches the glob (bitset over D_KEY)
__device__ __forceinline__ uint32_t pat_lookup_glob(const PatArgs& a, const uint2* doc, uint32_t m, uint32_t loc) {
  const uint32_t end = m + 1u + doc[PVD(m)].y;
  for (uint32_t c = m + 1u; c < end;) {
    const uint2 n = doc[PVD(c)];
    const uint32_t k1 = DN_KEY(n.x);
    if (k1 && DN_KIND(n.x) == DN_SCALAR && SC_TYPE(a.scal[PV(n.y, a.nscal, 7)].flags) == SC_T_STR &&
        ((a.pbuf[PV(loc + ((k1 - 1u) >> 5), a.npbuf, 10)] >> ((k1 - 1u) & 31u)) & 1u))
      return c;
    c += nd_skip(n);
  }
  return kNoNode;
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
  const bool m = pat_match(a.pats[PV(cd->pat, a.npats, 6)], a.pat_bytes, a.scal_text + v->text_off, (int)v->text_len);
  return op == PC_NE ? !m : m;
}
__device__ __forceinline__ int64_t go_f2i(double f) {
  return (f >= -9223372036854775808.0 && f < 9223372036854775808.0) ? (int64_t)f : INT64_MIN;
}
// pattern.Validate (pattern.go:26-50) of scalar `sid` (kNoNode: a map / list value)
__device__ __forceinline__ bool pat_leaf(const PatArgs& a, uint32_t sid, uint32_t li) {
  if (sid == kNoNode) return false;  // no scalar validator accepts a map / list
  const KpeLeaf* L = a.leaves + PV(li, a.nleaves, 4);
  const KpeScalar* v = a.scal + PV(sid, a.nscal, 7);
  const uint32_t vf = v->flags, t = SC_TYPE(vf);
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
      if (t == SC_T_STR && pat_match(a.pats[PV(L->exact, a.npats, 6)], a.pat_bytes, a.scal_text + v->text_off, (int)v->text_len))
        return true;  // value == pattern
      bool group = true;  // OR over `|` alternatives of an AND over their `&` terms
      const uint32_t c0 = L->c0, ce = c0 + L->nc;
      for (uint32_t i = c0; i < ce; ++i) {
        const KpeCond* cd = a.conds + PV(i, a.nconds, 5);
        const uint32_t cop = cd->op;
        if ((cop & PC_NEWGROUP) && i != c0) {
          if (group) return true;
          group = true;
        }
        bool r = group && pat_cond(a, v, vf, cd);
        if (cop & PC_OR2) {  // NotInRange: `< lo` OR `> hi`
          ++i;
          r = group && (r || pat_cond(a, v, vf, a.conds + PV(i, a.nconds, 5)));
        }
        group = group && r;
      }
      return group;
    }
    default: return false;
  }
}
// scalar id of node c (kNoNode for maps / lists); an absent member is null
__device__ __forceinline__ uint32_t node_sid(const PatArgs& a, const uint2* doc, uint32_t c) {
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

// Every VM member is inlined: a call would receive the lane's private frame stack through a
// generic pointer, and a flat access into the private aperture from a callee faults.
struct PatVM {
  const PatArgs& a;
  const uint2* doc;
  uint32_t reg, val;  // AnchorMap: slots registered / present in the resource
  int sp;
  PFrame st[kPatStack];

  __device__ __forceinline__ uint32_t leaf_all(uint32_t r, uint32_t li) {  // a scalar pattern vs a list
    const uint32_t end = r + 1u + doc[PVD(r)].y;
    for (uint32_t c = r + 1u; c < end; c += nd_skip(doc[PVD(c)]))
      if (!pat_leaf(a, node_sid(a, doc, c), li)) return PE_OTHER;
    return PE_OK;
  }
  __device__ __forceinline__ uint32_t push(uint32_t kind, uint32_t r, uint32_t pi, uint32_t cur) {
    if (sp + 1 >= kPatStack) return PE_OTHER;  // unreachable: the compiler bounds pattern depth
    ++sp;
    st[PV(sp, kPatStack, 11)] = PFrame{kind, r, pi, 0u, cur, 0u, 0u};
    return PE_PUSHED;
  }
  __device__ __forceinline__ uint32_t pop(uint32_t e) {
    --sp;
    return e;
  }
  // validateResourceElement (validate.go:71-114): a verdict, or PE_PUSHED with a new frame
  __device__ __forceinline__ uint32_t begin(uint32_t r, uint32_t pi) {
    const KpePNode pn = a.nodes[PV(pi, a.nnodes, 1)];
    const uint32_t rk = r == kNoNode ? 0xFFu : DN_KIND(doc[PVD(r)].x);
    if (pn.kind == PN_LEAF) {
      if (rk == DN_ARR) return leaf_all(r, pn.y);
      return pat_leaf(a, node_sid(a, doc, r), pn.y) ? PE_OK : PE_OTHER;
    }
    if (pn.kind == PN_MAP) {
      if (rk != DN_MAP) return PE_OTHER;
      const uint32_t nmem = pn.z >> 16;
      for (uint32_t k = 0; k < nmem; ++k) {  // AnchorMap.CheckAnchorInResource (anchormap.go:33-48)
        const uint4 m = a.members[PV(pn.y + k, a.nmembers, 2)];
        if (m.x & PMF_SLOT) {
          const uint32_t bit = 1u << PM_SLOT(m.x);
          reg |= bit;
          if (pat_lookup(a, doc, r, m.y) != kNoNode) val |= bit;
        }
      }
      return push(PF_MAP, r, pi, 0u);
    }
    if (rk != DN_ARR) return PE_OTHER;
    switch (pn.kind) {
      case PN_ARR_LEAF: return leaf_all(r, pn.y);
      case PN_ARR_MAPS: return push(PF_AMAPS, r, pi, r + 1u);
      case PN_ARR_POS: {
        uint32_t len = 0;
        const uint32_t end = r + 1u + doc[PVD(r)].y;
        for (uint32_t c = r + 1u; c < end; c += nd_skip(doc[PVD(c)])) ++len;
        if (len < pn.z) return PE_OTHER_NOPATH;  // length mismatch: a PatternError with no path
        return push(PF_APOS, r, pi, r + 1u);
      }
      default: return PE_OTHER;  // PN_ARR_EMPTY: "pattern Array empty"
    }
  }

  // validateMap (validate.go:118-175) + anchor handlers, resumed with the verdict `v` of
  // the child frame it waited on (PE_NONE: nothing pending)
  __device__ __forceinline__ uint32_t map_step(uint32_t v) {
    PFrame& F = st[PV(sp, kPatStack, 11)];
    const KpePNode pn = a.nodes[PV(F.pi, a.nnodes, 1)];
    const uint32_t m0 = pn.y, nanch = pn.z & 0xFFFFu, nmem = pn.z >> 16;
    uint32_t k = F.kind_k >> 2, applied = F.cnt & 0xFFFFu, skips = F.cnt >> 16;
    for (;;) {
      uint32_t e;
      if (v == PE_NONE) {
        if (k == nanch && applied == 0u && skips > 0u) return pop(PE_SKIP);  // every anchor skipped
        if (k == nmem) return pop(PE_OK);
        const uint4 m = a.members[PV(m0 + k, a.nmembers, 2)];
        const uint32_t h = PM_HANDLER(m.x);
        const uint32_t c = (m.x & PMF_GLOB) ? pat_lookup_glob(a, doc, F.r, m.w) : pat_lookup(a, doc, F.r, m.y);
        if (h == PM_NEG) {
          e = c == kNoNode ? PE_OK : PE_NEG;
        } else if (c == kNoNode && h != PM_DEFAULT) {
          e = h == PM_COND ? PE_SKIP : PE_OK;  // absent: condition skips, =() <() ^() hold
        } else if (m.x & PMF_STAR) {
          e = (c != kNoNode && node_sid(a, doc, c) != SC_NULL_ID) ? PE_OK : PE_OTHER;
        } else if (h == PM_EXIST) {
          if (DN_KIND(doc[PVD(c)].x) != DN_ARR || a.nodes[PV(m.z, a.nnodes, 1)].kind != PN_EXLIST) {
            e = PE_OTHER;
          } else {
            F.x = 1u, F.cur = c + 1u, F.c = c;
            e = PE_NONE;  // search below
          }
        } else {
          F.kind_k = PF_MAP | (k << 2), F.cnt = applied | (skips << 16);
          const uint32_t w = begin(c, m.z);
          if (w == PE_PUSHED) return PE_PUSHED;
          e = (h == PM_COND || h == PM_GLOBAL) ? (w == PE_OK ? PE_OK : PE_SKIP) : w;
        }
      } else {  // the child of member k finished with v
        const uint32_t h = PM_HANDLER(a.members[PV(m0 + k, a.nmembers, 2)].x);
        if (h == PM_EXIST) {
          if (v == PE_OK) F.x += 1u, F.cur = F.c + 1u;
          else F.cur += nd_skip(doc[PVD(F.cur)]);
          e = PE_NONE;
        } else {
          e = (h == PM_COND || h == PM_GLOBAL) ? (v == PE_OK ? PE_OK : PE_SKIP) : v;
        }
        v = PE_NONE;
      }
      if (e == PE_NONE) {  // existence anchor: each pattern map needs one matching element
        const KpePNode xl = a.nodes[PV(a.members[PV(m0 + k, a.nmembers, 2)].z, a.nnodes, 1)];
        const uint32_t end = F.c + 1u + doc[PVD(F.c)].y;
        e = PE_OK;
        while (F.x - 1u < xl.z) {
          const uint32_t pj = a.lists[PV(xl.y + F.x - 1u, a.nlists, 3)];
          if (a.nodes[PV(pj, a.nnodes, 1)].kind == PN_BAD || F.cur >= end) {
            e = PE_OTHER;
            break;
          }
          F.kind_k = PF_MAP | (k << 2), F.cnt = applied | (skips << 16);
          const uint32_t w = begin(F.cur, pj);
          if (w == PE_PUSHED) return PE_PUSHED;
          if (w == PE_OK) F.x += 1u, F.cur = F.c + 1u;
          else F.cur += nd_skip(doc[PVD(F.cur)]);
        }
        F.x = 0u;
      }
      if (k < nanch) {  // anchors: skips are counted, any other error ends the map
        if (e == PE_SKIP) ++skips;
        else if (e != PE_OK) return pop(e);
        else ++applied;
      } else if (e != PE_OK) {
        return pop(e);
      }
      ++k;
    }
  }

  // validateArrayOfMaps / positional validateArray (validate.go:177-261)
  __device__ __forceinline__ uint32_t arr_step(uint32_t v) {
    PFrame& F = st[PV(sp, kPatStack, 11)];
    const KpePNode pn = a.nodes[PV(F.pi, a.nnodes, 1)];
    const bool pos = (F.kind_k & 3u) == PF_APOS;
    const uint32_t end = F.r + 1u + doc[PVD(F.r)].y;
    uint32_t applied = F.cnt, skips = F.x, j = F.kind_k >> 2, cur = F.cur;
    for (;;) {
      if (v != PE_NONE) {  // element `cur` finished
        if (v == PE_SKIP) ++skips;
        else if (v != PE_OK) return pop(v);
        else ++applied;
        cur += nd_skip(doc[PVD(cur)]);
        ++j;
        v = PE_NONE;
      }
      if (pos ? j >= pn.z : cur >= end) return pop(applied == 0u && skips > 0u ? PE_SKIP : PE_OK);
      F.kind_k = (F.kind_k & 3u) | (j << 2), F.cnt = applied, F.x = skips, F.cur = cur;
      const uint32_t w = begin(cur, pos ? a.lists[PV(pn.y + j, a.nlists, 3)] : pn.y);
      if (w == PE_PUSHED) return PE_PUSHED;
      v = w;
    }
  }

  // validate.MatchPattern (validate.go:31-56) of pattern root node `pi`
  __device__ __forceinline__ uint32_t run(uint32_t pi) {
    sp = -1, reg = 0u, val = 0u;
    uint32_t v = begin(0u, pi);
    if (v != PE_PUSHED) return v;
    v = PE_NONE;
    for (;;) {
      const uint32_t w = (st[PV(sp, kPatStack, 11)].kind_k & 3u) == PF_MAP ? map_step(v) : arr_step(v);
      if (w == PE_PUSHED) {
        v = PE_NONE;
        continue;
      }
      if (sp < 0) return w;
      v = w;
    }
  }
};

// verdict of one pattern: pass / skip / fail, or error when the PatternError path is empty
__device__ __forceinline__ uint32_t pat_match_root(PatVM& vm, uint32_t root) {
  const PatArgs& a = vm.a;
  const uint32_t e = vm.run(a.roots[PV(2 * root, a.nroots, 8)]);
  if (e == PE_OK) return KPE_PASS_;
  if (e == PE_SKIP) return KPE_SKIP_;
  if (e == PE_NEG) return KPE_FAIL_;
  if (e == PE_OTHER_NOPATH || (vm.reg & ~vm.val)) return KPE_ERROR_;  // AnchorMap.KeysAreMissing
  return KPE_FAIL_;
}

// kpe_pattern_kernel's body for resource r: resolve the row's KPE_PENDING_ pattern cells
// (validate_resource.go:316-398: one pattern, or anyPattern's first pass / skip / fail)
__device__ __forceinline__ void pat_eval_row(const PatArgs& a, int64_t r) {
  PatVM vm{a, reinterpret_cast<const uint2*>(a.doc) + a.doc_off[r]};
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  for (uint32_t i = 0; i < a.npr; ++i) {
    const KpePatRule pr = a.rules[i];
    if (row[pr.col] != KPE_PENDING_) continue;
    uint32_t v;
    if (!(pr.flags & PR_ANY)) {
      v = pat_match_root(vm, pr.r0);
    } else if (pr.flags & PR_ANY_BAD) {
      v = KPE_ERROR_;  // anyPattern is not a list
    } else {
      uint32_t fails = 0, skips = 0;
      bool passed = false;
      for (uint32_t k = 0; k < pr.nr && !passed; ++k) {
        const uint32_t x = pat_match_root(vm, pr.r0 + k);
        if (x == KPE_PASS_) passed = true;
        else if (x == KPE_SKIP_) ++skips;
        else ++fails;  // an empty-path error counts as a failure here
      }
      v = passed ? KPE_PASS_ : (fails ? KPE_FAIL_ : (skips ? KPE_SKIP_ : KPE_PASS_));
    }
    row[pr.col] = (uint8_t)v;
  }
}
