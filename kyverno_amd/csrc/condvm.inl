// Condition VM: preconditions / deny / foreach-deny of the compiled program (program.cpp cq::*)
// evaluated per resource over the document tape. Device code included inside kernels.hip's
// anonymous namespace (after patvm.inl, whose tape helpers it shares).
//
// Restates, for the subset the compiler accepts:
//   variables/evaluate.go:14-125      Evaluate / evaluateAnyAllConditions / evaluateOldConditions
//   variables/operator/equal.go, notequal.go (+ operator.go:79-138 parseDuration),
//   anyin.go, allin.go, anynotin.go, allnotin.go, in.go, notin.go
//   engine.go:278-285 (preconditions), validate_resource.go:186-279 (foreach, deny),
//   utils/foreach.go:12-63 (EvaluateList, AddElementToContext)
//   go-jmespath (go.mod:33) field / index / flatten / projection / multi-select / keys / `||`
// Every function is forced inline and each heavy one has a single call site (cond_eval_row is a
// state machine around one block() call): a call would receive the lane's private list buffers
// through a generic `this` pointer (the same constraint as patvm.inl). Nothing recurses.
// Values a restated operator cannot decide on the device (a map or list printed by
// fmt.Sprint, a resource string that may be JSON, lists longer than CV_LIST_CAP) make the
// cell KPE_UNDECIDED_ instead of guessing.

#ifndef CV_LIST_CAP
#define CV_LIST_CAP 32
#endif
constexpr int kCvBufs = 6 + KPE_FE_DEPTH;  // key: 0,1 (+2 list template); value: 3,4 (+5); foreach
                                           // lists: 6 + nesting level

constexpr uint32_t VK_NULL = 0, VK_NODE = 1, VK_CONST = 2, VK_LIST = 3, VK_KEY = 4, VK_NUM = 5,
                   VK_TXT = 6;  // a string built by substitution (VT_TMPL) in the lane's LDS text area:
                                // p = byte offset | length << 8
#ifndef KPE_TXT_CAP
#define KPE_TXT_CAP 120  // bytes of one substituted string (key / value slot); longer: undecided
#endif
constexpr uint32_t JT_NULL = 0, JT_BOOL = 1, JT_NUM = 2, JT_STR = 3, JT_ARR = 4, JT_OBJ = 5;
constexpr int CS_OK = 0, CS_NOTFOUND = 1, CS_ERROR = 2, CS_UNDEC = 3;
constexpr int CB_FALSE = 0, CB_TRUE = 1, CB_ERROR = 2, CB_UNDEC = 3;

struct CV {
  uint32_t k, p;
};
__device__ __forceinline__ CV cv(uint32_t k, uint32_t p) { return CV{k, p}; }

struct SView {
  const uint8_t* s;
  int n;
};

struct CondVM {
  const CondArgs& a;
  const uint2* doc;
  uint32_t root;
  uint32_t img;  // the row's images map entry (kNoNode: no images in the context)
  CV buf[kCvBufs][CV_LIST_CAP];
  uint32_t blen[kCvBufs];
  int dep;                     // foreach nesting level of the current element (-1: none)
  CV els[KPE_FE_DEPTH];        // element<n>
  uint32_t elis[KPE_FE_DEPTH];  // elementIndex<n>
  char (*nb)[16];  // 2 x 16 bytes for fmt.Sprint of an elementIndex: LDS on the device, so that
                   // no generic pointer ever reaches the lane's private memory
  uint8_t* tx;       // 2 x KPE_TXT_CAP bytes of LDS: substituted key / value strings (VK_TXT), or
                     // null when the program has no partial-string variables
  uint32_t bt;  // where the last block() stopped: first true `any` | first false `all` << 7

  // ---- value access ----------------------------------------------------------------------
  __device__ __forceinline__ CV node(uint32_t e) const {  // a tape entry; a null scalar is the null value
    const uint2 n = doc[e];
    if (DN_KIND(n.x) == DN_SCALAR && SC_TYPE(a.scal[n.y].flags) == SC_T_NULL) return cv(VK_NULL, 0);
    return cv(VK_NODE, e);
  }
  __device__ __forceinline__ const KpeScalar* scalar(CV v, const uint8_t** text) const {
    if (v.k == VK_NODE) {
      *text = a.scal_text;
      return a.scal + doc[v.p].y;
    }
    *text = a.ctext;
    return a.ctab + v.p;
  }
  __device__ __forceinline__ uint32_t type(CV v) const {
    switch (v.k) {
      case VK_NODE: {
        const uint2 n = doc[v.p];
        if (DN_KIND(n.x) == DN_MAP) return JT_OBJ;
        if (DN_KIND(n.x) == DN_ARR) return JT_ARR;
        const uint32_t t = SC_TYPE(a.scal[n.y].flags);
        return t == SC_T_NULL ? JT_NULL : t == SC_T_BOOL ? JT_BOOL : t == SC_T_STR ? JT_STR : JT_NUM;
      }
      case VK_CONST: {
        const uint32_t t = SC_TYPE(a.ctab[v.p].flags);
        return t == SC_T_NULL ? JT_NULL : t == SC_T_BOOL ? JT_BOOL : t == SC_T_STR ? JT_STR : t == SC_T_ARR ? JT_ARR
                                                                                                            : JT_NUM;
      }
      case VK_LIST: return JT_ARR;
      case VK_KEY:
      case VK_TXT: return JT_STR;
      case VK_NUM: return JT_NUM;
      default: return JT_NULL;
    }
  }
  __device__ __forceinline__ uint32_t alen(CV v) const {
    if (v.k == VK_NODE) return doc[doc[v.p].y].x;
    if (v.k == VK_CONST) return a.ctab[v.p].text_len;
    return blen[v.p];
  }
  __device__ __forceinline__ CV aget(CV v, uint32_t i) const {
    if (v.k == VK_NODE) return node(doc[v.p].y + 1u + i);
    if (v.k == VK_CONST) {
      const uint32_t c = a.clist[a.ctab[v.p].text_off + i];
      return SC_TYPE(a.ctab[c].flags) == SC_T_NULL ? cv(VK_NULL, 0) : cv(VK_CONST, c);
    }
    return buf[v.p][i];
  }
  __device__ __forceinline__ SView str(CV v) const {  // a JT_STR value's text
    if (v.k == VK_KEY) return SView{a.key_bytes + a.key_off[v.p], (int)(a.key_off[v.p + 1] - a.key_off[v.p])};
    if (v.k == VK_TXT) return SView{tx + (v.p & 0xFFu), (int)(v.p >> 8)};
    const uint8_t* t;
    const KpeScalar* s = scalar(v, &t);
    return SView{t + s->text_off, (int)s->text_len};
  }
  __device__ __forceinline__ double num(CV v) const {
    if (v.k == VK_NUM) return (double)v.p;
    const uint8_t* t;
    const KpeScalar* s = scalar(v, &t);
    return SC_TYPE(s->flags) == SC_T_INT ? (double)s->ival : s->fval;
  }
  __device__ __forceinline__ bool btrue(CV v) const {
    const uint8_t* t;
    return (scalar(v, &t)->flags & SC_BTRUE) != 0u;
  }
  // fmt.Sprint of a scalar (false: a map or list, which the device does not print)
  __device__ __forceinline__ bool sprint(CV v, int slot, SView* out) {
    switch (type(v)) {
      case JT_NULL: *out = SView{reinterpret_cast<const uint8_t*>("<nil>"), 5}; return true;
      case JT_BOOL:
        *out = btrue(v) ? SView{reinterpret_cast<const uint8_t*>("true"), 4}
                        : SView{reinterpret_cast<const uint8_t*>("false"), 5};
        return true;
      case JT_STR: *out = str(v); return true;
      case JT_NUM: {
        if (v.k == VK_NUM) {  // a small non-negative integer: decimal digits
          if (v.p >= 1000000u) return false;  // %e form: not produced for list indexes
          uint32_t x = v.p;
          int n = 0;
          char t[12];
          do t[n++] = (char)('0' + x % 10u), x /= 10u;
          while (x);
          for (int i = 0; i < n; ++i) nb[slot][i] = t[n - 1 - i];
          *out = SView{reinterpret_cast<const uint8_t*>(nb[slot]), n};
          return true;
        }
        const uint8_t* t;
        const KpeScalar* s = scalar(v, &t);
        *out = SView{t + s->text_off + s->text_len, (int)s->sp_len};
        return true;
      }
      default: return false;
    }
  }
  __device__ __forceinline__ bool is_false(CV v) const {  // JMESPath false-like values
    switch (type(v)) {
      case JT_NULL: return true;
      case JT_BOOL: return !btrue(v);
      case JT_STR: return str(v).n == 0;
      case JT_ARR: return alen(v) == 0u;
      case JT_OBJ: return doc[doc[v.p].y].x == 0u;
      default: return false;
    }
  }
  __device__ __forceinline__ static bool seq(SView x, SView y) { return x.n == y.n && bytes_eq(x.s, y.s, x.n); }
  // a string with no scalar record (a member name, a substituted string): no parsed attributes
  __device__ __forceinline__ static bool raw(CV x) { return x.k == VK_KEY || x.k == VK_TXT; }
  __device__ __forceinline__ static bool wm(SView pat, SView s) { return glob(pat.s, pat.n, s.s, s.n); }

  // ---- JMESPath subset ------------------------------------------------------------------
  __device__ __forceinline__ int push(uint32_t b, CV x) {
    if (blen[b] >= (uint32_t)CV_LIST_CAP) return CS_UNDEC;
    buf[b][blen[b]++] = x;
    return CS_OK;
  }
  // member named key1 of map entry m (the flattener keeps the last of duplicate names)
  __device__ __forceinline__ uint32_t lookup(uint32_t m, uint32_t key1) const {
    if (key1 == 0u) return kNoNode;
    const uint32_t b = doc[m].y, c0 = b + 1u, end = c0 + doc[b].x;
    uint32_t i = c0;
    for (; i + 4u <= end; i += 4u) {
      const uint2 n0 = doc[i], n1 = doc[i + 1u], n2 = doc[i + 2u], n3 = doc[i + 3u];
      if (DN_KEY(n0.x) == key1) return i;
      if (DN_KEY(n1.x) == key1) return i + 1u;
      if (DN_KEY(n2.x) == key1) return i + 2u;
      if (DN_KEY(n3.x) == key1) return i + 3u;
    }
    for (; i < end; ++i)
      if (DN_KEY(doc[i].x) == key1) return i;
    return kNoNode;
  }
  __device__ __forceinline__ CV field(CV v, uint32_t fi, bool strict, int* st) {
    if (type(v) != JT_OBJ) return cv(VK_NULL, 0);
    const uint32_t m = lookup(v.p, a.fkeys[fi]);
    if (m == kNoNode) {
      if (strict) *st = CS_NOTFOUND;
      return cv(VK_NULL, 0);
    }
    return node(m);
  }
  __device__ __forceinline__ CV index(CV v, int32_t i) const {
    if (type(v) != JT_ARR) return cv(VK_NULL, 0);
    const int32_t n = (int32_t)alen(v);
    if (i < 0) i += n;
    if (i < 0 || i >= n) return cv(VK_NULL, 0);
    return aget(v, (uint32_t)i);
  }
  // splice arrays, keep everything else (nulls too): N_FLATTEN
  __device__ __forceinline__ int flatten_into(CV v, uint32_t out) {
    blen[out] = 0;
    const uint32_t n = alen(v);
    for (uint32_t i = 0; i < n; ++i) {
      const CV e = aget(v, i);
      if (type(e) == JT_ARR) {
        const uint32_t m = alen(e);
        for (uint32_t j = 0; j < m; ++j)
          if (push(out, aget(e, j))) return CS_UNDEC;
      } else if (push(out, e)) {
        return CS_UNDEC;
      }
    }
    return CS_OK;
  }
  __device__ __forceinline__ void drop_nulls(uint32_t b) {
    uint32_t k = 0;
    for (uint32_t i = 0; i < blen[b]; ++i)
      if (type(buf[b][i]) != JT_NULL) buf[b][k++] = buf[b][i];
    blen[b] = k;
  }
  __device__ __forceinline__ int keys_into(CV v, uint32_t out, bool append) {  // keys(@) of an object
    if (!append) blen[out] = 0;
    const uint32_t b = doc[v.p].y, c0 = b + 1u, end = c0 + doc[b].x;
    for (uint32_t c = c0; c < end; ++c)
      if (push(out, cv(VK_KEY, DN_KEY(doc[c].x) - 1u))) return CS_UNDEC;
    return CS_OK;
  }

  // One expression (no `||`): the result may be a list in buffer b0 or b1.
  __device__ __forceinline__ int run_ops(const KpeCExpr& e, uint32_t b0, uint32_t b1, CV* out) {
    const bool strict = e.flags & CE_STRICT;
    uint32_t mode = 0;  // 0 single value, 1 projection over list `lb`, 2 dead projection (null)
    CV cur = cv(VK_NULL, 0);
    uint32_t lb = b0;
    bool keys_pending = false;
    auto free_buf = [&]() -> uint32_t {  // the buffer not holding the current list
      const uint32_t held = mode == 1 ? lb : (cur.k == VK_LIST ? cur.p : b1);
      return held == b0 ? b1 : b0;
    };
    uint32_t i = e.op0;
    const uint32_t end = e.op0 + e.nops;
    while (i < end) {
      const uint2 o = a.ops[i++];
      const uint32_t op = QO_OP(o.x);
      if (mode == 2) {  // a projection over a non-list: the rest of the expression is null
        if (op == QO_LEN) return CS_ERROR;  // length(null): invalid type
        if (op == QO_MSL) {
          for (uint32_t k = 0; k < QO_ARG(o.x); ++k) i += 1u + QO_ARG(a.ops[i].x);
        }
        continue;
      }
      switch (op) {
        case QO_OBJ: cur = node(root); break;
        case QO_IMG:
          if (img == kNoNode) {  // no images: the context has no `images` key
            if (strict) return CS_NOTFOUND;
            cur = cv(VK_NULL, 0);
          } else {
            cur = node(img);
          }
          break;
        case QO_EL:
        case QO_IDX: {  // element<n> / elementIndex<n> (n = innermost by default) of the foreach levels
          const int lv = o.y == 0xFFFFFFFFu ? dep : (int)o.y;
          if (lv < 0 || lv > dep) {  // not in the context: NotFoundError for a plain chain
            if (strict) return CS_NOTFOUND;
            cur = cv(VK_NULL, 0);
          } else {
            cur = op == QO_EL ? els[lv] : cv(VK_NUM, elis[lv]);
          }
          break;
        }
        case QO_CONST: cur = SC_TYPE(a.ctab[o.y].flags) == SC_T_NULL ? cv(VK_NULL, 0) : cv(VK_CONST, o.y); break;
        case QO_FIELD:
        case QO_INDEX:
          if (mode == 0) {
            int st = CS_OK;
            cur = op == QO_FIELD ? field(cur, o.y, strict, &st) : index(cur, (int32_t)o.y);
            if (st != CS_OK) return st;
          } else {
            int st = CS_OK;
            for (uint32_t k = 0; k < blen[lb]; ++k)
              buf[lb][k] = op == QO_FIELD ? field(buf[lb][k], o.y, false, &st) : index(buf[lb][k], (int32_t)o.y);
          }
          break;
        case QO_KEYS:
          if (mode == 0) {
            if (type(cur) != JT_OBJ) return CS_ERROR;  // keys: invalid type
            const uint32_t fb = free_buf();
            if (keys_into(cur, fb, false)) return CS_UNDEC;
            cur = cv(VK_LIST, fb);
          } else {
            keys_pending = true;  // fused with the `[]` that follows (compile-time check)
          }
          break;
        case QO_VALS:  // (compile time: never inside a projection)
          if (type(cur) != JT_OBJ) {
            mode = 2;
            break;
          } else {
            const uint32_t fb = free_buf();
            blen[fb] = 0;
            const uint32_t b = doc[cur.p].y, c0 = b + 1u, end = c0 + doc[b].x;
            for (uint32_t c = c0; c < end; ++c)
              if (push(fb, node(c))) return CS_UNDEC;
            lb = fb, mode = 1;
          }
          break;
        case QO_FLAT:
        case QO_STAR:
          if (mode == 0) {
            if (type(cur) != JT_ARR) {
              mode = 2;
              break;
            }
            const uint32_t fb = free_buf();
            if (op == QO_FLAT) {
              if (flatten_into(cur, fb)) return CS_UNDEC;
            } else {
              blen[fb] = 0;
              const uint32_t n = alen(cur);
              for (uint32_t k = 0; k < n; ++k)
                if (push(fb, aget(cur, k))) return CS_UNDEC;
            }
            lb = fb, mode = 1;
          } else {
            const uint32_t fb = lb == b0 ? b1 : b0;
            if (keys_pending) {  // keys(@) per element (errors on any non-object), then flatten
              blen[fb] = 0;
              for (uint32_t k = 0; k < blen[lb]; ++k) {
                const CV x = buf[lb][k];
                if (type(x) != JT_OBJ) return CS_ERROR;
                if (keys_into(x, fb, true)) return CS_UNDEC;
              }
              keys_pending = false;
              lb = fb;
            } else {
              drop_nulls(lb);
              if (op == QO_FLAT) {
                if (flatten_into(cv(VK_LIST, lb), fb)) return CS_UNDEC;
                lb = fb;
              }
            }
          }
          break;
        case QO_MSL: {
          const uint32_t nitems = QO_ARG(o.x);
          if (type(cur) == JT_NULL) {
            for (uint32_t k = 0; k < nitems; ++k) i += 1u + QO_ARG(a.ops[i].x);
            cur = cv(VK_NULL, 0);
            break;
          }
          const uint32_t fb = free_buf();
          blen[fb] = 0;
          for (uint32_t k = 0; k < nitems; ++k) {
            const uint32_t len = QO_ARG(a.ops[i].x);
            ++i;
            CV x = cur;
            for (uint32_t j = 0; j < len; ++j, ++i) {
              const uint2 q = a.ops[i];
              int st = CS_OK;
              x = QO_OP(q.x) == QO_FIELD ? field(x, q.y, false, &st) : index(x, (int32_t)q.y);
            }
            if (push(fb, x)) return CS_UNDEC;
          }
          cur = cv(VK_LIST, fb);
          break;
        }
        case QO_LEN: {  // jpfLength (go-jmespath functions.go): runes / items / members
          uint32_t len = 0;
          if (mode == 1) {
            drop_nulls(lb);
            len = blen[lb];
            mode = 0;
          } else {
            const uint32_t t = type(cur);
            if (t == JT_ARR) {
              len = alen(cur);
            } else if (t == JT_OBJ) {
              len = doc[doc[cur.p].y].x;
            } else if (t == JT_STR) {
              const SView sv = str(cur);
              for (int k = 0; k < sv.n; ++k) len += (sv.s[k] & 0xC0u) != 0x80u;
            } else {
              return CS_ERROR;
            }
          }
          cur = cv(VK_NUM, len);
          break;
        }
        default: return CS_ERROR;  // QO_ERROR: an empty expression
      }
    }
    if (mode == 2) {
      *out = cv(VK_NULL, 0);
    } else if (mode == 1) {
      drop_nulls(lb);
      *out = cv(VK_LIST, lb);
    } else {
      *out = cur;
    }
    return CS_OK;
  }
  // A query with its `||` operands: the first truthy one, else the last one's value.
  __device__ __forceinline__ int query(uint32_t ei, uint32_t b0, uint32_t b1, CV* out) {
    for (;;) {
      const KpeCExpr e = a.exprs[ei];
      CV r;
      const int st = run_ops(e, b0, b1, &r);
      if (st == CS_NOTFOUND) return CS_ERROR;  // NotFoundError => "Unknown key" => RuleError
      if (st != CS_OK) return st;
      if (e.alt == CE_NONE || !is_false(r)) {
        *out = r;
        return CS_OK;
      }
      ei = e.alt;
    }
  }
  // substituteVariablesIfAny (variables/vars.go:311-389) of a string with variables inside it:
  // every {{ }} replaced by its value (substituteVarInPattern :403-420: a string as is, anything
  // else json.Marshal-ed), into the lane's LDS text slot `slot`. Undecided: a substituted text
  // holding "{{" (vars.go substitutes again), a map / list value, a number whose json.Marshal text
  // the device does not hold (an exponent, an integer past 2^53), a slot's strings past KPE_TXT_CAP
  // bytes together (the list elements of one side share its slot: `base` bytes are taken).
  static_assert(2 * KPE_TXT_CAP <= 256, "VK_TXT offsets are one byte");
  __device__ __forceinline__ int substitute(const KpeVTmpl& t, uint32_t b0, uint32_t b1, uint32_t slot, uint32_t base,
                                            CV* out) {
    uint8_t* d = tx + slot * KPE_TXT_CAP + base;
    uint32_t len = 0;
    auto put = [&](const uint8_t* p, uint32_t n) -> bool {
      if (base + len + n > (uint32_t)KPE_TXT_CAP) return false;
      for (uint32_t i = 0; i < n; ++i) d[len + i] = p[i];
      len += n;
      return true;
    };
    for (uint32_t k = 0; k < t.b; ++k) {
      const uint2 pc = a.tpieces[t.a + k];
      if ((pc.x & 1u) == PT_TEXT) {
        if (!put(a.ctext + pc.y, pc.x >> 1)) return CS_UNDEC;
        continue;
      }
      CV x;
      const int st = query(pc.y, b0, b1, &x);
      if (st != CS_OK) return st;
      switch (type(x)) {
        case JT_NULL:
          if (!put(reinterpret_cast<const uint8_t*>("null"), 4u)) return CS_UNDEC;
          break;
        case JT_BOOL:
          if (btrue(x) ? !put(reinterpret_cast<const uint8_t*>("true"), 4u)
                       : !put(reinterpret_cast<const uint8_t*>("false"), 5u))
            return CS_UNDEC;
          break;
        case JT_STR: {
          const SView sv = str(x);
          for (int i = 0; i + 1 < sv.n; ++i)
            if (sv.s[i] == '{' && sv.s[i + 1] == '{') return CS_UNDEC;
          if (!put(sv.s, (uint32_t)sv.n)) return CS_UNDEC;
          break;
        }
        case JT_NUM: {
          if (x.k == VK_NUM) {  // a count / index: its decimal digits
            uint8_t dg[10];
            uint32_t n = 0, y = x.p;
            do dg[9 - n++] = (uint8_t)('0' + y % 10u), y /= 10u;
            while (y);
            if (!put(dg + 10 - n, n)) return CS_UNDEC;
            break;
          }
          const uint8_t* tb;
          const KpeScalar* s = scalar(x, &tb);
          if (SC_TYPE(s->flags) == SC_T_INT) {  // a float64 in the JSON context: exact below 2^53
            if (s->ival > (1ll << 53) || s->ival < -(1ll << 53)) return CS_UNDEC;
            if (!put(tb + s->text_off, s->text_len)) return CS_UNDEC;
          } else {  // json.Marshal equals the fmt.Sprint text when that has no exponent
            const uint8_t* sp = tb + s->text_off + s->text_len;
            for (uint32_t i = 0; i < s->sp_len; ++i)
              if (sp[i] == 'e') return CS_UNDEC;
            if (!put(sp, s->sp_len)) return CS_UNDEC;
          }
          break;
        }
        default: return CS_UNDEC;  // json.Marshal of a map / list
      }
    }
    *out = cv(VK_TXT, (slot * KPE_TXT_CAP + base) | len << 8);
    return CS_OK;
  }
  // A condition key / value after substitution (template `ti`); lists go to buffer bl. One
  // query() call site: a single query is a one-element template walk that returns its value. A
  // string with variables inside it (alone, or elements of a list: program.cpp CondCompiler::tmpl)
  // is built in the side's lane text slot (key 0, value 1), a list's elements one after another.
  __device__ __forceinline__ int value(uint32_t ti, uint32_t b0, uint32_t b1, uint32_t bl, CV* out) {
    const KpeVTmpl t = a.tmpls[ti];
    const uint32_t slot = b0 == 3u ? 1u : 0u;
    if (t.kind == VT_TMPL) return substitute(t, b0, b1, slot, 0u, out);
    const bool arr = t.kind == VT_ARRAY;
    const uint32_t n = arr ? t.b : 1u;
    blen[bl] = 0;
    uint32_t fill = 0;                  // bytes of the slot taken by earlier template elements
    for (uint32_t k = 0; k < n; ++k) {  // list elements: constants, queries or templates
      const KpeVTmpl te = arr ? a.tmpls[t.a + k] : t;
      CV x;
      if (te.kind == VT_CONST) {
        x = SC_TYPE(a.ctab[te.a].flags) == SC_T_NULL ? cv(VK_NULL, 0) : cv(VK_CONST, te.a);
      } else if (te.kind == VT_TMPL) {
        const int st = substitute(te, b0, b1, slot, fill, &x);
        if (st != CS_OK) return st;
        fill += x.p >> 8;
      } else {
        const int st = query(te.a, b0, b1, &x);
        if (st != CS_OK) return st;
      }
      if (!arr) {
        *out = x;
        return CS_OK;
      }
      if (x.k == VK_LIST) return CS_UNDEC;  // a list inside a list
      if (push(bl, x)) return CS_UNDEC;
    }
    *out = cv(VK_LIST, bl);
    return CS_OK;
  }

  // ---- operators --------------------------------------------------------------------------
  // operator.go:79-138 parseDuration: a string (other than "0") that parses as a duration, or a
  // number of seconds beside one; -1 when neither side is a duration string
  __device__ __forceinline__ int duration2(CV k, CV v, double* ks, double* vs) const {
    auto dstr = [&](CV x, int64_t* d) -> bool {
      if (type(x) != JT_STR || raw(x)) return false;
      const uint8_t* t;
      const KpeScalar* s = scalar(x, &t);
      if (!(s->flags & SC_DUR)) return false;
      if (s->text_len == 1u && t[s->text_off] == '0') return false;
      *d = s->dur;
      return true;
    };
    auto ndur = [&](CV x, int64_t* d) -> bool {
      if (type(x) != JT_NUM) return false;
      const double tr = trunc(num(x));
      if (!(tr >= -9.2e18 && tr <= 9.2e18)) return false;
      *d = (int64_t)((uint64_t)(int64_t)tr * 1000000000ull);
      return true;
    };
    int64_t kd = 0, vd = 0;
    const bool hk = dstr(k, &kd), hv = dstr(v, &vd);
    if (!hk && !hv) return -1;
    if (!hk && !ndur(k, &kd)) return -1;
    if (!hv && !ndur(v, &vd)) return -1;
    auto secs = [](int64_t d) { return (double)(d / 1000000000) + (double)(d % 1000000000) / 1e9; };
    *ks = secs(kd), *vs = secs(vd);
    return 1;
  }
  // A member name (VK_KEY) carries no parsed attributes: undecided where it could parse as a
  // number, duration or quantity.
  // (durations and quantities start with [-+.0-9]; strconv.ParseFloat also takes inf / nan)
  __device__ __forceinline__ bool numeric_looking(CV x, bool floats) const {
    if (!raw(x)) return false;
    const SView s = str(x);
    if (s.n == 0) return false;
    const uint8_t c = s.s[0];
    if (!((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.') &&
        !(floats && (c == 'I' || c == 'i' || c == 'N' || c == 'n')))
      return false;
    // numbers (hex floats, Inf / NaN included), durations (µs) and quantities hold only ASCII
    // letters and digits, '+', '-', '.', '_' and the bytes of U+00B5: any other byte rules them out
    for (int i = 1; i < s.n; ++i) {
      const uint8_t b = s.s[i];
      if (!((b >= '0' && b <= '9') || (b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z') || b == '+' || b == '-' ||
            b == '.' || b == '_' || b == 0xC2u || b == 0xB5u))
        return false;
    }
    return true;
  }
  // equal.go / notequal.go
  __device__ __forceinline__ int op_equals(CV k, CV v, bool neg) {
    const uint32_t kt = type(k), vt = type(v);
    switch (kt) {
      case JT_NULL: return 0;
      case JT_BOOL: return vt != JT_BOOL ? neg : ((btrue(k) == btrue(v)) != neg);
      case JT_NUM:
        if (vt == JT_NUM) return (num(v) == num(k)) != neg;
        if (vt == JT_STR) {
          if (raw(v)) return numeric_looking(v, true) ? -1 : neg;
          const uint8_t* t;
          const KpeScalar* s = scalar(v, &t);
          if (!(s->flags & SC_PFLOAT)) return neg;
          return (s->fval == num(k)) != neg;
        }
        return neg;
      case JT_STR: {
        if (numeric_looking(k, false) || numeric_looking(v, false)) return -1;
        double ks, vs;
        if (duration2(k, v, &ks, &vs) > 0) return (ks == vs) != neg;
        const uint8_t *tk, *tv;
        const KpeScalar* sk = raw(k) ? nullptr : scalar(k, &tk);
        if (sk && (sk->flags & SC_QTY) && vt == JT_STR) {
          if (neg && str(v).n == 0) return !wm(str(v), str(k));
          const KpeScalar* sv = raw(v) ? nullptr : scalar(v, &tv);
          if (!sv || !(sv->flags & SC_QTY)) return 0;
          const int c = qcmp(sk->flags & SC_QNEG, sk->qexp, sk->qlo, sk->qhi, sv->flags & SC_QNEG, sv->qexp, sv->qlo,
                             sv->qhi);
          return (c == 0) != neg;
        }
        if (vt == JT_STR) return wm(str(v), str(k)) != neg;
        return neg;
      }
      case JT_ARR: {
        if (vt != JT_ARR) return neg;
        const int d = deep_equal_list(k, v);
        return d < 0 ? -1 : ((d == 1) != neg);
      }
      default: return vt != JT_OBJ ? neg : -1;  // map equality: undecided
    }
  }
  __device__ __forceinline__ int deep_equal_list(CV x, CV y) {  // reflect.DeepEqual of two lists of scalars
    const uint32_t n = alen(x);
    if (alen(y) != n) return 0;
    for (uint32_t i = 0; i < n; ++i) {
      const CV p = aget(x, i), q = aget(y, i);
      const uint32_t tp = type(p), tq = type(q);
      if (tp == JT_ARR || tp == JT_OBJ || tq == JT_ARR || tq == JT_OBJ) return -1;
      if (tp != tq) return 0;
      if (tp == JT_BOOL && btrue(p) != btrue(q)) return 0;
      if (tp == JT_NUM && num(p) != num(q)) return 0;
      if (tp == JT_STR && !seq(str(p), str(q))) return 0;
    }
    return 1;
  }
  // A string value of a set / In operator decoded as a JSON []string: 1 decoded (*c0, *cn list
  // of constants), 0 not JSON, 2 valid JSON that is not a []string, -1 undecided (a resource
  // string that may be JSON).
  __device__ __forceinline__ int json_list(CV v, uint32_t* c0, uint32_t* cn) const {
    if (v.k == VK_CONST) {
      const KpeScalar& s = a.ctab[v.p];
      if (!(s.flags & SC_JVALID)) return 0;
      if (!(s.flags & SC_JLIST)) return 2;
      *c0 = (uint32_t)s.ival, *cn = (uint32_t)((uint64_t)s.ival >> 32);
      return 1;
    }
    if (v.k == VK_NODE) {  // the flattener's json.Valid (SC_JVALID / SC_JARR)
      const uint8_t* t;
      const KpeScalar* s = scalar(v, &t);
      if (!(s->flags & SC_JVALID)) return 0;
      if (s->flags & SC_JARR) return -1;  // a JSON array: its []string decode stays on the host
      const SView x = str(v);
      int i = 0;
      while (i < x.n && (x.s[i] == ' ' || x.s[i] == '\t' || x.s[i] == '\n' || x.s[i] == '\r')) ++i;
      if (i < x.n && x.s[i] == 'n') {  // null: a nil slice
        *c0 = 0, *cn = 0;
        return 1;
      }
      return 2;  // valid JSON that is not a list: the Unmarshal error (invalid type)
    }
    const SView s = str(v);
    int i = 0;
    while (i < s.n && (s.s[i] == ' ' || s.s[i] == '\t' || s.s[i] == '\n' || s.s[i] == '\r')) ++i;
    if (i == s.n) return 0;
    const uint8_t c = s.s[i];
    if (c == '[' || c == '{' || c == '"' || c == '-' || (c >= '0' && c <= '9') || c == 't' || c == 'f' || c == 'n')
      return -1;
    return 0;
  }
  // anyin.go / allin.go / anynotin.go / allnotin.go
  __device__ __forceinline__ int op_set(uint32_t op, CV k, CV v, uint32_t rng) {
    const uint32_t kt = type(k), vt = type(v);
    if (kt == JT_NULL || kt == JT_OBJ) return 0;
    const bool notin = op == CO_ANYNOTIN || op == CO_ALLNOTIN;
    const bool single = kt != JT_ARR;
    const uint32_t nk = single ? 1u : alen(k);
    SView k0;
    if (single && !sprint(k, 0, &k0)) return -1;
    if (vt == JT_NULL || vt == JT_BOOL || vt == JT_NUM || vt == JT_OBJ) return 0;  // invalid type
    uint32_t vc0 = 0, vcn = 0;
    bool decoded = false;
    if (vt == JT_STR) {
      const SView vs = str(v);
      if (single && wm(vs, k0)) return !notin;
      if (!single && nk == 1u) {
        SView x;
        if (!sprint(aget(k, 0), 0, &x)) return -1;
        if (seq(x, vs)) return !notin;
      }
      bool rt = false;  // a resource string in the InRange form
      if (v.k == VK_NODE) {
        const uint8_t* t;
        const uint32_t f = scalar(v, &t)->flags;
        if (f & SC_RANGEU) return -1;
        rt = (f & SC_RANGE) != 0u;
      }
      if (rng || rt) {  // InRange value: handleRange per key (anyin.go:76-77,146-165; allin.go)
        const uint32_t li = rng - 1u;
        if (single) {
          const int h = rt ? range_rt(k, v, false) : range_holds(k, li);
          return h < 0 ? -1 : ((h == 1) != notin);
        }
        // AnyIn: some key in range; AnyNotIn: some key in the `!-` form; AllIn: every key;
        // AllNotIn: no key
        const uint32_t lj = op == CO_ANYNOTIN ? li + 1u : li;
        int undec = 0, hits = 0;
        for (uint32_t i = 0; i < nk; ++i) {
          const int h = rt ? range_rt(aget(k, i), v, op == CO_ANYNOTIN) : range_holds(aget(k, i), lj);
          if (h < 0) undec = 1;
          else hits += h;
        }
        if (op == CO_ANYIN || op == CO_ANYNOTIN) return hits ? 1 : (undec ? -1 : 0);
        if (op == CO_ALLIN) return (hits == (int)nk) ? 1 : (undec ? -1 : 0);
        return hits ? 0 : (undec ? -1 : 1);  // CO_ALLNOTIN
      }
      // member names carry no attributes (json_list leaves digit / sign starts undecided)
      if (raw(v) && vs.n > 0 && (vs.s[0] == '+' || vs.s[0] == '|')) return -1;
      const int j = json_list(v, &vc0, &vcn);
      if (j < 0) return -1;
      if (j == 2) return 0;
      if (j == 0) {  // not JSON: the string itself
        if (single) return seq(vs, k0) != notin;
        vcn = 1, decoded = false;
      } else {
        decoded = true;
      }
      if (single) {  // exact membership in the decoded list
        bool ex = false;
        for (uint32_t i = 0; i < vcn && !ex; ++i) ex = seq(str(cv(VK_CONST, a.clist[vc0 + i])), k0);
        return ex != notin;
      }
    }
    const uint32_t nv = vt == JT_STR ? vcn : alen(v);
    auto vtext = [&](uint32_t i, SView* out) -> bool {
      if (vt == JT_STR) {
        if (!decoded) {
          *out = str(v);
          return true;
        }
        *out = str(cv(VK_CONST, a.clist[vc0 + i]));
        return true;
      }
      return sprint(aget(v, i), 1, out);
    };
    auto found = [&](SView kk, int* undec) -> bool {
      for (uint32_t i = 0; i < nv; ++i) {
        SView vv;
        if (!vtext(i, &vv)) {
          *undec = 1;
          return false;
        }
        if (wm(kk, vv) || wm(vv, kk)) return true;
      }
      return false;
    };
    int undec = 0;
    if (single) {  // a scalar key against a list value (anyKeyExistsInArray)
      const bool ex = found(k0, &undec);
      return undec ? -1 : (ex != notin);
    }
    for (uint32_t i = 0; i < nk; ++i) {
      SView kk;
      if (!sprint(aget(k, i), 0, &kk)) return -1;
      const bool f = found(kk, &undec);
      if (undec) return -1;
      if ((op == CO_ANYIN) && f) return 1;
      if ((op == CO_ANYNOTIN) && !f) return 1;
      if ((op == CO_ALLIN) && !f) return 0;
      if ((op == CO_ALLNOTIN) && f) return 0;
    }
    return (op == CO_ALLIN || op == CO_ALLNOTIN) ? 1 : 0;
  }
  // in.go / notin.go (deprecated): keyExistsInArray / setExistsInArray
  __device__ __forceinline__ int op_in(CV k, CV v, bool notin) {
    const uint32_t kt = type(k), vt = type(v);
    if (kt == JT_NULL || kt == JT_OBJ) return 0;
    if (kt != JT_ARR) {
      SView k0;
      if (!sprint(k, 0, &k0)) return -1;
      int r;  // 1 in, 0 not in, -1 invalid type
      if (vt == JT_ARR) {
        r = 0;
        const uint32_t n = alen(v);
        for (uint32_t i = 0; i < n && r == 0; ++i) {
          SView s;
          if (!sprint(aget(v, i), 1, &s)) return -1;
          if (wm(s, k0) || wm(k0, s)) r = 1;
        }
      } else if (vt == JT_STR) {
        const SView vs = str(v);
        if (wm(vs, k0)) {
          r = 1;
        } else {
          uint32_t c0 = 0, cn = 0;
          const int j = json_list(v, &c0, &cn);
          if (j < 0) return -1;
          if (j != 1) {
            r = -1;
          } else {
            r = 0;
            for (uint32_t i = 0; i < cn && !r; ++i) r = seq(str(cv(VK_CONST, a.clist[c0 + i])), k0) ? 1 : 0;
          }
        }
      } else {
        r = -1;
      }
      if (r < 0) return 0;
      return (r == 1) != notin;
    }
    // a key list: every element must be a string (the reference panics otherwise: an error)
    const uint32_t nk = alen(k);
    for (uint32_t i = 0; i < nk; ++i)
      if (type(aget(k, i)) != JT_STR) return -2;
    uint32_t c0 = 0, cn = 0;
    bool from_const = false;
    if (vt == JT_ARR) {
      const uint32_t n = alen(v);
      for (uint32_t i = 0; i < n; ++i)
        if (type(aget(v, i)) != JT_STR) return 0;
    } else if (vt == JT_STR) {
      if (nk == 1u && seq(str(aget(k, 0)), str(v))) return 1;  // in.go:126-128, NotIn too
      const int j = json_list(v, &c0, &cn);
      if (j < 0) return -1;
      if (j != 1) return 0;
      from_const = true;
    } else {
      return 0;
    }
    bool all = true, any_missing = false;
    for (uint32_t i = 0; i < nk; ++i) {
      const SView kk = str(aget(k, i));
      bool f = false;
      const uint32_t n = from_const ? cn : alen(v);
      for (uint32_t j = 0; j < n && !f; ++j)
        f = seq(from_const ? str(cv(VK_CONST, a.clist[c0 + j])) : str(aget(v, j)), kk);
      all = all && f;
      any_missing = any_missing || !f;
    }
    return notin ? any_missing : all;
  }

  // ---- InRange values of the set operators -------------------------------------------------
  // anyin.go:103-109 handleRange: pattern.Validate(key, value) with the key as its fmt.Sprint
  // string: validateStringPatterns (pattern.go:152-215) of the compiled value leaf. 1 / 0, -1
  // where the key's Sprint text has no parsed attributes on the device.
  __device__ __forceinline__ bool rcond(const KpeScalar* v, uint32_t vf, SView vt, const KpeCond& cd) const {
    const uint32_t cop = cd.op, op = PC_OP(cop);
    if ((cop & PC_DUR) && (vf & SC_DUR)) return op_holds(op, v->dur < cd.dur ? -1 : (v->dur > cd.dur ? 1 : 0));
    if ((cop & PC_QTY) && (vf & SC_QTY))
      return op_holds(op, qcmp(vf & SC_QNEG, v->qexp, v->qlo, v->qhi, cop & PC_QNEG, cd.qexp, cd.qlo, cd.qhi));
    if (op != PC_EQ && op != PC_NE) return false;
    const bool m = pv_match(a.pats[cd.pat], a.pat_bytes, vt.s, vt.n);
    return op == PC_NE ? !m : m;
  }
  // The key as the Go string handleRange receives (fmt.Sprint): its text, and the parsed
  // duration / quantity attributes that stand for it (vf; *s holds the values). -1: undecided
  // (a member name that may parse, a map / list, 0 against a duration operand, a number whose
  // Sprint quantity is not its %f one).
  __device__ __forceinline__ int key_text(CV k, bool dur_operand, const KpeScalar** sp, uint32_t* vfp, SView* tp) const {
    const KpeScalar* s = nullptr;
    uint32_t vf = SC_TEXT;
    SView t;
    switch (type(k)) {
      case JT_NULL: t = SView{reinterpret_cast<const uint8_t*>("<nil>"), 5}; break;
      case JT_BOOL:
        t = btrue(k) ? SView{reinterpret_cast<const uint8_t*>("true"), 4}
                     : SView{reinterpret_cast<const uint8_t*>("false"), 5};
        break;
      case JT_STR:
        if (raw(k)) {
          if (numeric_looking(k, true)) return -1;
          t = str(k);
        } else {
          const uint8_t* tb;
          s = scalar(k, &tb);
          vf = s->flags & (SC_DUR | SC_QTY | SC_QNEG | SC_TEXT);
          t = SView{tb + s->text_off, (int)s->text_len};
        }
        break;
      case JT_NUM: {
        if (k.k == VK_NUM) return -1;
        const uint8_t* tb;
        s = scalar(k, &tb);
        // the Sprint text (after the compareString text); its quantity equals the %f one
        // (SC_SPQ); it is a duration only for 0 ("0")
        if (!(s->flags & SC_SPQ) || (dur_operand && num(k) == 0.0)) return -1;
        vf = (s->flags & (SC_QTY | SC_QNEG)) | SC_TEXT;
        t = SView{tb + s->text_off + s->text_len, (int)s->sp_len};
        break;
      }
      default: return -1;  // fmt.Sprint of a map / list
    }
    *sp = s, *vfp = vf, *tp = t;
    return 0;
  }
  __device__ __forceinline__ int range_holds(CV k, uint32_t li) const {
    const KpeLeaf L = a.leaves[li];
    const KpeScalar* s = nullptr;
    uint32_t vf;
    SView t;
    if (key_text(k, L.pad[0] != 0u, &s, &vf, &t) < 0) return -1;
    if (pv_match(a.pats[L.exact], a.pat_bytes, t.s, t.n)) return 1;  // value == pattern
    bool group = true;
    const uint32_t c0 = L.c0, ce = c0 + L.nc;
    for (uint32_t i = c0; i < ce; ++i) {
      const KpeCond cd = a.pconds[i];
      if ((cd.op & PC_NEWGROUP) && i != c0) {
        if (group) return 1;
        group = true;
      }
      bool r = group && rcond(s, vf, t, cd);
      if (cd.op & PC_OR2) {
        ++i;
        r = group && (r || rcond(s, vf, t, a.pconds[i]));
      }
      group = group && r;
    }
    return group ? 1 : 0;
  }

  // A resource string value in the InRange form (SC_RANGE: endpoints interned by the flattener).
  // notin: AnyNotIn's strings.Replace(value, "-", "!-", 1): `a!-b` (NotInRange), or for a value
  // with a leading `-` the `!` (NotEqual) prefix before the whole value.
  __device__ __forceinline__ bool bound(uint32_t op, const KpeScalar* ks, uint32_t vf, uint32_t id) const {
    const KpeScalar e = a.scal[id];
    if ((e.flags & SC_DUR) && (vf & SC_DUR)) return op_holds(op, ks->dur < e.dur ? -1 : (ks->dur > e.dur ? 1 : 0));
    if ((e.flags & SC_QTY) && (vf & SC_QTY))
      return op_holds(op, qcmp(vf & SC_QNEG, ks->qexp, ks->qlo, ks->qhi, e.flags & SC_QNEG, e.qexp, e.qlo, e.qhi));
    return false;  // compareString: >=, <=, >, < never hold for strings
  }
  __device__ __forceinline__ int range_rt(CV k, CV v, bool notin) const {
    const uint8_t* tb;
    const KpeScalar* rs = scalar(v, &tb);
    const SView r = str(v);
    const uint32_t lo = (uint32_t)(uint64_t)rs->ival, hi = (uint32_t)((uint64_t)rs->ival >> 32);
    const bool dur = ((a.scal[lo].flags | a.scal[hi].flags) & SC_DUR) != 0u;
    const KpeScalar* s = nullptr;
    uint32_t vf;
    SView t;
    if (key_text(k, dur, &s, &vf, &t) < 0) return -1;
    if (!notin) {
      if (seq(t, r)) return 1;  // value == pattern
      return bound(PC_GE, s, vf, lo) && bound(PC_LE, s, vf, hi);
    }
    int d = 0;
    while (d < r.n && r.s[d] != '-') ++d;
    bool eqm = t.n == r.n + 1 && t.s[d] == '!';  // value == the replaced pattern
    for (int i = 0; eqm && i < d; ++i) eqm = t.s[i] == r.s[i];
    for (int i = d; eqm && i < r.n; ++i) eqm = t.s[i + 1] == r.s[i];
    if (eqm) return 1;
    if (d == 0) return !seq(t, r);  // `!-lo-hi`: NotEqual of `-lo-hi` (no glob characters)
    return bound(PC_LT, s, vf, lo) || bound(PC_GT, s, vf, hi);
  }

  // ---- numeric.go / duration.go ---------------------------------------------------------------
  __device__ __forceinline__ static int cmp_by(uint32_t nop, double x, double y) {  // compareByCondition
    switch (nop) {
      case CN_GE: return x >= y;
      case CN_GT: return x > y;
      case CN_LE: return x <= y;
      case CN_LT: return x < y;
      default: return 0;
    }
  }
  // time.Duration(f) * time.Second: truncation, wrapping multiplication; false when out of range
  __device__ __forceinline__ static bool f2dur(double f, int64_t* d) {
    const double tr = trunc(f);
    if (!(tr >= -9.2e18 && tr <= 9.2e18)) return false;
    *d = (int64_t)((uint64_t)(int64_t)tr * 1000000000ull);
    return true;
  }
  __device__ __forceinline__ static double dsecs(int64_t d) {
    return (double)(d / 1000000000) + (double)(d % 1000000000) / 1e9;
  }
  // validateValueWithFloatPattern (numeric.go:102-128) of a float64 key
  __device__ __forceinline__ int num_float(uint32_t nop, double kf, CV v) const {
    const uint32_t vt = type(v);
    if (vt == JT_NUM) return cmp_by(nop, kf, num(v));
    if (vt != JT_STR) return 0;
    if (raw(v)) return numeric_looking(v, true) ? -1 : 0;
    const uint8_t* t;
    const KpeScalar* s = scalar(v, &t);
    int64_t kd;
    // parseDuration: the value a duration string other than "0", the key seconds
    if ((s->flags & SC_DUR) && !(s->text_len == 1u && t[s->text_off] == '0') && f2dur(kf, &kd))
      return cmp_by(nop, dsecs(kd), dsecs(s->dur));
    if (s->flags & SC_PFLOAT) return cmp_by(nop, kf, s->fval);
    return 0;
  }
  // blang/semver v4 Parse (oracle/conditions.hpp semver_parse): major, minor, patch and the
  // prerelease text [*p0, *p1); false when not a version
  __device__ __forceinline__ static bool sv_num(SView s, int b, int e, uint64_t* out) {
    if (e <= b || (e - b > 1 && s.s[b] == '0')) return false;
    uint64_t x = 0;
    for (int i = b; i < e; ++i) {
      const uint32_t c = s.s[i];
      if (c < '0' || c > '9') return false;
      const uint64_t d = c - '0';
      if (x > (0xFFFFFFFFFFFFFFFFull - d) / 10u) return false;
      x = x * 10u + d;
    }
    *out = x;
    return true;
  }
  __device__ __forceinline__ static bool sv_ident_ok(SView s, int b, int e, bool pre) {
    if (e <= b) return false;
    bool digits = true;
    for (int i = b; i < e; ++i) {
      const uint32_t c = s.s[i];
      const bool d = c >= '0' && c <= '9';
      if (!(d || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '-')) return false;
      digits = digits && d;
    }
    uint64_t x;
    return !(pre && digits) || sv_num(s, b, e, &x);
  }
  __device__ __forceinline__ static bool semver(SView s, uint64_t* mmp, int* p0, int* p1) {
    int d1 = -1, d2 = -1;
    for (int i = 0; i < s.n && d2 < 0; ++i)
      if (s.s[i] == '.') (d1 < 0 ? d1 : d2) = i;
    if (d2 < 0) return false;
    if (!sv_num(s, 0, d1, &mmp[0]) || !sv_num(s, d1 + 1, d2, &mmp[1])) return false;
    int plus = s.n, minus = -1;
    for (int i = d2 + 1; i < s.n; ++i)
      if (s.s[i] == '+') {
        plus = i;
        break;
      }
    for (int i = d2 + 1; i < plus; ++i)
      if (s.s[i] == '-') {
        minus = i;
        break;
      }
    if (!sv_num(s, d2 + 1, minus >= 0 ? minus : plus, &mmp[2])) return false;
    *p0 = minus >= 0 ? minus + 1 : plus, *p1 = plus;
    if (minus >= 0)  // prerelease identifiers
      for (int b = minus + 1;;) {
        int e = b;
        while (e < plus && s.s[e] != '.') ++e;
        if (!sv_ident_ok(s, b, e, true)) return false;
        if (e >= plus) break;
        b = e + 1;
      }
    if (plus < s.n)  // build identifiers
      for (int b = plus + 1;;) {
        int e = b;
        while (e < s.n && s.s[e] != '.') ++e;
        if (!sv_ident_ok(s, b, e, false)) return false;
        if (e >= s.n) break;
        b = e + 1;
      }
    return true;
  }
  __device__ __forceinline__ static int semver_cmp(SView x, SView y) {  // both valid
    uint64_t a[3], b[3];
    int xa, xb, ya, yb;
    semver(x, a, &xa, &xb);
    semver(y, b, &ya, &yb);
    for (int i = 0; i < 3; ++i)
      if (a[i] != b[i]) return a[i] > b[i] ? 1 : -1;
    const bool xp = xa < xb, yp = ya < yb;
    if (!xp && !yp) return 0;
    if (!xp) return 1;
    if (!yp) return -1;
    int i = xa, j = ya;
    for (;;) {  // identifiers in lockstep
      int ie = i, je = j;
      while (ie < xb && x.s[ie] != '.') ++ie;
      while (je < yb && y.s[je] != '.') ++je;
      bool xn = true, yn = true;
      for (int k = i; k < ie; ++k) xn = xn && x.s[k] >= '0' && x.s[k] <= '9';
      for (int k = j; k < je; ++k) yn = yn && y.s[k] >= '0' && y.s[k] <= '9';
      int c = 0;
      if (xn && !yn) c = -1;
      else if (!xn && yn) c = 1;
      else if (xn) {  // no leading zeros: longer is larger, else digit order
        c = (ie - i) != (je - j) ? ((ie - i) > (je - j) ? 1 : -1) : 0;
        for (int k = 0; c == 0 && k < ie - i; ++k)
          if (x.s[i + k] != y.s[j + k]) c = x.s[i + k] > y.s[j + k] ? 1 : -1;
      } else {  // byte order
        const int n = (ie - i) < (je - j) ? (ie - i) : (je - j);
        for (int k = 0; c == 0 && k < n; ++k)
          if (x.s[i + k] != y.s[j + k]) c = x.s[i + k] > y.s[j + k] ? 1 : -1;
        if (c == 0 && (ie - i) != (je - j)) c = (ie - i) > (je - j) ? 1 : -1;
      }
      if (c) return c;
      const bool xend = ie >= xb, yend = je >= yb;
      if (xend && yend) return 0;
      if (xend) return -1;
      if (yend) return 1;
      i = ie + 1, j = je + 1;
    }
  }
  // NumericOperatorHandler.Evaluate (numeric.go:62-77, 130-165)
  __device__ __forceinline__ int op_num(uint32_t nop, CV k, CV v) {
    const uint32_t kt = type(k);
    if (kt == JT_NUM) return num_float(nop, num(k), v);
    if (kt != JT_STR) return 0;
    if (numeric_looking(k, true) || numeric_looking(v, true)) return -1;  // member names: no parsed attributes
    double ks, vs;
    if (duration2(k, v, &ks, &vs) > 0) return cmp_by(nop, ks, vs);
    if (!raw(k)) {
      const uint8_t* tk;
      const KpeScalar* sk = scalar(k, &tk);
      if ((sk->flags & SC_QTY) && type(v) == JT_STR && !raw(v)) {
        const uint8_t* tv;
        const KpeScalar* sv = scalar(v, &tv);
        if (sv->flags & SC_QTY)
          return cmp_by(nop, (double)qcmp(sk->flags & SC_QNEG, sk->qexp, sk->qlo, sk->qhi, sv->flags & SC_QNEG, sv->qexp,
                                          sv->qlo, sv->qhi), 0.0);
      }
      if (sk->flags & SC_PFLOAT) return num_float(nop, sk->fval, v);
    }
    uint64_t m[3];
    int p0, p1;
    const SView ksv = str(k);
    if (!semver(ksv, m, &p0, &p1)) return 0;
    if (type(v) != JT_STR) return 0;
    const SView vsv = str(v);
    if (!semver(vsv, m, &p0, &p1)) return 0;
    return cmp_by(nop, (double)semver_cmp(ksv, vsv), 0.0);
  }
  // DurationOperatorHandler.Evaluate (duration.go:42-120): int64 durations
  __device__ __forceinline__ int dur_of(CV x, int64_t* d) const {  // 1 ok, 0 not a duration, -1 undecided
    const uint32_t t = type(x);
    if (t == JT_NUM) return f2dur(num(x), d) ? 1 : 0;
    if (t != JT_STR) return 0;
    if (raw(x)) return numeric_looking(x, false) ? -1 : 0;
    const uint8_t* tb;
    const KpeScalar* s = scalar(x, &tb);
    if (!(s->flags & SC_DUR)) return 0;
    *d = s->dur;
    return 1;
  }
  __device__ __forceinline__ int op_dur(uint32_t nop, CV k, CV v) {
    int64_t kd = 0, vd = 0;
    const int a1 = dur_of(k, &kd);
    if (a1 <= 0) return a1;
    const int a2 = dur_of(v, &vd);
    if (a2 <= 0) return a2;
    switch (nop) {
      case CN_GE: return kd >= vd;
      case CN_GT: return kd > vd;
      case CN_LE: return kd <= vd;
      case CN_LT: return kd < vd;
      default: return 0;
    }
  }

  // ---- conditions ---------------------------------------------------------------------------
  __device__ __forceinline__ int condition(uint32_t ci) {
    const KpeCCond c = a.conds[ci];
    CV kv[2];
    for (int side = 0; side < 2; ++side) {  // key (buffers 0, 1, 2), then value (3, 4, 5)
      const uint32_t b = side ? 3u : 0u;
      const int st = value(side ? c.value : c.key, b, b + 1u, b + 2u, &kv[side]);
      if (st == CS_UNDEC) return CB_UNDEC;
      if (st != CS_OK) {
        bt = (uint32_t)side << 7;  // the substitution error's side (CT_ERR_SIDE)
        return CB_ERROR;
      }
    }
    bt = 2u << 7;  // an operator error
    const CV k = kv[0], v = kv[1];
    int r;
    if (c.op <= CO_NE) r = op_equals(k, v, c.op == CO_NE);
    else if (c.op == CO_NUM) r = op_num(c.aux, k, v);
    else if (c.op == CO_DUR) r = op_dur(c.aux, k, v);
    else if (c.op == CO_BAD) r = -2;  // no operator handler: an error once key and value substituted
    else if (c.op >= CO_IN) r = op_in(k, v, c.op == CO_NOTIN);
    else r = op_set(c.op, k, v, c.aux);
    if (r == -2) return CB_ERROR;
    if (r < 0) return CB_UNDEC;
    return r ? CB_TRUE : CB_FALSE;
  }
  // evaluateAnyAllConditions: any (when present) then all, each short-circuiting
  __device__ __forceinline__ int block(uint32_t bi) {
    const KpeCBlock b = a.blocks[bi];
    const bool has_any = b.flags & CB_HAS_ANY;
    bool any_ok = !has_any;
    uint32_t as = b.nany;
    const uint32_t n = b.nany + b.nall;
    for (uint32_t i = has_any ? 0u : b.nany; i < n; ++i) {  // any (when present), then all
      const int r = condition(b.c0 + i);
      if (r >= CB_ERROR) {
        bt |= i;  // CT_ERR_COND: the condition that raised it
        return r;
      }
      if (i < b.nany) {
        if (r == CB_TRUE) {  // the first true `any` condition ends the any loop
          any_ok = true;
          as = i;
          i = b.nany - 1u;
        }
      } else if (r == CB_FALSE) {
        bt = as | (i - b.nany) << 7;
        return CB_FALSE;
      }
    }
    bt = as | b.nall << 7;
    return any_ok ? CB_TRUE : CB_FALSE;
  }
};

// kpe_cond_kernel's body for resource r: every condition rule whose cell the scan matched.
// A state machine so that block() (conditions), value() (foreach lists and pattern variables)
// and the pattern VM (foreach pattern entries) are each called from one place: everything is
// inlined, and every extra call site would be another copy.
//
// Foreach (validateForEach / validateElements, validate_resource.go:186-254): a stack of
// KPE_FE_DEPTH frames, one per nesting level; an element's verdict `ev` goes to the frame's
// loop (FE_RES): nil / skip continue, an error counts only on the last element, a failure
// ends the level, a pass counts; a level's result goes to its parent element (or the cell).
// Pattern rules with {{ }} variables (substitutePatterns, :456-476): the rule's variables are
// resolved after its preconditions into pvals (an error => RuleError, a value the pattern VM
// cannot use => undecided) and the cell stays pending for kpe_pattern_kernel.
constexpr uint32_t PH_PRE = 0, PH_HANDLER = 1, PH_DENY = 2, PH_FE_LIST = 3, PH_FE_EL = 4, PH_FE_PRE = 5,
                   PH_FE_DENY = 6, PH_DONE = 7, PH_PV = 8, PH_FE_BODY = 9, PH_FE_PAT = 10, PH_FE_RES = 11,
                   PH_FE_POP = 12, PH_EXC = 13;
struct FeFrame {
  KpeCForeach fe;
  uint32_t f, fend, idx, n, count, applied;
  CV lst;
  bool one;
  uint32_t scoped;  // the innermost scoped element's tape entry (kNoNode: the resource)
};
// A resolved pattern variable (kpe_pattern_kernel reads it): 0 ok, else the cell's verdict
__device__ __forceinline__ uint32_t pv_store(CondVM& vm, CV x, uint32_t flags, uint2* dst) {
  const uint32_t t = vm.type(x);
  if (flags & PVF_KEY) {  // a whole-string variable naming a map key (traverse.go:90-117)
    if (t == JT_NULL) return KPE_UNDECIDED_;  // the key stays as written
    if (t != JT_STR) return KPE_ERROR_;       // "expected string after substituting variables in key"
  }
  if (t == JT_NULL) {
    *dst = make_uint2(PVK_NULL, 0u);
    return 0u;
  }
  if (t == JT_ARR || t == JT_OBJ || CondVM::raw(x) || x.k == VK_LIST) return KPE_UNDECIDED_;  // a subtree / key text
  if (x.k == VK_NUM) {
    *dst = make_uint2(PVK_NUM, x.p);
    return 0u;
  }
  const uint8_t* tb;
  const KpeScalar* sc = vm.scalar(x, &tb);
  const uint32_t f = sc->flags;
  if ((flags & PVF_WHOLE) && t == JT_STR && !(f & SC_PSIMPLE)) return KPE_UNDECIDED_;
  if (flags & PVF_TEXT) {  // json.Marshal of a float64 equals its fmt.Sprint text only without exponent
    if (t == JT_STR) {  // a substituted "{{" would be substituted again (vars.go nested loop)
      for (uint32_t i = 0; i + 1u < sc->text_len; ++i)
        if (tb[sc->text_off + i] == '{' && tb[sc->text_off + i + 1u] == '{') return KPE_UNDECIDED_;
    }
    if (SC_TYPE(f) == SC_T_INT && (sc->ival > (1ll << 53) || sc->ival < -(1ll << 53))) return KPE_UNDECIDED_;
    if (SC_TYPE(f) == SC_T_FLOAT)
      for (uint32_t i = 0; i < sc->sp_len; ++i)
        if (tb[sc->text_off + sc->text_len + i] == 'e') return KPE_UNDECIDED_;
  }
  *dst = make_uint2(x.k == VK_NODE ? PVK_SCAL : PVK_CONST, x.k == VK_NODE ? vm.doc[x.p].y : x.p);
  return 0u;
}

// A substituted key equal to another substituted key of its map (PVF_GROUP: the map's keys with
// variables, resolved in slot order): jsonutils/traverse.go:104-114 renames them in Go's random
// map order, so which value the shared key keeps is not defined (the cell is undecided)
__device__ __forceinline__ bool pv_key_collides(const CondArgs& a, const uint2* pvrow, uint32_t k0, uint32_t k) {
  const uint32_t g = PVF_GROUP(a.pvars[k].flags);
  auto view = [&](uint2 x) {
    const KpeScalar* s = x.x == PVK_SCAL ? a.scal + x.y : a.ctab + x.y;
    return SView{(x.x == PVK_SCAL ? a.scal_text : a.ctext) + s->text_off, (int)s->text_len};
  };
  const SView v = view(pvrow[k]);
  for (uint32_t j = k0; j < k; ++j)
    if (PVF_GROUP(a.pvars[j].flags) == g) {
      const SView w = view(pvrow[j]);
      if (w.n == v.n && bytes_eq(w.s, v.s, v.n)) return true;
    }
  return false;
}

template <bool FEPAT>
__device__ __forceinline__ void cond_eval_row(const CondArgs& a, int64_t r, char (*nb)[16], uint8_t* tx) {
  const uint64_t im = a.img_off ? a.img_off[r] : ~0ull;
  CondVM vm{a, reinterpret_cast<const uint2*>(a.doc), (uint32_t)a.doc_off[r], im == ~0ull ? kNoNode : (uint32_t)im,
            {}, {}, -1, {}, {}, nb, tx, 0u};
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  uint2* pvrow = a.pvals ? a.pvals + (size_t)r * a.nvars : nullptr;
  for (uint32_t i = 0; i < a.ncr; ++i) {
    const KpeCRule cr = a.rules[i];
    const uint8_t cell = row[cr.col];
    uint32_t* mt = cr.mslot && a.mtrace ? a.mtrace + (size_t)r * a.nmsg + (cr.mslot - 1u) : nullptr;
    uint32_t mtv = 0;
    if (mt) *mt = 0u;
    if (cell == KPE_NA_) continue;  // the rule did not match
    const bool fe_tr = mt && cr.kind == CR_FOREACH;  // four trace words (KPE_FE_TRACE_WORDS)
    if (fe_tr) mt[1] = 0u;
    // A PolicyException the scan decided already made the cell RuleSkip (validate_resource.go:
    // 44-56 returns before the deny / foreach is evaluated). A deferred one (XC_DEFER) is applied
    // here after the preconditions, in the cells whose exception match held (KPE_XDEFER_).
    const bool xd = (cr.xflags & XC_DEFER) && (cell & KPE_XDEFER_);
    uint32_t v = xd ? cell & ~(uint32_t)KPE_XDEFER_ : cell;
    if (cr.pre == CE_NONE && !xd && cell != KPE_PENDING_) continue;
    uint32_t ph = cr.pre != CE_NONE ? PH_PRE : xd ? PH_EXC : PH_HANDLER;
    FeFrame fr[KPE_FE_DEPTH];
    vm.dep = -1;
    uint32_t ev = 0;            // the current element's verdict (PH_FE_RES) / a level's result (PH_FE_POP)
    uint32_t pk = 0, pk0 = 0, pend = 0;  // pattern variable slots being resolved
    // a foreach element whose verdict may decide the cell (FAIL / ERROR): its path, what decided
    // it and its tape entries (schema.h FT_*); a later candidate replaces it, and the one that
    // propagates to the cell is always the last
    auto cand = [&](uint32_t kind, uint32_t ct, CV el, uint32_t scoped) {
      if (!fe_tr) return;
      uint32_t b = (uint32_t)vm.dep | kind << 2 | FT_VALID;
      for (int l = 0; l <= vm.dep; ++l) {
        const uint32_t left = fr[l].fend - fr[l].f, idx = fr[l].idx;
        if (left > 7u || idx > 31u) b |= FT_OVERFLOW;
        b |= ((left & 7u) | (idx & 31u) << 3) << (8u + 8u * (uint32_t)l);
      }
      mt[1] = b;
      mt[2] = el.k == VK_NODE ? el.p : 0xFFFFFFFFu;
      mt[3] = scoped;
      mtv = (mtv & 0xFFFFu) | ct << 16;
    };
    while (ph != PH_DONE) {
      if (ph == PH_HANDLER) {
        if (cr.kind == CR_DENY) {
          ph = PH_DENY;
        } else if (cr.kind == CR_FOREACH) {
          vm.dep = 0;
          fr[0].f = cr.fe0, fr[0].fend = cr.fe0 + cr.nfe, fr[0].applied = 0, fr[0].scoped = kNoNode;
          ph = PH_FE_LIST;
        } else if (cr.npv) {
          pk = pk0 = cr.pv0, pend = cr.pv0 + cr.npv;
          ph = PH_PV;
        } else {
          if (cr.kind == CR_NONE) v = KPE_NA_;  // no handler: no response
          ph = PH_DONE;
        }
        continue;
      }
      if (ph == PH_FE_POP) {  // level vm.dep finished with ev
        if (vm.dep == 0) {
          v = ev;
          ph = PH_DONE;
        } else {
          --vm.dep;
          ph = PH_FE_RES;
        }
        continue;
      }
      FeFrame& F = fr[vm.dep < 0 ? 0 : vm.dep];
      if (ph == PH_FE_LIST && F.f >= F.fend) {  // every entry done: pass if any element applied
        ev = F.applied ? KPE_PASS_ : KPE_NA_;
        ph = PH_FE_POP;
        continue;
      }
      if (ph == PH_FE_LIST || ph == PH_PV) {  // the one value() call site
        uint32_t ti;
        if (ph == PH_FE_LIST) {
          F.fe = a.fes[F.f];
          ti = F.fe.list;
        } else {
          if (pk >= pend) {  // every variable resolved
            ph = vm.dep < 0 ? PH_DONE : PH_FE_PAT;
            continue;
          }
          ti = a.pvars[pk].tmpl;
        }
        const uint32_t lb = 6u + (uint32_t)(vm.dep < 0 ? 0 : vm.dep);
        const int saved = vm.dep;
        if (ph == PH_FE_LIST) --vm.dep;  // a level's list is evaluated in its parent's context
        CV res;
        const int st = vm.value(ti, 0, 1, 2, &res);
        vm.dep = saved;
        if (st == CS_UNDEC) {
          v = KPE_UNDECIDED_;
          ph = PH_DONE;
          continue;
        }
        if (ph == PH_PV) {
          uint32_t bad = st != CS_OK ? (uint32_t)KPE_ERROR_ : pv_store(vm, res, a.pvars[pk].flags, pvrow + pk);
          if (!bad && PVF_GROUP(a.pvars[pk].flags) && pv_key_collides(a, pvrow, pk0, pk)) bad = KPE_UNDECIDED_;
          ++pk;
          if (bad == KPE_UNDECIDED_) {
            v = KPE_UNDECIDED_;
            ph = PH_DONE;
          } else if (bad) {  // "variable substitution failed": RuleError
            if (vm.dep < 0) {
              v = KPE_ERROR_;
              ph = PH_DONE;
            } else {
              cand(FT_PVAR_ERR, 0u, vm.els[vm.dep], F.scoped);
              ev = KPE_ERROR_;
              ph = PH_FE_RES;
            }
          }
          continue;
        }
        // EvaluateList (utils/foreach.go:12-24)
        if (st != CS_OK) {  // "failed to evaluate list": the entry is skipped
          ++F.f;
          continue;
        }
        F.one = vm.type(res) != JT_ARR;  // a non-list result is a one-element list
        if (!F.one && res.k == VK_LIST) {  // keep a computed list out of the key / value buffers
          vm.blen[lb] = vm.blen[res.p];
          for (uint32_t k = 0; k < vm.blen[lb]; ++k) vm.buf[lb][k] = vm.buf[res.p][k];
          res = cv(VK_LIST, lb);
        }
        F.lst = res;
        F.n = F.one ? 1u : vm.alen(res);
        F.idx = 0, F.count = 0;
        ph = PH_FE_EL;
        continue;
      }
      if (ph == PH_FE_EL) {
        if (F.idx >= F.n) {
          F.applied += F.count;
          ++F.f;
          ph = PH_FE_LIST;
          continue;
        }
        const CV el = F.one ? F.lst : vm.aget(F.lst, F.idx);
        if (vm.type(el) == JT_NULL) {
          ++F.idx;
          continue;
        }
        const bool is_map = vm.type(el) == JT_OBJ;
        if (F.fe.scope == 2u && !is_map) {  // AddElementToContext: elementScope needs a map (RuleError)
          cand(FT_SCOPE_ERR, 0u, el, kNoNode);
          ev = KPE_ERROR_;
          ph = PH_FE_POP;
          continue;
        }
        vm.els[vm.dep] = el, vm.elis[vm.dep] = F.idx;
        const bool scoped = F.fe.scope == 0u ? is_map : F.fe.scope == 2u;
        const uint32_t parent = vm.dep > 0 ? fr[vm.dep - 1].scoped : kNoNode;
        // a scoped element is a map: a tape entry (VK_NODE) or a constant the pattern VM cannot walk
        F.scoped = scoped ? (el.k == VK_NODE ? el.p : 0xFFFFFFFEu) : parent;
        ph = F.fe.pre != CE_NONE ? PH_FE_PRE : PH_FE_BODY;
        continue;
      }
      if (ph == PH_FE_BODY) {
        if (F.fe.kind == FE_DENY) {
          ph = PH_FE_DENY;
        } else if (F.fe.kind == FE_PAT && FEPAT) {
          pk = pk0 = F.fe.c & 0xFFFFu, pend = pk + (F.fe.c >> 16);
          ph = PH_PV;
        } else if (F.fe.kind == FE_NEST && vm.dep + 1 < KPE_FE_DEPTH) {
          FeFrame& G = fr[vm.dep + 1];
          G.f = F.fe.a, G.fend = F.fe.a + F.fe.b, G.applied = 0, G.scoped = F.scoped;
          ++vm.dep;
          ph = PH_FE_LIST;
        } else if (F.fe.kind == FE_NONE) {
          ev = KPE_NA_;  // a nil response
          ph = PH_FE_RES;
        } else {
          v = KPE_UNDECIDED_;  // not compiled into this kernel instance
          ph = PH_DONE;
        }
        continue;
      }
      if (ph == PH_FE_PAT) {  // the entry's pattern / anyPattern (validatePatterns) on the element
        if constexpr (FEPAT) {
          if (F.scoped == 0xFFFFFFFEu) {
            v = KPE_UNDECIDED_;
            ph = PH_DONE;
            continue;
          }
          const PatArgs& pa = *a.pat;
          PatVM pvm{pa, PV_DOCVIEW(pa, vm.doc, 0u, pa.ndoc), F.scoped == kNoNode ? vm.root : F.scoped, pvrow, 0u};
          const uint32_t nr = F.fe.b & 0xFFFFu, pf = F.fe.b >> 16;
          uint32_t fails = 0, skips = 0, last = KPE_PASS_;
          bool passed = false, undec = false;
          if (pf & PR_ANY_BAD) last = KPE_ERROR_;
          for (uint32_t k = 0; k < nr && !passed && !undec && !(pf & PR_ANY_BAD); ++k) {
            last = pat_match_root(pvm, F.fe.a + k);
            if (last == KPE_PASS_) passed = true;
            else if (last == KPE_SKIP_) ++skips;
            else if (last == KPE_UNDECIDED_) undec = true;
            else ++fails;
          }
          if (undec) {
            v = KPE_UNDECIDED_;
            ph = PH_DONE;
            continue;
          }
          ev = !(pf & PR_ANY) || (pf & PR_ANY_BAD) ? last
                                                   : passed ? KPE_PASS_ : (fails ? KPE_FAIL_ : (skips ? KPE_SKIP_ : KPE_PASS_));
          if (ev == KPE_FAIL_ || ev == KPE_ERROR_) cand(FT_PAT, 0u, vm.els[vm.dep], F.scoped);
        }
        ph = PH_FE_RES;
        continue;
      }
      if (ph == PH_FE_RES) {  // the element's verdict ev
        if (ev == KPE_UNDECIDED_) {
          v = KPE_UNDECIDED_;
          ph = PH_DONE;
        } else if (ev == KPE_FAIL_ || (ev == KPE_ERROR_ && F.idx + 1u >= F.n)) {
          ph = PH_FE_POP;  // the level ends with ev
        } else {
          if (ev == KPE_PASS_) ++F.count;
          ++F.idx;
          ph = PH_FE_EL;
        }
        continue;
      }
      const bool elem = ph == PH_FE_PRE || ph == PH_FE_DENY;
      const uint32_t bi = ph == PH_PRE   ? cr.pre
                          : ph == PH_EXC ? cr.exc
                          : ph == PH_DENY ? cr.deny
                          : ph == PH_FE_PRE ? F.fe.pre
                                            : F.fe.deny;
      const int saved = vm.dep;
      if (!elem) vm.dep = -1;  // rule-level conditions: no element in the context
      const int res = bi == CE_NONE ? CB_TRUE : vm.block(bi);  // the one call site (an exception
                                                               // without conditions holds)
      vm.dep = saved;
      if (res == CB_UNDEC) {
        v = KPE_UNDECIDED_;
        ph = PH_DONE;
        continue;
      }
      if (mt && (ph == PH_PRE || ph == PH_DENY)) {  // the block's messages (CT_*) or its error
        const uint32_t t = res == CB_ERROR ? (vm.bt & 0x1FFu) | CT_ERR
                                           : (vm.bt & 0x3FFFu) | CT_EVAL | (res == CB_TRUE ? CT_TRUE : 0u);
        mtv |= t << (ph == PH_DENY ? 16u : 0u);
      }
      if (ph == PH_PRE) {  // engine.go:278-285: false => skip, error => error
        if (res == CB_TRUE) {
          ph = xd ? PH_EXC : PH_HANDLER;
        } else {
          v = res == CB_FALSE ? KPE_SKIP_ : KPE_ERROR_;
          ph = PH_DONE;
        }
      } else if (ph == PH_EXC) {  // MatchesException (exceptions.go:33-41): only true applies it
        if (res == CB_TRUE) {
          // validate_resource.go:43-56 skips; validate_pss.go:45-104 with podSecurity controls
          // evaluates the pod under the exception's exclusions (kpe_pssx_kernel, KPE_XFAIL_)
          if (cr.xflags & XC_PSS) v = v == KPE_FAIL_ ? KPE_XFAIL_ : v;
          else v = KPE_SKIP_;
          ph = PH_DONE;
        } else {
          ph = PH_HANDLER;
        }
      } else if (ph == PH_DENY) {  // validateDeny (validate_resource.go:268-279)
        v = res == CB_TRUE ? KPE_FAIL_ : res == CB_FALSE ? KPE_PASS_ : KPE_ERROR_;
        ph = PH_DONE;
      } else if (ph == PH_FE_PRE) {  // an element's preconditions: false => skip, error => error
        if (res == CB_TRUE) {
          ph = PH_FE_BODY;
        } else {
          if (res == CB_ERROR) cand(FT_PRE_ERR, (vm.bt & 0x1FFu) | CT_ERR, vm.els[vm.dep], F.scoped);
          ev = res == CB_FALSE ? KPE_SKIP_ : KPE_ERROR_;
          ph = PH_FE_RES;
        }
      } else {  // an element's deny: true => fail
        if (res == CB_TRUE) cand(FT_DENY, (vm.bt & 0x3FFFu) | CT_EVAL | CT_TRUE, vm.els[vm.dep], F.scoped);
        else if (res == CB_ERROR) cand(FT_DENY, (vm.bt & 0x1FFu) | CT_ERR, vm.els[vm.dep], F.scoped);
        ev = res == CB_TRUE ? KPE_FAIL_ : res == CB_FALSE ? KPE_PASS_ : KPE_ERROR_;
        ph = PH_FE_RES;
      }
    }
    row[cr.col] = (uint8_t)v;
    if (mtv) *mt = mtv;
  }
}
