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
constexpr int kCvBufs = 7;  // key: 0,1 (+2 list template); value: 3,4 (+5); foreach list: 6

constexpr uint32_t VK_NULL = 0, VK_NODE = 1, VK_CONST = 2, VK_LIST = 3, VK_KEY = 4, VK_NUM = 5;
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
  CV buf[kCvBufs][CV_LIST_CAP];
  uint32_t blen[kCvBufs];
  char (*nb)[16];  // 2 x 16 bytes for fmt.Sprint of an elementIndex: LDS on the device, so that
                   // no generic pointer ever reaches the lane's private memory

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
      case VK_KEY: return JT_STR;
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
  __device__ __forceinline__ int run_ops(const KpeCExpr& e, CV el, uint32_t eli, uint32_t b0, uint32_t b1, CV* out) {
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
        if (op == QO_MSL) {
          for (uint32_t k = 0; k < QO_ARG(o.x); ++k) i += 1u + QO_ARG(a.ops[i].x);
        }
        continue;
      }
      switch (op) {
        case QO_OBJ: cur = node(root); break;
        case QO_EL: cur = el; break;
        case QO_IDX: cur = cv(VK_NUM, eli); break;
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
  __device__ __forceinline__ int query(uint32_t ei, CV el, uint32_t eli, uint32_t b0, uint32_t b1, CV* out) {
    for (;;) {
      const KpeCExpr e = a.exprs[ei];
      CV r;
      const int st = run_ops(e, el, eli, b0, b1, &r);
      if (st == CS_NOTFOUND) return CS_ERROR;  // NotFoundError => "Unknown key" => RuleError
      if (st != CS_OK) return st;
      if (e.alt == CE_NONE || !is_false(r)) {
        *out = r;
        return CS_OK;
      }
      ei = e.alt;
    }
  }
  // A condition key / value after substitution (template `ti`); lists go to buffer bl. One
  // query() call site: a single query is a one-element template walk that returns its value.
  __device__ __forceinline__ int value(uint32_t ti, CV el, uint32_t eli, uint32_t b0, uint32_t b1, uint32_t bl, CV* out) {
    const KpeVTmpl t = a.tmpls[ti];
    const bool arr = t.kind == VT_ARRAY;
    const uint32_t n = arr ? t.b : 1u;
    blen[bl] = 0;
    for (uint32_t k = 0; k < n; ++k) {  // list elements: constants or queries (no nested lists)
      const KpeVTmpl te = arr ? a.tmpls[t.a + k] : t;
      CV x;
      if (te.kind == VT_CONST) {
        x = SC_TYPE(a.ctab[te.a].flags) == SC_T_NULL ? cv(VK_NULL, 0) : cv(VK_CONST, te.a);
      } else {
        const int st = query(te.a, el, eli, b0, b1, &x);
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
      if (type(x) != JT_STR || x.k == VK_KEY) return false;
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
    if (x.k != VK_KEY) return false;
    const SView s = str(x);
    if (s.n == 0) return false;
    const uint8_t c = s.s[0];
    if ((c >= '0' && c <= '9') || c == '+' || c == '-' || c == '.') return true;
    return floats && (c == 'I' || c == 'i' || c == 'N' || c == 'n');
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
          if (v.k == VK_KEY) return numeric_looking(v, true) ? -1 : neg;
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
        const KpeScalar* sk = k.k == VK_KEY ? nullptr : scalar(k, &tk);
        if (sk && (sk->flags & SC_QTY) && vt == JT_STR) {
          if (neg && str(v).n == 0) return !wm(str(v), str(k));
          const KpeScalar* sv = v.k == VK_KEY ? nullptr : scalar(v, &tv);
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
  __device__ __forceinline__ int op_set(uint32_t op, CV k, CV v) {
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

  // ---- conditions ---------------------------------------------------------------------------
  __device__ __forceinline__ int condition(uint32_t ci, CV el, uint32_t eli) {
    const KpeCCond c = a.conds[ci];
    CV kv[2];
    for (int side = 0; side < 2; ++side) {  // key (buffers 0, 1, 2), then value (3, 4, 5)
      const uint32_t b = side ? 3u : 0u;
      const int st = value(side ? c.value : c.key, el, eli, b, b + 1u, b + 2u, &kv[side]);
      if (st == CS_UNDEC) return CB_UNDEC;
      if (st != CS_OK) return CB_ERROR;
    }
    const CV k = kv[0], v = kv[1];
    int r;
    if (c.op <= CO_NE) r = op_equals(k, v, c.op == CO_NE);
    else if (c.op >= CO_IN) r = op_in(k, v, c.op == CO_NOTIN);
    else r = op_set(c.op, k, v);
    if (r == -2) return CB_ERROR;
    if (r < 0) return CB_UNDEC;
    return r ? CB_TRUE : CB_FALSE;
  }
  // evaluateAnyAllConditions: any (when present) then all, each short-circuiting
  __device__ __forceinline__ int block(uint32_t bi, CV el, uint32_t eli) {
    const KpeCBlock b = a.blocks[bi];
    const bool has_any = b.flags & CB_HAS_ANY;
    bool any_ok = !has_any;
    const uint32_t n = b.nany + b.nall;
    for (uint32_t i = has_any ? 0u : b.nany; i < n; ++i) {  // any (when present), then all
      const int r = condition(b.c0 + i, el, eli);
      if (r >= CB_ERROR) return r;
      if (i < b.nany) {
        if (r == CB_TRUE) {  // the first true `any` condition ends the any loop
          any_ok = true;
          i = b.nany - 1u;
        }
      } else if (r == CB_FALSE) {
        return CB_FALSE;
      }
    }
    return any_ok ? CB_TRUE : CB_FALSE;
  }
};

// kpe_cond_kernel's body for resource r: every condition rule whose cell the scan matched.
// A small state machine so that block() (and the foreach list's value()) are each called
// from one place: everything is inlined, and every extra call site would be another copy.
constexpr uint32_t PH_PRE = 0, PH_HANDLER = 1, PH_DENY = 2, PH_FE_LIST = 3, PH_FE_EL = 4, PH_FE_PRE = 5,
                   PH_FE_DENY = 6, PH_DONE = 7;
__device__ __forceinline__ void cond_eval_row(const CondArgs& a, int64_t r, char (*nb)[16]) {
  CondVM vm{a, reinterpret_cast<const uint2*>(a.doc), (uint32_t)a.doc_off[r], {}, {}, nb};
  uint8_t* row = a.verdicts + (size_t)r * a.R;
  for (uint32_t i = 0; i < a.ncr; ++i) {
    const KpeCRule cr = a.rules[i];
    const uint8_t cell = row[cr.col];
    if (cell == KPE_NA_) continue;  // the rule did not match
    uint32_t v = cell;
    uint32_t ph = cr.pre != CE_NONE ? PH_PRE : PH_HANDLER;
    // foreach state (validateForEach / validateElements, validate_resource.go:186-254)
    uint32_t f = 0, idx = 0, n = 0, count = 0, applied = 0;
    KpeCForeach fe{};
    CV lst = cv(VK_NULL, 0), el = cv(VK_NULL, 0);
    bool one = false;
    while (ph != PH_DONE) {
      uint32_t bi = CE_NONE;
      if (ph == PH_HANDLER) {
        if (cr.kind == CR_DENY) {
          ph = PH_DENY;
        } else if (cr.kind == CR_FOREACH) {
          ph = PH_FE_LIST;
        } else {
          if (cr.kind == CR_NONE) v = KPE_NA_;  // no handler: no response
          ph = PH_DONE;
        }
        continue;
      }
      if (ph == PH_FE_LIST) {  // next entry: EvaluateList (utils/foreach.go:12-24)
        if (f >= cr.nfe) {
          v = applied ? KPE_PASS_ : KPE_NA_;
          ph = PH_DONE;
          continue;
        }
        fe = a.fes[cr.fe0 + f];
        const int st = vm.value(fe.list, cv(VK_NULL, 0), 0, 0, 1, 2, &lst);
        if (st == CS_UNDEC) {
          v = KPE_UNDECIDED_;
          ph = PH_DONE;
          continue;
        }
        if (st != CS_OK) {  // "failed to evaluate list": the entry is skipped
          ++f;
          continue;
        }
        one = vm.type(lst) != JT_ARR;  // a non-list result is a one-element list
        if (!one && lst.k == VK_LIST) {  // keep a computed list out of the key / value buffers
          vm.blen[6] = vm.blen[lst.p];
          for (uint32_t k = 0; k < vm.blen[6]; ++k) vm.buf[6][k] = vm.buf[lst.p][k];
          lst = cv(VK_LIST, 6);
        }
        n = one ? 1u : vm.alen(lst);
        idx = 0, count = 0;
        ph = PH_FE_EL;
        continue;
      }
      if (ph == PH_FE_EL) {
        if (idx >= n) {
          applied += count;
          ++f;
          ph = PH_FE_LIST;
          continue;
        }
        el = one ? lst : vm.aget(lst, idx);
        if (vm.type(el) == JT_NULL) {
          ++idx;
          continue;
        }
        if (fe.scope == 2u && vm.type(el) != JT_OBJ) {  // AddElementToContext: elementScope needs a map
          v = KPE_ERROR_;
          ph = PH_DONE;
          continue;
        }
        ph = fe.pre != CE_NONE ? PH_FE_PRE : PH_FE_DENY;
        continue;
      }
      const bool elem = ph == PH_FE_PRE || ph == PH_FE_DENY;
      bi = ph == PH_PRE ? cr.pre : ph == PH_DENY ? cr.deny : ph == PH_FE_PRE ? fe.pre : fe.deny;
      const int res = vm.block(bi, elem ? el : cv(VK_NULL, 0), elem ? idx : 0u);  // the one call site
      if (res == CB_UNDEC) {
        v = KPE_UNDECIDED_;
        ph = PH_DONE;
        continue;
      }
      if (ph == PH_PRE) {  // engine.go:278-285: false => skip, error => error
        if (res == CB_TRUE) {
          ph = PH_HANDLER;
        } else {
          v = res == CB_FALSE ? KPE_SKIP_ : KPE_ERROR_;
          ph = PH_DONE;
        }
      } else if (ph == PH_DENY) {  // validateDeny (validate_resource.go:268-279)
        v = res == CB_TRUE ? KPE_FAIL_ : res == CB_FALSE ? KPE_PASS_ : KPE_ERROR_;
        ph = PH_DONE;
      } else {  // an element's preconditions (false => skip) or deny (true => fail)
        uint32_t ev;
        if (res == CB_ERROR) ev = KPE_ERROR_;
        else if (ph == PH_FE_PRE) ev = res == CB_FALSE ? KPE_SKIP_ : 0u;
        else ev = res == CB_TRUE ? KPE_FAIL_ : KPE_PASS_;
        if (ev == 0u) {  // preconditions hold: evaluate the deny conditions
          ph = PH_FE_DENY;
          continue;
        }
        ph = PH_FE_EL;
        ++idx;
        if (ev == KPE_PASS_) {
          ++count;
        } else if (ev == KPE_FAIL_) {
          v = KPE_FAIL_;
          ph = PH_DONE;
        } else if (ev == KPE_ERROR_ && idx >= n) {  // an error counts only on the last element
          v = KPE_ERROR_;
          ph = PH_DONE;
        }
      }
    }
    row[cr.col] = (uint8_t)v;
  }
}
