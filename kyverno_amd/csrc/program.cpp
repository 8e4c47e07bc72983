// Policy compiler: ClusterPolicy/Policy JSON -> autogen -> device rule program.
//
// Follows, in order:
//   autogen.ComputeRules / CanAutoGen / generateRules   pkg/autogen/autogen.go:67-116,192-270
//   generateRule / generateRuleForControllers / generateCronJobRule  pkg/autogen/rule.go:73-322
//   rule handler precedence (manifest > PSS > CEL > resource) pkg/engine/validation.go:32-63
//   match/exclude structure  pkg/engine/utils/match.go:168-300 (lowered to filter/term tables)
//   kind selectors           pkg/utils/kube/kind.go:11-46
//   PSS version selection    pkg/pss/evaluate.go:24-70 + ParseVersion :221-239 (folded into cv_mask)
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "goval.hpp"
#include "jscan.hpp"
#include "program.hpp"
#include "pss_msg.hpp"
#include "pss_fixed.hpp"

namespace kpe {

// ---------------------------------------------------------------------------
// Minimal JSON DOM for policies (small inputs; resources never use this).
struct JV {
  enum T { Null, Bool, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  double n = 0;
  bool is_int = false;
  int64_t i = 0;
  std::string s;
  std::vector<JV> a;
  std::vector<std::pair<std::string, JV>> o;
  const JV* get(const char* k) const {
    if (t != Obj) return nullptr;
    const JV* r = nullptr;
    for (auto& kv : o)
      if (kv.first == k) r = &kv.second;
    return r;
  }
  JV* getm(const char* k) {
    if (t != Obj) return nullptr;
    JV* r = nullptr;
    for (auto& kv : o)
      if (kv.first == k) r = &kv.second;
    return r;
  }
  void set(const std::string& k, JV v) {
    for (auto& kv : o)
      if (kv.first == k) {
        kv.second = std::move(v);
        return;
      }
    o.emplace_back(k, std::move(v));
  }
  static JV str(const std::string& x) {
    JV v;
    v.t = Str;
    v.s = x;
    return v;
  }
  static JV obj() {
    JV v;
    v.t = Obj;
    return v;
  }
  static JV strs(const std::vector<std::string>& l) {
    JV v;
    v.t = Arr;
    for (auto& x : l) v.a.push_back(str(x));
    return v;
  }
};

namespace {

JV parse_value(JCur& c) {
  JV v;
  std::string sc;
  switch (c.peek()) {
    case JK::Null: c.null(); break;
    case JK::Bool:
      v.t = JV::Bool;
      c.boolean(&v.b);
      break;
    case JK::Num: {
      JNum n;
      c.number(&n);
      v.t = JV::Num;
      v.is_int = n.is_int;
      v.i = n.i;
      v.n = n.is_int ? (double)n.i : n.f;
      break;
    }
    case JK::Str: {
      std::string_view sv;
      c.str(&sv, sc);
      v.t = JV::Str;
      v.s.assign(sv);
      break;
    }
    case JK::Arr: {
      v.t = JV::Arr;
      c.arr_begin();
      bool f = true;
      while (c.arr_next(f)) v.a.push_back(parse_value(c));
      break;
    }
    case JK::Obj: {
      v.t = JV::Obj;
      c.obj_begin();
      bool f = true;
      std::string_view k;
      std::string ks;
      while (c.obj_next(f, &k, ks)) {
        std::string key(k);
        JV child = parse_value(c);
        v.set(key, std::move(child));  // duplicate keys: last wins
      }
      break;
    }
    default: c.fail();
  }
  return v;
}

void write(const JV& v, std::string& o) {
  switch (v.t) {
    case JV::Null: o += "null"; break;
    case JV::Bool: o += v.b ? "true" : "false"; break;
    case JV::Num: {
      if (v.is_int) o += std::to_string(v.i);
      else {
        char b[64];
        snprintf(b, sizeof b, "%.17g", v.n);
        o += b;
        if (!strpbrk(b, ".eEni")) o += ".0";  // stays a float64 through a re-parse
      }
      break;
    }
    case JV::Str: {
      o += '"';
      for (unsigned char ch : v.s) {
        if (ch == '"' || ch == '\\') {
          o += '\\';
          o += (char)ch;
        } else if (ch < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", ch);
          o += b;
        } else {
          o += (char)ch;
        }
      }
      o += '"';
      break;
    }
    case JV::Arr:
      o += '[';
      for (size_t k = 0; k < v.a.size(); ++k) {
        if (k) o += ',';
        write(v.a[k], o);
      }
      o += ']';
      break;
    case JV::Obj:
      o += '{';
      for (size_t k = 0; k < v.o.size(); ++k) {
        if (k) o += ',';
        write(JV::str(v.o[k].first), o);
        o += ':';
        write(v.o[k].second, o);
      }
      o += '}';
      break;
  }
}

JV parse_all(const char* p, size_t n) {
  JCur c(p, p + n);
  JV v = parse_value(c);
  c.ws();
  if (!c.ok() || c.pos() != p + n) throw std::invalid_argument("malformed policy JSON");
  return v;
}
// document-order JSON of a policy fragment (reparsed by the message renderers)
std::string doc_text(const JV& v) {
  std::string o;
  write(v, o);
  return o;
}
// the JSON type encoding/json's UnmarshalTypeError names (decode.go: "object", "string", ...)
const char* json_type_name(const JV& v) {
  switch (v.t) {
    case JV::Obj: return "object";
    case JV::Str: return "string";
    case JV::Bool: return "bool";
    case JV::Num: return "number";
    case JV::Arr: return "array";
    default: return "null";
  }
}

std::string sv(const JV* v) { return (v && v->t == JV::Str) ? v->s : std::string(); }
std::vector<std::string> svl(const JV* v) {
  std::vector<std::string> o;
  if (v && v->t == JV::Arr)
    for (auto& e : v->a)
      if (e.t == JV::Str) o.push_back(e.s);
  return o;
}
bool nonempty(const JV* v) {  // !DeepEqual(x, zero value)
  if (!v) return false;
  switch (v->t) {
    case JV::Null: return false;
    case JV::Bool: return v->b;
    case JV::Num: return v->n != 0;
    case JV::Str: return !v->s.empty();
    case JV::Arr: return !v->a.empty();
    case JV::Obj:
      for (auto& kv : v->o)
        if (nonempty(&kv.second)) return true;
      return false;
  }
  return false;
}

std::vector<std::string> split(const std::string& s, char d) {
  std::vector<std::string> o;
  size_t i = 0;
  while (true) {
    size_t j = s.find(d, i);
    if (j == std::string::npos) {
      o.push_back(s.substr(i));
      break;
    }
    o.push_back(s.substr(i, j - i));
    i = j + 1;
  }
  return o;
}

// host glob (go-wildcard v1.0.3 semantics, runes) — only for compile-time constant folding
bool glob_host(const std::string& pat, const std::string& s) {
  if (pat.empty()) return s.empty();
  if (pat == "*") return true;
  auto runes = [](const std::string& x) {
    std::vector<uint32_t> r;
    for (size_t i = 0; i < x.size();) {
      unsigned char ch = (unsigned char)x[i];
      int n = ch < 0x80 ? 1 : (ch >> 5) == 6 ? 2 : (ch >> 4) == 14 ? 3 : (ch >> 3) == 30 ? 4 : 1;
      uint32_t cp = 0;
      for (int k = 0; k < n && i + k < x.size(); ++k) cp = (cp << 8) | (unsigned char)x[i + k];
      r.push_back(cp);
      i += n;
    }
    return r;
  };
  auto p = runes(pat), t = runes(s);
  size_t pi = 0, si = 0, star = SIZE_MAX, mark = 0;
  while (si < t.size()) {
    if (pi < p.size() && (p[pi] == '?' || (p[pi] != '*' && p[pi] == t[si]))) {
      ++pi;
      ++si;
    } else if (pi < p.size() && p[pi] == '*') {
      star = pi++;
      mark = si;
    } else if (star != SIZE_MAX) {
      pi = star + 1;
      si = ++mark;
    } else {
      return false;
    }
  }
  while (pi < p.size() && p[pi] == '*') ++pi;
  return pi == p.size();
}

// ---- kind helpers (pkg/utils/kube/kind.go) ----
// k8s.io/apimachinery v0.29.1 util/validation, restated (third-party; pinned by
// pkg/utils/match/labels_test.go and the selector cases of tests/golden).
bool qname_char(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
bool name_part_ok(const std::string& s) {  // qualifiedNameFmt, <= 63 bytes
  if (s.empty() || s.size() > 63 || !qname_char(s.front()) || !qname_char(s.back())) return false;
  for (char c : s)
    if (!(qname_char(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
bool dns1123_subdomain_ok(const std::string& s) {  // dns1123SubdomainFmt, <= 253 bytes
  if (s.empty() || s.size() > 253) return false;
  size_t i = 0;
  while (true) {
    size_t j = s.find('.', i);
    if (j == std::string::npos) j = s.size();
    if (j == i) return false;
    for (size_t k = i; k < j; ++k) {
      char c = s[k];
      bool an = (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9');
      if (!(an || (c == '-' && k != i && k + 1 != j))) return false;
    }
    if (j == s.size()) return true;
    i = j + 1;
  }
}
bool qualified_name_ok(const std::string& s) {  // IsQualifiedName
  size_t p = s.find('/');
  if (p == std::string::npos) return name_part_ok(s);
  if (s.find('/', p + 1) != std::string::npos) return false;
  return dns1123_subdomain_ok(s.substr(0, p)) && name_part_ok(s.substr(p + 1));
}
bool label_value_ok(const std::string& s) { return s.empty() || name_part_ok(s); }  // IsValidLabelValue
bool has_wildcard(const std::string& s) {  // wildcard.ContainsWildcard
  return s.find('*') != std::string::npos || s.find('?') != std::string::npos;
}

bool version_regex(const std::string& s) {  // `^v\d((alpha|beta)\d)?|\*$`
  if (s.size() >= 2 && s[0] == 'v' && s[1] >= '0' && s[1] <= '9') return true;
  return !s.empty() && s.back() == '*';
}
struct KindSel {
  std::string g, v, k, sub;
};
KindSel parse_kind_selector(const std::string& in) {
  auto parts = split(in, '/');
  auto last = split(parts.back(), '.');
  parts.pop_back();
  for (auto& x : last) parts.push_back(x);
  auto lower = [](std::string x) {
    for (auto& ch : x) ch = (char)tolower((unsigned char)ch);
    return x;
  };
  switch (parts.size()) {
    case 1: return {"*", "*", parts[0], ""};
    case 2:
      if (parts[0] == "*" && parts[1] == "*") return {"*", "*", "*", "*"};
      if (parts[0] == "*" && lower(parts[1]) == parts[1]) return {"*", "*", parts[0], parts[1]};
      if (version_regex(parts[0])) return {"*", parts[0], parts[1], ""};
      return {"*", "*", parts[0], parts[1]};
    case 3:
      if (version_regex(parts[0])) return {"*", parts[0], parts[1], parts[2]};
      return {parts[0], parts[1], parts[2], ""};
    case 4: return {parts[0], parts[1], parts[2], parts[3]};
    default: return {"", "", "", ""};
  }
}
bool contains_kind(const std::vector<std::string>& list, const std::string& kind) {  // kube.ContainsKind
  for (auto& e : list) {
    auto parts = split(e, '/');
    auto fmt = [](std::string s) {
      size_t d = s.find('.');
      if (d != std::string::npos) s[d] = '/';
      return s;
    };
    std::string k;
    switch (parts.size()) {
      case 1: k = fmt(e); break;
      case 2:
        if (parts[0] == "*" && parts[1] == "*") k = "*/*";
        else if (version_regex(parts[0])) k = fmt(parts[1]);
        else k = parts[0] + "/" + parts[1];
        break;
      case 3: k = version_regex(parts[0]) ? parts[1] + "/" + parts[2] : fmt(parts[2]); break;
      case 4: k = parts[2] + "/" + parts[3]; break;
      default: k = "";
    }
    auto sp = split(k, '/');
    if (sp.size() == 2) k = sp[0];
    if (k == kind) return true;
  }
  return false;
}

// ---- autogen (pkg/autogen) ----
const char* kPodControllers = "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController,CronJob";

bool autogen_support(bool* needed, const JV* rd) {
  if (!rd || rd->t != JV::Obj) return true;
  static const std::set<std::string> pc = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                           "ReplicationController", "CronJob", "Pod"};
  auto kinds = svl(rd->get("kinds"));
  const JV* ann = rd->get("annotations");
  const JV* sel = rd->get("selector");
  if (!sv(rd->get("name")).empty() || !svl(rd->get("names")).empty() || (sel && sel->t != JV::Null) ||
      (ann && ann->t != JV::Null) || (kinds.size() > 1 && contains_kind(kinds, "Pod")))
    return false;
  for (auto& k : kinds)
    if (pc.count(k)) *needed = true;
  return true;
}
bool can_autogen(const JV& spec) {
  bool needed = false;
  const JV* rules = spec.get("rules");
  if (!rules || rules->t != JV::Arr) return false;
  for (auto& r : rules->a) {
    const JV* mut = r.get("mutate");
    if (mut && !sv(mut->get("patchesJson6902")).empty()) return false;
    if (nonempty(r.get("generate"))) return false;
    if (mut && mut->get("foreach") && mut->get("foreach")->t == JV::Arr)
      for (auto& fe : mut->get("foreach")->a)
        if (!sv(fe.get("patchesJson6902")).empty()) return false;
    const JV* m = r.get("match");
    const JV* x = r.get("exclude");
    if (!autogen_support(&needed, m ? m->get("resources") : nullptr)) return false;
    if (!autogen_support(&needed, x ? x->get("resources") : nullptr)) return false;
    for (const JV* blk : {m, x}) {
      if (!blk) continue;
      for (const char* k : {"any", "all"}) {
        const JV* l = blk->get(k);
        if (l && l->t == JV::Arr)
          for (auto& f : l->a)
            if (!autogen_support(&needed, f.get("resources"))) return false;
      }
    }
  }
  return needed;
}
std::vector<std::string> block_kinds(const JV* blk) {  // MatchResources.GetKinds
  std::vector<std::string> k;
  if (!blk) return k;
  if (const JV* rd = blk->get("resources"))
    for (auto& s : svl(rd->get("kinds"))) k.push_back(s);
  for (const char* key : {"all", "any"}) {
    const JV* l = blk->get(key);
    if (l && l->t == JV::Arr)
      for (auto& f : l->a)
        if (const JV* r = f.get("resources"))
          for (auto& s : svl(r->get("kinds"))) k.push_back(s);
  }
  return k;
}
std::string autogen_name(const std::string& prefix, const std::string& name) {
  std::string n = prefix + "-" + name;
  return n.size() > 63 ? n.substr(0, 63) : n;
}
bool is_autogen_name(const std::string& n) { return n.compare(0, 8, "autogen-") == 0; }

bool generate_rule(JV& out, const std::string& name, const JV& rule, const char* tpl,
                   const std::vector<std::string>& kinds, bool all_filters) {
  out = rule;
  out.set("name", JV::str(name));
  auto grf = [&](JV& list) {
    for (auto& f : list.a) {
      JV* rd = f.getm("resources");
      if (!rd) continue;
      if (all_filters || contains_kind(svl(rd->get("kinds")), "Pod")) rd->set("kinds", JV::strs(kinds));
    }
  };
  for (const char* bk : {"match", "exclude"}) {
    bool is_match = !strcmp(bk, "match");
    JV* blk = out.getm(bk);
    if (!blk || blk->t != JV::Obj) {
      if (is_match) {
        JV m = JV::obj(), rd = JV::obj();
        rd.set("kinds", JV::strs(kinds));
        m.set("resources", rd);
        out.set(bk, m);
      }
      continue;
    }
    JV* any = blk->getm("any");
    JV* all = blk->getm("all");
    if (any && any->t == JV::Arr && !any->a.empty()) grf(*any);
    else if (all && all->t == JV::Arr && !all->a.empty()) grf(*all);
    else {
      JV* rd = blk->getm("resources");
      if (is_match) {
        if (!rd) {
          blk->set("resources", JV::obj());
          rd = blk->getm("resources");
        }
        rd->set("kinds", JV::strs(kinds));
      } else if (rd && !svl(rd->get("kinds")).empty()) {
        rd->set("kinds", JV::strs(kinds));
      }
    }
  }
  const JV* val = rule.get("validate");
  // SetPattern(ToJSON(...)) (autogen rule.go:130-183): json.Marshal writes a whole float64
  // below 1e21 as an integer literal, which decodes back as int64 when it fits.
  std::function<void(JV&)> marshal = [&](JV& x) {
    if (x.t == JV::Num && !x.is_int && std::isfinite(x.n) && x.n == std::trunc(x.n) && std::fabs(x.n) < 1e21 &&
        x.n >= -9223372036854775808.0 && x.n < 9223372036854775808.0)
      x.is_int = true, x.i = (int64_t)x.n;
    for (auto& y : x.a) marshal(y);
    for (auto& kv : x.o) marshal(kv.second);
  };
  auto wrap = [&](const JV& target0) {
    JV target = target0;
    marshal(target);
    JV inner = JV::obj(), outer = JV::obj();
    inner.set(tpl, target);
    outer.set("spec", inner);
    return outer;
  };
  JV nv = JV::obj();
  if (val && val->get("message")) nv.set("message", *val->get("message"));
  auto present = [&](const char* k) { return val && val->get(k) && val->get(k)->t != JV::Null; };
  if (present("pattern")) nv.set("pattern", wrap(*val->get("pattern")));
  else if (present("deny")) nv.set("deny", *val->get("deny"));
  else if (present("podSecurity")) nv.set("podSecurity", *val->get("podSecurity"));
  else if (val && val->get("anyPattern") && val->get("anyPattern")->t == JV::Arr) {
    JV arr;
    arr.t = JV::Arr;
    for (auto& p : val->get("anyPattern")->a) arr.a.push_back(wrap(p));
    nv.set("anyPattern", arr);
  } else if (val && val->get("foreach") && val->get("foreach")->t == JV::Arr && !val->get("foreach")->a.empty())
    nv.set("foreach", *val->get("foreach"));
  else
    return false;
  out.set("validate", nv);
  return true;
}
bool gen_for_controllers(JV& out, const JV& rule, const std::string& controllers) {
  std::string name = sv(rule.get("name"));
  if (is_autogen_name(name) || controllers.empty()) return false;
  auto mk = block_kinds(rule.get("match"));
  auto xk = block_kinds(rule.get("exclude"));
  if (!contains_kind(mk, "Pod") || (!xk.empty() && !contains_kind(xk, "Pod"))) return false;
  static const std::set<std::string> valid = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                              "ReplicationController"};
  std::vector<std::string> kinds;
  if (controllers == "all") kinds = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"};
  else {
    for (auto& c : split(controllers, ','))
      if (valid.count(c)) kinds.push_back(c);
    if (kinds.empty()) kinds = split(controllers, ',');
  }
  return generate_rule(out, autogen_name("autogen", name), rule, "template", kinds, false);
}
std::string replace_all(std::string s, const std::string& a, const std::string& b) {
  size_t p = 0;
  while ((p = s.find(a, p)) != std::string::npos) {
    s.replace(p, a.size(), b);
    p += b.size();
  }
  return s;
}
JV convert_rule(const JV& r, bool cron) {  // autogen.go updateGenRuleByte
  std::string s;
  write(r, s);
  std::string mid = cron ? "spec.jobTemplate.spec.template." : "spec.template.";
  for (const char* o : {"request.object.", "request.oldObject."}) {
    s = replace_all(s, std::string(o) + "spec", std::string(o) + mid + "spec");
    s = replace_all(s, std::string(o) + "metadata", std::string(o) + mid + "metadata");
  }
  return parse_all(s.data(), s.size());
}
std::vector<JV> compute_rules(const JV& policy) {
  const JV* spec = policy.get("spec");
  std::vector<JV> orig;
  if (spec && spec->get("rules") && spec->get("rules")->t == JV::Arr) orig = spec->get("rules")->a;
  if (!spec) return orig;
  bool apply = can_autogen(*spec);
  std::string controllers = apply ? kPodControllers : "none";
  const JV* meta = policy.get("metadata");
  const JV* ann = meta ? meta->get("annotations") : nullptr;
  const JV* ac = ann ? ann->get("pod-policies.kyverno.io/autogen-controllers") : nullptr;
  if (ac && apply) controllers = sv(ac);
  if (controllers == "none") return orig;
  std::string nocron;
  for (auto& c : split(controllers, ','))
    if (c != "CronJob") nocron += (nocron.empty() ? "" : ",") + c;
  std::vector<JV> gen;
  for (auto& r : orig) {
    JV g;
    if (gen_for_controllers(g, r, nocron)) gen.push_back(convert_rule(g, false));
    if (controllers.find("CronJob") != std::string::npos || controllers.find("all") != std::string::npos) {
      JV inter;
      if (gen_for_controllers(inter, r, controllers)) {
        JV g2;
        if (generate_rule(g2, autogen_name("autogen-cronjob", sv(r.get("name"))), inter, "jobTemplate",
                          {"CronJob"}, true))
          gen.push_back(convert_rule(g2, true));
      }
    }
  }
  if (gen.empty()) return orig;
  std::vector<JV> out;
  for (auto& r : orig)
    if (!is_autogen_name(sv(r.get("name")))) out.push_back(r);
  for (auto& g : gen) out.push_back(g);
  return out;
}

// ---- pattern compilation (validate.pattern / anyPattern) ----------------------------------
// Restates, at compile time, every decision of the reference's tree walk that depends only
// on the pattern: anchor parsing (anchor/anchor.go:8-123), the anchor / non-anchor split and
// evaluation order of validateMap (validate/validate.go:118-175, validate/utils.go:11-69),
// array shapes (validate.go:177-261), the string-pattern grammar (pattern.go:152-215,
// operator/operator.go:7-61) and the ExpandInMetadata targets (wildcards/wildcards.go:83-162).
// Everything that depends on the resource is left to kpe_pattern_kernel.
namespace pc {

enum AK { AK_NONE, AK_COND, AK_GLOBAL, AK_NEG, AK_ADD, AK_EQ, AK_EXIST };
struct Anc {
  AK k = AK_NONE;
  std::string key;
};
inline bool ws_ascii(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r'; }
std::string trim_ws(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && ws_ascii(s[a])) ++a;
  while (b > a && ws_ascii(s[b - 1])) --b;
  return s.substr(a, b - a);
}
std::string trim_sp(const std::string& s) {
  size_t a = s.find_first_not_of(' ');
  if (a == std::string::npos) return "";
  return s.substr(a, s.find_last_not_of(' ') - a + 1);
}
// ^([+<=X^])?\((.+)\)$ on the TrimSpace-d key
Anc anchor_of(const std::string& raw) {
  Anc r;
  const std::string t = trim_ws(raw);
  if (t.size() < 3 || t.back() != ')') return r;
  static const char mods[] = "+<=X^";
  static const AK kinds[] = {AK_ADD, AK_GLOBAL, AK_EQ, AK_NEG, AK_EXIST};
  size_t open = 0;
  AK k = AK_COND;
  if (const char* m = strchr(mods, t[0]); m && t[0]) k = kinds[m - mods], open = 1;
  if (t[open] != '(') return r;
  std::string inner = t.substr(open + 1, t.size() - open - 2);
  if (inner.empty() || inner.find('\n') != std::string::npos) return r;
  r.k = k;
  r.key = std::move(inner);
  return r;
}
bool phase1(AK k) { return k == AK_COND || k == AK_EXIST || k == AK_EQ || k == AK_NEG; }
bool nested_anchor(const JV& v) {
  if (v.t == JV::Obj) {
    for (auto& kv : v.o) {
      const AK k = anchor_of(kv.first).k;
      if (phase1(k) || k == AK_GLOBAL) return true;
    }
    for (auto& kv : v.o)
      if (nested_anchor(kv.second)) return true;
  } else if (v.t == JV::Arr) {
    for (auto& x : v.a)
      if (nested_anchor(x)) return true;
  }
  return false;
}
bool has_glob(const std::string& s) { return s.find_first_of("*?") != std::string::npos; }
bool has_vars(const JV& v) {
  auto bad = [](const std::string& x) { return x.find("{{") != std::string::npos || x.find("$(") != std::string::npos; };
  if (v.t == JV::Str) return bad(v.s);
  for (auto& x : v.a)
    if (has_vars(x)) return true;
  for (auto& kv : v.o)
    if (bad(kv.first) || has_vars(kv.second)) return true;
  return false;
}
// one range endpoint, anchored: [-|+]?\d+(\.\d+)?[A-Za-z]*
bool endpoint(const std::string& x) {
  size_t i = 0;
  auto dg = [&](size_t j) { return j < x.size() && x[j] >= '0' && x[j] <= '9'; };
  if (i < x.size() && (x[i] == '-' || x[i] == '|' || x[i] == '+')) ++i;
  if (!dg(i)) return false;
  while (dg(i)) ++i;
  if (i < x.size() && x[i] == '.') {
    if (!dg(i + 1)) return false;
    ++i;
    while (dg(i)) ++i;
  }
  while (i < x.size() && isalpha((unsigned char)x[i])) ++i;
  return i == x.size();
}
bool split_range(const std::string& t, const char* sep, std::string* l, std::string* r) {
  const size_t n = strlen(sep);
  for (size_t k = 1; k + n <= t.size(); ++k)
    if (!t.compare(k, n, sep) && endpoint(t.substr(0, k)) && endpoint(t.substr(k + n))) {
      *l = t.substr(0, k), *r = t.substr(k + n);
      return true;
    }
  return false;
}

class PatCompiler {
 public:
  PatCompiler(PatProgram& pp, std::function<int32_t(const std::string&)> key_pred) : PP(pp), key_pred_(key_pred) {}
  // Strings with {{ }} variables (substitutePatterns, validate_resource.go:456-476): fills a
  // PL_VAR / PL_TMPL leaf and returns true; false for a plain string
  std::function<bool(const std::string&, KpeLeaf&)> var_leaf;
  // A map key with {{ }} variables (jsonutils/traverse.go:90-117): its template leaf (PMF_VKEY)
  std::function<bool(const std::string&, KpeLeaf&)> key_leaf;

  // one root (validate.MatchPattern call); returns the root table index
  uint32_t root(const JV& pattern) {
    slots_.clear();
    expand_.clear();
    const uint32_t n = node(pattern, 0, false);
    PP.roots.push_back(n);
    PP.roots.push_back((uint32_t)slots_.size());
    return (uint32_t)(PP.roots.size() / 2 - 1);
  }

 private:
  // compile recursion bound only: walks deeper than the VM's frame stack (patvm.inl kPatStack)
  // make their cells KPE_UNDECIDED at run time
  static constexpr int kMaxDepth = 64;
  PatProgram& PP;
  std::function<int32_t(const std::string&)> key_pred_;
  std::map<std::string, uint32_t> slots_;  // AnchorMap key -> slot
  std::set<const JV*> expand_;             // labels/annotations maps ExpandInMetadata rewrites

  uint32_t push_node(KpePNode n) {
    PP.nodes.push_back(n);
    return (uint32_t)PP.nodes.size() - 1;
  }
  uint32_t operand(const std::string& text, bool exact) {
    PP.operands.push_back(text);
    PP.operand_exact.push_back(exact ? 1 : 0);
    return (uint32_t)PP.operands.size() - 1;
  }
  void cond(uint32_t op, const std::string& operand_text, uint32_t flags) {
    KpeCond c{};
    c.op = op | flags;
    c.pat = operand(operand_text, false);
    int64_t d;
    if (goval::parse_duration(operand_text, &d)) c.op |= PC_DUR, c.dur = d;
    goval::Quantity q;
    if (goval::parse_quantity(operand_text, &q)) {
      c.op |= PC_QTY | (q.neg ? PC_QNEG : 0u);
      goval::qty_key(q, &c.qexp, &c.qlo, &c.qhi);
    }
    PP.conds.push_back(c);
  }
  // A scalar pattern leaf (pattern.Validate's pattern side). Also the InRange values of the
  // condition set operators (anyin.go:103-109 handleRange: pattern.Validate(key, value)).
 public:
  uint32_t leaf(const JV& v) {
    KpeLeaf l{};
    switch (v.t) {
      case JV::Bool: l.type = PL_BOOL, l.bval = v.b ? 1u : 0u; break;
      case JV::Num:
        if (v.is_int) l.type = PL_INT, l.ival = v.i;
        else l.type = PL_FLOAT, l.fval = v.n;
        break;
      case JV::Null: l.type = PL_NIL; break;
      case JV::Str: {
        if (var_leaf && var_leaf(v.s, l)) break;
        l.type = PL_STR;
        l.exact = operand(v.s, true);
        l.c0 = (uint32_t)PP.conds.size();
        size_t a = 0;
        const std::string& pat = v.s;
        for (size_t i = 0; i <= pat.size(); ++i) {  // strings.Split(pattern, "|")
          if (i < pat.size() && pat[i] != '|') continue;
          const std::string alt = trim_sp(pat.substr(a, i - a));
          a = i + 1;
          uint32_t group = PC_NEWGROUP;
          size_t b = 0;
          for (size_t j = 0; j <= alt.size(); ++j) {  // strings.Split(alternative, "&")
            if (j < alt.size() && alt[j] != '&') continue;
            const std::string t = trim_sp(alt.substr(b, j - b));
            b = j + 1;
            std::string lo, hi;
            // operator.GetOperatorFromStringPattern
            uint32_t op = PC_EQ;
            size_t oplen = 0;
            if (t.size() >= 2) {
              if (!t.compare(0, 2, ">=")) op = PC_GE, oplen = 2;
              else if (!t.compare(0, 2, "<=")) op = PC_LE, oplen = 2;
              else if (t[0] == '>') op = PC_GT, oplen = 1;
              else if (t[0] == '<') op = PC_LT, oplen = 1;
              else if (t[0] == '!') op = PC_NE, oplen = 1;
              else if (split_range(t, "!-", &lo, &hi)) {  // NotInRange: < lo | > hi
                cond(PC_LT, lo, group | PC_OR2);
                cond(PC_GT, hi, 0);
                group = 0;
                continue;
              } else if (split_range(t, "-", &lo, &hi)) {  // InRange: >= lo & <= hi
                cond(PC_GE, lo, group);
                cond(PC_LE, hi, 0);
                group = 0;
                continue;
              }
            }
            cond(op, trim_ws(t.substr(oplen)), group);
            group = 0;
          }
        }
        l.nc = (uint32_t)PP.conds.size() - l.c0;
        for (uint32_t i = l.c0; i < l.c0 + l.nc; ++i)
          if (PP.conds[i].op & PC_DUR) l.pad[0] = 1u;  // some operand is a duration
        break;
      }
      default: l.type = PL_NEVER; break;
    }
    PP.leaves.push_back(l);
    return (uint32_t)PP.leaves.size() - 1;
  }
 private:

  uint32_t node(const JV& v, int depth, bool repeated) {
    if (depth > kMaxDepth) throw CompileError("pattern nested deeper than 64 levels");
    if (v.t == JV::Obj) return map(v, depth, repeated);
    if (v.t == JV::Arr) {
      if (v.a.empty()) return push_node({PN_ARR_EMPTY, 0, 0, 0});
      const JV& e0 = v.a[0];
      if (e0.t == JV::Obj) {
        const uint32_t n = node(e0, depth + 1, true);
        return push_node({PN_ARR_MAPS, n, 0, 0});
      }
      if (e0.t != JV::Arr) return push_node({PN_ARR_LEAF, leaf(e0), 0, 0});
      std::vector<uint32_t> kids;
      for (auto& e : v.a) kids.push_back(node(e, depth + 1, true));
      const uint32_t at = (uint32_t)PP.lists.size();
      PP.lists.insert(PP.lists.end(), kids.begin(), kids.end());
      return push_node({PN_ARR_POS, at, (uint32_t)kids.size(), 0});
    }
    return push_node({PN_LEAF, leaf(v), 0, 0});
  }

  uint32_t map(const JV& v, int depth, bool repeated) {
    // ExpandInMetadata targets below this map (getPatternValue: plain or anchored key)
    const JV* meta = nullptr;
    for (auto& kv : v.o)
      if (kv.first == "metadata" || anchor_of(kv.first).key == "metadata") {
        meta = &kv.second;
        break;
      }
    if (meta && meta->t == JV::Obj)
      for (const char* tag : {"labels", "annotations"})
        for (auto& kv : meta->o)
          if (kv.first == tag || anchor_of(kv.first).key == tag) {
            if (kv.second.t == JV::Obj) expand_.insert(&kv.second);
            break;
          }
    const bool expanding = expand_.count(&v) > 0;
    std::vector<std::string> first, front, back;
    std::vector<std::string> vkeys;  // the map's keys with variables
    for (auto& kv : v.o) {
      const Anc a = anchor_of(kv.first);
      if (kv.first.find("$(") != std::string::npos)
        throw CompileError("$(...) references in pattern keys are not supported on the device");
      if (kv.first.find("{{") != std::string::npos) {
        if (!key_leaf) throw CompileError("variables in pattern keys are not supported here");
        if (a.k != AK_NONE) {
          // an anchor whose key has variables: traverse.go:90-117 renames "=({{x}})" to "=(value)"
          // before validateMap parses the anchor, so the anchor is the written one and its key the
          // substituted text inside the parentheses (kpe: PMF_VKEY with the anchor's handler)
          if (!phase1(a.k)) throw CompileError("global / add anchors with variables in their key are not supported");
          if (trim_ws(kv.first) != kv.first || kv.first.find("{{") < kv.first.find('('))
            throw CompileError("an anchored pattern key with variables outside its parentheses");
        }
        if (expanding && has_glob(kv.first)) throw CompileError("wildcard metadata keys with variables");
        if (expanding && repeated) throw CompileError("metadata keys with variables under an array pattern");
        vkeys.push_back(kv.first);
      }
      if (expanding && has_glob(kv.first) && repeated)  // the reference rewrites the shared pattern per element
        throw CompileError("wildcard metadata keys under an array pattern are not supported");
      if (phase1(a.k)) first.push_back(kv.first);
    }
    if (expanding) {
      // anchored glob keys are expanded per resource (wildcards.go:145-162) and the anchor phase
      // / global members run in the sorted order of the expanded keys (validate.go:118-175): the
      // order of the compile-time keys is the same unless another such member's key starts with
      // the glob key's literal prefix
      for (auto& kv : v.o) {
        const AK ka = anchor_of(kv.first).k;
        if (!has_glob(kv.first) || (!phase1(ka) && ka != AK_GLOBAL)) continue;
        const std::string pre = kv.first.substr(0, kv.first.find_first_of("*?"));
        for (auto& other : v.o) {
          const AK ko = anchor_of(other.first).k;
          if (&other == &kv || (phase1(ka) ? !phase1(ko) : ko != AK_GLOBAL)) continue;
          if (other.first.compare(0, pre.size(), pre) == 0)
            throw CompileError("anchored wildcard metadata keys whose expansion can reorder the anchors");
        }
      }
    }
    // several keys with variables in one map: each must be one whole-string variable, whose
    // substituted value kpe_cond_kernel compares with the map's other substituted keys (a rename
    // of one onto another, traverse.go:108-114, depends on Go's map order: the cell is undecided)
    if (vkeys.size() > 1)
      for (auto& k : vkeys) {
        if (anchor_of(k).k != AK_NONE)
          throw CompileError("an anchored pattern key with variables beside another key with variables");
        const bool whole = k.size() >= 4 && k.compare(0, 2, "{{") == 0 && k.find("{{", 2) == std::string::npos &&
                           k.find("}}") == k.size() - 2;
        if (!whole)
          throw CompileError("several pattern keys with variables in one map, one of them a partial string");
      }
    const uint32_t vgroup = vkeys.size() > 1 ? ++PP.vkey_groups : 0u;
    auto is_vkey = [&](const std::string& k) { return std::find(vkeys.begin(), vkeys.end(), k) != vkeys.end(); };
    std::sort(first.begin(), first.end());
    std::vector<std::string> rest;
    for (auto& kv : v.o)
      if (!phase1(anchor_of(kv.first).k)) rest.push_back(kv.first);
    // a key with variables takes the place of its text before the first variable (any place is
    // correct: the device checks per row that the substituted key sorts between the same
    // neighbours, else the cell is undecided)
    auto sort_text = [&](const std::string& k) { return is_vkey(k) ? k.substr(0, k.find("{{")) : k; };
    std::sort(rest.begin(), rest.end(),
              [&](const std::string& x, const std::string& y) { return sort_text(x) < sort_text(y); });
    for (auto& k : rest) {
      if (anchor_of(k).k == AK_GLOBAL || nested_anchor(*v.get(k.c_str()))) front.insert(front.begin(), k);
      else back.push_back(k);
    }
    std::vector<std::string> order = first;
    order.insert(order.end(), front.begin(), front.end());
    order.insert(order.end(), back.begin(), back.end());
    // members are written after the values are compiled (values append members too)
    std::vector<uint32_t> mem;
    for (auto& k : order) {
      const JV& val = *v.get(k.c_str());
      const Anc a = anchor_of(k);
      uint32_t h = PM_DEFAULT, flags = 0, slot = 0, w = 0xFFFFFFFFu, vn = 0xFFFFFFFFu;  // w: PRED_NONE
      std::string name = k;
      switch (a.k) {
        case AK_COND: h = PM_COND; break;
        case AK_GLOBAL: h = PM_GLOBAL; break;
        case AK_EXIST: h = PM_EXIST; break;
        case AK_EQ: h = PM_EQ; break;
        case AK_NEG: h = PM_NEG; break;
        default: break;  // plain keys and "+(...)" keys are looked up verbatim
      }
      if (h != PM_DEFAULT) name = a.key;
      if (h == PM_COND || h == PM_EXIST) {
        auto it = slots_.find(k);
        if (it == slots_.end()) it = slots_.emplace(k, (uint32_t)slots_.size()).first;
        if (it->second < 32) flags |= PMF_SLOT, slot = it->second;
        else flags |= PMF_XSLOT;
      }
      if (h == PM_DEFAULT && val.t == JV::Str && val.s == "*") flags |= PMF_STAR;
      if (is_vkey(k)) {
        // validateMap walks the plain keys without nested anchors in sorted order and returns the
        // first error; such members can only fail plainly, so the verdict does not depend on where
        // the substituted key sorts (only the failure path of a message does: checked per row by
        // the trace walk). A key whose value holds anchors would move among members that skip.
        // An anchored key (phase 1, validate.go:118-175) is walked in the sorted order of the
        // substituted anchor keys, and the first non-skip error decides: its place among the map's
        // anchors is checked per row in every walk (bit 2), else the cell is undecided.
        const bool anc = a.k != AK_NONE;
        if (!anc && nested_anchor(val)) throw CompileError("a pattern key with variables whose value holds anchors");
        KpeLeaf kl{};
        if (!key_leaf(k, kl)) throw CompileError("pattern key template");
        kl.bval = expanding ? 1u : 0u;
        if (anc) {
          if (kl.type != PL_TMPL) throw CompileError("pattern key template");
          kl.bval |= 4u;
          kl.pad[2] = (uint32_t)(k.find('(') + 1u) | 1u << 16;  // anchor text before / after the key
        }
        if (vgroup) {  // bit 1: other keys of the map have variables too (their order is not tracked)
          kl.bval |= 2u;
          PP.vars[kl.c0].flags |= (vgroup & 0xFFFFFFu) << PVF_GROUP_SH;
        }
        // the map's other plain keys in walk order, [u16 length][bytes] each, and this key's place
        kl.pad[0] = (uint32_t)PP.ttext.size();
        uint32_t nsib = 0, at = 0;
        for (auto& t : anc ? first : rest) {
          if (t == k) {
            at = nsib;
            continue;
          }
          if (t.size() >= 0xFFFFu) throw CompileError("pattern key longer than 64 KiB");
          PP.ttext.push_back((uint8_t)(t.size() & 0xFF)), PP.ttext.push_back((uint8_t)(t.size() >> 8));
          PP.ttext.insert(PP.ttext.end(), t.begin(), t.end());
          ++nsib;
        }
        if (nsib > 0xFFFFu) throw CompileError("pattern map with too many keys");
        kl.pad[1] = nsib | at << 16;
        PP.leaves.push_back(kl);
        flags |= PMF_VKEY;
        w = (uint32_t)PP.leaves.size() - 1;
      }
      if (expanding && has_glob(k) && a.k != AK_ADD) {  // "+(...)" keys stay verbatim
        flags |= PMF_GLOB;
        w = (uint32_t)key_pred_(name);
      }
      if (h == PM_EXIST) {
        if (val.t != JV::Arr) {
          vn = push_node({PN_BAD, 0, 0, 0});
        } else {
          std::vector<uint32_t> kids;
          for (auto& e : val.a)
            kids.push_back(e.t == JV::Obj ? node(e, depth + 1, true) : push_node({PN_BAD, 0, 0, 0}));
          const uint32_t at = (uint32_t)PP.lists.size();
          PP.lists.insert(PP.lists.end(), kids.begin(), kids.end());
          vn = push_node({PN_EXLIST, at, (uint32_t)kids.size(), 0});
        }
      } else if (h != PM_NEG && !(flags & PMF_STAR)) {
        vn = node(val, depth + 1, repeated);
        if (PP.nodes[vn].kind == PN_LEAF) {
          flags |= PMF_LEAF;
          const uint32_t lt = PP.leaves[PP.nodes[vn].y].type;
          if (h == PM_DEFAULT && (lt == PL_VAR || lt == PL_TMPL)) flags |= PMF_VSTAR;
        }
      }
      uint32_t ki = 0;
      for (; ki < PP.keys.size() && PP.keys[ki] != name; ++ki) {
      }
      if (ki == PP.keys.size()) PP.keys.push_back(name);
      mem.insert(mem.end(), {h | flags | (slot << 8), ki, vn, w});
    }
    const uint32_t m0 = (uint32_t)(PP.members.size() / 4);
    PP.members.insert(PP.members.end(), mem.begin(), mem.end());
    uint32_t depth_in = order.size() <= 8 ? 1u : 0u;  // inline depth (schema.h PNF_FLAT)
    for (size_t i = 0; i < mem.size() && depth_in; i += 4) {
      const uint32_t x = mem[i], h = PM_HANDLER(x);
      if (h == PM_EXIST || (x & (PMF_GLOB | PMF_XSLOT | PMF_VKEY))) {
        depth_in = 0;
      } else if (h != PM_NEG && !(x & (PMF_STAR | PMF_LEAF))) {  // a map (or list) value
        const KpePNode& c = PP.nodes[mem[i + 2]];
        const uint32_t cw = c.w & PNW_DEPTH;
        depth_in = (c.kind == PN_MAP && cw && cw < PNF_MAXDEPTH) ? std::max(depth_in, cw + 1u) : 0u;
      }
    }
    const bool chain = mem.size() == 4 && first.empty() && mem[0] == PM_DEFAULT && PP.nodes[mem[2]].kind != PN_LEAF;
    return push_node({PN_MAP, m0, (uint32_t)first.size() | ((uint32_t)order.size() << 16),
                      depth_in | (chain ? PNW_CHAIN : 0u)});
  }
};

}  // namespace pc

// ---- lowering ----
// ---- compile-time condition folding ---------------------------------------------------
// Preconditions and deny conditions whose keys are letter-only literals or the whole-string
// variable {{request.operation}}, and whose values are letter-only literals that may add `*`
// and `?` globs, are decided here: the CLI and background scans evaluate with
// request.operation = CREATE (policy_processor.go / scanner.go build CREATE contexts).
// Letter-only strings are never durations, quantities or InRange patterns, and the key is
// never a glob, so the two-way wildcard.Match of the operators reduces to value-as-pattern:
// equal.go / notequal.go wildcard.Match(value, key), anyin.go:65 / allin.go:60 / in.go:64
// Match(sprint(v), k) || Match(k, sprint(v)). A scalar string value that does not match is
// then decoded as a JSON []string: "null" is a valid empty list, "true" / "false" fail to
// decode (invalid type => the operator is false), and any other letter-only text is not JSON,
// which anyin.go:81-88 (and allin / anynotin / allnotin) reads as a one-element list but
// in.go:74-78 / notin.go (keyExistsInArray) reads as an invalid type. Anything else is refused.
enum Fold { F_NO = 0, F_FALSE = 1, F_TRUE = 2 };

bool fold_scalar(const JV& v, std::string* out, bool glob = false) {
  if (v.t != JV::Str) return false;
  std::string t = v.s;
  if (t.find("{{") != std::string::npos) {
    // replaceBracesAndTrimSpaces (variables/vars.go:422-427) on a whole-string reference
    if (t.size() < 4 || t.compare(0, 2, "{{") != 0 || t.compare(t.size() - 2, 2, "}}") != 0) return false;
    std::string in = t.substr(2, t.size() - 4);
    size_t a = in.find_first_not_of(" \t"), b = in.find_last_not_of(" \t");
    if (a == std::string::npos) return false;
    in = in.substr(a, b - a + 1);
    if (in != "request.operation") {
      // `request.operation || '<raw string>'` (the chart idiom): CREATE is truthy, so `||`
      // returns it; the right operand only has to parse
      if (in.compare(0, 17, "request.operation") != 0) return false;
      size_t i = in.find_first_not_of(" \t", 17);
      if (i == std::string::npos || in.compare(i, 2, "||") != 0) return false;
      i = in.find_first_not_of(" \t", i + 2);
      if (i == std::string::npos || in[i] != '\'' || in.back() != '\'' || i + 1 >= in.size()) return false;
      for (size_t k = i + 1; k + 1 < in.size(); ++k)
        if (in[k] == '\'' || in[k] == '\\') return false;
    }
    *out = "CREATE";
    return true;
  }
  if (t.empty()) return false;
  for (char c : t)
    if (!((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (glob && (c == '*' || c == '?')))) return false;
  *out = t;
  return true;
}

Fold fold_condition(const JV& c) {
  if (c.t != JV::Obj) return F_NO;
  const JV* k = c.get("key");
  const JV* v = c.get("value");
  std::string key, op;
  if (!k || !fold_scalar(*k, &key)) return F_NO;
  for (char ch : sv(c.get("operator"))) op += (char)tolower((unsigned char)ch);
  std::vector<std::string> vals;
  bool list = false;
  if (!v) return F_NO;
  if (v->t == JV::Arr) {
    list = true;
    for (auto& e : v->a) {
      std::string x;
      if (!fold_scalar(e, &x, true)) return F_NO;
      vals.push_back(x);
    }
  } else {
    std::string x;
    if (!fold_scalar(*v, &x, true)) return F_NO;
    vals.push_back(x);
  }
  // values may be go-wildcard globs; the key never is (see above)
  bool in = false;
  for (auto& x : vals) in = in || glob_host(x, key);
  const bool legacy = op == "in" || op == "notin";
  bool invalid = false;  // the value fails to decode as a []string: every such operator is false
  if (!list && !in) {
    const std::string& x = vals[0];
    if (x == "true" || x == "false") invalid = true;   // valid JSON, not a []string
    else if (x != "null" && legacy) invalid = true;    // not JSON: keyExistsInArray's Unmarshal error
  }
  bool r;
  if (op == "equal" || op == "equals") r = !list && in;          // equal.go: string key vs string value
  else if (op == "notequal" || op == "notequals") r = list || !in;  // notequal.go: other value types => true
  else if (op == "anyin" || op == "allin" || op == "in") r = !invalid && in;  // a single key against the value set
  else if (op == "anynotin" || op == "allnotin" || op == "notin") r = !invalid && !in;
  else return F_NO;
  return r ? F_TRUE : F_FALSE;
}

// variables/evaluate.go:29-125 (EvaluateConditions / evaluateAnyAllConditions); null or absent
// conditions are true.
Fold fold_conditions(const JV* j) {
  if (!j || j->t == JV::Null) return F_TRUE;
  auto all_of = [](const JV& arr) {
    Fold out = F_TRUE;
    for (auto& e : arr.a) {
      Fold f = fold_condition(e);
      if (f == F_NO) return F_NO;
      if (f == F_FALSE) out = F_FALSE;
    }
    return out;
  };
  if (j->t == JV::Arr) return all_of(*j);
  if (j->t != JV::Obj) return F_NO;
  const JV* any = j->get("any");
  const JV* all = j->get("all");
  if ((any && any->t != JV::Arr && any->t != JV::Null) || (all && all->t != JV::Arr && all->t != JV::Null)) return F_NO;
  Fold any_ok = F_TRUE, all_ok = F_TRUE;
  if (any && any->t == JV::Arr) {
    any_ok = F_FALSE;
    for (auto& e : any->a) {
      Fold f = fold_condition(e);
      if (f == F_NO) return F_NO;
      if (f == F_TRUE) any_ok = F_TRUE;
    }
  }
  if (all && all->t == JV::Arr) all_ok = all_of(*all);
  if (all_ok == F_NO) return F_NO;
  return (any_ok == F_TRUE && all_ok == F_TRUE) ? F_TRUE : F_FALSE;
}

// where a block that folds (fold_conditions != F_NO) stops: its first true `any` condition and
// first false `all` condition (schema.h CT_ANY / CT_ALL)
void fold_stops(const JV* j, uint32_t* as, uint32_t* ls) {
  *as = *ls = 0;
  if (!j || j->t == JV::Null) return;
  auto first = [](const JV& arr, Fold want) {
    uint32_t i = 0;
    for (auto& e : arr.a) {
      if (fold_condition(e) == want) break;
      ++i;
    }
    return i;
  };
  if (j->t == JV::Arr) {
    *ls = first(*j, F_FALSE);
    return;
  }
  const JV* any = j->get("any");
  const JV* all = j->get("all");
  if (any && any->t == JV::Arr) *as = first(*any, F_TRUE);
  if (all && all->t == JV::Arr) *ls = first(*all, F_FALSE);
}

// The `message` of every condition of a block (utils.TransformConditions: a list is the
// deprecated form, an object holds `any` / `all`), in the order CondCompiler::block lays them out
CondMsgs cond_msgs(const JV* j) {
  CondMsgs m;
  if (!j || j->t == JV::Null) return m;
  m.present = true;
  auto text = [](const JV& c) {
    const JV* x = c.t == JV::Obj ? c.get("message") : nullptr;
    return x && x->t == JV::Str ? x->s : std::string();
  };
  if (j->t == JV::Arr) {
    m.old = true;
    for (auto& e : j->a) m.all.push_back(text(e));
    return m;
  }
  if (j->t != JV::Obj) return m;
  const JV* any = j->get("any");
  const JV* all = j->get("all");
  if (any && any->t == JV::Arr) {
    m.has_any = true;
    for (auto& e : any->a) m.any.push_back(text(e));
  }
  if (all && all->t == JV::Arr)
    for (auto& e : all->a) m.all.push_back(text(e));
  return m;
}

// ---- condition programs evaluated per resource (kpe_cond_kernel) -------------------------
// Conditions that read the resource (or a foreach element) are compiled to the device program
// of schema.h QO_* / KpeC*. The restated subset, with everything else refused (CompileError):
//   * substitution (variables/vars.go:311-389): a key / value is a constant, a string that is
//     exactly one {{ }} variable (which keeps its JSON type), or a list of those; `$(...)`,
//     partial-string and nested variables are refused;
//   * JMESPath (github.com/kyverno/go-jmespath, go.mod:33) over request.object,
//     request.operation ("CREATE"), element / elementIndex: fields, quoted fields, [n], `[]`,
//     `[*]`, `.[a, b]` multi-select of relative field chains, keys(@), `||` with a literal or
//     another chain, raw-string and JSON literals, length(<chain>) and `<chain> | length(@)`
//     (functions.go jpfLength: runes of a string, items of an array, members of an object, else
//     an invalid-type error). Parse errors of an empty expression are run-time errors; anything
//     outside the subset is refused;
//   * operators Equals / NotEquals / AnyIn / AllIn / AnyNotIn / AllNotIn / In / NotIn
//     (variables/operator/*.go); InRange values of set operators are refused (as the oracle).
namespace cq {

enum Tok { T_EOF, T_ID, T_QID, T_NUM, T_DOT, T_STAR, T_FLAT, T_LBRACK, T_RBRACK, T_COMMA, T_LPAREN, T_RPAREN,
           T_CUR, T_OR, T_LIT, T_RAW, T_PIPE, T_OTHER };
struct Token {
  Tok t;
  std::string s;
  long n = 0;
  JV lit;
};
// go-jmespath lexer.go, the token subset above (anything else is T_OTHER => refused)
std::vector<Token> lex(const std::string& q) {
  std::vector<Token> out;
  size_t i = 0;
  while (i < q.size()) {
    const char c = q[i];
    if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
      ++i;
      continue;
    }
    if (isalpha((unsigned char)c) || c == '_') {
      size_t j = i;
      while (j < q.size() && (isalnum((unsigned char)q[j]) || q[j] == '_')) ++j;
      out.push_back({T_ID, q.substr(i, j - i)});
      i = j;
      continue;
    }
    if (isdigit((unsigned char)c) || (c == '-' && i + 1 < q.size() && isdigit((unsigned char)q[i + 1]))) {
      size_t j = i + 1;
      while (j < q.size() && isdigit((unsigned char)q[j])) ++j;
      Token t{T_NUM, q.substr(i, j - i)};
      t.n = atol(t.s.c_str());
      out.push_back(t);
      i = j;
      continue;
    }
    if (c == '"') {  // quoted identifier (a JSON string)
      size_t j = i + 1;
      while (j < q.size() && q[j] != '"') j += q[j] == '\\' ? 2 : 1;
      if (j >= q.size()) throw CompileError("JMESPath: unclosed quoted identifier");
      const std::string body = q.substr(i, j + 1 - i);
      JCur jc(body.data(), body.data() + body.size());
      JV v = parse_value(jc);
      if (!jc.ok() || v.t != JV::Str) throw CompileError("JMESPath: bad quoted identifier");
      out.push_back({T_QID, v.s});
      i = j + 1;
      continue;
    }
    if (c == '\'') {  // raw string literal
      std::string s;
      size_t j = i + 1;
      while (j < q.size() && q[j] != '\'') {
        if (q[j] == '\\' && j + 1 < q.size() && q[j + 1] == '\'') {
          s += '\'';
          j += 2;
        } else {
          s += q[j++];
        }
      }
      if (j >= q.size()) throw CompileError("JMESPath: unclosed raw string");
      Token t{T_RAW, s};
      t.lit = JV::str(s);
      out.push_back(t);
      i = j + 1;
      continue;
    }
    if (c == '`') {  // JSON literal (an invalid one is a deprecated string literal)
      std::string s;
      size_t j = i + 1;
      while (j < q.size() && q[j] != '`') {
        if (q[j] == '\\' && j + 1 < q.size() && q[j + 1] == '`') {
          s += '`';
          j += 2;
        } else {
          s += q[j++];
        }
      }
      if (j >= q.size()) throw CompileError("JMESPath: unclosed JSON literal");
      Token t{T_LIT, s};
      JCur jc(s.data(), s.data() + s.size());
      JV v = parse_value(jc);
      jc.ws();
      if (jc.ok() && jc.pos() == s.data() + s.size()) t.lit = v;
      else t.lit = JV::str(s);
      out.push_back(t);
      i = j + 1;
      continue;
    }
    auto two = [&](char a, char b) { return c == a && i + 1 < q.size() && q[i + 1] == b; };
    if (two('[', ']')) {
      out.push_back({T_FLAT});
      i += 2;
      continue;
    }
    if (two('|', '|')) {
      out.push_back({T_OR});
      i += 2;
      continue;
    }
    Tok t = T_OTHER;
    switch (c) {
      case '.': t = T_DOT; break;
      case '*': t = T_STAR; break;
      case '[': t = (i + 1 < q.size() && q[i + 1] == '?') ? T_OTHER : T_LBRACK; break;
      case ']': t = T_RBRACK; break;
      case ',': t = T_COMMA; break;
      case '(': t = T_LPAREN; break;
      case ')': t = T_RPAREN; break;
      case '@': t = T_CUR; break;
      case '|': t = T_PIPE; break;
      default: break;
    }
    if (t == T_OTHER) throw CompileError(std::string("JMESPath construct '") + c + "' is not supported on the device");
    out.push_back({t});
    ++i;
  }
  out.push_back({T_EOF});
  return out;
}

// Constant table shared by the policy's literals, JSON literals and request.operation.
class Consts {
 public:
  explicit Consts(CondProgram& cp) : CP(cp) {}
  uint32_t scalar(const JV& v) {
    KpeScalar e{};
    switch (v.t) {
      case JV::Null: e.flags = SC_T_NULL; break;
      case JV::Bool:
        e.flags = SC_T_BOOL | SC_TEXT | (v.b ? SC_BTRUE : 0u);
        text(e, v.b ? "true" : "false");
        break;
      case JV::Num: {  // the JSON context holds float64 numbers (encoding/json into interface{})
        const double f = v.is_int ? (double)v.i : v.n;
        e.flags = SC_T_FLOAT | SC_TEXT;
        e.fval = f;
        text(e, goval::fmt_E(f));
        const std::string sp = goval::sprint_float(f);
        CP.ctext.insert(CP.ctext.end(), sp.begin(), sp.end());
        e.sp_len = (uint32_t)sp.size();
        attrs(e, goval::fmt_f(f));  // as the flattener's float scalars (convertNumberToString)
        if (goval::sprint_qty_same(sp, e.flags & SC_QTY, e.flags & SC_QNEG, e.qexp, e.qlo, e.qhi)) e.flags |= SC_SPQ;
        break;
      }
      case JV::Str: {
        e.flags = SC_T_STR | SC_TEXT;
        text(e, v.s);
        int64_t i;
        double f;
        if (goval::parse_int(v.s, &i)) e.flags |= SC_PINT, e.ival = i;
        if (goval::parse_float(v.s, &f)) e.flags |= SC_PFLOAT, e.fval = f;
        attrs(e, v.s);
        if (goval::pattern_simple(v.s)) e.flags |= SC_PSIMPLE;
        json_list(e, v.s);
        break;
      }
      default: throw CompileError("condition constant: objects are not supported on the device");
    }
    CP.consts.push_back(e);
    return (uint32_t)CP.consts.size() - 1;
  }
  // a list of constants (SC_T_ARR)
  uint32_t list(const std::vector<uint32_t>& items) {
    KpeScalar e{};
    e.flags = SC_T_ARR;
    e.text_off = (uint32_t)CP.clist.size();
    e.text_len = (uint32_t)items.size();
    CP.clist.insert(CP.clist.end(), items.begin(), items.end());
    CP.consts.push_back(e);
    return (uint32_t)CP.consts.size() - 1;
  }
  uint32_t value(const JV& v) {
    if (v.t == JV::Arr) {
      std::vector<uint32_t> items;
      for (auto& x : v.a) {
        if (x.t == JV::Arr || x.t == JV::Obj) throw CompileError("condition constant: nested lists are not supported");
        items.push_back(scalar(x));
      }
      return list(items);
    }
    return scalar(v);
  }

 private:
  CondProgram& CP;
  static void attrs(KpeScalar& e, const std::string& s) {  // ParseDuration / ParseQuantity of a text form
    int64_t d;
    if (goval::parse_duration(s, &d)) e.flags |= SC_DUR, e.dur = d;
    goval::Quantity q;
    if (goval::parse_quantity(s, &q)) {
      e.flags |= SC_QTY | (q.neg ? SC_QNEG : 0u);
      goval::qty_key(q, &e.qexp, &e.qlo, &e.qhi);
    }
  }
  void text(KpeScalar& e, const std::string& s) {
    e.text_off = (uint32_t)CP.ctext.size();
    e.text_len = (uint32_t)s.size();
    CP.ctext.insert(CP.ctext.end(), s.begin(), s.end());
  }
  // A string value of a set / In operator is decoded as a JSON []string when json.Valid
  // (anyin.go:81-88; in.go:74-78 decodes it straight away): SC_JVALID marks valid JSON, SC_JLIST
  // a successful []string decode whose elements are the constant list packed in ival.
  void json_list(KpeScalar& e, const std::string& s) {
    JCur c(s.data(), s.data() + s.size());
    c.ws();
    if (c.pos() == s.data() + s.size()) return;  // empty / blank: not JSON
    JV v = parse_value(c);
    c.ws();
    if (!c.ok() || c.pos() != s.data() + s.size()) return;
    e.flags |= SC_JVALID;
    if (v.t == JV::Null) {  // null decodes to a nil slice
      e.flags |= SC_JLIST;
      e.ival = (int64_t)CP.clist.size();  // count 0
      return;
    }
    if (v.t != JV::Arr) return;
    std::vector<uint32_t> items;
    for (auto& x : v.a) {
      if (x.t == JV::Null) items.push_back(scalar(JV::str("")));  // null => "" in a []string
      else if (x.t == JV::Str) items.push_back(scalar(x));
      else return;                                                 // Unmarshal type error
    }
    e.flags |= SC_JLIST;
    e.ival = (int64_t)CP.clist.size() | ((int64_t)items.size() << 32);
    CP.clist.insert(CP.clist.end(), items.begin(), items.end());
  }
};

// Parser of the restated JMESPath subset into schema.h QO_* ops.
class QueryParser {
 public:
  QueryParser(CondProgram& cp, Consts& k) : CP(cp), K(k) {}

  // a whole query (a {{ }} variable text or a foreach list); returns the expression index
  uint32_t compile(const std::string& q0) {
    std::string q = q0;
    while (!q.empty() && isspace((unsigned char)q.back())) q.pop_back();
    size_t b = 0;
    while (b < q.size() && isspace((unsigned char)q[b])) ++b;
    q = q.substr(b);
    if (q.empty()) {  // "invalid query (nil)": an evaluation error at run time
      KpeCExpr e{(uint32_t)CP.ops.size() / 2, 1, 0, CE_NONE};
      CP.ops.insert(CP.ops.end(), {QO_ERROR, 0u});
      CP.exprs.push_back(e);
      return (uint32_t)CP.exprs.size() - 1;
    }
    t_ = lex(q);
    i_ = 0;
    if (std::any_of(t_.begin(), t_.end(), [](const Token& t) { return t.t == T_PIPE; })) {
      // `<chain> | length(@)`, the one pipe on the device: the pipe binds loosest (a `||` would
      // sit inside one of its sides), so no `||` is accepted with it
      if (std::any_of(t_.begin(), t_.end(), [](const Token& t) { return t.t == T_OR; }))
        throw CompileError("JMESPath pipe with `||` is not supported on the device: " + q);
      bool pl = true;
      std::vector<uint32_t> c = chain(&pl);
      if (!(cur().t == T_PIPE && peek().t == T_ID && peek().s == "length" && peek(2).t == T_LPAREN &&
            peek(3).t == T_CUR && peek(4).t == T_RPAREN && peek(5).t == T_EOF))
        throw CompileError("JMESPath pipe other than `| length(@)` is not supported on the device: " + q);
      op(c, QO_LEN);
      KpeCExpr e{(uint32_t)CP.ops.size() / 2, (uint32_t)c.size() / 2, 0, CE_NONE};  // a pipe: not strict
      CP.ops.insert(CP.ops.end(), c.begin(), c.end());
      CP.exprs.push_back(e);
      return (uint32_t)CP.exprs.size() - 1;
    }
    std::vector<std::vector<uint32_t>> chains;
    std::vector<bool> plain;
    for (;;) {
      bool pl = true;
      chains.push_back(chain(&pl));
      plain.push_back(pl);
      if (cur().t == T_OR) {
        ++i_;
        continue;
      }
      break;
    }
    if (cur().t != T_EOF) throw CompileError("JMESPath expression outside the device subset: " + q);
    // `a || b || c`: left-associative N_OR nodes; the first truthy operand wins, else the last
    uint32_t next = CE_NONE;
    for (size_t k = chains.size(); k-- > 0;) {
      KpeCExpr e{(uint32_t)CP.ops.size() / 2, (uint32_t)chains[k].size() / 2, 0, next};
      // strict (NotFoundError on a missing member) only for a query that is one plain chain
      if (chains.size() == 1 && plain[k]) e.flags |= CE_STRICT;
      CP.ops.insert(CP.ops.end(), chains[k].begin(), chains[k].end());
      CP.exprs.push_back(e);
      next = (uint32_t)CP.exprs.size() - 1;
    }
    return next;
  }

 private:
  CondProgram& CP;
  Consts& K;
  std::vector<Token> t_;
  size_t i_ = 0;
  const Token& cur() const { return t_[i_]; }
  const Token& peek(size_t k = 1) const { return t_[std::min(i_ + k, t_.size() - 1)]; }
  static void op(std::vector<uint32_t>& o, uint32_t x, uint32_t y = 0) { o.push_back(x), o.push_back(y); }
  uint32_t field(const std::string& name) {
    for (size_t k = 0; k < CP.fields.size(); ++k)
      if (CP.fields[k] == name) return (uint32_t)k;
    CP.fields.push_back(name);
    return (uint32_t)CP.fields.size() - 1;
  }
  bool name_tok() const { return cur().t == T_ID || cur().t == T_QID; }
  // relative chain inside a multi-select list: fields and indexes only
  std::vector<uint32_t> rel_chain() {
    std::vector<uint32_t> o;
    if (!name_tok()) throw CompileError("JMESPath multi-select item outside the device subset");
    op(o, QO_FIELD, field(cur().s));
    ++i_;
    for (;;) {
      if (cur().t == T_DOT && (peek().t == T_ID || peek().t == T_QID)) {
        op(o, QO_FIELD, field(peek().s));
        i_ += 2;
      } else if (cur().t == T_LBRACK && peek().t == T_NUM && peek(2).t == T_RBRACK) {
        op(o, QO_INDEX, (uint32_t)(int32_t)peek().n);
        i_ += 3;
      } else {
        return o;
      }
    }
  }
  std::vector<uint32_t> chain(bool* plain) {
    std::vector<uint32_t> o;
    // ---- root ----
    if (cur().t == T_RAW || cur().t == T_LIT) {
      op(o, QO_CONST, K.value(cur().lit));
      ++i_;
      *plain = false;
      if (cur().t != T_OR && cur().t != T_EOF) throw CompileError("JMESPath: steps after a literal are not supported");
      return o;
    }
    if (cur().t != T_ID) throw CompileError("JMESPath root outside the device subset");
    const std::string r = cur().s;
    ++i_;
    if (r == "length" && cur().t == T_LPAREN) {  // length(<chain>): a number, no further steps
      ++i_;
      bool pl = true;
      o = chain(&pl);
      if (cur().t != T_RPAREN) throw CompileError("length() argument outside the device subset");
      ++i_;
      op(o, QO_LEN);
      *plain = false;
      return o;
    }
    if (r == "request") {
      if (cur().t != T_DOT || peek().t != T_ID || (peek().s != "object" && peek().s != "operation"))
        throw CompileError("context value request." + (peek().t == T_ID ? peek().s : std::string("?")) +
                           " is not available to device conditions");
      if (peek().s == "object") op(o, QO_OBJ);
      else op(o, QO_CONST, K.scalar(JV::str("CREATE")));  // background scans / CLI: CREATE
      i_ += 2;
    } else if (r == "images") {
      op(o, QO_IMG);  // AddImageInfos (context.go:306-348), built by the flattener
    } else if (r == "element" || r == "elementIndex") {
      op(o, r == "element" ? QO_EL : QO_IDX, 0xFFFFFFFFu);  // the innermost foreach element
    } else if ((r.size() == 8 && !r.compare(0, 7, "element") && r[7] >= '0' && r[7] < '0' + KPE_FE_DEPTH) ||
               (r.size() == 13 && !r.compare(0, 12, "elementIndex") && r[12] >= '0' && r[12] < '0' + KPE_FE_DEPTH)) {
      op(o, r.size() == 8 ? QO_EL : QO_IDX, (uint32_t)(r.back() - '0'));  // element<n>: nesting level n
    } else {
      throw CompileError("context value " + r + " is not available to device conditions");
    }
    // ---- steps ----
    bool proj = false;  // inside a projection (steps apply per element)
    bool keys_open = false;
    for (;;) {
      const Token& t = cur();
      if (keys_open && t.t != T_FLAT) throw CompileError("keys(@) inside a projection must be flattened");
      if (t.t == T_DOT && (peek().t == T_ID || peek().t == T_QID)) {
        if (peek().t == T_ID && peek().s == "keys" && peek(2).t == T_LPAREN) {
          if (peek(3).t != T_CUR || peek(4).t != T_RPAREN) throw CompileError("keys() argument other than @");
          op(o, QO_KEYS);
          *plain = false;
          keys_open = proj;
          i_ += 5;
          continue;
        }
        op(o, QO_FIELD, field(peek().s));
        i_ += 2;
      } else if (t.t == T_LBRACK && peek().t == T_NUM && peek(2).t == T_RBRACK) {
        op(o, QO_INDEX, (uint32_t)(int32_t)peek().n);
        i_ += 3;
      } else if (t.t == T_FLAT) {
        op(o, QO_FLAT);
        *plain = false;
        proj = true, keys_open = false;
        ++i_;
      } else if (t.t == T_DOT && peek().t == T_STAR) {
        // `.*` value projection over an object (go-jmespath ASTValueProjection); nested in
        // another projection it would produce lists per element: not on the device
        if (proj) throw CompileError("`.*` inside a projection is not supported on the device");
        op(o, QO_VALS);
        *plain = false;
        proj = true;
        i_ += 2;
      } else if (t.t == T_LBRACK && peek().t == T_STAR && peek(2).t == T_RBRACK) {
        op(o, QO_STAR);
        *plain = false;
        proj = true;
        i_ += 3;
      } else if (t.t == T_DOT && peek().t == T_LBRACK) {
        if (proj) throw CompileError("multi-select inside a projection is not supported on the device");
        i_ += 2;
        std::vector<std::vector<uint32_t>> items;
        for (;;) {
          items.push_back(rel_chain());
          if (cur().t == T_RBRACK) break;
          if (cur().t != T_COMMA) throw CompileError("JMESPath multi-select outside the device subset");
          ++i_;
        }
        ++i_;
        op(o, QO_MSL | (uint32_t)items.size() << 8);
        for (auto& it : items) {
          op(o, QO_ITEM | (uint32_t)(it.size() / 2) << 8);
          o.insert(o.end(), it.begin(), it.end());
        }
        *plain = false;
      } else {
        break;
      }
    }
    if (keys_open) throw CompileError("keys(@) inside a projection must be flattened");
    return o;
  }
};

// variables.replaceBracesAndTrimSpaces on the text of one {{ }} match
std::string var_text(const std::string& v) {
  std::string s;
  for (size_t i = 0; i < v.size(); ++i) {
    if ((v[i] == '{' || v[i] == '}') && i + 1 < v.size() && v[i + 1] == v[i]) {
      ++i;
      continue;
    }
    s += v[i];
  }
  return pc::trim_ws(s);
}
// regex.RegexVariables `(^|[^\\])(\{\{(?:\{[^{}]*\}|[^{}])*\}\})`: the first match at or after from
bool next_var(const std::string& s, size_t from, size_t* st, size_t* en) {
  for (size_t i = from; i + 1 < s.size(); ++i) {
    if (s[i] != '{' || s[i + 1] != '{') continue;
    if (i > 0 && s[i - 1] == '\\') continue;
    size_t j = i + 2;
    bool ok = false;
    while (j < s.size()) {
      if (s[j] == '}' && j + 1 < s.size() && s[j + 1] == '}') {
        ok = true;
        break;
      }
      if (s[j] == '{') {
        size_t k = j + 1;
        while (k < s.size() && s[k] != '{' && s[k] != '}') ++k;
        if (k >= s.size() || s[k] != '}') break;
        j = k + 1;
        continue;
      }
      if (s[j] == '}') break;
      ++j;
    }
    if (ok) {
      *st = i, *en = j + 2;
      return true;
    }
  }
  return false;
}

class CondCompiler {
 public:
  explicit CondCompiler(CondProgram& cp) : CP(cp), K(cp), Q(cp, K) {}
  std::function<uint32_t(const std::string&)> range_leaf;  // string-pattern leaf of the pattern program

  // a condition key / value after substitution
  uint32_t tmpl(const JV& v, int depth = 0) {
    KpeVTmpl t{};
    if (v.t == JV::Str) {
      if (v.s.find("$(") != std::string::npos) throw CompileError("$(...) references in conditions are not supported");
      size_t st, en;
      if (!next_var(v.s, 0, &st, &en)) {
        if (v.s.find("\\{{") != std::string::npos) throw CompileError("escaped variables in conditions");
        t.kind = VT_CONST, t.a = K.scalar(v);
      } else if (st == 0 && en == v.s.size()) {  // the whole string: the value keeps its JSON type
        const std::string q = var_text(v.s);
        if (q == "@" || q.find("{{") != std::string::npos) throw CompileError("{{@}} / nested variables");
        t.kind = VT_QUERY, t.a = Q.compile(q);
      } else {  // variables inside a string (vars.go:311-389): text and variable pieces
        // list elements are substituted one after another into the side's lane text slot
        // (condvm.inl value(): KPE_TXT_CAP bytes together, else the cell is undecided)
        if (v.s.find("\\{{") != std::string::npos) throw CompileError("escaped variables in conditions");
        t.kind = VT_TMPL, t.a = (uint32_t)CP.tpieces.size() / 2;
        auto text = [&](size_t b, size_t e) {
          if (e <= b) return;
          const std::string piece = v.s.substr(b, e - b);
          if (piece.find("{{") != std::string::npos || piece.find("}}") != std::string::npos)
            throw CompileError("nested variables in conditions");  // vars.go substitutes the result again
          CP.tpieces.push_back(PT_TEXT | (uint32_t)(e - b) << 1);
          CP.tpieces.push_back((uint32_t)CP.ctext.size());
          CP.ctext.insert(CP.ctext.end(), v.s.begin() + b, v.s.begin() + e);
        };
        size_t pos = 0;
        while (next_var(v.s, pos, &st, &en)) {
          text(pos, st);
          const std::string q = var_text(v.s.substr(st, en - st));
          if (q == "@" || q.find("{{") != std::string::npos) throw CompileError("{{@}} / nested variables");
          CP.tpieces.push_back(PT_VAR);
          CP.tpieces.push_back(Q.compile(q));
          pos = en;
        }
        text(pos, v.s.size());
        t.b = (uint32_t)CP.tpieces.size() / 2 - t.a;
      }
    } else if (v.t == JV::Arr && depth == 0 && has_var(v)) {
      std::vector<uint32_t> el;
      for (auto& x : v.a) {
        if (x.t == JV::Arr || x.t == JV::Obj) throw CompileError("nested lists with variables");
        el.push_back(tmpl(x, 1));
      }
      t.kind = VT_ARRAY, t.a = el.empty() ? 0u : el[0], t.b = (uint32_t)el.size();
      // element templates are contiguous: re-emit them in order
      const uint32_t base = (uint32_t)CP.tmpls.size();
      for (uint32_t k : el) CP.tmpls.push_back(CP.tmpls[k]);
      t.a = base;
    } else if (v.t == JV::Obj) {
      throw CompileError("object condition keys / values are not supported on the device");
    } else {
      t.kind = VT_CONST, t.a = K.value(v);
    }
    CP.tmpls.push_back(t);
    return (uint32_t)CP.tmpls.size() - 1;
  }
  uint32_t condition(const JV& c) {
    if (c.t != JV::Obj) throw CompileError("condition is not an object");
    // CreateOperatorHandler (operator.go:27-67) dispatches on the lower-cased name; the numeric
    // and duration handlers then compare the name as written with the canonical spelling
    // (numeric.go:32-45, duration.go:27-40), so another spelling always gives false
    const std::string opw = sv(c.get("operator"));
    std::string op;
    for (char ch : opw) op += (char)tolower((unsigned char)ch);
    uint32_t o = CO_BAD, aux = 0;
    if (op == "equal" || op == "equals") o = CO_EQ;
    else if (op == "notequal" || op == "notequals") o = CO_NE;
    else if (op == "anyin") o = CO_ANYIN;
    else if (op == "allin") o = CO_ALLIN;
    else if (op == "anynotin") o = CO_ANYNOTIN;
    else if (op == "allnotin") o = CO_ALLNOTIN;
    else if (op == "in") o = CO_IN;
    else if (op == "notin") o = CO_NOTIN;
    static const char* const kNum[4] = {"GreaterThanOrEquals", "GreaterThan", "LessThanOrEquals", "LessThan"};
    for (uint32_t d = 0; d < 2 && o == CO_BAD; ++d)
      for (uint32_t i = 0; i < 4; ++i) {
        const std::string canon = std::string(d ? "Duration" : "") + kNum[i];
        std::string lc;
        for (char ch : canon) lc += (char)tolower((unsigned char)ch);
        if (op == lc) {
          o = d ? CO_DUR : CO_NUM;
          aux = opw == canon ? i : CN_NONE;
          break;
        }
      }
    static const JV null_v;
    const JV* k = c.get("key");
    const JV* v = c.get("value");
    const JV& vv = v ? *v : null_v;
    if (vv.t == JV::Str && o >= CO_ANYIN && o <= CO_ALLNOTIN) {
      size_t st, en;
      if (!next_var(vv.s, 0, &st, &en) && in_range(vv.s)) {
        // an InRange constant value (GetOperatorFromStringPattern): handleRange compares each key
        // as pattern.Validate(key, value); AnyNotIn uses the value with its first `-` as `!-`
        if (!range_leaf) throw CompileError("InRange values of set operators");
        aux = 1u + range_leaf(vv.s);
        std::string nr = vv.s;
        nr.replace(nr.find('-'), 1, "!-");
        range_leaf(nr);  // the next leaf
      }
    }
    KpeCCond cc{o, tmpl(k ? *k : null_v), tmpl(vv), aux};
    CP.conds.push_back(cc);
    return (uint32_t)CP.conds.size() - 1;
  }
  // utils.TransformConditions: a list => the deprecated form; a map => any / all
  uint32_t block(const JV* j) {
    KpeCBlock b{};
    std::vector<KpeCCond> any, all;
    auto collect = [&](const JV& arr, std::vector<KpeCCond>& dst) {
      for (auto& e : arr.a) dst.push_back(CP.conds[condition(e)]);
    };
    if (j && j->t == JV::Arr) {
      collect(*j, all);
    } else if (j && j->t == JV::Obj) {
      const JV* a = j->get("any");
      const JV* l = j->get("all");
      if (a && a->t == JV::Arr) b.flags |= CB_HAS_ANY, collect(*a, any);
      else if (a && a->t != JV::Null) throw CompileError("condition block 'any' is not a list");
      if (l && l->t == JV::Arr) collect(*l, all);
      else if (l && l->t != JV::Null) throw CompileError("condition block 'all' is not a list");
    } else if (j && j->t != JV::Null) {
      throw CompileError("condition block");
    }
    b.c0 = (uint32_t)CP.conds.size();
    b.nany = (uint32_t)any.size(), b.nall = (uint32_t)all.size();
    CP.conds.insert(CP.conds.end(), any.begin(), any.end());
    CP.conds.insert(CP.conds.end(), all.begin(), all.end());
    CP.blocks.push_back(b);
    return (uint32_t)CP.blocks.size() - 1;
  }
  // a foreach list: a query template (the device evaluates it through the condition-value path)
  uint32_t list_query(const std::string& q) {
    KpeVTmpl t{};
    t.kind = VT_QUERY, t.a = Q.compile(q);
    CP.tmpls.push_back(t);
    return (uint32_t)CP.tmpls.size() - 1;
  }

 private:
  CondProgram& CP;
  Consts K;
  QueryParser Q;
  static bool has_var(const JV& v) {
    size_t a, b;
    if (v.t == JV::Str) return next_var(v.s, 0, &a, &b);
    for (auto& x : v.a)
      if (has_var(x)) return true;
    return false;
  }
  // operator.GetOperatorFromStringPattern == InRange (operator/operator.go:7-61)
  static bool in_range(const std::string& s) {
    for (const char* p : {">=", "<=", ">", "<", "!"})
      if (!s.compare(0, strlen(p), p)) return false;
    std::string l, r;
    if (pc::split_range(s, "!-", &l, &r)) return false;
    return pc::split_range(s, "-", &l, &r);
  }
};

}  // namespace cq

class Lowerer {
 public:
  explicit Lowerer(Program& p) : P(p), CC(p.cond) {
    CC.range_leaf = [this](const std::string& text) {
      pc::PatCompiler pcomp(P.pat, [](const std::string&) { return (int32_t)-1; });
      return pcomp.leaf(JV::str(text));
    };
    var_leaf_ = [this](const std::string& s, KpeLeaf& l) { return var_leaf(s, l); };
    key_leaf_ = [this](const std::string& s, KpeLeaf& l) { return var_leaf(s, l, PVF_KEY); };
  }
  // validate.foreach entries of one level (newForEachValidator, validate_resource.go:76-119);
  // nested levels are appended first, so each level's entries are contiguous. Returns the first.
  uint32_t foreach_entries(const JV& arr, uint32_t depth) {
    std::vector<KpeCForeach> fes;
    std::vector<FeReport> reps;
    for (auto& e : arr.a) {
      if (e.t != JV::Obj) throw CompileError("foreach entry is not an object");
      if (nonempty(e.get("context"))) throw CompileError("foreach context entries are not supported on the device");
      KpeCForeach f{};
      FeReport fr;
      f.list = CC.list_query(sv(e.get("list")));
      const JV* fp = e.get("preconditions");
      f.pre = (fp && fp->t != JV::Null) ? CC.block(fp) : CE_NONE;
      if (f.pre != CE_NONE) fr.pre_json = doc_text(*fp);
      const JV* sc = e.get("elementScope");
      f.scope = (sc && sc->t == JV::Bool) ? (sc->b ? 2u : 1u) : 0u;
      auto present = [&](const char* key) { return e.get(key) && e.get(key)->t != JV::Null; };
      if (present("deny")) {
        const JV* dn = e.get("deny");
        f.kind = FE_DENY;
        f.deny = CC.block(dn->t == JV::Obj ? dn->get("conditions") : nullptr);
        if (dn->t == JV::Obj && dn->get("conditions")) {
          fr.deny_json = doc_text(*dn->get("conditions"));
          fr.deny_msgs = cond_msgs(dn->get("conditions"));
        }
      } else if (present("pattern") || present("anyPattern")) {
        f.kind = FE_PAT;
        fe_pat_ = true;
        pc::PatCompiler pcomp(P.pat, [&](const std::string& g) {
          const int32_t id = pred(D_KEY, {g});
          P.preds[id].global_only = true;
          return id;
        });
        pcomp.var_leaf = var_leaf_;
        pcomp.key_leaf = key_leaf_;
        const uint32_t pv0 = (uint32_t)P.pat.vars.size();
        f.a = (uint32_t)(P.pat.roots.size() / 2);
        uint32_t nr = 0, flags = 0;
        if (present("pattern")) {
          pcomp.root(*e.get("pattern"));
          nr = 1;
          fr.pattern_json = doc_text(*e.get("pattern"));
        } else {
          const JV& ap = *e.get("anyPattern");
          flags = PR_ANY;
          fr.any = true;
          fr.pattern_json = doc_text(ap);
          if (ap.t != JV::Arr) {
            flags |= PR_ANY_BAD;
            fr.any_bad_type = json_type_name(ap);
          } else {
            for (auto& x : ap.a) {
              JV g = x;
              to_float(g);  // deserializeAnyPattern's encoding/json round trip
              pcomp.root(g);
              ++nr;
            }
          }
        }
        const uint32_t npv = (uint32_t)P.pat.vars.size() - pv0;
        if (nr > 0xFFFFu || pv0 > 0xFFFFu || npv > 0xFFFFu) throw CompileError("foreach pattern tables too large");
        f.b = nr | flags << 16;
        f.c = pv0 | npv << 16;
        fr.root0 = f.a, fr.nroots = nr;
      } else if (present("foreach")) {
        const JV& nf = *e.get("foreach");
        if (nf.t != JV::Arr) throw CompileError("nested foreach is not a list");
        if (depth + 1 >= KPE_FE_DEPTH) throw CompileError("foreach nested deeper than the device evaluates");
        f.kind = FE_NEST;
        f.a = nf.a.empty() ? 0u : foreach_entries(nf, depth + 1);
        f.b = (uint32_t)nf.a.size();
        fr.nested0 = f.a, fr.nnested = f.b;
      } else {
        f.kind = FE_NONE;  // "invalid validation rule": a nil response
      }
      fr.kind = f.kind;
      fes.push_back(f);
      reps.push_back(std::move(fr));
    }
    const uint32_t f0 = (uint32_t)P.cond.fes.size();
    P.cond.fes.insert(P.cond.fes.end(), fes.begin(), fes.end());
    P.fe_reports.insert(P.fe_reports.end(), std::make_move_iterator(reps.begin()), std::make_move_iterator(reps.end()));
    return f0;
  }
  bool fe_pat_ = false;

  // A pattern string with {{ }} variables (vars.go:311-389 substituteVariablesIfAny): a
  // whole-string variable keeps the value's JSON type (PL_VAR); otherwise the variables'
  // texts are spliced into the string (PL_TMPL: substituteVarInPattern). Each variable is a
  // query of the condition program, resolved per row by kpe_cond_kernel.
  bool var_leaf(const std::string& s, KpeLeaf& l, uint32_t key_flags = 0) {
    if (s.find("$(") != std::string::npos) throw CompileError("$(...) references in patterns are not supported");
    size_t st, en;
    if (!cq::next_var(s, 0, &st, &en)) return false;  // no complete {{ }}: a plain string
    if (s.find("\\{{") != std::string::npos) throw CompileError("escaped variables in patterns are not supported");
    auto slot = [&](const std::string& raw, uint32_t flags) {
      const std::string q = cq::var_text(raw);
      if (q == "@" || q.find("{{") != std::string::npos || q.find("}}") != std::string::npos)
        throw CompileError("{{@}} / nested variables in patterns are not supported");
      KpePVar pv{CC.list_query(q), flags};
      P.pat.vars.push_back(pv);
      return (uint32_t)P.pat.vars.size() - 1;
    };
    if (st == 0 && en == s.size()) {
      l.type = PL_VAR;
      l.c0 = slot(s, key_flags ? key_flags : PVF_WHOLE);
      return true;
    }
    l.type = PL_TMPL;
    l.c0 = (uint32_t)P.pat.tpieces.size() / 2;
    size_t pos = 0;
    auto text = [&](size_t a, size_t b) {
      if (b <= a) return;
      P.pat.tpieces.push_back(PT_TEXT | (uint32_t)(b - a) << 1);
      P.pat.tpieces.push_back((uint32_t)P.pat.ttext.size());
      P.pat.ttext.insert(P.pat.ttext.end(), s.begin() + a, s.begin() + b);
    };
    while (cq::next_var(s, pos, &st, &en)) {
      text(pos, st);
      P.pat.tpieces.push_back(PT_VAR);
      P.pat.tpieces.push_back(slot(s.substr(st, en - st), PVF_TEXT));
      pos = en;
    }
    text(pos, s.size());
    l.nc = (uint32_t)P.pat.tpieces.size() / 2 - l.c0;
    if (l.nc > 8) throw CompileError("pattern string with more than 8 pieces around variables");
    return true;
  }

  static void to_float(JV& v) {
    if (v.t == JV::Num && v.is_int) v.is_int = false, v.n = (double)v.i;
    for (auto& x : v.a) to_float(x);
    for (auto& kv : v.o) to_float(kv.second);
  }
  int32_t pred(uint32_t domain, std::vector<std::string> globs) {
    for (size_t i = 0; i < P.preds.size(); ++i)
      if (P.preds[i].domain == domain && P.preds[i].globs == globs) return (int32_t)i;
    P.preds.push_back({domain, std::move(globs)});
    return (int32_t)P.preds.size() - 1;
  }
  static std::string glob_escape_check(const std::string& lit) {
    if (lit.find('*') != std::string::npos || lit.find('?') != std::string::npos)
      throw CompileError("literal namespace contains wildcard characters");
    return lit;
  }

  void pss_preds() {  // the PSA library's fixed sets (pss_fixed.hpp)
    auto& s = P.pss;
    if (s.apparmor_key >= 0) return;
    s.apparmor_key = pred(D_ANNK, pssfix::kApparmorKey);
    s.apparmor_val_ok = pred(D_ANNV, pssfix::kApparmorOk);
    s.seccomp_pod_key = pred(D_ANNK, pssfix::kSeccompPodKey);
    s.seccomp_ann_ok = pred(D_ANNV, pssfix::kSeccompAnnOk);
    s.caps_baseline_ok = pred(D_CAP, pssfix::kCapsBaselineOk);
    s.cap_nbs = pred(D_CAP, pssfix::kCapNbs);
    s.cap_all = pred(D_CAP, pssfix::kCapAll);
    for (int v = 0; v < 3; ++v) s.sysctl[v] = pred(D_SYSCTL, pssfix::sysctls(v));
  }

  // a predicate read only by a kernel after the scan: its bitset is always written to pbuf
  int32_t gpred(uint32_t domain, std::vector<std::string> globs) {
    for (size_t i = 0; i < P.preds.size(); ++i)
      if (P.preds[i].global_only && P.preds[i].domain == domain && P.preds[i].globs == globs) return (int32_t)i;
    P.preds.push_back({domain, std::move(globs)});
    P.preds.back().global_only = true;
    return (int32_t)P.preds.size() - 1;
  }

  // restrictedField -> XRF_* (the field paths the PSA checks report, digit runs as "*")
  static void restricted_field(const std::string& f, KpeXExcl* x, std::vector<std::string>& ann) {
    static const char* sfx[] = {"securityContext.allowPrivilegeEscalation", "securityContext.capabilities.add",
                                "securityContext.capabilities.drop", "ports[*].hostPort",
                                "securityContext.privileged", "securityContext.procMount",
                                "securityContext.runAsNonRoot", "securityContext.runAsUser",
                                "securityContext.seLinuxOptions.type", "securityContext.seLinuxOptions.user",
                                "securityContext.seLinuxOptions.role", "securityContext.seccompProfile.type",
                                "securityContext.windowsOptions.hostProcess"};
    static const char* ctn[] = {"initContainers", "containers", "ephemeralContainers"};
    // corev1.VolumeSource JSON names by VS_* index
    static const char* vs[] = {"hostPath", "emptyDir", "gcePersistentDisk", "awsElasticBlockStore", "gitRepo",
                               "secret", "nfs", "iscsi", "glusterfs", "persistentVolumeClaim", "rbd",
                               "flexVolume", "cinder", "cephfs", "flocker", "downwardAPI", "fc", "azureFile",
                               "configMap", "vsphereVolume", "quobyte", "azureDisk", "photonPersistentDisk",
                               "projected", "portworxVolume", "scaleIO", "storageos", "csi", "ephemeral"};
    static_assert(sizeof(vs) / sizeof(vs[0]) == KPE_NUM_VOLUME_SOURCES, "volume sources");
    x->rf_kind = XRF_NEVER;
    if (f.empty()) {
      x->rf_kind = XRF_ANY;
      return;
    }
    auto set = [&](uint32_t fc, uint32_t ct) { x->rf_kind = XRF_FIELD, x->rf_key = XKEY(fc, ct); };
    for (uint32_t c = 0; c < 3; ++c)
      for (uint32_t k = 0; k <= XF_WHP; ++k)
        if (f == std::string("spec.") + ctn[c] + "[*]." + sfx[k]) set(k, c);
    for (uint32_t k : {XF_RNR, XF_RAU, XF_SEL_TYPE, XF_SEL_USER, XF_SEL_ROLE, XF_SECCOMP, XF_WHP})
      if (f == std::string("spec.") + sfx[k]) set(k, XT_POD);
    if (f == "spec.hostNetwork") set(XF_HOSTNET, XT_POD);
    if (f == "spec.hostPID") set(XF_HOSTPID, XT_POD);
    if (f == "spec.hostIPC") set(XF_HOSTIPC, XT_POD);
    if (f == "spec.securityContext.sysctls[*].name") set(XF_SYSCTL, XT_POD);
    for (uint32_t v = 0; v < KPE_NUM_VOLUME_SOURCES; ++v)
      if (f == std::string("spec.volumes[*].") + vs[v]) set(XF_VOL + v, XT_POD);
    if (f == "spec.volumes[*].unknown") set(XF_VOL + 31, XT_POD);
    const std::string pre = "metadata.annotations[";
    if (f.size() > pre.size() + 1 && f.compare(0, pre.size(), pre) == 0 && f.back() == ']') {
      x->rf_kind = XRF_ANN;
      x->rf_key = (uint32_t)ann.size();
      ann.push_back(f.substr(pre.size(), f.size() - pre.size() - 1));
    }
  }

  // podSecurity.exclude (pkg/pss/evaluate.go:72-317; exclude.Validate, common_types.go:472-478)
  void pss_exclusions(const JV& ex, uint32_t col, uint32_t cvm, const std::string& rname) {
    KpeXRule xr{};
    xr.col = col, xr.cv_mask = cvm;
    pending_excl_.clear();
    const int64_t last_invalid = excl_list(ex, "rule '" + rname + "'", &xr.excl0, &xr.nexcl, &xr.kx, &pending_excl_);
    if (last_invalid >= 0)
      xr.force = last_invalid == (int64_t)ex.a.size() - 1 ? XR_FORCE_FAIL : XR_FORCE_PASS;
    pssx_fixed_preds();
    P.pssx.rules.push_back(xr);
  }
  // A PolicyException's podSecurity controls on PSS rule col: the rule's KpeXRule (one with no
  // excludes of its own when it has none) also holds the exception's excludes
  void pss_exception(const JV& ex, uint32_t col, uint32_t cvm, const std::string& what) {
    size_t i = 0;
    while (i < P.pssx.rules.size() && P.pssx.rules[i].col != col) ++i;
    if (i == P.pssx.rules.size()) {
      KpeXRule xr{};
      xr.col = col, xr.cv_mask = cvm, xr.excl0 = (uint32_t)P.pssx.excl.size();
      pssx_fixed_preds();
      P.pssx.rules.push_back(xr);
    }
    uint32_t x0, n, kx = 0;
    std::vector<PssExcl> specs;
    const int64_t last_invalid = excl_list(ex, what, &x0, &n, &kx, &specs);
    KpeXRule& xr = P.pssx.rules[i];
    P.reports[col].pss_excl = true;  // fail messages are the checks after the exception's excludes
    P.reports[col].pss_xexcludes = std::move(specs);
    P.reports[col].pss_has_xexcl = true;
    if (n > 0xFFFFFFu) throw CompileError(what + ": too many podSecurity controls");
    xr.kx |= kx, xr.xexcl0 = x0;
    xr.xn = n | (last_invalid < 0 ? XR_FORCE_NONE
                 : last_invalid == (int64_t)ex.a.size() - 1 ? XR_FORCE_FAIL : XR_FORCE_PASS) << 24;
  }
  // The compiled KpeXExcl entries of one podSecurity exclude list (rule or PolicyException);
  // returns the index of the last invalid entry (Validate: restrictedField and values go
  // together), or -1
  int64_t excl_list(const JV& ex, const std::string& who, uint32_t* x0, uint32_t* n, uint32_t* kx,
                    std::vector<PssExcl>* specs) {
    static const std::map<std::string, uint32_t> controls = {  // pkg/pss/utils/mapping.go:45-107
        {"Capabilities", (1u << CK_CAPS_BASELINE) | (1u << CK_CAPS_RESTRICTED)},
        {"Seccomp", (1u << CK_SECCOMP_BASELINE) | (1u << CK_SECCOMP_RESTRICTED)},
        {"Privileged Containers", 1u << CK_PRIVILEGED},
        {"Host Ports", 1u << CK_HOST_PORTS},
        {"/proc Mount Type", 1u << CK_PROC_MOUNT},
        {"HostProcess", 1u << CK_WIN_HOST_PROCESS},
        {"SELinux", 1u << CK_SELINUX},
        {"Host Namespaces", 1u << CK_HOST_NS},
        {"HostPath Volumes", 1u << CK_HOST_PATH},
        {"Sysctls", 1u << CK_SYSCTLS},
        {"AppArmor", 1u << CK_APPARMOR},
        {"Privilege Escalation", 1u << CK_APE},
        {"Running as Non-root", 1u << CK_RUN_AS_NON_ROOT},
        {"Running as Non-root user", 1u << CK_RUN_AS_USER},
        {"Volume Types", 1u << CK_RESTRICTED_VOLUMES},
    };
    auto strs = [&](const JV* j, const char* what) {
      std::vector<std::string> out;
      if (!j || j->t == JV::Null) return out;
      if (j->t != JV::Arr) throw CompileError(who + ": podSecurity.exclude " + what + " is not a list");
      for (auto& e : j->a) {
        if (e.t != JV::Str) throw CompileError(who + ": podSecurity.exclude " + what + " entry");
        out.push_back(e.s);
      }
      return out;
    };
    auto str = [&](const JV* j, const char* what) {
      if (!j || j->t == JV::Null) return std::string();
      if (j->t != JV::Str) throw CompileError(who + ": podSecurity.exclude " + what + " is not a string");
      return j->s;
    };
    *x0 = (uint32_t)P.pssx.excl.size(), *n = (uint32_t)ex.a.size();
    int64_t last_invalid = -1;
    for (size_t i = 0; i < ex.a.size(); ++i) {
      const JV& e = ex.a[i];
      if (e.t != JV::Obj) throw CompileError(who + ": podSecurity.exclude entry is not an object");
      const std::string cn = str(e.get("controlName"), "controlName");
      const std::vector<std::string> images = strs(e.get("images"), "images");
      const std::string rf = str(e.get("restrictedField"), "restrictedField");
      const std::vector<std::string> values = strs(e.get("values"), "values");
      specs->push_back(PssExcl{cn, images, rf, values});
      if ((!rf.empty() && values.empty()) || (rf.empty() && !values.empty())) last_invalid = (int64_t)i;
      KpeXExcl x{};
      auto it = controls.find(cn);
      x.checks = it == controls.end() ? 0u : it->second;
      x.img = images.empty() ? -1 : gpred(D_IMAGE, images);
      restricted_field(rf, &x, P.pssx.rf_ann);
      x.has_values = values.empty() ? 0u : 1u;
      x.pv_misc = x.pv_annv = x.pv_sys = x.pv_cap = -1;
      if (!values.empty()) {
        auto any = [&](const char* s) {
          for (auto& v : values)
            if (glob_host(v, s)) return true;
          return false;
        };
        x.vconst = (any("true") ? XV_TRUE : 0u) | (any("false") ? XV_FALSE : 0u) | (any("0") ? XV_ZERO : 0u);
        x.pv_misc = gpred(D_MISC, values);
        x.pv_annv = gpred(D_ANNV, values);
        x.pv_sys = gpred(D_SYSCTL, values);
        x.pv_cap = gpred(D_CAP, values);
      }
      *kx |= x.checks;
      P.pssx.excl.push_back(x);
    }
    return last_invalid;
  }
  void pssx_fixed_preds() {
    if (P.pssx.rules.empty()) {  // fixed PSA predicates, read from pbuf by kpe_pssx_kernel
      auto& g = P.pssx_preds;
      g[0] = gpred(D_ANNK, pssfix::kApparmorKey);
      g[1] = gpred(D_ANNV, pssfix::kApparmorOk);
      g[2] = gpred(D_ANNV, pssfix::kSeccompAnnOk);
      g[3] = gpred(D_CAP, pssfix::kCapsBaselineOk);
      g[4] = gpred(D_CAP, pssfix::kCapNbs);
      g[5] = gpred(D_CAP, pssfix::kCapAll);
      for (int v = 0; v < 3; ++v) g[6 + v] = gpred(D_SYSCTL, P.preds[P.pss.sysctl[v]].globs);
    }
  }

  uint32_t term(const KpeTerm& t) {  // distinct terms are evaluated once per resource
    for (size_t i = 0; i < P.terms.size(); ++i) {
      const KpeTerm& u = P.terms[i];
      if (u.type == t.type && u.a == t.a && u.b == t.b && u.pad == t.pad) return (uint32_t)i;
    }
    P.terms.push_back(t);
    return (uint32_t)P.terms.size() - 1;
  }

  // one filter block -> terms; returns filter index
  // exc: a PolicyException filter (pkg/utils/match/match.go:76-193 checkResourceFilter): no
  // operations term, and userInfo is checked against the (empty) background admission info
  uint32_t filter(const JV* rd, bool has_userinfo, bool is_exclude, bool exc = false) {
    KpeFilter f{(uint32_t)P.fterms.size(), 0};
    auto push = [&](KpeTerm t) {
      P.fterms.push_back(term(t));
      f.nt++;
    };
    // ResourceDescription{} DeepEqual: a present selector pointer is never zero, even `{}`
    auto sel_obj = [&](const char* k) {
      const JV* x = rd ? rd->get(k) : nullptr;
      return x && x->t == JV::Obj;
    };
    bool rd_empty = !nonempty(rd) && !sel_obj("selector") && !sel_obj("namespaceSelector");
    if (exc) {
      // "statement cannot be empty"; roles / clusterRoles / subjects never match the empty
      // admission info of a background scan (checkUserInfo, match.go:105-126)
      if (rd_empty || has_userinfo) push({T_FALSE, 0, 0, 0});
    } else if (!is_exclude) {
      // userInfo is cleared for empty admission info (utils/match.go:263-265)
      if (rd_empty) push({T_FALSE, 0, 0, 0});  // "match cannot be empty"
    } else {
      if (rd_empty && !has_userinfo) push({T_FALSE, 0, 0, 0});  // filter never excludes
      if (has_userinfo) push({T_FALSE, 0, 0, 0});  // empty admission info never satisfies userInfo
    }
    if (!rd_empty) {
      auto ops = svl(rd->get("operations"));
      if (!exc && !ops.empty() && std::find(ops.begin(), ops.end(), "CREATE") == ops.end()) push({T_FALSE, 0, 0, 0});
      auto kinds = svl(rd->get("kinds"));
      if (!kinds.empty()) {
        // CheckKind (pkg/utils/match/kind.go:14-26): OR over selectors of
        // glob(g)&&glob(v)&&glob(k)&&glob(sub,""). Selectors whose group and
        // version are "*" fold into one predicate over the kind dictionary.
        std::vector<KindSel> sels;
        for (auto& k : kinds) sels.push_back(parse_kind_selector(k));
        bool kind_only = true;
        std::vector<std::string> kpats;
        for (auto& s : sels) {
          if (!glob_host(s.sub, "")) continue;  // never matches a scan (no subresource)
          if (s.g != "*" || s.v != "*") kind_only = false;
          kpats.push_back(s.k);
        }
        if (kpats.empty()) {
          push({T_FALSE, 0, 0, 0});
        } else if (kind_only) {
          push({T_KIND_PRED, (uint32_t)pred(D_KIND, kpats), 0, 0});
        } else {
          std::vector<KpeKindSel> run;
          for (auto& s : sels) {
            KpeKindSel ks{};
            ks.pg = s.g == "*" ? -1 : pred(D_GROUP, {s.g});
            ks.pv = s.v == "*" ? -1 : pred(D_VERSION, {s.v});
            ks.pk = s.k == "*" ? -1 : pred(D_KIND, {s.k});
            ks.sub_ok = glob_host(s.sub, "") ? 1u : 0u;
            run.push_back(ks);
          }
          // an identical selector list already in the table is reused, so filters with the same
          // kinds share one term (C3's 200 policies draw their kinds from 15 lists)
          auto same = [](const KpeKindSel& x, const KpeKindSel& y) {
            return x.pg == y.pg && x.pv == y.pv && x.pk == y.pk && x.sub_ok == y.sub_ok;
          };
          uint32_t k0 = (uint32_t)P.kindsels.size();
          for (size_t i = 0; i + run.size() <= P.kindsels.size(); ++i) {
            size_t j = 0;
            while (j < run.size() && same(P.kindsels[i + j], run[j])) ++j;
            if (j == run.size()) {
              k0 = (uint32_t)i;
              break;
            }
          }
          if (k0 == (uint32_t)P.kindsels.size()) P.kindsels.insert(P.kindsels.end(), run.begin(), run.end());
          push({T_KINDS, k0, (uint32_t)run.size(), 0});
        }
      }
      std::string name = sv(rd->get("name"));
      if (!name.empty()) push({T_PRED, (uint32_t)pred(D_NAME, {name}), COL_NAME, 0});
      auto names = svl(rd->get("names"));
      if (!names.empty()) push({T_PRED, (uint32_t)pred(D_NAME, names), COL_NAME, 0});
      auto nss = svl(rd->get("namespaces"));
      if (!nss.empty()) push({T_PRED, (uint32_t)pred(D_NS, nss), COL_MNS, 0});
      const JV* ann = rd->get("annotations");
      if (ann && ann->t == JV::Obj && !ann->o.empty()) {
        uint32_t a0 = (uint32_t)P.annpairs.size();
        for (auto& kv : ann->o) P.annpairs.push_back({pred(D_ANNK, {kv.first}), pred(D_ANNV, {sv(&kv.second)})});
        push({T_ANNOTATIONS, a0, (uint32_t)ann->o.size(), 0});
      }
      const JV* sel = rd->get("selector");
      if (sel && sel->t != JV::Null) selector(sel, false, false, push);
      const JV* nsel = rd->get("namespaceSelector");
      if (nsel && nsel->t != JV::Null) {
        bool star = std::find(kinds.begin(), kinds.end(), "*") != kinds.end();
        sel_exc_ = exc;
        selector(nsel, true, star, push);
        sel_exc_ = false;
      }
    }
    // a term list equal to one already in the table is shared (smaller LDS tables for the scan:
    // C3's 482 filters hold 189 distinct lists)
    for (uint32_t o = 0; o + f.nt <= f.t0; ++o)
      if (std::equal(P.fterms.begin() + f.t0, P.fterms.begin() + f.t0 + f.nt, P.fterms.begin() + o)) {
        P.fterms.resize(f.t0);
        f.t0 = o;
        break;
      }
    P.filters.push_back(f);
    return (uint32_t)P.filters.size() - 1;
  }
  int32_t special_pred(uint32_t domain, uint32_t special) {
    for (size_t i = 0; i < P.preds.size(); ++i)
      if (P.preds[i].domain == domain && P.preds[i].special == special) return (int32_t)i;
    P.preds.push_back({domain, {}, special});
    return (int32_t)P.preds.size() - 1;
  }
  // CheckSelector (pkg/utils/match/labels.go:9-24): ReplaceInSelector then
  // metav1.LabelSelectorAsSelector + Matches. A selector that fails to build is a
  // non-match ("failed to parse selector", pkg/engine/utils/match.go:114-123).
  template <class Push>
  void selector(const JV* sel, bool ns_sel, bool star_kind, Push&& push) {
    if (sel->t != JV::Obj) throw std::invalid_argument("label selector must be an object");
    const JV* ml = sel->get("matchLabels");
    const JV* me = sel->get("matchExpressions");
    if (ml && ml->t != JV::Null && ml->t != JV::Obj) throw std::invalid_argument("matchLabels must be an object");
    if (me && me->t != JV::Null && me->t != JV::Arr) throw std::invalid_argument("matchExpressions must be a list");
    const size_t nml = ml && ml->t == JV::Obj ? ml->o.size() : 0, nme = me && me->t == JV::Arr ? me->a.size() : 0;
    KpeSelector S{};
    S.req0 = (uint32_t)P.selreqs.size();
    S.p_kind_ns = S.p_kind_empty = -1;
    if (ns_sel) {
      S.p_kind_ns = pred(D_KIND, {"Namespace"});
      S.p_kind_empty = pred(D_KIND, {""});
      S.star_kind = star_kind ? 1u : 0u;
      S.exc = sel_exc_ ? 1u : 0u;
    }
    bool invalid = false;
    std::vector<KpeSelReq> reqs;
    if (nml) {
      // Wildcard keys can make two entries resolve to the same key; the result
      // then depends on Go map iteration order in the reference. Refuse those.
      std::vector<std::string> keys;
      for (auto& kv : ml->o) keys.push_back(kv.first);
      for (size_t i = 0; i < keys.size(); ++i) {
        if (!has_wildcard(keys[i])) continue;
        std::string rk = keys[i];
        for (auto& c : rk)
          if (c == '*' || c == '?') c = '0';
        for (size_t j = 0; j < keys.size(); ++j)
          if (j != i && (has_wildcard(keys[j]) || glob_host(keys[i], keys[j]) || rk == keys[j]))
            throw CompileError("label selector with colliding wildcard keys (order-dependent in the reference)");
      }
      for (auto& kv : ml->o) {
        if (kv.second.t != JV::Str) throw std::invalid_argument("matchLabels values must be strings");
        const std::string& k = kv.first;
        const std::string& v = kv.second.s;
        KpeSelReq q{};
        q.pk_ok = q.pv_ok = -1;
        if (has_wildcard(k) || has_wildcard(v)) {
          q.op = SR_WILD;
          q.pk = pred(D_LABK, {k});
          q.pv = pred(D_LABV, {v});
          q.pk_ok = special_pred(D_LABK, PRED_SPECIAL_QNAME);
          q.pv_ok = special_pred(D_LABV, PRED_SPECIAL_LABVAL);
        } else {
          if (!qualified_name_ok(k) || !label_value_ok(v)) invalid = true;
          q.op = SR_EQ;
          q.pk = pred(D_LABK, {k});
          q.pv = pred(D_LABV, {v});
        }
        reqs.push_back(q);
      }
    }
    for (size_t i = 0; i < nme; ++i) {
      const JV& e = me->a[i];
      std::string key = sv(e.get("key")), op = sv(e.get("operator"));
      auto vals = svl(e.get("values"));
      KpeSelReq q{};
      q.pk_ok = q.pv_ok = -1;
      if (!qualified_name_ok(key)) invalid = true;
      if (op == "In" || op == "NotIn") {
        if (vals.empty()) invalid = true;
        q.op = op == "In" ? SR_IN : SR_NOTIN;
      } else if (op == "Exists" || op == "DoesNotExist") {
        if (!vals.empty()) invalid = true;
        q.op = op == "Exists" ? SR_EXISTS : SR_NOTEXIST;
      } else {
        invalid = true;
      }
      for (auto& v : vals)
        if (!label_value_ok(v)) invalid = true;
      if (invalid) break;
      q.pk = pred(D_LABK, {key});
      q.pv = vals.empty() ? -1 : pred(D_LABV, vals);  // valid values hold no '*'/'?': exact patterns
      reqs.push_back(q);
    }
    if (invalid) {
      // A label selector that never builds is constant false. A namespaceSelector
      // is still skipped for an empty kind without "*" kinds (match.go:125-138).
      if (!ns_sel) {
        push({T_FALSE, 0, 0, 0});
        return;
      }
      S.invalid = 1;
      reqs.clear();
    }
    if (reqs.empty() && !ns_sel && !S.invalid) return;  // labels.Everything()
    S.nreq = (uint32_t)reqs.size();
    P.selreqs.insert(P.selreqs.end(), reqs.begin(), reqs.end());
    P.selectors.push_back(S);
    push({ns_sel ? T_NSSELECTOR : T_SELECTOR, (uint32_t)P.selectors.size() - 1, 0, 0});
  }

  static bool has_ui(const JV* f) {
    if (!f) return false;
    for (const char* k : {"roles", "clusterRoles", "subjects"})
      if (nonempty(f->get(k))) return true;
    return false;
  }
  void block(const JV* blk, bool is_exclude, uint32_t* mode, uint32_t* f0, uint32_t* nf) {
    *f0 = (uint32_t)P.filters.size();
    const JV* any = blk ? blk->get("any") : nullptr;
    const JV* all = blk ? blk->get("all") : nullptr;
    if (any && any->t == JV::Arr && !any->a.empty()) {
      *mode = MODE_ANY;
      for (auto& f : any->a) filter(f.get("resources"), has_ui(&f), is_exclude);
    } else if (all && all->t == JV::Arr && !all->a.empty()) {
      *mode = MODE_ALL;
      for (auto& f : all->a) filter(f.get("resources"), has_ui(&f), is_exclude);
    } else {
      *mode = MODE_LEGACY;
      filter(blk ? blk->get("resources") : nullptr, has_ui(blk), is_exclude);
    }
    *nf = (uint32_t)P.filters.size() - *f0;
  }

  static uint32_t cv_mask(const std::string& level, const std::string& version, bool* ok) {
    // pss.ParseVersion + evaluatePSS version selection, folded at compile time.
    bool latest = version.empty() || version == "latest";
    int minor = 0;
    *ok = true;
    if (!latest) {
      if (version.size() < 4 || version.compare(0, 3, "v1.") != 0) *ok = false;
      std::string mi = *ok ? version.substr(3) : "";
      if (mi.empty() || mi.size() > 9 || (mi.size() > 1 && mi[0] == '0')) *ok = false;
      for (char ch : mi)
        if (ch < '0' || ch > '9') *ok = false;
      if (!*ok) return 0;
      minor = atoi(mi.c_str());
    }
    bool baseline = level == "baseline";
    struct VC {
      int check;
      bool restricted;
      std::vector<std::pair<int, int>> versions;  // (minor, cv)
    };
    static const std::vector<VC> table = {
        {CK_APE, true, {{8, CV_APE_1_8}, {25, CV_APE_1_25}}},
        {CK_APPARMOR, false, {{0, CV_APPARMOR_1_0}}},
        {CK_CAPS_BASELINE, false, {{0, CV_CAPS_BASELINE_1_0}}},
        {CK_CAPS_RESTRICTED, true, {{22, CV_CAPS_RESTRICTED_1_22}, {25, CV_CAPS_RESTRICTED_1_25}}},
        {CK_HOST_NS, false, {{0, CV_HOST_NS_1_0}}},
        {CK_HOST_PATH, false, {{0, CV_HOST_PATH_1_0}}},
        {CK_HOST_PORTS, false, {{0, CV_HOST_PORTS_1_0}}},
        {CK_PRIVILEGED, false, {{0, CV_PRIVILEGED_1_0}}},
        {CK_PROC_MOUNT, false, {{0, CV_PROC_MOUNT_1_0}}},
        {CK_RESTRICTED_VOLUMES, true, {{0, CV_RESTRICTED_VOLUMES_1_0}}},
        {CK_RUN_AS_NON_ROOT, true, {{0, CV_RUN_AS_NON_ROOT_1_0}}},
        {CK_RUN_AS_USER, true, {{23, CV_RUN_AS_USER_1_23}}},
        {CK_SELINUX, false, {{0, CV_SELINUX_1_0}}},
        {CK_SECCOMP_BASELINE, false, {{0, CV_SECCOMP_BASELINE_1_0}, {19, CV_SECCOMP_BASELINE_1_19}}},
        {CK_SECCOMP_RESTRICTED, true, {{19, CV_SECCOMP_RESTRICTED_1_19}, {25, CV_SECCOMP_RESTRICTED_1_25}}},
        {CK_SYSCTLS, false, {{0, CV_SYSCTLS_1_0}, {27, CV_SYSCTLS_1_27}, {29, CV_SYSCTLS_1_29}}},
        {CK_WIN_HOST_PROCESS, false, {{0, CV_WIN_HOST_PROCESS_1_0}}},
    };
    uint32_t m = 0;
    for (auto& c : table) {
      if (baseline && c.restricted) continue;  // level "privileged"/other: every check runs
      if (latest) {
        m |= 1u << c.versions.back().second;  // newest MinimumVersion
      } else {
        for (auto& v : c.versions)
          if (v.first <= minor) m |= 1u << v.second;
      }
    }
    return m;
  }

  void rule(const JV& r, uint32_t policy, bool apply_one, const std::string& pol_name, bool namespaced,
            const std::string& pol_ns) {
    KpeRule k{};
    k.policy = policy;
    k.apply_one = apply_one ? 1u : 0u;
    k.pol_term = -1;
    block(r.get("match"), false, &k.match_mode, &k.match_f0, &k.match_nf);
    block(r.get("exclude"), true, &k.excl_mode, &k.excl_f0, &k.excl_nf);
    if (namespaced || !pol_ns.empty()) {
      if (namespaced && pol_ns.empty()) {  // checkNamespacedPolicy can never pass
        k.match_f0 = (uint32_t)P.filters.size();
        P.filters.push_back({(uint32_t)P.fterms.size(), 1});
        P.fterms.push_back(term({T_FALSE, 0, 0, 0}));
        k.match_nf = 1;
        k.match_mode = MODE_LEGACY;
      } else {
        k.pol_term = (int32_t)term({T_PRED, (uint32_t)pred(D_NS, {glob_escape_check(pol_ns)}), COL_NSA, 0});
      }
    }
    const JV* v = r.get("validate");
    bool has_validate = nonempty(v);
    const JV* ps = v ? v->get("podSecurity") : nullptr;
    std::string rname = sv(r.get("name"));
    // preconditions (engine.go:278-285): folded at compile time, else evaluated per resource by
    // kpe_cond_kernel
    Fold pre = F_TRUE;
    uint32_t pre_block = CE_NONE;
    const JV* pre_raw = r.get("preconditions");  // any non-null block is evaluated (utils.go:78-95)
    if (has_validate && nonempty(r.get("context")))
      throw CompileError("rule '" + rname + "': context entries are not supported on the device");
    if (has_validate && pre_raw && pre_raw->t != JV::Null) {
      pre = fold_conditions(pre_raw);
      if (pre == F_NO) {
        try {
          pre_block = CC.block(pre_raw);
        } catch (const CompileError& e) {
          throw CompileError("rule '" + rname + "': preconditions: " + e.what());
        }
      }
    }
    KpeCRule crule{(uint32_t)P.rules.size(), pre_block, CR_PRE_ONLY, CE_NONE, 0, 0, 0, 0, CE_NONE, 0};
    crule.pv0 = (uint32_t)P.pat.vars.size();
    bool pss_excl = false, msg_pattern = false, pat_may_skip = true;
    struct { bool on, any; uint32_t roots; } pat_report{false, false, 0u};
    if (!has_validate) {
      k.handler = H_NONE;  // mutate/generate/verifyImages-only rules give no validate response
      if (nonempty(r.get("verifyImages"))) throw CompileError("rule '" + rname + "': verifyImages is not supported");
    } else if (nonempty(v->get("manifests"))) {
      throw CompileError("rule '" + rname + "': validate.manifests is not supported");
    } else if (ps && ps->t == JV::Obj && nonempty(ps)) {
      bool ok;
      k.cv_mask = cv_mask(sv(ps->get("level")), sv(ps->get("version")), &ok);
      k.handler = ok ? H_PSS : H_ERROR;
      pss_preds();
      const JV* ex = ps->get("exclude");
      if (ok && ex && ex->t != JV::Null) {
        if (ex->t != JV::Arr) throw CompileError("rule '" + rname + "': podSecurity.exclude is not a list");
        if (!ex->a.empty()) {
          pss_excl = true;
          pss_exclusions(*ex, (uint32_t)P.rules.size(), k.cv_mask, rname);
        }
      }
      P.any_pss = true;
      P.cv_union |= k.cv_mask;
      auto it = std::find(P.cv_classes.begin(), P.cv_classes.end(), k.cv_mask);
      k.cv_class = (uint32_t)(it - P.cv_classes.begin());
      if (it == P.cv_classes.end()) P.cv_classes.push_back(k.cv_mask);
    } else {
      // validate_resource.go:121-170: deny, then pattern / anyPattern, then foreach
      auto present = [&](const char* key) { return v->get(key) && v->get(key)->t != JV::Null; };
      if (present("deny")) {
        // validateDeny (validate_resource.go:268-279): conditions true => fail, else pass
        const JV* d = v->get("deny");
        if (d->t != JV::Obj) throw CompileError("rule '" + rname + "': validate.deny is not an object");
        const Fold f = fold_conditions(d->get("conditions"));
        if (f != F_NO) {
          k.handler = f == F_TRUE ? H_CONST_FAIL : H_CONST_PASS;
        } else {
          try {
            crule.deny = CC.block(d->get("conditions"));
          } catch (const CompileError& e) {
            throw CompileError("rule '" + rname + "': validate.deny: " + e.what());
          }
          crule.kind = CR_DENY;
          k.handler = H_COND;
        }
      } else if (pre == F_FALSE && (present("pattern") || present("anyPattern"))) {
        k.handler = H_CONST_SKIP;  // patterns are never evaluated
      } else if (present("pattern") || present("anyPattern")) {
        pc::PatCompiler pcomp(P.pat, [&](const std::string& g) {
          const int32_t id = pred(D_KEY, {g});
          P.preds[id].global_only = true;
          return id;
        });
        pcomp.var_leaf = var_leaf_;
        pcomp.key_leaf = key_leaf_;
        crule.pv0 = (uint32_t)P.pat.vars.size();
        KpePatRule pr{(uint32_t)P.rules.size(), 0, (uint32_t)(P.pat.roots.size() / 2), 0};
        try {
          if (present("pattern")) {
            msg_pattern = true;
            const JV& pt = *v->get("pattern");
            msg_pattern = !pc::has_vars(pt);  // pass message of a substituted pattern: rendered alike
            pcomp.root(pt);
            pr.nr = 1;
          } else {
            const JV& ap = *v->get("anyPattern");
            pr.flags = PR_ANY;
            if (ap.t != JV::Arr) {
              pr.flags |= PR_ANY_BAD;  // deserializeAnyPattern fails: RuleStatusError
            } else {
              for (auto& e : ap.a) {
                JV f = e;
                to_float(f);  // encoding/json round trip (validate_resource.go:400-416)
                pcomp.root(f);
                ++pr.nr;
              }
            }
          }
        } catch (const CompileError& e) {
          throw CompileError("rule '" + rname + "': " + e.what());
        }
        crule.npv = (uint32_t)P.pat.vars.size() - crule.pv0;
        pr.flags |= PR_NO_MEMO << PR_MEMO_SH;
        if (!crule.npv) {  // equal patterns give equal verdicts on a row: memo candidates
          std::string sig = std::to_string(pr.flags & 0xFFFFu) + "|";
          if (present("pattern")) jv_sig(*v->get("pattern"), sig);
          else jv_sig(*v->get("anyPattern"), sig);
          pat_sigs_.emplace_back((uint32_t)P.pat.rules.size(), std::move(sig));
        }
        if (P.pat.rules.size() >= 65535) throw CompileError("more than 65535 pattern rules in one program");
        P.pat.rules.push_back(pr);
        k.handler = H_PATTERN;
        // a pattern skips only through conditional / global anchors (validate.go: pe.Skip)
        pat_may_skip = present("pattern") ? anchor_skips(*v->get("pattern")) : anchor_skips(*v->get("anyPattern"));
        if (!(pr.flags & PR_ANY_BAD)) pat_report = {true, (pr.flags & PR_ANY) != 0u, pr.nr};
      } else if (v->get("foreach") && v->get("foreach")->t == JV::Arr && !v->get("foreach")->a.empty()) {
        // validateForEach (validate_resource.go:186-254): deny, pattern / anyPattern and nested
        // entries
        crule.kind = CR_FOREACH;
        try {
          crule.fe0 = foreach_entries(*v->get("foreach"), 0);
        } catch (const CompileError& e) {
          throw CompileError("rule '" + rname + "': validate.foreach: " + e.what());
        }
        crule.nfe = (uint32_t)v->get("foreach")->a.size();
        P.any_fe_pat = P.any_fe_pat || fe_pat_;
        k.handler = H_COND;
      } else if (nonempty(v->get("foreach")) || nonempty(v->get("cel"))) {
        throw CompileError("rule '" + rname + "': validate.foreach/cel are not supported on the device yet");
      } else {
        k.handler = H_NONE;  // no podSecurity/cel/pattern/deny/foreach: the validator returns nil
      }
    }
    // invokeRuleHandler (engine.go:278-285) checks preconditions before any handler runs, and
    // every validate rule has one (validation.go:37-53: at least NewValidateResourceHandler,
    // even when its validator then returns nil)
    if (pre == F_FALSE && (k.handler != H_NONE || has_validate)) k.handler = H_CONST_SKIP;
    if (pre_block != CE_NONE && k.handler == H_NONE && has_validate) {
      k.handler = H_COND;  // matched cells need the preconditions' skip / error
      crule.kind = CR_NONE;
    }
    if (k.handler >= H_CONST_SKIP || pre_block != CE_NONE) P.any_const = true;
    RuleReport rr;
    // condition messages (variables/evaluate.go:31-125): the preconditions skip (engine.go:282-284)
    // and getDenyMessage (validate_resource.go:279-300). A block evaluated per resource whose
    // message depends on where it stopped gets a condition trace slot (KpeCRule::mslot).
    const bool is_pss = ps && ps->t == JV::Obj && nonempty(ps);
    if (has_validate && pre_raw && pre_raw->t != JV::Null) {
      rr.pre_msgs = cond_msgs(pre_raw);
      if (pre == F_FALSE) {
        uint32_t as, ls;
        fold_stops(pre_raw, &as, &ls);
        rr.pre_const_skip = true;
        rr.pre_skip_msg = join_non_empty({"preconditions not met", rr.pre_msgs.render(as, ls, false)}, "; ");
      }
      rr.msg_pre_skip = !rr.pre_msgs.has_text();
    }
    if (has_validate && !is_pss && v->get("deny") && v->get("deny")->t == JV::Obj) {
      const JV* m = v->get("message");
      const JV* dc = v->get("deny")->get("conditions");
      rr.msg_deny = true;
      rr.deny_vmsg = (m && m->t == JV::Str) ? m->s : std::string();
      rr.deny_msgs = cond_msgs(dc);
      if (crule.kind != CR_DENY) {  // folded: the message the block gives when it holds
        uint32_t as, ls;
        fold_stops(dc, &as, &ls);
        rr.deny_cm = rr.deny_msgs.render(as, ls, true);
      } else {
        rr.cond_deny = rr.deny_msgs.has_text();
      }
    }
    // a trace slot for every rule whose conditions are evaluated per resource (their messages and
    // RuleError texts depend on where a block stopped or which condition raised the error), four
    // words for foreach rules (schema.h FT_*)
    auto fits = [](const CondMsgs& m) { return m.any.size() <= CT_MAXC && m.all.size() <= CT_MAXC; };
    if ((pre_block != CE_NONE || crule.kind == CR_DENY || crule.kind == CR_FOREACH) && fits(rr.pre_msgs) &&
        fits(rr.deny_msgs)) {
      crule.mslot = P.cond.nmsg + 1u;
      P.cond.nmsg += crule.kind == CR_FOREACH ? KPE_FE_TRACE_WORDS : 1u;
      rr.cond_slot = true;
    }
    if (pre_block != CE_NONE) rr.pre_json = doc_text(*pre_raw);
    if (crule.kind == CR_DENY && v->get("deny")->get("conditions")) rr.deny_json = doc_text(*v->get("deny")->get("conditions"));
    if (crule.kind == CR_FOREACH) {
      rr.foreach = true, rr.fe0 = crule.fe0, rr.nfe = crule.nfe;
      const JV* m = v->get("message");
      rr.vmsg = (m && m->t == JV::Str) ? m->s : std::string();
    }
    rule_info_.push_back({pre_block != CE_NONE, has_validate, rname, k.handler == H_PATTERN && !pat_may_skip});
    if (pre_block != CE_NONE || k.handler == H_COND || crule.npv) P.cond.rules.push_back(crule);
    if (k.apply_one) P.any_apply_one = true;
    P.rules.push_back(k);
    P.rule_names.push_back(pol_name + "/" + rname);
    rr.rule = rname;
    rr.has_validate = has_validate;
    if (ps && ps->t == JV::Obj && nonempty(ps)) {
      rr.pss = true;
      rr.pss_level = sv(ps->get("level"));
      rr.pss_version = sv(ps->get("version"));
    }
    rr.pss_excl = pss_excl;
    rr.pss_cv = k.cv_mask;
    if (pss_excl) rr.pss_excludes = std::move(pending_excl_);
    rr.msg_pattern = msg_pattern;
    if (k.handler == H_PATTERN) {  // RuleError texts of substitutePatterns / deserializeAnyPattern
      const JV* pt = v->get("pattern") && v->get("pattern")->t != JV::Null ? v->get("pattern") : v->get("anyPattern");
      rr.pattern_json = doc_text(*pt);
      rr.pat_vars = crule.npv != 0;
      if (pt == v->get("anyPattern") && pt->t != JV::Arr) rr.any_bad_type = json_type_name(*pt);
      const JV* m = v->get("message");
      rr.vmsg = (m && m->t == JV::Str) ? m->s : std::string();
    }
    if (pat_report.on) {
      rr.pat_rule = true, rr.any_pattern = pat_report.any, rr.pat_roots = pat_report.roots;
      const JV* m = v ? v->get("message") : nullptr;
      rr.vmsg = (m && m->t == JV::Str) ? m->s : std::string();
      rr.vmsg_vars = rr.vmsg.find("{{") != std::string::npos || rr.vmsg.find("$(") != std::string::npos;
    }
    P.reports.push_back(std::move(rr));
  }

 private:
  // PolicyExceptions (api/kyverno/v2beta1/policy_exception_types.go; engine.go:286-293,
  // pkg/engine/utils/exceptions.go:14-47). An exception lists (policy key, rule-name globs)
  // and a match block; a matched cell of such a rule whose preconditions held is RuleSkip when
  // the block holds. The device evaluates the block like a rule's match (KpeRule::exc).
  // An exception's conditions (CheckAnyAllConditions, pkg/utils/conditions/condition.go:14-30)
  // that fold at compile time keep the decision in the scan; conditions that read the resource,
  // and rules whose preconditions read it (preconditions run first, engine.go:278-293), defer it
  // (XE_DEFER): the scan marks a cell whose exception match holds (KPE_XDEFER_ | its verdict
  // without the exception) and kpe_cond_kernel evaluates preconditions, then the exception's
  // conditions (error or false: no exception), then the handler. Refused (KPE_E_UNSUPPORTED):
  // several exceptions on a rule when one has conditions that do not fold to true or podSecurity
  // controls (MatchesException stops at the first matching one, so it decides which applies),
  // and several exceptions that are not all `any` blocks.
 public:
  void exceptions(const JV& root, bool background, const std::vector<std::string>& rule_pol_key) {
    std::vector<const JV*> xs;
    if (root.t == JV::Arr)
      for (auto& e : root.a) xs.push_back(&e);
    else if (root.t != JV::Null)
      xs.push_back(&root);
    struct X {
      const JV* spec;
      std::string key;
      const JV* pss;  // spec.podSecurity when non-empty (HasPodSecurity)
      JV cond;        // spec.conditions, an empty `any` dropped (CheckAnyAllConditions: it holds)
      Fold fold;      // F_TRUE: no conditions, or conditions true for every resource
      std::string name;
    };
    std::vector<X> keep;
    for (const JV* e : xs) {
      if (e->t != JV::Obj) throw std::invalid_argument("PolicyException is not an object");
      const JV* spec = e->get("spec");
      if (!spec || spec->t != JV::Obj) throw std::invalid_argument("PolicyException without spec");
      const JV* meta = e->get("metadata");
      const std::string name = meta ? sv(meta->get("name")) : "", ns = meta ? sv(meta->get("namespace")) : "";
      const std::string key = ns.empty() ? name : ns + "/" + name;
      // background scans only fetch exceptions with background processing enabled
      // (pkg/controllers/report/utils/utils.go:113-124); kyverno apply uses every one given
      const JV* bg = spec->get("background");
      if (background && bg && bg->t == JV::Bool && !bg->b) continue;
      const JV* pss = spec->get("podSecurity");
      if (pss && pss->t != JV::Null && pss->t != JV::Arr)
        throw CompileError("PolicyException " + key + ": podSecurity is not a list");
      if (pss && (pss->t != JV::Arr || pss->a.empty())) pss = nullptr;
      // CheckAnyAllConditions (pkg/utils/conditions/condition.go:14-30): every `all` holds and
      // some `any` holds, or `any` is empty. Only true matters (an error or false both mean no
      // exception, exceptions.go:33-41), and on that the preconditions' evaluation order agrees
      // (variables/evaluate.go:57-100) once an empty `any` list is dropped.
      X x{spec, key, pss, JV(), F_TRUE, name};
      const JV* cond = spec->get("conditions");
      if (cond && cond->t != JV::Null) {
        if (cond->t != JV::Obj) throw CompileError("PolicyException " + key + ": conditions is not an object");
        x.cond = *cond;
        JV* any = x.cond.getm("any");
        if (any && any->t == JV::Arr && any->a.empty()) *any = JV();
        x.fold = fold_conditions(&x.cond);
      }
      keep.push_back(std::move(x));
    }
    for (size_t r = 0; r < P.rules.size(); ++r) {
      std::vector<const JV*> mine;  // match blocks of the exceptions that contain this rule
      std::vector<const X*> mine_x;
      const X* with_pss = nullptr;
      for (auto& x : keep) {
        bool has = false;
        const JV* ex = x.spec->get("exceptions");
        if (ex && ex->t == JV::Arr)
          for (auto& it : ex->a) {  // Exception.Contains: policy key, then rule-name globs
            if (it.t != JV::Obj || sv(it.get("policyName")) != rule_pol_key[r]) continue;
            for (auto& rn : svl(it.get("ruleNames")))
              if (glob_host(rn, rule_info_[r].name)) has = true;
          }
        if (has) mine.push_back(x.spec->get("match")), mine_x.push_back(&x);
        if (has && x.pss) with_pss = &x;
      }
      if (mine.empty()) continue;
      const std::string rname = rule_names_at(r);
      bool dyn_cond = false;
      for (const X* x : mine_x) dyn_cond = dyn_cond || x->fold == F_NO;
      if (mine.size() > 1)
        for (const X* x : mine_x)
          if (x->fold != F_TRUE)
            throw CompileError("rule '" + rname + "': several PolicyExceptions, one with conditions (" + x->key + ")");
      if (mine_x[0]->fold == F_FALSE) continue;  // its conditions never hold: the exception never applies
      // validate_pss.go:45-58: on a podSecurity rule an exception with podSecurity controls does
      // not skip; an unparsable level / version (H_ERROR) errors with or without it
      if (with_pss && P.rules[r].handler == H_ERROR) continue;
      const bool xpss = with_pss && P.rules[r].handler == H_PSS;
      if (xpss && mine.size() > 1)  // MatchesException: the first matching one decides
        throw CompileError("rule '" + rname + "': several PolicyExceptions, one with podSecurity controls");
      const bool defer = rule_info_[r].pre_dyn || dyn_cond;
      if (P.rules[r].handler == H_NONE) {
        if (rule_info_[r].has_validate)
          throw CompileError("rule '" + rname + "': PolicyExceptions on a validate rule without a handler");
        continue;  // no validate handler: the rule gives no response either way
      }
      auto blocks = [&](const JV* m, const char* k) -> const JV* {
        const JV* b = m ? m->get(k) : nullptr;
        return (b && b->t == JV::Arr && !b->a.empty()) ? b : nullptr;
      };
      bool always = false, any_only = true;
      for (const JV* m : mine) {
        if (!blocks(m, "any") && !blocks(m, "all")) always = true;  // CheckMatchesResources: no error
        else if (!blocks(m, "any") && blocks(m, "all")->a.size() > 1) any_only = false;
      }
      uint32_t x = XE_PRESENT;
      const uint32_t f0 = (uint32_t)P.filters.size();
      if (always) {
        x |= XE_ALL;  // no filters: holds
      } else if (mine.size() == 1 && !blocks(mine[0], "any")) {
        x |= XE_ALL;
        for (auto& f : blocks(mine[0], "all")->a) filter(f.get("resources"), has_ui(&f), false, true);
      } else {
        if (!any_only) throw CompileError("rule '" + rname + "': several PolicyExceptions with `all` blocks");
        for (const JV* m : mine) {
          const JV* b = blocks(m, "any") ? blocks(m, "any") : blocks(m, "all");
          for (auto& f : b->a) filter(f.get("resources"), has_ui(&f), false, true);
        }
      }
      const uint32_t nf = (uint32_t)P.filters.size() - f0;
      static_assert(((XE_PRESENT | XE_ALL | XE_PSS | XE_DEFER) & (0xFFu << 20 | 0xFFFFFu)) == 0,
                    "KpeRule::exc fields overlap");
      if (f0 > 0xFFFFFu || nf > 0xFFu) throw CompileError("rule '" + rname + "': too many PolicyException filters");
      if (xpss) {
        x |= XE_PSS;
        pss_exception(*with_pss->pss, (uint32_t)r, P.rules[r].cv_mask, "PolicyException " + with_pss->key);
      }
      if (defer) {  // kpe_cond_kernel decides: the rule's condition record carries the exception
        x |= XE_DEFER;
        uint32_t xb = CE_NONE;
        if (dyn_cond) {
          try {
            xb = CC.block(&mine_x[0]->cond);
          } catch (const CompileError& e) {
            throw CompileError("PolicyException " + mine_x[0]->key + ": conditions: " + e.what());
          }
        }
        KpeCRule* cr = nullptr;
        for (auto& c : P.cond.rules)
          if (c.col == (uint32_t)r) cr = &c;
        if (!cr) {
          P.cond.rules.push_back(KpeCRule{(uint32_t)r, CE_NONE, CR_PRE_ONLY, CE_NONE, 0, 0, 0, 0, CE_NONE, 0});
          cr = &P.cond.rules.back();
        }
        cr->exc = xb;
        cr->xflags = XC_DEFER | (xpss ? XC_PSS : 0u);
        P.any_const = true;
      }
      P.rules[r].exc = x | f0 | nf << 20;
      P.any_exc = true;
      // the report of a skip this exception caused (validate_resource.go:43-55): unambiguous when
      // it is the rule's only exception and no other skip is possible (no resource-reading
      // preconditions; a podSecurity, deny or constant handler, or a pattern without conditional /
      // global anchors: no anchor or foreach skip)
      const uint32_t hd = P.rules[r].handler;
      // (resource-reading preconditions: a skip after they held, which the condition trace shows)
      if (mine.size() == 1 && !xpss && (!rule_info_[r].pre_dyn || P.reports[r].cond_slot) &&
          (hd == H_PSS || hd == H_CONST_PASS || hd == H_CONST_FAIL || P.reports[r].msg_deny ||
           rule_info_[r].pat_noskip)) {
        P.reports[r].exc_key = mine_x[0]->key;
        P.reports[r].exc_name = mine_x[0]->name;
        P.reports[r].exc_after_pre = rule_info_[r].pre_dyn;
      }
    }
  }
  std::string rule_names_at(size_t r) const { return P.rule_names[r]; }
  // memo slots of the pattern rules (KpePatRule::flags >> PR_MEMO_SH): patterns shared by several
  // rules, the most shared first, KPE_PAT_MEMO of them
  void assign_pattern_memo() {
    std::map<std::string, std::vector<uint32_t>> by;
    for (auto& x : pat_sigs_) by[x.second].push_back(x.first);
    std::vector<const std::vector<uint32_t>*> groups;
    for (auto& kv : by)
      if (kv.second.size() > 1) groups.push_back(&kv.second);
    std::stable_sort(groups.begin(), groups.end(), [](auto* x, auto* y) { return x->size() > y->size(); });
    for (size_t g = 0; g < groups.size() && g < KPE_PAT_MEMO; ++g)
      for (uint32_t pi : *groups[g])
        P.pat.rules[pi].flags = (P.pat.rules[pi].flags & 0xFFFFu) | ((uint32_t)g << PR_MEMO_SH);
  }
 private:
  // type-tagged canonical text of a pattern value (members in document order, as compiled)
  static void jv_sig(const JV& v, std::string& o) {
    switch (v.t) {
      case JV::Null: o += 'n'; break;
      case JV::Bool: o += v.b ? 't' : 'f'; break;
      case JV::Num:
        o += v.is_int ? 'i' : 'd';
        o += v.is_int ? std::to_string(v.i) : goval::fmt_E(v.n);
        o += ';';
        break;
      case JV::Str:
        o += 's' + std::to_string(v.s.size()) + ':' + v.s;
        break;
      case JV::Arr:
        o += '[';
        for (auto& x : v.a) jv_sig(x, o);
        o += ']';
        break;
      case JV::Obj:
        o += '{';
        for (auto& kv : v.o) {
          o += std::to_string(kv.first.size()) + ':' + kv.first;
          jv_sig(kv.second, o);
        }
        o += '}';
        break;
    }
  }
  std::vector<std::pair<uint32_t, std::string>> pat_sigs_;

  Program& P;
  cq::CondCompiler CC;
  std::function<bool(const std::string&, KpeLeaf&)> var_leaf_, key_leaf_;
  std::vector<PssExcl> pending_excl_;  // the podSecurity.exclude entries of the rule being lowered
  struct RuleInfo {
    bool pre_dyn, has_validate;
    std::string name;
    bool pat_noskip;  // a pattern rule without conditional / global anchors: it never skips
  };
  // a key with a conditional "(k)" or global "<(k)" anchor anywhere in the pattern
  static bool anchor_skips(const JV& v) {
    if (v.t == JV::Arr) {
      for (auto& e : v.a)
        if (anchor_skips(e)) return true;
    } else if (v.t == JV::Obj) {
      for (auto& kv : v.o)
        if (kv.first.rfind("(", 0) == 0 || kv.first.rfind("<(", 0) == 0 || anchor_skips(kv.second)) return true;
    }
    return false;
  }
  std::vector<RuleInfo> rule_info_;
  bool sel_exc_ = false;
};

}  // namespace

Program::~Program() = default;

std::unique_ptr<Program> compile_policies(const char* json, size_t len, const char* exceptions, size_t exc_len,
                                          bool background) {
  JV root = parse_all(json, len);
  std::vector<const JV*> pols;
  if (root.t == JV::Arr)
    for (auto& p : root.a) pols.push_back(&p);
  else
    pols.push_back(&root);
  auto prog = std::make_unique<Program>();
  Lowerer L(*prog);
  for (size_t pi = 0; pi < pols.size(); ++pi) {
    const JV& p = *pols[pi];
    if (p.t != JV::Obj) throw std::invalid_argument("policy is not an object");
    const JV* meta = p.get("metadata");
    std::string name = meta ? sv(meta->get("name")) : "";
    std::string ns = meta ? sv(meta->get("namespace")) : "";
    bool namespaced = sv(p.get("kind")) == "Policy";
    const JV* spec = p.get("spec");
    bool apply_one = spec && sv(spec->get("applyRules")) == "One";
    const size_t r0 = prog->reports.size();
    for (auto& r : compute_rules(p)) L.rule(r, (uint32_t)pi, apply_one, name, namespaced, ns);
    // results.go:94-108: policy key, scored / category / severity annotations
    const JV* ann = meta ? meta->get("annotations") : nullptr;
    auto annv = [&](const char* k) { return ann ? sv(ann->get(k)) : std::string(); };
    std::string sev = annv("policies.kyverno.io/severity");
    if (sev != "critical" && sev != "high" && sev != "medium" && sev != "low" && sev != "info") sev.clear();
    const std::string vfa = spec ? sv(spec->get("validationFailureAction")) : std::string();
    const JV* ovr = spec ? spec->get("validationFailureActionOverrides") : nullptr;
    for (size_t i = r0; i < prog->reports.size(); ++i) {
      RuleReport& rr = prog->reports[i];
      rr.audit = !(vfa == "Enforce" || vfa == "enforce");
      rr.overrides = ovr && ovr->t == JV::Arr && !ovr->a.empty();
      rr.name_mult = 0;
      for (size_t j = r0; j < prog->reports.size(); ++j)
        if (prog->reports[j].has_validate && prog->reports[j].rule == rr.rule) ++rr.name_mult;
      rr.policy_key = ns.empty() ? name : ns + "/" + name;
      rr.scored = annv("policies.kyverno.io/scored") != "false";
      rr.category = annv("policies.kyverno.io/category");
      rr.severity = sev;
    }
  }
  if (exceptions && exc_len) {
    std::vector<std::string> keys;
    for (auto& rr : prog->reports) keys.push_back(rr.policy_key);
    L.exceptions(parse_all(exceptions, exc_len), background, keys);
  }
  L.assign_pattern_memo();
  return prog;
}

// ---------------------------------------------------------------------------
// variables.SubstituteAll of a rule message (pkg/engine/variables/vars.go:161-167,311-389) on a
// background scan's context, where `request.object` is the resource decoded as
// map[string]interface{} (numbers float64). Restated for `request.object` paths of identifiers,
// quoted identifiers and [N] indexes; anything else (other roots, functions, `@`, `$(...)`
// references, a variable inside a substituted value) returns false and the message is left to the
// Go engine, as does a substitution error (a member missing from an object: the message is then
// empty in the reference too).
namespace {

// encoding/json float64 (encode.go floatEncoder): 'f' with the shortest round-trip digits, 'e'
// below 1e-6 or from 1e21, exponent without leading zeros
void go_json_float(std::string& o, double f) {
  char buf[64];
  const double a = std::fabs(f);
  if (a != 0 && (a < 1e-6 || a >= 1e21)) {
    auto r = std::to_chars(buf, buf + sizeof buf, f, std::chars_format::scientific);
    std::string t(buf, r.ptr);
    const size_t e = t.find('e');
    if (e != std::string::npos && e + 3 < t.size() && t[e + 2] == '0') t.erase(e + 2, 1);  // e-07 -> e-7
    o += t;
    return;
  }
  auto r = std::to_chars(buf, buf + sizeof buf, f, std::chars_format::fixed);
  o.append(buf, r.ptr);
}

// encoding/json string with HTML escaping (encode.go appendString, escapeHTML)
void go_json_str(std::string& o, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  for (size_t i = 0; i < s.size(); ++i) {
    const unsigned char c = (unsigned char)s[i];
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c == '\n') {
      o += "\\n";
    } else if (c == '\r') {
      o += "\\r";
    } else if (c == '\t') {
      o += "\\t";
    } else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      o += "\\u00";
      o += hex[c >> 4];
      o += hex[c & 15];
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

// json.Marshal of a decoded value (maps: sorted keys, the last of duplicate keys)
void go_json(std::string& o, const JV& v) {
  switch (v.t) {
    case JV::Null: o += "null"; break;
    case JV::Bool: o += v.b ? "true" : "false"; break;
    case JV::Num: go_json_float(o, v.is_int ? (double)v.i : v.n); break;
    case JV::Str: go_json_str(o, v.s); break;
    case JV::Arr:
      o += '[';
      for (size_t k = 0; k < v.a.size(); ++k) {
        if (k) o += ',';
        go_json(o, v.a[k]);
      }
      o += ']';
      break;
    case JV::Obj: {
      std::map<std::string, const JV*> m;
      for (auto& kv : v.o) m[kv.first] = &kv.second;
      o += '{';
      bool first = true;
      for (auto& kv : m) {
        if (!first) o += ',';
        first = false;
        go_json_str(o, kv.first);
        o += ':';
        go_json(o, *kv.second);
      }
      o += '}';
      break;
    }
  }
}

// A plain chain of the message context (the queries kpe_cond_kernel marks CE_STRICT): the roots
// request.object (the resource), request.operation ("CREATE", background scans and the CLI),
// element / element<depth> and elementIndex / elementIndex<depth> (the foreach element, when
// given), then identifiers, "quoted" identifiers and [N] (negative from the end). A member
// missing from an object is the kyverno go-jmespath fork's NotFoundError (*missing_key: the
// member; SubstituteAll fails); a member of a non-object or an index past a list is null.
// false: not this grammar (another root, a projection, a function).
bool ctx_path(const std::string& q, const JV& res, const JV* el, const MsgElem* me, JV* scratch, const JV** out,
              std::string* missing_key) {
  missing_key->clear();
  static const JV kNull;
  auto ident0 = [](char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; };
  auto ident1 = [&](char c) { return ident0(c) || (c >= '0' && c <= '9'); };
  auto root_is = [&](const std::string& r) {
    return q.compare(0, r.size(), r) == 0 && (q.size() == r.size() || q[r.size()] == '.' || q[r.size()] == '[');
  };
  const JV* cur = nullptr;
  size_t i = 0;
  if (root_is("request.object")) {
    cur = &res, i = 14;
  } else if (root_is("request.operation")) {
    *scratch = JV::str("CREATE");
    cur = scratch, i = 17;
  } else if (me && el && q.compare(0, 7, "element") == 0) {
    size_t j = 7;
    const bool index = q.compare(0, 12, "elementIndex") == 0;
    if (index) j = 12;
    if (j < q.size() && q[j] >= '0' && q[j] <= '9') {  // element<n>: only the innermost level is kept
      if (q[j] - '0' != me->depth) return false;
      ++j;
    }
    if (j < q.size() && q[j] != '.' && q[j] != '[') return false;
    if (index) {
      JV x;
      x.t = JV::Num, x.is_int = true, x.i = me->index, x.n = (double)me->index;
      *scratch = x;
      cur = scratch;
    } else {
      cur = el;
    }
    i = j;
  } else {
    return false;
  }
  bool missing = false;
  while (i < q.size()) {
    if (q[i] == '.') {
      ++i;
      std::string key;
      if (i < q.size() && q[i] == '"') {
        const size_t e = q.find('"', i + 1);
        if (e == std::string::npos) return false;
        key = q.substr(i + 1, e - i - 1);
        if (key.find('\\') != std::string::npos) return false;
        i = e + 1;
      } else {
        if (i >= q.size() || !ident0(q[i])) return false;
        const size_t b = i;
        while (i < q.size() && ident1(q[i])) ++i;
        key = q.substr(b, i - b);
      }
      const JV* nx = cur && cur->t == JV::Obj ? cur->get(key.c_str()) : nullptr;
      if (cur && cur->t == JV::Obj && !nx && !missing) missing = true, *missing_key = key;
      cur = nx;
    } else if (q[i] == '[') {
      size_t e = q.find(']', i);
      if (e == std::string::npos) return false;
      const std::string num = q.substr(i + 1, e - i - 1);
      if (num.empty() || num.size() > 9) return false;
      size_t d = num[0] == '-' ? 1 : 0;
      if (d == num.size()) return false;
      for (size_t k = d; k < num.size(); ++k)
        if (num[k] < '0' || num[k] > '9') return false;
      long idx = std::stol(num);
      if (cur && cur->t == JV::Arr) {
        if (idx < 0) idx += (long)cur->a.size();
        cur = idx >= 0 && idx < (long)cur->a.size() ? &cur->a[(size_t)idx] : nullptr;
      } else {
        cur = nullptr;
      }
      i = e + 1;
    } else {
      return false;
    }
  }
  *out = cur ? cur : &kNull;
  return true;
}
bool object_path(const std::string& q, const JV& res, const JV** out, bool* missing) {
  JV scratch;
  std::string mk;
  if (q.compare(0, 14, "request.object") != 0) return false;
  const bool ok = ctx_path(q, res, nullptr, nullptr, &scratch, out, &mk);
  *missing = !mk.empty();
  return ok;
}

// the end of the variable starting at s[i] == '{' s[i+1] == '{' (RegexVariables: `{...}` groups
// or non-brace bytes, then "}}"); npos: none
size_t var_end(const std::string& s, size_t i) {
  size_t j = i + 2;
  while (j < s.size()) {
    if (s[j] == '}') return j + 1 < s.size() && s[j + 1] == '}' ? j + 2 : std::string::npos;
    if (s[j] == '{') {
      const size_t e = s.find_first_of("{}", j + 1);
      if (e == std::string::npos || s[e] != '}') return std::string::npos;
      j = e + 1;
      continue;
    }
    ++j;
  }
  return std::string::npos;
}

}  // namespace

bool go_wildcard(const std::string& pattern, const std::string& s) { return glob_host(pattern, s); }

std::string join_non_empty(const std::vector<std::string>& v, const std::string& sep) {
  std::string o;
  for (auto& x : v)
    if (!x.empty()) o += (o.empty() ? "" : sep) + x;
  return o;
}

bool CondMsgs::has_text() const {
  for (auto& x : any)
    if (!x.empty()) return true;
  for (auto& x : all)
    if (!x.empty()) return true;
  return false;
}

// evaluateOldConditions: the first false condition's message, else the true ones joined by ";";
// evaluateAnyAllConditions: the true ones (the first true `any`, every `all`) joined by "; "
// when the block held, else the false ones (the `any` conditions before the first true one,
// the first false `all`)
std::string CondMsgs::render(uint32_t as, uint32_t ls, bool held) const {
  if (old) return held ? join_non_empty(all, ";") : (ls < all.size() ? all[ls] : std::string());
  std::vector<std::string> v;
  if (held) {
    if (has_any && as < any.size()) v.push_back(any[as]);
    v.insert(v.end(), all.begin(), all.end());
  } else {
    for (size_t i = 0; i < std::min<size_t>(as, any.size()); ++i) v.push_back(any[i]);
    if (ls < all.size()) v.push_back(all[ls]);
  }
  return join_non_empty(v, "; ");
}

namespace {
// The message context: the resource and, in a foreach, the element's document
struct MsgCtx {
  JV res;
  JV el;
  const MsgElem* me = nullptr;
  bool ok = false;
  MsgCtx(const char* json, size_t n, const MsgElem* e) : me(e) {
    try {
      res = parse_all(json, n);
      if (e) el = parse_all(e->json.data(), e->json.size());
      ok = true;
    } catch (...) {
      ok = false;
    }
  }
  bool path(const std::string& q, JV* scratch, const JV** out, std::string* missing) const {
    return ctx_path(q, res, me ? &el : nullptr, me, scratch, out, missing);
  }
};
std::string trim_var(const std::string& v) {  // replaceBracesAndTrimSpaces (vars.go:422-427)
  std::string q = v;
  for (size_t p; (p = q.find("{{")) != std::string::npos;) q.erase(p, 2);
  for (size_t p; (p = q.find("}}")) != std::string::npos;) q.erase(p, 2);
  const size_t b = q.find_first_not_of(" \t\n\r\f\v"), z = q.find_last_not_of(" \t\n\r\f\v");
  return b == std::string::npos ? std::string() : q.substr(b, z - b + 1);
}
// substituteVariablesIfAny (vars.go:311-389) over one string leaf at `path`, checking for the
// resolver errors only: 0 no error (*whole: the leaf is one variable, its value), 1 an error
// (*err: the reference's text), 2 a variable whose error the host cannot tell (a construct
// outside the plain chains that may raise one).
int leaf_error(const std::string& s, const MsgCtx& cx, const std::string& path, std::string* err, const JV** whole,
               JV* scratch) {
  *whole = nullptr;
  for (size_t i = 0; i + 1 < s.size();) {
    if (!(s[i] == '{' && s[i + 1] == '{') || (i > 0 && s[i - 1] == '\\')) {
      ++i;
      continue;
    }
    const size_t e = var_end(s, i);
    if (e == std::string::npos) {
      ++i;
      continue;
    }
    const std::string q = trim_var(s.substr(i, e - i));
    const std::string pre = "failed to resolve " + q + " at path " + path + ": ";
    if (q.empty()) {  // context/evaluate.go:16-19
      *err = pre + "invalid query (nil)";
      return 1;
    }
    const JV* v = nullptr;
    std::string missing;
    if (!cx.path(q, scratch, &v, &missing)) {
      // not a plain chain of the context: a projection, `||` or a literal raises no NotFoundError
      // (the device's CE_STRICT queries); a function (length) or a plain chain over a root the
      // host does not hold (images, an outer foreach element) may raise one
      const bool projects = q.find("||") != std::string::npos || q.find("[]") != std::string::npos ||
                            q.find("[*]") != std::string::npos || q.find(".*") != std::string::npos ||
                            q.find(".[") != std::string::npos || q.find('|') != std::string::npos ||
                            q.find('`') != std::string::npos || q.find('\'') != std::string::npos;
      if (!projects || q.find('(') != std::string::npos || q.find("{{") != std::string::npos) return 2;
    } else if (!missing.empty()) {
      *err = pre + "JMESPath query failed: Unknown key \"" + missing + "\" in path";
      return 1;
    } else if (i == 0 && e == s.size()) {
      *whole = v;
    }
    i = e;
  }
  return 0;
}
// jsonutils traverse.go:64-130 with OnlyForLeafsAndKeys: keys (at their map's path) and leaves;
// the first error in traversal order (document order for maps)
int doc_error(const JV& d, const MsgCtx& cx, const std::string& path, std::string* err) {
  JV scratch;
  const JV* whole = nullptr;
  switch (d.t) {
    case JV::Str: return leaf_error(d.s, cx, path, err, &whole, &scratch);
    case JV::Arr:
      for (size_t k = 0; k < d.a.size(); ++k)
        if (int r = doc_error(d.a[k], cx, path + "/" + std::to_string(k), err)) return r;
      return 0;
    case JV::Obj:
      for (auto& kv : d.o) {
        if (int r = leaf_error(kv.first, cx, path, err, &whole, &scratch)) return r;
        if (whole && whole->t != JV::Null && whole->t != JV::Str) {  // traverse.go:97-104
          *err = "expected string after substituting variables in key \"" + kv.first + "\"";
          return 1;
        }
        std::string kp;
        for (char ch : kv.first) kp += ch == '/' ? std::string("\\/") : std::string(1, ch);
        if (int r = doc_error(kv.second, cx, path + "/" + kp, err)) return r;
      }
      return 0;
    default: return 0;
  }
}
}  // namespace

bool substitute_message(const std::string& msg, const char* json, size_t n, std::string* out, bool* nonstring,
                        bool* subst_err, const MsgElem* elem) {
  *nonstring = false;
  if (subst_err) *subst_err = false;
  if (msg.find("$(") != std::string::npos) return false;  // substituteReferences: not restated
  if (msg.find("{{") == std::string::npos) {
    *out = msg;
    return true;
  }
  MsgCtx cx(json, n, elem);
  if (!cx.ok) return false;
  std::string o;
  size_t i = 0;
  JV scratch;
  while (i < msg.size()) {
    if (msg[i] == '{' && i + 1 < msg.size() && msg[i + 1] == '{') {
      const size_t e = var_end(msg, i);
      if (e == std::string::npos) {
        o += msg[i++];
        continue;
      }
      if (i > 0 && msg[i - 1] == '\\') {  // escaped: RegexEscpVariables drops the backslash
        o.pop_back();
        o.append(msg, i, e - i);
        i = e;
        continue;
      }
      const std::string q = trim_var(msg.substr(i, e - i));
      const JV* v = nullptr;
      std::string missing;
      if (!cx.path(q, &scratch, &v, &missing)) return false;
      if (!missing.empty()) {
        if (subst_err) *subst_err = true;
        return false;
      }
      if (i == 0 && e == msg.size()) {  // the whole message is the variable: its value as is
        if (v->t == JV::Str) {
          if (v->s.find("{{") != std::string::npos) return false;
          *out = v->s;
          return true;
        }
        *nonstring = true;
        out->clear();
        go_json(*out, *v);
        return true;
      }
      std::string val;
      if (v->t == JV::Str) val = v->s;
      else go_json(val, *v);
      if (val.find("{{") != std::string::npos) return false;  // a second round would substitute it
      o += val;
      i = e;
      continue;
    }
    o += msg[i++];
  }
  *out = std::move(o);
  return true;
}

std::string doc_subst_error(const std::string& doc_json, const char* json, size_t n, const MsgElem* el) {
  MsgCtx cx(json, n, el);
  if (!cx.ok) return "";
  JV d;
  try {
    d = parse_all(doc_json.data(), doc_json.size());
  } catch (...) {
    return "";
  }
  std::string err;
  return doc_error(d, cx, "", &err) == 1 ? err : std::string();
}

std::string block_error_text(const std::string& block_json, uint32_t t, const char* json, size_t n,
                             const MsgElem* el) {
  if (!CT_IS_ERR(t) || block_json.empty()) return "";
  JV b;
  try {
    b = parse_all(block_json.data(), block_json.size());
  } catch (...) {
    return "";
  }
  // the conditions in the device's order: `any` then `all`, or the deprecated list
  std::vector<const JV*> cs;
  if (b.t == JV::Arr) {
    for (auto& c : b.a) cs.push_back(&c);
  } else if (b.t == JV::Obj) {
    for (const char* k : {"any", "all"})
      if (const JV* l = b.get(k))
        if (l->t == JV::Arr)
          for (auto& c : l->a) cs.push_back(&c);
  }
  const uint32_t ci = CT_ERR_COND(t), side = CT_ERR_SIDE(t);
  if (ci >= cs.size() || cs[ci]->t != JV::Obj) return "";
  const JV& c = *cs[ci];
  if (side == 2) {  // CreateOperatorHandler found no handler (evaluate.go:22-25; the value's err is nil)
    std::string op;
    for (char ch : sv(c.get("operator"))) op += (char)tolower((unsigned char)ch);
    static const char* const kOps[] = {"equal", "equals", "notequal", "notequals", "anyin", "allin", "anynotin",
                                       "allnotin", "in", "notin", "greaterthanorequals", "greaterthan",
                                       "lessthanorequals", "lessthan", "durationgreaterthanorequals",
                                       "durationgreaterthan", "durationlessthanorequals", "durationlessthan"};
    for (const char* k : kOps)
      if (op == k) return "";  // an operator's own error (In / NotIn over a non-string list): not restated
    return "failed to create handler for condition operator: %!w(<nil>)";
  }
  MsgCtx cx(json, n, el);
  if (!cx.ok) return "";
  static const JV kNull;
  const JV* d = c.get(side ? "value" : "key");
  std::string err;
  if (doc_error(d ? *d : kNull, cx, "", &err) != 1) return "";
  return std::string(side ? "failed to substitute variables in condition value: "
                          : "failed to substitute variables in condition key: ") + err;
}

}  // namespace kpe
