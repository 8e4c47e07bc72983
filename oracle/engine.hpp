// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the validate rule loop for one (policy, resource) pair:
//   engine.Validate                 pkg/engine/engine.go:87-101
//   MatchPolicyContext              pkg/engine/internal/match.go:19-67
//   engine.validate (rule loop)     pkg/engine/validation.go:16-80
//   invokeRuleHandler / matches     pkg/engine/engine.go:190-299
//   MatchesResourceDescription      pkg/engine/utils/match.go:168-300
//   doesResourceMatchConditionBlock pkg/engine/utils/match.go:52-160
//   CheckKind / ParseKindSelector   pkg/utils/match/kind.go:14-26, pkg/utils/kube/kind.go:11-46
//   CheckSelector / ReplaceInSelector pkg/utils/match/labels.go:9-24, pkg/engine/wildcards/wildcards.go:13-58
//     (+ apimachinery v0.29.1 LabelSelectorAsSelector / labels.Requirement, third-party, restated)
//   autogen.ComputeRules            pkg/autogen/autogen.go:67-116,236-270; rule.go:73-338
//   validatePssHandler.Process      pkg/engine/handlers/validation/validate_pss.go:31-112
// Rules whose handler is not restated here (pattern/anyPattern/deny/foreach,
// preconditions, context entries, CEL, manifests, image verification) yield the
// oracle-only status UNSUPPORTED so tests never compare them silently.
#pragma once
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "conditions.hpp"
#include "json_dom.hpp"
#include "k8s_typed.hpp"
#include "pattern.hpp"
#include "pss.hpp"
#include "wildcard.hpp"

namespace oracle {

enum Status : uint8_t { NA = 0, PASS = 1, FAIL = 2, WARN = 3, ERROR = 4, SKIP = 5, UNSUPPORTED = 7 };

// ---- JSON helpers -----------------------------------------------------------
inline void json_write(const JVal& v, std::string& o) {
  switch (v.t) {
    case JT::Null: o += "null"; break;
    case JT::Bool: o += v.b ? "true" : "false"; break;
    case JT::Int: o += std::to_string(v.i); break;
    case JT::Float: {
      char b[64];
      snprintf(b, sizeof b, "%.17g", v.f);
      o += b;
      if (!strpbrk(b, ".eEni")) o += ".0";  // keep the float64 type through a re-parse
      break;
    }
    case JT::Str: {
      o += '"';
      for (unsigned char c : v.s) {
        if (c == '"' || c == '\\') {
          o += '\\';
          o += (char)c;
        } else if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
      }
      o += '"';
      break;
    }
    case JT::Arr:
      o += '[';
      for (size_t i = 0; i < v.a.size(); ++i) {
        if (i) o += ',';
        json_write(*v.a[i], o);
      }
      o += ']';
      break;
    case JT::Obj:
      o += '{';
      for (size_t i = 0; i < v.o.size(); ++i) {
        if (i) o += ',';
        JVal k;
        k.t = JT::Str;
        k.s = v.o[i].first;
        json_write(k, o);
        o += ':';
        json_write(*v.o[i].second, o);
      }
      o += '}';
      break;
  }
}
inline JPtr deep_copy(const JVal& v) {
  std::string s;
  json_write(v, s);
  return parse_json(s);
}
inline std::string jstr(const JVal* v) { return (v && v->t == JT::Str) ? v->s : std::string(); }
inline std::vector<std::string> jstrlist(const JVal* v) {
  std::vector<std::string> o;
  if (v && v->t == JT::Arr)
    for (auto& e : v->a)
      if (e->t == JT::Str) o.push_back(e->s);
  return o;
}
inline bool jnonempty(const JVal* v) {  // Go DeepEqual(x, zero) == false
  if (!v) return false;
  switch (v->t) {
    case JT::Null: return false;
    case JT::Bool: return v->b;
    case JT::Int: return v->i != 0;
    case JT::Float: return v->f != 0;
    case JT::Str: return !v->s.empty();
    case JT::Arr: return !v->a.empty();
    case JT::Obj:
      for (auto& kv : v->o)
        if (jnonempty(kv.second.get())) return true;
      return false;
  }
  return false;
}
inline void jset(JVal& obj, const std::string& k, JPtr v) {
  for (auto& kv : obj.o)
    if (kv.first == k) {
      kv.second = v;
      return;
    }
  obj.o.emplace_back(k, v);
}
inline JPtr jstrarr(const std::vector<std::string>& l) {
  auto a = std::make_shared<JVal>();
  a->t = JT::Arr;
  for (auto& s : l) {
    auto e = std::make_shared<JVal>();
    e->t = JT::Str;
    e->s = s;
    a->a.push_back(e);
  }
  return a;
}
inline JPtr jobj() {
  auto o = std::make_shared<JVal>();
  o->t = JT::Obj;
  return o;
}

// ---- unstructured accessors (apimachinery unstructured, NestedString etc.) ---------
struct Unstructured {
  const JVal* obj;
  std::string str_at(const char* a, const char* b = nullptr) const {
    const JVal* v = obj->get(a);
    if (b) v = (v && v->t == JT::Obj) ? v->get(b) : nullptr;
    return jstr(v);
  }
  std::string kind() const { return str_at("kind"); }
  std::string api_version() const { return str_at("apiVersion"); }
  std::string name() const { return str_at("metadata", "name"); }
  std::string generate_name() const { return str_at("metadata", "generateName"); }
  std::string ns() const { return str_at("metadata", "namespace"); }
  // NestedStringMap: any non-string value => error => nil map
  std::vector<std::pair<std::string, std::string>> strmap(const char* k) const {
    std::vector<std::pair<std::string, std::string>> o;
    const JVal* m = obj->get("metadata");
    const JVal* v = (m && m->t == JT::Obj) ? m->get(k) : nullptr;
    if (!v || v->t != JT::Obj) return o;
    for (auto& kv : v->o) {
      if (kv.second->t != JT::Str) return {};
      o.emplace_back(kv.first, kv.second->s);
    }
    return o;
  }
};

// ---- label selectors (apimachinery labels, restated) -------------------------------
inline bool is_dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t i = 0;
  while (i <= s.size()) {
    size_t j = s.find('.', i);
    if (j == std::string::npos) j = s.size();
    std::string lab = s.substr(i, j - i);
    if (lab.empty()) return false;  // dns1123SubdomainFmt has no per-label length limit
    for (size_t k = 0; k < lab.size(); ++k) {
      char c = lab[k];
      bool alnum = (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9');
      if (!(alnum || (c == '-' && k > 0 && k + 1 < lab.size()))) return false;
    }
    i = j + 1;
    if (j == s.size()) break;
  }
  return true;
}
inline bool is_name_part(const std::string& s) {  // qualifiedNameFmt, <= 63
  if (s.empty() || s.size() > 63) return false;
  auto alnum = [](char c) { return isalnum((unsigned char)c) != 0; };
  if (!alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!(alnum(c) || c == '-' || c == '_' || c == '.')) return false;
  return true;
}
inline bool is_qualified_name(const std::string& s) {
  size_t p = s.find('/');
  if (p == std::string::npos) return is_name_part(s);
  if (s.find('/', p + 1) != std::string::npos) return false;
  return is_dns1123_subdomain(s.substr(0, p)) && is_name_part(s.substr(p + 1));
}
inline bool is_label_value(const std::string& s) { return s.empty() || is_name_part(s); }

using Labels = std::vector<std::pair<std::string, std::string>>;
inline const std::string* label_get(const Labels& l, const std::string& k) {
  for (auto& kv : l)
    if (kv.first == k) return &kv.second;
  return nullptr;
}

struct SelReq {
  std::string key, op;
  std::vector<std::string> values;
};
struct Selector {
  bool present = false;
  std::vector<std::pair<std::string, std::string>> match_labels;  // Go map (unique keys)
  std::vector<SelReq> exprs;
};
inline Selector parse_selector(const JVal* v) {
  Selector s;
  if (!v || v->t != JT::Obj) return s;
  s.present = true;
  const JVal* ml = v->get("matchLabels");
  if (ml && ml->t == JT::Obj)
    for (auto& kv : ml->o) s.match_labels.emplace_back(kv.first, jstr(kv.second.get()));
  const JVal* me = v->get("matchExpressions");
  if (me && me->t == JT::Arr)
    for (auto& e : me->a) s.exprs.push_back({jstr(e->get("key")), jstr(e->get("operator")), jstrlist(e->get("values"))});
  return s;
}
// CheckSelector: returns 1 match, 0 no match, -1 parse error (=> "failed to parse selector")
inline int check_selector(const Selector& sel, const Labels& actual) {
  if (!sel.present) return 0;
  // wildcards.ReplaceInSelector (map; first matching actual label in iteration order)
  std::vector<std::pair<std::string, std::string>> ml;
  auto put = [&](const std::string& k, const std::string& v) {
    for (auto& kv : ml)
      if (kv.first == k) {
        kv.second = v;
        return;
      }
    ml.emplace_back(k, v);
  };
  auto has_wc = [](const std::string& x) { return x.find('*') != std::string::npos || x.find('?') != std::string::npos; };
  for (auto& kv : sel.match_labels) {
    if (has_wc(kv.first) || has_wc(kv.second)) {
      bool found = false;
      for (auto& a : actual)
        if (wildcard_match(kv.first, a.first) && wildcard_match(kv.second, a.second)) {
          put(a.first, a.second);
          found = true;
          break;
        }
      if (!found) {
        std::string k = kv.first, v = kv.second;
        for (auto& c : k)
          if (c == '*' || c == '?') c = '0';
        for (auto& c : v)
          if (c == '*' || c == '?') c = '0';
        put(k, v);
      }
    } else {
      put(kv.first, kv.second);
    }
  }
  if (ml.empty() && sel.exprs.empty()) return 1;  // labels.Everything()
  // build + validate requirements
  for (auto& kv : ml)
    if (!is_qualified_name(kv.first) || !is_label_value(kv.second)) return -1;
  for (auto& r : sel.exprs) {
    if (!is_qualified_name(r.key)) return -1;
    if (r.op == "In" || r.op == "NotIn") {
      if (r.values.empty()) return -1;
    } else if (r.op == "Exists" || r.op == "DoesNotExist") {
      if (!r.values.empty()) return -1;
    } else {
      return -1;
    }
    for (auto& v : r.values)
      if (!is_label_value(v)) return -1;
  }
  for (auto& kv : ml) {
    auto a = label_get(actual, kv.first);
    if (!a || *a != kv.second) return 0;
  }
  for (auto& r : sel.exprs) {
    auto a = label_get(actual, r.key);
    bool inset = false;
    if (a)
      for (auto& v : r.values)
        if (v == *a) inset = true;
    if (r.op == "In" && !(a && inset)) return 0;
    if (r.op == "NotIn" && a && inset) return 0;
    if (r.op == "Exists" && !a) return 0;
    if (r.op == "DoesNotExist" && a) return 0;
  }
  return 1;
}

// ---- kinds ---------------------------------------------------------------------
inline bool version_regex(const std::string& s) {  // `^v\d((alpha|beta)\d)?|\*$`
  if (s.size() >= 2 && s[0] == 'v' && isdigit((unsigned char)s[1])) return true;
  return !s.empty() && s.back() == '*';
}
inline std::vector<std::string> split(const std::string& s, char d) {
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
struct KindSel {
  std::string g, v, k, sub;
};
inline KindSel parse_kind_selector(const std::string& in) {
  auto parts = split(in, '/');
  auto last = split(parts.back(), '.');
  parts.pop_back();
  for (auto& x : last) parts.push_back(x);
  auto lower = [](std::string x) {
    for (auto& c : x) c = (char)tolower((unsigned char)c);
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
struct GVK {
  std::string g, v, k;
};
inline GVK gvk_of(const Unstructured& u) {
  std::string av = u.api_version();
  GVK r;
  size_t p = av.find('/');
  if (p == std::string::npos) r.v = av;
  else {
    r.g = av.substr(0, p);
    r.v = av.substr(p + 1);
  }
  r.k = u.kind();
  return r;
}
inline bool check_kind(const std::vector<std::string>& kinds, const GVK& gvk, const std::string& sub) {
  for (auto& k : kinds) {
    KindSel s = parse_kind_selector(k);
    if (wildcard_match(s.g, gvk.g) && wildcard_match(s.v, gvk.v) && wildcard_match(s.k, gvk.k)) {
      if (wildcard_match(s.sub, sub)) return true;
      if (gvk.g.empty() && gvk.v == "v1" && gvk.k == "Pod" && sub == "ephemeralcontainers") return true;
    }
  }
  return false;
}
// kube.GetKindFromGVK + SplitSubresource, for ContainsKind
inline bool contains_kind(const std::vector<std::string>& list, const std::string& kind) {
  for (auto& e : list) {
    auto parts = split(e, '/');
    std::string k;
    auto fmt_sub = [](std::string s) {
      size_t d = s.find('.');
      if (d != std::string::npos) s[d] = '/';
      return s;
    };
    switch (parts.size()) {
      case 1: k = fmt_sub(e); break;
      case 2:
        if (parts[0] == "*" && parts[1] == "*") k = "*/*";
        else if (version_regex(parts[0])) k = fmt_sub(parts[1]);
        else k = parts[0] + "/" + parts[1];
        break;
      case 3:
        if (version_regex(parts[0])) k = parts[1] + "/" + parts[2];
        else k = fmt_sub(parts[2]);
        break;
      case 4: k = parts[2] + "/" + parts[3]; break;
      default: k = "";
    }
    auto sp = split(k, '/');
    if (sp.size() == 2) k = sp[0];
    if (k == kind) return true;
  }
  return false;
}

// ---- policy model -----------------------------------------------------------------
struct ResourceDescription {
  bool empty = true;  // DeepEqual(rd, ResourceDescription{})
  std::vector<std::string> kinds, names, namespaces, operations;
  std::string name;
  bool has_annotations = false;
  std::vector<std::pair<std::string, std::string>> annotations;
  Selector selector, ns_selector;
};
struct UserInfo {
  bool empty = true;
};
struct Filter {
  ResourceDescription rd;
  UserInfo ui;
};
struct MatchRes {
  std::vector<Filter> any, all;
  Filter legacy;
};
struct Rule {
  std::string name;
  JPtr raw;
  MatchRes match, exclude;
  bool has_validate = false, has_pss = false, unsupported = false;
  JPtr pattern, any_pattern;  // validate.pattern / validate.anyPattern (validate_resource.go:316-398)
  std::string pss_level, pss_version;
  std::vector<PSSExclude> pss_excludes;
  cond::Conditions pre;   // rule.preconditions (engine.go:278-286)
  cond::Conditions deny;  // validate.deny.conditions (validate_resource.go:268-279)
  bool has_deny = false;
  bool pattern_vars = false;  // {{ }} variables in pattern / anyPattern (substitutePatterns)
  std::string vmsg;           // validate.message (Validation.Message)
  struct ForEach {        // validate.foreach entry (validate_resource.go:186-254, newForEachValidator)
    cond::Query list;
    cond::Conditions pre, deny;
    bool has_deny = false;
    JPtr pattern, any_pattern;  // the entry's pattern / anyPattern
    bool pattern_vars = false;
    std::vector<ForEach> nested;  // a nested foreach (nesting + 1)
    int scope = -1;       // elementScope: -1 unset, 0 false, 1 true
  };
  std::vector<ForEach> foreach;
};
// PolicyException (api/kyverno/v2beta1/policy_exception_types.go): the exceptions that name
// a (policy key, rule) pair, their match block and conditions.
struct PolicyException {
  std::string key;  // cache.MetaNamespaceKeyFunc
  bool background = true;
  std::vector<Filter> any, all;  // MatchResources (no legacy form)
  bool has_conditions = false;
  std::vector<cond::Condition> c_any, c_all;  // AnyAllConditions
  bool has_pss = false;                  // HasPodSecurity: spec.podSecurity non-empty
  std::vector<PSSExclude> pss_excludes;  // spec.podSecurity
  bool unsupported = false;  // a condition this restatement does not cover
  std::vector<std::pair<std::string, std::vector<std::string>>> refs;  // (policyName, ruleNames)
  // Exception.Contains (policy_exception_types.go:136-145): policy key equal, a rule-name glob
  bool contains(const std::string& policy, const std::string& rule) const {
    for (auto& r : refs)
      if (r.first == policy)
        for (auto& g : r.second)
          if (wildcard_match(g, rule)) return true;
    return false;
  }
};
struct Policy {
  std::string name, ns;
  bool namespaced = false;
  bool apply_one = false;
  std::vector<Rule> rules;  // after autogen
  std::string key() const { return ns.empty() ? name : ns + "/" + name; }
  // per rule: the exceptions that contain it (pkg/engine/exceptions.go:12-35), in list order
  std::vector<std::vector<const PolicyException*>> exceptions;
};

inline ResourceDescription parse_rd(const JVal* v) {
  ResourceDescription r;
  if (!v || v->t != JT::Obj) return r;
  // DeepEqual(rd, ResourceDescription{}): a present selector pointer is non-zero even for `{}`
  auto sel_obj = [&](const char* k) {
    const JVal* x = v->get(k);
    return x && x->t == JT::Obj;
  };
  r.empty = !jnonempty(v) && !sel_obj("selector") && !sel_obj("namespaceSelector");
  r.kinds = jstrlist(v->get("kinds"));
  r.names = jstrlist(v->get("names"));
  r.namespaces = jstrlist(v->get("namespaces"));
  r.operations = jstrlist(v->get("operations"));
  r.name = jstr(v->get("name"));
  const JVal* a = v->get("annotations");
  if (a && a->t == JT::Obj) {
    r.has_annotations = true;
    for (auto& kv : a->o) r.annotations.emplace_back(kv.first, jstr(kv.second.get()));
  }
  r.selector = parse_selector(v->get("selector"));
  r.ns_selector = parse_selector(v->get("namespaceSelector"));
  return r;
}
inline UserInfo parse_ui(const JVal* v) {
  UserInfo u;
  if (!v) return u;
  for (const char* k : {"roles", "clusterRoles", "subjects"})
    if (jnonempty(v->get(k))) u.empty = false;
  return u;
}
inline MatchRes parse_match(const JVal* v) {
  MatchRes m;
  if (!v || v->t != JT::Obj) return m;
  auto filters = [](const JVal* a) {
    std::vector<Filter> o;
    if (a && a->t == JT::Arr)
      for (auto& f : a->a) o.push_back({parse_rd(f->get("resources")), parse_ui(f.get())});
    return o;
  };
  m.any = filters(v->get("any"));
  m.all = filters(v->get("all"));
  m.legacy = {parse_rd(v->get("resources")), parse_ui(v)};
  return m;
}

// ---- autogen (pkg/autogen) --------------------------------------------------------------
static const char* kPodControllers = "DaemonSet,Deployment,Job,StatefulSet,ReplicaSet,ReplicationController,CronJob";

inline bool check_autogen_support(bool* needed, const JVal* rd) {
  if (!rd || rd->t != JT::Obj) return true;
  static const std::set<std::string> pc = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                           "ReplicationController", "CronJob", "Pod"};
  auto kinds = jstrlist(rd->get("kinds"));
  const JVal* ann = rd->get("annotations");
  bool is_other = kinds.size() > 1 && contains_kind(kinds, "Pod");
  if (!jstr(rd->get("name")).empty() || !jstrlist(rd->get("names")).empty() ||
      (rd->get("selector") && !rd->get("selector")->is_null()) || (ann && !ann->is_null()) || is_other)
    return false;
  for (auto& k : kinds)
    if (pc.count(k)) *needed = true;
  return true;
}
inline bool can_autogen(const JVal* spec) {
  bool needed = false;
  const JVal* rules = spec->get("rules");
  if (!rules || rules->t != JT::Arr) return false;
  for (auto& r : rules->a) {
    const JVal* mut = r->get("mutate");
    if (mut && !jstr(mut->get("patchesJson6902")).empty()) return false;
    if (jnonempty(r->get("generate"))) return false;
    if (mut && mut->get("foreach") && mut->get("foreach")->t == JT::Arr)
      for (auto& fe : mut->get("foreach")->a)
        if (!jstr(fe->get("patchesJson6902")).empty()) return false;
    const JVal* m = r->get("match");
    const JVal* x = r->get("exclude");
    if (!check_autogen_support(&needed, m ? m->get("resources") : nullptr)) return false;
    if (!check_autogen_support(&needed, x ? x->get("resources") : nullptr)) return false;
    for (const JVal* blk : {m, x}) {
      if (!blk) continue;
      for (const char* k : {"any", "all"}) {
        const JVal* l = blk->get(k);
        if (l && l->t == JT::Arr)
          for (auto& f : l->a)
            if (!check_autogen_support(&needed, f->get("resources"))) return false;
      }
    }
  }
  return needed;
}
inline std::vector<std::string> match_kinds(const JVal* blk) {  // MatchResources.GetKinds
  std::vector<std::string> k;
  if (!blk) return k;
  const JVal* rd = blk->get("resources");
  if (rd)
    for (auto& s : jstrlist(rd->get("kinds"))) k.push_back(s);
  for (const char* key : {"all", "any"}) {
    const JVal* l = blk->get(key);
    if (l && l->t == JT::Arr)
      for (auto& f : l->a) {
        const JVal* r = f->get("resources");
        if (r)
          for (auto& s : jstrlist(r->get("kinds"))) k.push_back(s);
      }
  }
  return k;
}
inline std::string autogen_name(const std::string& prefix, const std::string& name) {
  std::string n = prefix + "-" + name;
  if (n.size() > 63) n = n.substr(0, 63);
  return n;
}
inline bool is_autogen_name(const std::string& n) { return n.compare(0, 8, "autogen-") == 0; }

// rule.go:73-216 generateRule (validate subset: pattern, anyPattern, deny, podSecurity, foreach)
inline JPtr generate_rule(const std::string& name, const JVal* rule, const char* tpl_key,
                          const std::vector<std::string>& kinds, bool all_filters) {
  if (!rule) return nullptr;
  JPtr r = deep_copy(*rule);
  jset(*r, "name", std::make_shared<JVal>(JVal{JT::Str, false, 0, 0, name}));
  auto grf = [&](JVal* list) {
    for (auto& f : list->a) {
      JVal* rd = nullptr;
      for (auto& kv : f->o)
        if (kv.first == "resources") rd = kv.second.get();
      if (!rd) continue;
      if (all_filters || contains_kind(jstrlist(rd->get("kinds")), "Pod")) jset(*rd, "kinds", jstrarr(kinds));
    }
  };
  auto fix_block = [&](const char* bk, bool is_match) {
    JVal* blk = nullptr;
    for (auto& kv : r->o)
      if (kv.first == bk) blk = kv.second.get();
    if (!blk || blk->t != JT::Obj) {
      if (is_match) {
        auto m = jobj();
        auto rd = jobj();
        jset(*rd, "kinds", jstrarr(kinds));
        jset(*m, "resources", rd);
        jset(*r, bk, m);
      }
      return;
    }
    JVal* any = nullptr;
    JVal* all = nullptr;
    for (auto& kv : blk->o) {
      if (kv.first == "any" && kv.second->t == JT::Arr && !kv.second->a.empty()) any = kv.second.get();
      if (kv.first == "all" && kv.second->t == JT::Arr && !kv.second->a.empty()) all = kv.second.get();
    }
    if (any) grf(any);
    else if (all) grf(all);
    else {
      JVal* rd = nullptr;
      for (auto& kv : blk->o)
        if (kv.first == "resources") rd = kv.second.get();
      if (is_match) {
        if (!rd) {
          auto nrd = jobj();
          jset(*blk, "resources", nrd);
          rd = nrd.get();
        }
        jset(*rd, "kinds", jstrarr(kinds));
      } else if (rd && !jstrlist(rd->get("kinds")).empty()) {
        jset(*rd, "kinds", jstrarr(kinds));
      }
    }
  };
  fix_block("match", true);
  fix_block("exclude", false);
  const JVal* val = rule->get("validate");
  auto wrap = [&](const JVal* target) {
    auto inner = jobj();
    JPtr c = deep_copy(*target);
    pat::marshal_roundtrip(*c);
    jset(*inner, tpl_key, c);
    auto outer = jobj();
    jset(*outer, "spec", inner);
    return outer;
  };
  auto msg = val ? val->get("message") : nullptr;
  auto nv = jobj();
  if (msg) jset(*nv, "message", deep_copy(*msg));
  if (val && val->get("pattern") && !val->get("pattern")->is_null()) {
    jset(*nv, "pattern", wrap(val->get("pattern")));
  } else if (val && val->get("deny") && !val->get("deny")->is_null()) {
    jset(*nv, "deny", deep_copy(*val->get("deny")));
  } else if (val && val->get("podSecurity") && !val->get("podSecurity")->is_null()) {
    jset(*nv, "podSecurity", deep_copy(*val->get("podSecurity")));
  } else if (val && val->get("anyPattern") && val->get("anyPattern")->t == JT::Arr) {
    auto arr = std::make_shared<JVal>();
    arr->t = JT::Arr;
    for (auto& p : val->get("anyPattern")->a) arr->a.push_back(wrap(p.get()));
    jset(*nv, "anyPattern", arr);
  } else if (val && val->get("foreach") && val->get("foreach")->t == JT::Arr && !val->get("foreach")->a.empty()) {
    jset(*nv, "foreach", deep_copy(*val->get("foreach")));
  } else {
    return nullptr;  // mutate / verifyImages / CEL autogen: out of the restated subset
  }
  jset(*r, "validate", nv);
  return r;
}
inline JPtr gen_for_controllers(const JVal* rule, const std::string& controllers) {
  std::string name = jstr(rule->get("name"));
  if (is_autogen_name(name) || controllers.empty()) return nullptr;
  auto mk = match_kinds(rule->get("match"));
  auto xk = match_kinds(rule->get("exclude"));
  if (!contains_kind(mk, "Pod") || (!xk.empty() && !contains_kind(xk, "Pod"))) return nullptr;
  static const std::set<std::string> valid = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet",
                                              "ReplicationController"};
  std::vector<std::string> kinds;
  if (controllers == "all") kinds = {"DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController"};
  else if (controllers != "none") {
    for (auto& c : split(controllers, ','))
      if (valid.count(c)) kinds.push_back(c);
    if (kinds.empty()) kinds = split(controllers, ',');
  } else {
    kinds = split(controllers, ',');
  }
  return generate_rule(autogen_name("autogen", name), rule, "template", kinds, false);
}
inline std::string replace_all(std::string s, const std::string& a, const std::string& b) {
  size_t p = 0;
  while ((p = s.find(a, p)) != std::string::npos) {
    s.replace(p, a.size(), b);
    p += b.size();
  }
  return s;
}
inline JPtr convert_rule(const JPtr& r, bool cron) {  // autogen.go:192-234 updateGenRuleByte
  std::string s;
  json_write(*r, s);
  std::string mid = cron ? "spec.jobTemplate.spec.template." : "spec.template.";
  for (const char* o : {"request.object.", "request.oldObject."}) {
    s = replace_all(s, std::string(o) + "spec", std::string(o) + mid + "spec");
    s = replace_all(s, std::string(o) + "metadata", std::string(o) + mid + "metadata");
  }
  return parse_json(s);
}
inline std::vector<JPtr> compute_rules(const JVal& policy) {
  const JVal* spec = policy.get("spec");
  std::vector<JPtr> orig;
  if (spec && spec->get("rules") && spec->get("rules")->t == JT::Arr)
    for (auto& r : spec->get("rules")->a) orig.push_back(r);
  if (!spec) return orig;
  bool apply = can_autogen(spec);
  std::string controllers = apply ? kPodControllers : "none";
  const JVal* meta = policy.get("metadata");
  const JVal* ann = meta ? meta->get("annotations") : nullptr;
  const JVal* ac = ann ? ann->get("pod-policies.kyverno.io/autogen-controllers") : nullptr;
  if (ac && apply) controllers = jstr(ac);
  if (controllers == "none") return orig;
  std::vector<JPtr> gen;
  std::string nocron;
  {
    std::vector<std::string> keep;
    for (auto& c : split(controllers, ','))
      if (c != "CronJob") keep.push_back(c);
    for (size_t i = 0; i < keep.size(); ++i) nocron += (i ? "," : "") + keep[i];
  }
  for (auto& r : orig) {
    if (JPtr g = gen_for_controllers(r.get(), nocron)) gen.push_back(convert_rule(g, false));
    bool has_cron = controllers.find("CronJob") != std::string::npos || controllers.find("all") != std::string::npos;
    if (has_cron) {
      JPtr inter = gen_for_controllers(r.get(), controllers);
      if (inter) {
        JPtr g = generate_rule(autogen_name("autogen-cronjob", jstr(r->get("name"))), inter.get(), "jobTemplate",
                               {"CronJob"}, true);
        if (g) gen.push_back(convert_rule(g, true));
      }
    }
  }
  if (gen.empty()) return orig;
  std::vector<JPtr> out;
  for (auto& r : orig)
    if (!is_autogen_name(jstr(r->get("name")))) out.push_back(r);
  for (auto& g : gen) out.push_back(g);
  return out;
}

// Variables in a pattern (validate_resource.go:456-476 substitutePatterns, vars.go:311-389):
// true when present; throws cond::Unsupported for what this restatement does not cover ($(...)
// references, escaped or nested variables, {{@}}, queries outside the JMESPath restatement).
inline bool pattern_vars_ok(const JVal& v) {
  if (!pat::has_variables(v)) return false;
  std::function<void(const JVal&)> walk = [&](const JVal& x) {
    auto str = [](const std::string& t) {
      if (t.find("$(") != std::string::npos) throw cond::Unsupported("$(...) references");
      if (t.find("\\{{") != std::string::npos) throw cond::Unsupported("escaped variables");
    };
    if (x.t == JT::Str) str(x.s);
    for (auto& e : x.a) walk(*e);
    for (auto& kv : x.o) str(kv.first), walk(*kv.second);
  };
  walk(v);
  cond::precompile_value(std::make_shared<JVal>(v));
  return true;
}
// A validate.foreach entry (newForEachValidator): list, preconditions, then one of deny,
// pattern / anyPattern, nested foreach. Context entries are not restated.
inline Rule::ForEach parse_foreach(const JVal& e, int depth) {
  if (e.t != JT::Obj || jnonempty(e.get("context"))) throw cond::Unsupported("foreach entry");
  if (depth > 3) throw cond::Unsupported("foreach nested deeper than 4 levels");
  Rule::ForEach f;
  f.list = cond::compile_query(jstr(e.get("list")));
  f.pre = cond::parse_conditions(e.get("preconditions"));
  cond::precompile(f.pre);
  const JVal* sc = e.get("elementScope");
  if (sc && sc->t == JT::Bool) f.scope = sc->b ? 1 : 0;
  const JVal* dn = e.get("deny");
  const JVal* pt = e.get("pattern");
  const JVal* ap = e.get("anyPattern");
  const JVal* nf = e.get("foreach");
  if (dn && !dn->is_null()) {
    f.has_deny = true;
    f.deny = cond::parse_conditions(dn->get("conditions"));
    cond::precompile(f.deny);
  } else if (pt && !pt->is_null()) {
    f.pattern = deep_copy(*pt);
    f.pattern_vars = pattern_vars_ok(*f.pattern);
  } else if (ap && !ap->is_null()) {
    f.any_pattern = deep_copy(*ap);
    f.pattern_vars = pattern_vars_ok(*f.any_pattern);
    if (!f.pattern_vars) pat::numbers_to_float(*f.any_pattern);
  } else if (nf && !nf->is_null()) {
    // api.DeserializeJSONArray[ForEachValidation]: a list of entries
    if (nf->t != JT::Arr) throw cond::Unsupported("nested foreach is not a list");
    for (auto& x : nf->a) f.nested.push_back(parse_foreach(*x, depth + 1));
  }
  return f;
}

// kyvernov1.PodSecurityStandard entries (common_types.go:440-478)
inline std::vector<PSSExclude> parse_pss_excludes(const JVal* ex) {
  std::vector<PSSExclude> out;
  if (ex && ex->t == JT::Arr)
    for (auto& e : ex->a)
      out.push_back({jstr(e->get("controlName")), jstrlist(e->get("images")), jstr(e->get("restrictedField")),
                     jstrlist(e->get("values"))});
  return out;
}

inline Rule compile_rule(const JPtr& raw) {
  Rule r;
  r.raw = raw;
  r.name = jstr(raw->get("name"));
  r.match = parse_match(raw->get("match"));
  r.exclude = parse_match(raw->get("exclude"));
  const JVal* v = raw->get("validate");
  r.has_validate = jnonempty(v);
  const JVal* ps = v ? v->get("podSecurity") : nullptr;
  if (v && jnonempty(v->get("manifests"))) r.unsupported = true;
  else if (ps && ps->t == JT::Obj && jnonempty(ps)) {
    r.has_pss = true;
    r.pss_level = jstr(ps->get("level"));
    r.pss_version = jstr(ps->get("version"));
    r.pss_excludes = parse_pss_excludes(ps->get("exclude"));
  } else if (r.has_validate) {
    if (const JVal* m = v->get("message"); m && m->t == JT::Str) r.vmsg = m->s;
    // validate_resource.go:121-170: deny, then pattern/anyPattern, then foreach
    const JVal* deny = v->get("deny");
    const JVal* pt = v->get("pattern");
    const JVal* ap = v->get("anyPattern");
    const JVal* fe = v->get("foreach");
    if (deny && !deny->is_null()) {
      try {
        r.deny = cond::parse_conditions(deny->get("conditions"));
        r.has_deny = true;
        cond::precompile(r.deny);
      } catch (const cond::Unsupported&) {
        r.unsupported = true;
      }
    } else if (pt && !pt->is_null()) {
      r.pattern = deep_copy(*pt);
      try {
        r.pattern_vars = pattern_vars_ok(*r.pattern);
      } catch (const cond::Unsupported&) {
        r.unsupported = true;
      }
    } else if (ap && !ap->is_null()) {
      r.any_pattern = deep_copy(*ap);
      try {
        r.pattern_vars = pattern_vars_ok(*r.any_pattern);
      } catch (const cond::Unsupported&) {
        r.unsupported = true;
      }
      // encoding/json round trip (validate_resource.go:400-416); with variables it follows the
      // substitution
      if (!r.pattern_vars) pat::numbers_to_float(*r.any_pattern);
    } else if (fe && fe->t == JT::Arr && !fe->a.empty()) {
      try {
        for (auto& e : fe->a) r.foreach.push_back(parse_foreach(*e, 0));
      } catch (const cond::Unsupported&) {
        r.unsupported = true;
      } catch (const cond::EvalError&) {
        r.unsupported = true;  // an unparsable list expression: not restated
      }
    } else if (jnonempty(v->get("cel"))) {
      r.unsupported = true;
    }
  }
  if (jnonempty(raw->get("context"))) r.unsupported = r.has_validate;
  // any non-null block is evaluated: TransformConditions (engine/utils/utils.go:78-95) decodes
  // `any: []` to a non-nil empty list, which evaluateAnyAllConditions reads as false
  if (raw->get("preconditions") && !raw->get("preconditions")->is_null()) {
    try {
      r.pre = cond::parse_conditions(raw->get("preconditions"));
      cond::precompile(r.pre);
    } catch (const cond::Unsupported&) {
      r.unsupported = r.has_validate;
    }
  }
  return r;
}
inline Policy compile_policy(const JVal& p) {
  Policy out;
  const JVal* meta = p.get("metadata");
  out.name = meta ? jstr(meta->get("name")) : "";
  out.ns = meta ? jstr(meta->get("namespace")) : "";
  out.namespaced = jstr(p.get("kind")) == "Policy";
  const JVal* spec = p.get("spec");
  out.apply_one = spec && jstr(spec->get("applyRules")) == "One";
  for (auto& r : compute_rules(p)) out.rules.push_back(compile_rule(r));
  return out;
}

// ---- match -----------------------------------------------------------------------------
struct MatchCtx {
  const Unstructured& res;
  GVK gvk;
  const Labels& ns_labels;
  std::string operation = "CREATE";
};

// utils/match.go:52-160; returns number of errors (0 => block matched)
inline int block_errors(const ResourceDescription& rd, const UserInfo& ui, bool clear_ui, const MatchCtx& c) {
  if (!rd.operations.empty()) {
    bool ok = false;
    for (auto& o : rd.operations)
      if (o == c.operation) ok = true;
    if (!ok) return 1;
  }
  int errs = 0;
  if (!rd.kinds.empty() && !check_kind(rd.kinds, c.gvk, "")) ++errs;
  std::string rname = c.res.name();
  if (rname.empty()) rname = c.res.generate_name();
  if (!rd.name.empty() && !wildcard_match(rd.name, rname)) ++errs;
  if (!rd.names.empty()) {
    bool any = false;
    for (auto& n : rd.names)
      if (wildcard_match(n, rname)) any = true;
    if (!any) ++errs;
  }
  if (!rd.namespaces.empty()) {
    std::string ns = c.res.kind() == "Namespace" ? c.res.name() : c.res.ns();
    bool any = false;
    for (auto& n : rd.namespaces)
      if (wildcard_match(n, ns)) any = true;
    if (!any) ++errs;
  }
  if (!rd.annotations.empty()) {
    auto actual = c.res.strmap("annotations");
    for (auto& kv : rd.annotations) {
      bool m = false;
      for (auto& a : actual)
        if (wildcard_match(kv.first, a.first) && wildcard_match(kv.second, a.second)) {
          m = true;
          break;
        }
      if (!m) {
        ++errs;
        break;
      }
    }
  }
  if (rd.selector.present) {
    if (check_selector(rd.selector, c.res.strmap("labels")) != 1) ++errs;
  }
  if (rd.ns_selector.present) {
    std::string k = c.res.kind();
    bool star = false;
    for (auto& x : rd.kinds)
      if (x == "*") star = true;
    if (k == "Namespace") ++errs;
    else if (!k.empty() || star) {
      if (check_selector(rd.ns_selector, c.ns_labels) != 1) ++errs;
    }
  }
  if (!clear_ui && !ui.empty) ++errs;  // empty admission info never satisfies user-info conditions
  return errs;
}
inline int match_helper(const Filter& f, const MatchCtx& c) {
  // admission info is empty in background scans / CLI => userInfo cleared
  if (!f.rd.empty) return block_errors(f.rd, f.ui, true, c);
  return 1;  // "match cannot be empty"
}
inline int exclude_helper(const Filter& f, const MatchCtx& c) {
  if (!f.rd.empty || !f.ui.empty) {
    if (block_errors(f.rd, f.ui, false, c) == 0) return 1;  // excluded
  }
  return 0;
}
inline bool matches_resource_description(const Rule& r, const Policy& p, const MatchCtx& c) {
  if (!p.ns.empty() && p.ns != c.res.ns()) return false;
  int fails = 0;
  if (!r.match.any.empty()) {
    bool one = false;
    for (auto& f : r.match.any)
      if (match_helper(f, c) == 0) {
        one = true;
        break;
      }
    if (!one) ++fails;
  } else if (!r.match.all.empty()) {
    for (auto& f : r.match.all) fails += match_helper(f, c);
  } else {
    fails += match_helper(r.match.legacy, c);
  }
  if (fails == 0) {
    if (!r.exclude.any.empty()) {
      for (auto& f : r.exclude.any) fails += exclude_helper(f, c);
    } else if (!r.exclude.all.empty()) {
      bool all = true;
      for (auto& f : r.exclude.all)
        if (exclude_helper(f, c) == 0) {
          all = false;
          break;
        }
      if (all) ++fails;
    } else {
      fails += exclude_helper(r.exclude.legacy, c);
    }
  }
  return fails == 0;
}

// RuleResponse messages of validatePatterns (validate_resource.go:316-454): *msg gets the text, or
// kNeedsErrText when the reference's text embeds a Go error string (skips, empty-path
// failures: PatternError.Error(), a failed message substitution) or the message resolves to a
// non-string (a Go type-assertion panic)
constexpr const char* kNeedsErrText = "\x01";
struct PatMsg {
  const std::string* rule;
  const std::string* vmsg;
  std::string* out;
  const cond::Ctx* cx = nullptr;  // the JSON context (request.object) for SubstituteAll of vmsg
};
inline const std::string* pm_rule(const PatMsg* pm) {
  static const std::string none;
  return pm ? pm->rule : &none;
}
inline std::string build_error_message(const PatMsg& pm, const std::string& path) {  // :418-441
  if (path.empty()) return kNeedsErrText;  // "... execution error: <err>"
  if (pm.vmsg->empty()) return "validation error: rule " + *pm.rule + " failed at path " + path;
  std::string m = *pm.vmsg;
  if (pm.vmsg->find("$(") != std::string::npos) return kNeedsErrText;  // substituteReferences: not restated
  if (pm.vmsg->find("{{") != std::string::npos) {  // variables.SubstituteAll (:428-433)
    if (!pm.cx || !pm.cx->root) return kNeedsErrText;
    try {
      const JPtr r = cond::substitute_string(*pm.vmsg, *pm.cx);
      if (cond::is_null(r) || r->t != JT::Str) return kNeedsErrText;  // msgRaw.(string) panics
      m = r->s;
    } catch (const cond::EvalError&) {
      return kNeedsErrText;  // "variables substitution error in rule ... execution error: <err>"
    } catch (const cond::Unsupported&) {
      return kNeedsErrText;
    }
  }
  if (m.empty() || m.back() != '.') m += '.';
  return "validation error: " + m + " rule " + *pm.rule + " failed at path " + path;
}

// validate_resource.go:316-398 validatePatterns (no exceptions, CREATE operation), after
// substitutePatterns (:456-476: an error is RuleError "variable substitution failed")
inline Status pattern_handler(const JPtr& pattern0, const JPtr& any0, bool vars, const JVal& res, const cond::Ctx* cx,
                              const PatMsg* pm = nullptr) {
  JPtr pattern = pattern0, any = any0;
  auto say = [&](const std::string& m) {
    if (pm) *pm->out = m;
  };
  if (vars) {
    try {
      if (pattern) {
        pattern = cond::substitute(pattern, *cx);
      } else {
        any = cond::substitute(any, *cx);
        if (!cond::is_null(any)) any = deep_copy(*any), pat::numbers_to_float(*any);  // deserializeAnyPattern
      }
    } catch (const cond::EvalError& e) {  // RuleError "variable substitution failed" (:139-141)
      say(e.restated ? "variable substitution failed: " + e.msg : std::string(kNeedsErrText));
      return ERROR;
    } catch (const cond::Unsupported&) {
      return UNSUPPORTED;
    }
  }
  if (pattern) {
    pat::MatchResult m = pat::match_pattern(res, *pattern);
    if (m.k == pat::M_PASS) return say("validation rule '" + *pm_rule(pm) + "' passed."), PASS;
    if (m.k == pat::M_SKIP) return say(kNeedsErrText), SKIP;  // pe.Error()
    if (pm) say(build_error_message(*pm, m.path));
    return m.path.empty() ? ERROR : FAIL;
  }
  if (cond::is_null(any) || any->t != JT::Arr) {  // deserializeAnyPattern: json.Unmarshal into []interface{}
    const char* t = cond::is_null(any) ? nullptr
                    : any->t == JT::Obj ? "object"
                    : any->t == JT::Str ? "string"
                    : any->t == JT::Bool ? "bool"
                                         : "number";
    say(t ? std::string("failed to deserialize anyPattern, expected type array: json: cannot unmarshal ") + t +
                " into Go value of type []interface {}"
          : std::string(kNeedsErrText));
    return ERROR;
  }
  int fails = 0, skips = 0, idx = 0;
  std::string errs;
  bool err_text = false;
  for (auto& p : any->a) {
    pat::MatchResult m = pat::match_pattern(res, *p);
    if (m.k == pat::M_PASS)
      return say("validation rule '" + *pm_rule(pm) + "' anyPattern[" + std::to_string(idx) + "] passed."), PASS;
    if (m.k == pat::M_SKIP) {
      ++skips;
    } else {
      ++fails;  // an empty-path PatternError counts as a failure here
      if (m.path.empty()) err_text = true;  // "rule %s[%d] failed: <err>"
      errs += (errs.empty() ? "" : " ") + ("rule " + *pm_rule(pm) + "[" + std::to_string(idx) + "] failed at path " + m.path);
    }
    ++idx;
  }
  if (skips > 0 && fails == 0) return say(kNeedsErrText), SKIP;
  if (fails > 0) {
    if (pm) {  // buildAnyPatternErrorMessage (:443-454)
      const std::string& vm = *pm->vmsg;
      say(err_text ? std::string(kNeedsErrText)
                   : vm.empty() ? "validation error: " + errs
                                : vm.back() == '.' ? "validation error: " + vm + " " + errs
                                                   : "validation error: " + vm + ". " + errs);
    }
    return FAIL;
  }
  return say(pm ? *pm->vmsg : std::string()), PASS;  // RulePass(rule.Validation.Message)
}

// validate_resource.go:268-300 validateDeny + getDenyMessage over a deny block `d` in context cx
// (the rule's deny, or a foreach entry's with the element in cx): conditions true => FAIL, false
// => PASS, error => ERROR ("failed to check deny conditions: <err>", :269-271). *msg: the
// RuleResponse message (a `$(...)` reference in the rule message is not restated: no message;
// kNeedsErrText: an error text the restatement does not hold)
inline Status deny_eval(const std::string& name, const std::string& vmsg, const cond::Conditions& d,
                        const cond::Ctx& cx, std::string* msg) {
  try {
    std::string cm;
    const bool deny = cond::eval_conditions_msg(d, cx, &cm);
    if (msg) {
      if (!deny) {
        *msg = "validation rule '" + name + "' passed.";
      } else if (vmsg.empty() && cm.empty()) {
        *msg = "validation error: rule " + name + " failed";
      } else {
        const std::string j = cond::join_non_empty({vmsg, cm}, "; ");
        if (j.find("$(") != std::string::npos) {
          msg->clear();
        } else {
          try {
            const JPtr v = cond::substitute_string(j, cx);
            *msg = (!cond::is_null(v) && v->t == JT::Str)
                       ? v->s
                       : "the produced message didn't resolve to a string, check your policy definition.";
          } catch (const cond::EvalError&) {
            *msg = cm;  // SubstituteAll failed: the condition message as is
          } catch (const cond::Unsupported&) {
            msg->clear();
          }
        }
      }
    }
    return deny ? FAIL : PASS;
  } catch (const cond::EvalError& e) {
    if (msg) *msg = e.restated ? "failed to check deny conditions: " + e.msg : std::string(kNeedsErrText);
    return ERROR;
  } catch (const cond::Unsupported&) {
    return UNSUPPORTED;
  }
}
inline Status deny_handler(const Rule& r, const cond::Ctx& cx, std::string* msg = nullptr) {
  return deny_eval(r.name, r.vmsg, r.deny, cx, msg);
}

// %T of a JSON-context value (encoding/json into interface{}), for AddElementToContext's error
inline const char* go_type_name(const JPtr& v) {
  if (cond::is_null(v)) return "<nil>";
  switch (v->t) {
    case JT::Str: return "string";
    case JT::Bool: return "bool";
    case JT::Arr: return "[]interface {}";
    case JT::Obj: return "map[string]interface {}";
    default: return "float64";
  }
}
// validateElements wraps an element's failing (or last erroring) response: "validation failure:
// <message>" (validate_resource.go:239-247)
inline std::string fe_wrap(const std::string& m) { return m == kNeedsErrText ? m : "validation failure: " + m; }

// validate_resource.go:186-254 validateForEach / validateElements, utils/foreach.go: each entry's
// list, then per non-null element (AddElementToContext at `nesting`) the entry's validator
// (newForEachValidator: the rule's name and validate.message, the entry's body): preconditions,
// then deny / pattern / anyPattern / nested foreach. `scoped` is the element the patterns validate
// (policyContext.Element(): the innermost scoped element), or null for the resource itself.
// *msg: the level's response message (the deciding element's, wrapped), when it is FAIL / ERROR.
inline Status foreach_entries(const Rule& r, const std::vector<Rule::ForEach>& fes, const cond::Ctx& cx,
                              const JPtr& scoped, const JVal& res, int nesting, std::string* msg) {
  int apply_count = 0;
  for (auto& f : fes) {
    JPtr lst;
    try {
      lst = cond::run_query(f.list, cx.root);  // EvaluateList
    } catch (const cond::NotFound&) {
      continue;  // "failed to evaluate list": the entry is skipped
    } catch (const cond::EvalError&) {
      continue;
    }
    std::vector<JPtr> elems;
    if (!cond::is_null(lst) && lst->t == JT::Arr) elems = lst->a;
    else elems = {lst};
    int count = 0;
    for (size_t idx = 0; idx < elems.size(); ++idx) {
      const JPtr& el = elems[idx];
      if (cond::is_null(el)) continue;
      const bool is_map = el->t == JT::Obj;
      if (f.scope == 1 && !is_map) {  // AddElementToContext: RuleError "failed to process foreach" (:218-221)
        if (msg)
          *msg = std::string("failed to process foreach: cannot use elementScope=true foreach rules for elements "
                             "that are not maps, expected type=map got type=") + go_type_name(el);
        return ERROR;
      }
      const bool scope = f.scope == -1 ? is_map : f.scope == 1;
      cond::Ctx ex{cond::with_element(cx.root, el, (int64_t)idx, nesting)};
      const JPtr el_scoped = scope ? el : scoped;
      Status st = NA;
      std::string em;  // the element validator's response message
      bool done = false;
      try {
        if (f.pre.present) {
          try {
            if (!cond::eval_conditions(f.pre, ex)) st = SKIP, done = true;
          } catch (const cond::EvalError& e) {  // validate_resource.go:125-128
            st = ERROR, done = true;
            em = e.restated ? "failed to evaluate preconditions: " + e.msg : std::string(kNeedsErrText);
          }
        }
        if (done) {
        } else if (f.has_deny) {
          st = deny_eval(r.name, r.vmsg, f.deny, ex, msg ? &em : nullptr);
        } else if (f.pattern || f.any_pattern) {
          PatMsg pm{&r.name, &r.vmsg, &em, &ex};
          st = pattern_handler(f.pattern, f.any_pattern, f.pattern_vars, el_scoped ? *el_scoped : res, &ex,
                               msg ? &pm : nullptr);
        } else if (!f.nested.empty()) {
          st = foreach_entries(r, f.nested, ex, el_scoped, res, nesting + 1, msg ? &em : nullptr);
        } else {
          st = NA;  // "invalid validation rule": nil response
        }
      } catch (const cond::EvalError&) {
        st = ERROR;
        em = kNeedsErrText;
      }
      if (st == UNSUPPORTED) return UNSUPPORTED;
      if (st == NA || st == SKIP) continue;
      if (st == ERROR) {
        if (idx + 1 < elems.size()) continue;
        if (msg) *msg = fe_wrap(em);
        return ERROR;
      }
      if (st == FAIL) {
        if (msg) *msg = fe_wrap(em);
        return FAIL;
      }
      ++count;
    }
    apply_count += count;
  }
  return apply_count == 0 ? NA : PASS;
}
inline Status foreach_handler(const Rule& r, const cond::Ctx& cx, const JVal& res, std::string* msg = nullptr) {
  try {
    const Status s = foreach_entries(r, r.foreach, cx, nullptr, res, 0, msg);
    if (msg && s == PASS) *msg = "rule passed";  // validate_resource.go:203
    if (msg && s == NA) msg->clear();
    return s;
  } catch (const cond::Unsupported&) {
    return UNSUPPORTED;
  }
}

// validate_pss.go:31-112 (CREATE operation). exc: the matching PolicyException when it has
// podSecurity controls (:88-104): a pod they clear entirely (no error) is skipped
inline Status pss_handler(const Rule& r, const JVal& res, const std::string& kind,
                          const PolicyException* exc = nullptr) {
  Pod pod;
  try {
    pod = get_spec(res, kind);
  } catch (const DecodeError&) {
    return ERROR;
  }
  Version v;
  if (!parse_version(r.pss_version, &v)) return ERROR;
  LevelVersion lv{r.pss_level == "baseline" ? Level::Baseline
                                            : (r.pss_level == "restricted" ? Level::Restricted : Level::Privileged),
                  v};
  try {
    std::vector<PSSCheckResult> checks;
    if (evaluate_pod(lv, r.pss_excludes, pod, &checks)) return PASS;
    if (!exc) return FAIL;
    convert_checks(checks, kind);
    bool err = false;
    checks = apply_exclusion(lv, exc->pss_excludes, checks, pod, &err);
    return checks.empty() && !err ? SKIP : FAIL;
  } catch (const std::out_of_range&) {
    return ERROR;  // the Go reference would panic here
  }
}

// ---- PolicyExceptions: pkg/utils/match/match.go:26-193 CheckMatchesResources ----------------
inline int exc_filter_errors(const Filter& f, const MatchCtx& c) {
  if (f.rd.empty && f.ui.empty) return 1;  // "statement cannot be empty"
  const ResourceDescription& rd = f.rd;
  int errs = 0;
  if (!rd.kinds.empty() && !check_kind(rd.kinds, c.gvk, "")) ++errs;
  std::string rname = c.res.name();
  if (rname.empty()) rname = c.res.generate_name();
  if (!rd.name.empty() && !wildcard_match(rd.name, rname)) ++errs;
  if (!rd.names.empty()) {
    bool any = false;
    for (auto& n : rd.names) any = any || wildcard_match(n, rname);
    if (!any) ++errs;
  }
  if (!rd.namespaces.empty()) {
    std::string ns = c.res.kind() == "Namespace" ? c.res.name() : c.res.ns();
    bool any = false;
    for (auto& n : rd.namespaces) any = any || wildcard_match(n, ns);
    if (!any) ++errs;
  }
  if (!rd.annotations.empty()) {  // CheckAnnotations: every pair matched by some annotation
    auto actual = c.res.strmap("annotations");
    for (auto& kv : rd.annotations) {
      bool m = false;
      for (auto& a : actual) m = m || (wildcard_match(kv.first, a.first) && wildcard_match(kv.second, a.second));
      if (!m) {
        ++errs;
        break;
      }
    }
  }
  if (rd.selector.present && check_selector(rd.selector, c.res.strmap("labels")) != 1) ++errs;
  if (rd.ns_selector.present && c.res.kind() != "Namespace" && !c.res.kind().empty() &&
      check_selector(rd.ns_selector, c.ns_labels) != 1)
    ++errs;
  if (!f.ui.empty) ++errs;  // checkUserInfo against the empty admission info of a scan
  return errs;
}
inline bool exc_matches(const PolicyException& e, const MatchCtx& c) {
  if (!e.any.empty()) {
    for (auto& f : e.any)
      if (exc_filter_errors(f, c) == 0) return true;
    return false;
  }
  for (auto& f : e.all)
    if (exc_filter_errors(f, c) != 0) return false;
  return true;  // no any / all: no error
}
// MatchesException (pkg/engine/utils/exceptions.go:14-47): the first exception whose match
// block holds decides; its conditions (CheckAnyAllConditions, pkg/utils/conditions/condition.go:
// 14-30) failing or erroring mean no exception. Returns the exception or null; throws
// cond::Unsupported for conditions outside this restatement.
inline const PolicyException* matches_exception(const std::vector<const PolicyException*>& xs, const MatchCtx& c,
                                                const JVal& res, cond::Ctx& cx) {
  for (const PolicyException* e : xs) {
    if (!exc_matches(*e, c)) continue;
    if (e->has_conditions) {
      if (e->unsupported) throw cond::Unsupported("exception conditions");
      if (!cx.root) cx.root = cond::request_context(res);
      try {
        for (auto& k : e->c_all)
          if (!cond::eval_condition(k, cx)) return nullptr;
        if (e->c_any.empty()) return e;
        for (auto& k : e->c_any)
          if (cond::eval_condition(k, cx)) return e;
        return nullptr;
      } catch (const cond::EvalError&) {
        return nullptr;
      }
    }
    return e;
  }
  return nullptr;
}
inline PolicyException parse_exception(const JVal& x) {
  PolicyException e;
  const JVal* meta = x.get("metadata");
  const std::string name = meta ? jstr(meta->get("name")) : "", ns = meta ? jstr(meta->get("namespace")) : "";
  e.key = ns.empty() ? name : ns + "/" + name;
  const JVal* spec = x.get("spec");
  if (!spec) return e;
  const JVal* bg = spec->get("background");
  e.background = !(bg && bg->t == JT::Bool && !bg->b);
  MatchRes m = parse_match(spec->get("match"));
  e.any = m.any, e.all = m.all;
  const JVal* ps = spec->get("podSecurity");
  e.has_pss = ps && ps->t == JT::Arr && !ps->a.empty();
  if (e.has_pss) e.pss_excludes = parse_pss_excludes(ps);
  const JVal* cnd = spec->get("conditions");
  if (cnd && !cnd->is_null()) {
    e.has_conditions = true;
    try {
      for (const char* k : {"any", "all"}) {
        const JVal* l = cnd->get(k);
        if (!l || l->t != JT::Arr) continue;
        for (auto& c : l->a) {
          cond::Condition cc = cond::parse_condition(*c);
          cond::Conditions one;
          one.present = true, one.old_list = true, one.list.push_back(cc);
          cond::precompile(one);
          (k[1] == 'n' ? e.c_any : e.c_all).push_back(cc);
        }
      }
    } catch (const cond::Unsupported&) {
      e.unsupported = true;
    }
  }
  const JVal* ex = spec->get("exceptions");
  if (ex && ex->t == JT::Arr)
    for (auto& it : ex->a) e.refs.emplace_back(jstr(it->get("policyName")), jstrlist(it->get("ruleNames")));
  return e;
}
inline void attach_exceptions(Policy& p, const std::vector<PolicyException>& xs, bool background) {
  p.exceptions.assign(p.rules.size(), {});
  for (size_t i = 0; i < p.rules.size(); ++i)
    for (auto& e : xs)
      if ((!background || e.background) && e.contains(p.key(), p.rules[i].name)) p.exceptions[i].push_back(&e);
}

// engine.go:87-101 + validation.go:16-80. out[i] = status of computed rule i.
inline void validate(const Policy& p, const JVal& res, const Labels& ns_labels, std::vector<uint8_t>& out,
                     std::vector<std::string>* msgs = nullptr) {
  out.assign(p.rules.size(), NA);
  if (msgs) msgs->assign(p.rules.size(), std::string());
  try {  // NewPolicyContext -> AddImageInfos (policy_context.go:230): an error means no response at all
    img::extract_images(res);
  } catch (const img::ImageError&) {
    out.assign(p.rules.size(), UNSUPPORTED);
    return;
  }
  Unstructured u{&res};
  if (p.namespaced) {  // internal/match.go:54-67
    std::string rns = u.ns();
    if (rns != p.ns || rns.empty()) return;
  }
  MatchCtx c{u, gvk_of(u), ns_labels};
  int applied = 0;
  cond::Ctx cx;  // JSON context, built on first use
  for (size_t i = 0; i < p.rules.size(); ++i) {
    const Rule& r = p.rules[i];
    if (!matches_resource_description(r, p, c)) continue;
    if (!r.has_validate) continue;  // handler factory returns nil => no response
    Status s;
    if (r.unsupported) {
      s = UNSUPPORTED;
    } else {
      if ((r.pre.present || r.has_deny || !r.foreach.empty() || r.pattern_vars ||
           (msgs && r.vmsg.find("{{") != std::string::npos)) && !cx.root)
        cx.root = cond::request_context(res);
      s = NA;
      bool done = false;
      if (r.pre.present) {  // engine.go:278-286: error => ERROR, false => SKIP
        try {
          std::string pm;
          if (!cond::eval_conditions_msg(r.pre, cx, &pm)) {
            s = SKIP, done = true;
            if (msgs) (*msgs)[i] = cond::join_non_empty({"preconditions not met", pm}, "; ");
          }
        } catch (const cond::EvalError& e) {  // engine.go:279-281: RuleError "failed to evaluate preconditions"
          s = ERROR, done = true;
          if (msgs) (*msgs)[i] = e.restated ? "failed to evaluate preconditions: " + e.msg : std::string(kNeedsErrText);
        } catch (const cond::Unsupported&) {
          s = UNSUPPORTED, done = true;
        }
      }
      // engine.go:286-293 + the handlers' first step: a matching PolicyException skips the
      // rule (validate_resource.go:43-56 always; validate_pss.go:45-58 when it has no
      // podSecurity controls, else the PSS handler applies them to a failing pod)
      const PolicyException* pss_exc = nullptr;
      if (!done && i < p.exceptions.size() && !p.exceptions[i].empty()) {
        try {
          if (const PolicyException* e = matches_exception(p.exceptions[i], c, res, cx)) {
            if (r.has_pss && e->has_pss) pss_exc = e;
            else s = SKIP, done = true;
          }
        } catch (const cond::Unsupported&) {
          s = UNSUPPORTED, done = true;
        }
      }
      if (!done) {
        if (r.has_pss) s = pss_handler(r, res, u.kind(), pss_exc);
        else if (r.has_deny) s = deny_handler(r, cx, msgs ? &(*msgs)[i] : nullptr);
        else if (r.pattern || r.any_pattern) {
          PatMsg pm{&r.name, &r.vmsg, msgs ? &(*msgs)[i] : nullptr, &cx};
          s = pattern_handler(r.pattern, r.any_pattern, r.pattern_vars, res, &cx, msgs ? &pm : nullptr);
        }
        else if (!r.foreach.empty()) s = foreach_handler(r, cx, res, msgs ? &(*msgs)[i] : nullptr);
      }
    }
    out[i] = s;
    if (s == PASS || s == FAIL) ++applied;
    if (p.apply_one && applied > 0) break;
  }
}

}  // namespace oracle
