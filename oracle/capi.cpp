// ORACLE — test infrastructure only. This library is loaded by tests/, by
// __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the CHECKER /
// CPU baseline; it is never part of the product path (kyverno_amd / libkpe).
//
// C ABI over the CPU restatement (oracle/*.hpp) of the reference's validate path.
#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "engine.hpp"

using namespace oracle;

namespace {
thread_local std::string g_err;

std::vector<std::pair<const char*, size_t>> split_lines(const char* buf, size_t len) {
  std::vector<std::pair<const char*, size_t>> out;
  size_t i = 0;
  while (i < len) {
    size_t j = i;
    while (j < len && buf[j] != '\n') ++j;
    size_t a = i, b = j;
    while (a < b && (buf[a] == ' ' || buf[a] == '\t' || buf[a] == '\r')) ++a;
    while (b > a && (buf[b - 1] == ' ' || buf[b - 1] == '\t' || buf[b - 1] == '\r')) --b;
    if (b > a) out.emplace_back(buf + a, b - a);
    i = j + 1;
  }
  return out;
}

std::vector<Policy> load_policies(const char* json) {
  JPtr arr = parse_json(json);
  std::vector<Policy> ps;
  if (arr->t == JT::Arr) {
    for (auto& p : arr->a) ps.push_back(compile_policy(*p));
  } else {
    ps.push_back(compile_policy(*arr));
  }
  return ps;
}
}  // namespace

extern "C" {

const char* oracle_last_error() { return g_err.c_str(); }

int oracle_wildcard_match(const char* pattern, const char* text) { return wildcard_match(pattern, text) ? 1 : 0; }

// pkg/pss/evaluate_test.go:13-59 driver: decode pod + PodSecurity rule, ParseVersion, EvaluatePod.
// Returns 1 allowed, 0 denied, -1 decode/version error.
int oracle_pss_evaluate(const char* rule_json, const char* pod_json) {
  try {
    JPtr rule = parse_json(rule_json);
    JPtr podj = parse_json(pod_json);
    Pod pod = get_spec(*podj, "Pod");
    Version v;
    if (!parse_version(jstr(rule->get("version")), &v)) return -1;
    std::string lvl = jstr(rule->get("level"));
    LevelVersion lv{lvl == "baseline" ? Level::Baseline : (lvl == "restricted" ? Level::Restricted : Level::Privileged),
                    v};
    std::vector<PSSExclude> ex;
    const JVal* e = rule->get("exclude");
    if (e && e->t == JT::Arr)
      for (auto& x : e->a)
        ex.push_back({jstr(x->get("controlName")), jstrlist(x->get("images")), jstr(x->get("restrictedField")),
                      jstrlist(x->get("values"))});
    return evaluate_pod(lv, ex, pod) ? 1 : 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  } catch (const DecodeError& de) {
    g_err = de.msg;
    return -1;
  }
}

// Failing check IDs (comma separated, evaluation order) for one pod, no exclusions.
int oracle_pss_failing_checks(const char* level, const char* version, const char* pod_json, char* buf, size_t cap) {
  try {
    JPtr podj = parse_json(pod_json);
    Pod pod = get_spec(*podj, "Pod");
    Version v;
    if (!parse_version(version, &v)) return -1;
    std::string lvl = level;
    LevelVersion lv{lvl == "baseline" ? Level::Baseline : (lvl == "restricted" ? Level::Restricted : Level::Privileged),
                    v};
    std::string s;
    for (auto& r : evaluate_pss(lv, pod)) s += (s.empty() ? "" : ",") + r.id;
    snprintf(buf, cap, "%s", s.c_str());
    return 0;
  } catch (...) {
    return -1;
  }
}

// Failing versioned checks of one pod as a bit mask, bit = flat index of (check, version) in
// default_checks() order (the kpe_fetch_cv_masks layout); evaluate.go:24-70 without exclusions.
static long long failing_cv_mask(const Pod& pod, const std::string& lvl, const Version& v) {
  const Level L = lvl == "baseline" ? Level::Baseline : (lvl == "restricted" ? Level::Restricted : Level::Privileged);
  long long m = 0;
  int flat = 0;
  for (auto& check : default_checks()) {
    const int base = flat;
    flat += (int)check.versions.size();
    if (L == Level::Baseline && check.level != L) continue;
    size_t latest = 0;
    for (size_t i = 1; i < check.versions.size(); ++i)
      if (!check.versions[i].min.older(check.versions[latest].min)) latest = i;
    for (size_t i = 0; i < check.versions.size(); ++i) {
      const bool run = v.latest ? i == latest : !v.older(check.versions[i].min);
      if (run && !check.versions[i].fn(pod.meta, pod.spec).allowed) m |= 1ll << (base + (int)i);
    }
  }
  return m;
}
long long oracle_pss_failing_cv(const char* level, const char* version, const char* pod_json) {
  try {
    JPtr podj = parse_json(pod_json);
    Pod pod = get_spec(*podj, "Pod");
    Version v;
    if (!parse_version(version, &v)) return -1;
    return failing_cv_mask(pod, level, v);
  } catch (...) {
    return -1;
  }
}
// The same for every row of an NDJSON batch, each decoded by its own kind (getSpec,
// validate_pss.go:137-188: a controller's pod template, a CronJob's job template); -1 for a row
// getSpec rejects. out: N entries. Returns N or -1.
long oracle_pss_failing_cv_batch(const char* level, const char* version, const char* ndjson, size_t len, long long* out,
                                 size_t out_cap, int nthreads) {
  Version v;
  if (!parse_version(version, &v)) return -1;
  auto lines = split_lines(ndjson, len);
  const size_t N = lines.size();
  if (N > out_cap) return -1;
  const std::string lvl = level;
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < N;) {
      try {
        JPtr res = parse_json(std::string(lines[i].first, lines[i].second));
        Unstructured u{res.get()};
        out[i] = failing_cv_mask(get_spec(*res, u.kind()), lvl, v);
      } catch (...) {
        out[i] = -1;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return (long)N;
}

// RuleResponse message of a podSecurity rule without exclusions for one resource
// (validate_pss.go:64-110): "Validation rule '<rule>' passed." or the FormatChecksPrint
// failure text after convertChecks. Returns 1 pass, 0 fail, -1 getSpec / version error.
// variables.SubstituteAll of a rule message (vars.go:311-389) over the background-scan context of
// one resource ({"request": {"operation", "object"}}): 0 a string (in buf), 1 a non-string value
// (its JSON in buf), -1 a substitution error, -2 outside the restated JMESPath subset.
int oracle_substitute(const char* resource_json, const char* msg, char* buf, size_t cap) {
  try {
    JPtr res = parse_json(resource_json);
    cond::Ctx cx{cond::request_context(*res)};
    const JPtr r = cond::substitute_string(msg, cx);
    if (!cond::is_null(r) && r->t == JT::Str) {
      snprintf(buf, cap, "%s", r->s.c_str());
      return 0;
    }
    snprintf(buf, cap, "%s", cond::json_marshal(r).c_str());
    return 1;
  } catch (const cond::EvalError&) {
    return -1;
  } catch (const cond::Unsupported&) {
    return -2;
  } catch (...) {
    return -1;
  }
}

// variables.SubstituteAll of a JSON document (vars.go:311-313 OnlyForLeafsAndKeys: every leaf
// and every map key, jsonutils/traverse.go:64-130) over one resource's background-scan context:
// 0 the substituted document's JSON in buf, -1 a substitution error, -2 outside the restatement.
int oracle_substitute_doc(const char* resource_json, const char* doc_json, char* buf, size_t cap) {
  try {
    JPtr res = parse_json(resource_json);
    cond::Ctx cx{cond::request_context(*res)};
    const JPtr r = cond::substitute(parse_json(doc_json), cx);
    snprintf(buf, cap, "%s", cond::json_marshal(r).c_str());
    return 0;
  } catch (const cond::EvalError&) {
    return -1;
  } catch (const cond::Unsupported&) {
    return -2;
  } catch (...) {
    return -1;
  }
}

int oracle_pss_message(const char* rule, const char* level, const char* version, const char* resource_json, char* buf,
                       size_t cap) {
  try {
    JPtr res = parse_json(resource_json);
    const std::string kind = jstr(res->get("kind"));
    Pod pod = get_spec(*res, kind);
    Version v;
    if (!parse_version(version, &v)) return -1;
    std::string lvl = level;
    LevelVersion lv{lvl == "baseline" ? Level::Baseline : (lvl == "restricted" ? Level::Restricted : Level::Privileged),
                    v};
    auto checks = evaluate_pss(lv, pod);
    std::string msg;
    if (checks.empty()) {
      msg = std::string("Validation rule '") + rule + "' passed.";
    } else {
      convert_checks(checks, kind);
      msg = std::string("Validation rule '") + rule + "' failed. It violates PodSecurity \"" + level + ":" + version +
            "\": " + format_checks_print(checks);
    }
    snprintf(buf, cap, "%s", msg.c_str());
    return checks.empty() ? 1 : 0;
  } catch (const DecodeError& de) {
    g_err = de.msg;
    return -1;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// The fail / pass message of a podSecurity rule with podSecurity.exclude entries (`excludes`, a
// JSON array or null) and, when a podSecurity PolicyException matched the resource, its entries
// (`xexcludes`, or null): validate_pss.go:76-110 (EvaluatePod with the rule's exclusions,
// convertChecks, ApplyPodSecurityExclusion of the exception's). After an exclusion pass the
// reference's check order is Go map order: here, evaluation order (exempt_exclusions). Returns 1
// pass, 0 fail, 2 skip (the exception left no check), -1 an error.
int oracle_pss_message_ex(const char* rule, const char* level, const char* version, const char* resource_json,
                          const char* excludes_json, const char* xexcludes_json, char* buf, size_t cap) {
  try {
    JPtr res = parse_json(resource_json);
    const std::string kind = jstr(res->get("kind"));
    Pod pod = get_spec(*res, kind);
    Version v;
    if (!parse_version(version, &v)) return -1;
    std::string lvl = level;
    LevelVersion lv{lvl == "baseline" ? Level::Baseline : (lvl == "restricted" ? Level::Restricted : Level::Privileged),
                    v};
    JPtr ej = parse_json(excludes_json), xj = parse_json(xexcludes_json);
    const auto ex = parse_pss_excludes(ej.get());
    std::vector<PSSCheckResult> checks;
    const bool allowed = evaluate_pod(lv, ex, pod, &checks);
    if (allowed) {
      snprintf(buf, cap, "Validation rule '%s' passed.", rule);
      return 1;
    }
    convert_checks(checks, kind);
    if (xj && xj->t == JT::Arr) {
      bool err = false;
      checks = apply_exclusion(lv, parse_pss_excludes(xj.get()), checks, pod, &err);
      if (checks.empty() && !err) {
        snprintf(buf, cap, "%s", "");
        return 2;
      }
    }
    const std::string msg = std::string("Validation rule '") + rule + "' failed. It violates PodSecurity \"" + level + ":" +
                            version + "\": " + format_checks_print(checks);
    snprintf(buf, cap, "%s", msg.c_str());
    return 0;
  } catch (const DecodeError& de) {
    g_err = de.msg;
    return -1;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// Number of rules after autogen for a JSON array of policies; names written
// newline-separated into buf as "<policy>/<rule>".
int oracle_rule_names(const char* policies_json, char* buf, size_t cap) {
  try {
    auto ps = load_policies(policies_json);
    std::string s;
    int n = 0;
    for (auto& p : ps)
      for (auto& r : p.rules) {
        s += p.name + "/" + r.name + "\n";
        ++n;
      }
    if (buf && cap) snprintf(buf, cap, "%s", s.c_str());
    return n;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// Verdict matrix for NDJSON resources x rules(after autogen) of all policies.
//   ns_labels_json: {"<namespace>": {"k": "v"}, ...} or NULL.
//   out: N x R bytes (row-major), values in oracle::Status.
// Returns N (number of resources) or -1.
long oracle_validate_ex(const char* policies_json, const char* exceptions_json, int background, const char* ndjson,
                        size_t len, const char* ns_labels_json, uint8_t* out, size_t out_cap, int nthreads);
long oracle_validate(const char* policies_json, const char* ndjson, size_t len, const char* ns_labels_json,
                     uint8_t* out, size_t out_cap, int nthreads) {
  return oracle_validate_ex(policies_json, nullptr, 0, ndjson, len, ns_labels_json, out, out_cap, nthreads);
}
// oracle_validate with PolicyExceptions (a JSON array or object; background: drop those with
// spec.background false, as FetchPolicyExceptions does).
long oracle_validate_ex(const char* policies_json, const char* exceptions_json, int background, const char* ndjson,
                        size_t len, const char* ns_labels_json, uint8_t* out, size_t out_cap, int nthreads) {
  try {
    auto ps = load_policies(policies_json);
    std::vector<PolicyException> xs;
    if (exceptions_json && *exceptions_json) {
      JPtr x = parse_json(exceptions_json);
      if (x->t == JT::Arr)
        for (auto& e : x->a) xs.push_back(parse_exception(*e));
      else
        xs.push_back(parse_exception(*x));
    }
    for (auto& p : ps) attach_exceptions(p, xs, background != 0);
    size_t R = 0;
    for (auto& p : ps) R += p.rules.size();
    std::vector<std::pair<std::string, Labels>> nsl;
    if (ns_labels_json && *ns_labels_json) {
      JPtr m = parse_json(ns_labels_json);
      for (auto& kv : m->o) {
        Labels l;
        for (auto& x : kv.second->o) l.emplace_back(x.first, jstr(x.second.get()));
        nsl.emplace_back(kv.first, l);
      }
    }
    auto lines = split_lines(ndjson, len);
    size_t N = lines.size();
    if (N * R > out_cap) {
      g_err = "output buffer too small";
      return -1;
    }
    if (nthreads < 1) nthreads = 1;
    std::atomic<size_t> next{0};
    std::atomic<bool> bad{false};
    std::string bad_msg;
    static const Labels empty;
    auto work = [&]() {
      std::vector<uint8_t> row;
      while (true) {
        size_t i = next.fetch_add(64);
        if (i >= N) break;
        size_t e = std::min(N, i + 64);
        for (; i < e; ++i) {
          JPtr res;
          try {
            res = parse_json(std::string(lines[i].first, lines[i].second));
          } catch (const std::exception& ex) {
            bad = true;
            continue;
          }
          Unstructured u{res.get()};
          std::string ns = u.ns();
          const Labels* l = &empty;
          for (auto& kv : nsl)
            if (kv.first == ns) l = &kv.second;
          size_t col = 0;
          for (auto& p : ps) {
            validate(p, *res, *l, row);
            memcpy(out + i * R + col, row.data(), row.size());
            col += row.size();
          }
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (bad) {
      g_err = "malformed resource JSON";
      return -1;
    }
    return (long)N;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// Per row, per rule: the RuleResponse message of pattern / anyPattern rules (validate_resource.go
// :316-454; "" for other rules or no response, "\u0001" where the reference's text embeds a Go
// error string). JSON array of rows. Single-threaded; test sizes only.
long oracle_pattern_messages(const char* policies_json, const char* ndjson, size_t len, char* buf, size_t cap) {
  try {
    auto ps = load_policies(policies_json);
    auto lines = split_lines(ndjson, len);
    static const Labels empty;
    std::string o = "[";
    std::vector<uint8_t> row;
    std::vector<std::string> msgs;
    for (size_t i = 0; i < lines.size(); ++i) {
      JPtr res = parse_json(std::string(lines[i].first, lines[i].second));
      o += i ? ",[" : "[";
      bool first = true;
      for (auto& p : ps) {
        validate(p, *res, empty, row, &msgs);
        for (auto& m : msgs) {
          o += first ? "\"" : ",\"";
          first = false;
          for (unsigned char ch : m) {
            if (ch == '"' || ch == '\\') o += '\\', o += (char)ch;
            else if (ch < 0x20) {
              char t[8];
              snprintf(t, sizeof t, "\\u%04x", ch);
              o += t;
            } else o += (char)ch;
          }
          o += '"';
        }
      }
      o += ']';
    }
    o += ']';
    if (o.size() + 1 <= cap) memcpy(buf, o.c_str(), o.size() + 1);
    return (long)o.size();
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// ---- pattern path (pkg/engine/{pattern,validate}) ----------------------------------
// Values are JSON texts; numbers keep their literal type (integer literal -> int, else
// float), so Go literals such as `7`, `7.0`, `nil`, `"x"` map 1:1. all_float=1 decodes
// every number as float64 (encoding/json into interface{}, as the Go tests do).
static JPtr pjson(const char* s, int all_float) {
  JPtr v = parse_json(s);
  if (all_float) pat::numbers_to_float(*v);
  return v;
}

// pattern.Validate(value, pattern)
int oracle_pattern_validate(const char* value_json, const char* pattern_json) {
  try {
    JPtr v = pjson(value_json, 0), p = pjson(pattern_json, 0);
    return pat::validate_leaf(v.get(), *p) ? 1 : 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// validateString(value, pattern, op) with op one of "", ">=", "<=", "!", ">", "<"
int oracle_validate_string(const char* value_json, const char* pattern, const char* op) {
  try {
    JPtr v = pjson(value_json, 0);
    std::string o = op;
    pat::Op k = o == ">=" ? pat::OP_GE
              : o == "<=" ? pat::OP_LE
              : o == "!"  ? pat::OP_NE
              : o == ">"  ? pat::OP_GT
              : o == "<"  ? pat::OP_LT
                          : pat::OP_EQ;
    return pat::validate_string(v.get(), pattern, k) ? 1 : 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// which = 0: validateStringPattern, 1: validateStringPatterns, 2: compareString(op "" / "!")
int oracle_string_pattern(const char* value_json, const char* pattern, int which, const char* op) {
  try {
    JPtr v = pjson(value_json, 0);
    if (which == 0) return pat::validate_string_pattern(v.get(), pattern) ? 1 : 0;
    if (which == 1) return pat::validate_string_patterns(v.get(), pattern) ? 1 : 0;
    return pat::compare_string(v.get(), pattern, std::string(op) == "!" ? pat::OP_NE : pat::OP_EQ) ? 1 : 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// operator.GetOperatorFromStringPattern -> index into {"", ">=", "<=", "!", ">", "<", "-", "!-"}
int oracle_get_operator(const char* pattern) { return (int)pat::get_operator(pattern); }

// convertNumberToString: 0 ok (text in buf), 1 error
int oracle_number_to_string(const char* value_json, char* buf, size_t cap) {
  try {
    JPtr v = pjson(value_json, 0);
    std::string s;
    if (!pat::number_to_string(v.get(), &s)) return 1;
    snprintf(buf, cap, "%s", s.c_str());
    return 0;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// validateResourceElement(resource, pattern, "/") (mode 0) or validateMap (mode 1).
// Returns the error kind (0 none, 1 conditional, 2 global, 3 negation, 4 other,
// 5 skip aggregate) and writes the returned path into buf.
int oracle_validate_element(const char* resource_json, const char* pattern_json, int mode, int all_float, char* buf,
                            size_t cap) {
  try {
    JPtr r = pjson(resource_json, all_float), p = pjson(pattern_json, all_float);
    pat::Walker w;
    pat::Err e = mode == 1 ? w.map(*r, *p, "/") : w.element(r.get(), *p, "/");
    snprintf(buf, cap, "%s", e.path.c_str());
    return (int)e.k;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// validate.MatchPattern: 0 pass, 1 skip, 2 fail (path in buf; empty path => rule error)
int oracle_match_pattern(const char* resource_json, const char* pattern_json, int all_float, char* buf, size_t cap) {
  try {
    JPtr r = pjson(resource_json, all_float), p = pjson(pattern_json, all_float);
    pat::MatchResult m = pat::match_pattern(*r, *p);
    snprintf(buf, cap, "%s", m.path.c_str());
    return (int)m.k;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// variables.Evaluate of one condition with constant key / value (JSON texts, decoded as the
// context does: numbers float64) and the operator as written: 1 true, 0 false, -1 evaluation
// error, -2 outside the restatement
int oracle_condition(const char* key_json, const char* op, const char* value_json) {
  try {
    auto c = std::make_shared<JVal>();
    c->t = JT::Obj;
    c->o.push_back({"key", parse_json(key_json)});
    c->o.push_back({"operator", cond::mk_str(op)});
    c->o.push_back({"value", parse_json(value_json)});
    cond::Condition cc = cond::parse_condition(*c);
    cond::Ctx cx{cond::request_context(JVal())};
    return cond::eval_condition(cc, cx) ? 1 : 0;
  } catch (const cond::EvalError& e) {
    g_err = e.msg;
    return -1;
  } catch (const std::exception& ex) {
    g_err = ex.what();
    return -2;
  }
}

// GetImageInfo with the default configuration: 0 and the info as JSON in buf, 1 an error
int oracle_image_info(const char* image, char* buf, size_t cap) {
  try {
    img::Info in = img::get_image_info(image);
    JVal o;
    o.t = JT::Obj;
    for (auto& kv : {std::pair<const char*, std::string*>{"registry", &in.registry}, {"name", &in.name},
                     {"path", &in.path}, {"tag", &in.tag}, {"digest", &in.digest}, {"reference", &in.reference},
                     {"referenceWithTag", &in.reference_with_tag}})
      o.o.push_back({kv.first, cond::mk_str(*kv.second)});
    std::string out;
    json_write(o, out);
    snprintf(buf, cap, "%s", out.c_str());
    return 0;
  } catch (const img::ImageError& e) {
    g_err = e.msg;
    return 1;
  }
}
// The `images` context of a resource as JSON ("null" when absent); 1 when extraction fails
int oracle_images_context(const char* resource_json, char* buf, size_t cap) {
  try {
    JPtr r = parse_json(resource_json);
    JPtr ctx = cond::request_context(*r);
    img::extract_images(*r);  // throws on an extraction error
    const JVal* im = ctx->get("images");
    std::string out = "null";
    if (im) out.clear(), json_write(*im, out);
    snprintf(buf, cap, "%s", out.c_str());
    return 0;
  } catch (const img::ImageError& e) {
    g_err = e.msg;
    return 1;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

}  // extern "C"
