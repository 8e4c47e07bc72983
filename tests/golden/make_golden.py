#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the reference's own tests.

Run ONLY in the build container (where /root/reference exists). The Go sources
are read as text and never executed; every fixture is data (inputs + expected
outputs) lifted from the reference's tests:

  pss_evaluate_cases.json  <- pkg/pss/evaluate_test.go (testCase{name,rawRule,rawPod,allowed})
  wildcard_match.json      <- ext/wildcard/match_test.go (TestMatch table) and
                              ext/wildcard/utils_test.go (TestCheckPatterns)
  chainsaw_psa.json        <- test/conformance/chainsaw/validate/clusterpolicy/standard/psa/*
                              (policy.yaml + bad/good/excluded pods; expectation
                              taken from each chainsaw-test.yaml apply step:
                              `($error != null): true` => fail, otherwise pass)
  background_report.json   <- test/conformance/chainsaw/reports/background/test-report-background-mode
                              (restricted:latest policy, badpod01, expected report result)
  report_message_cases.json <- test/conformance/chainsaw/reports/admission/update (disallow-latest-tag
                              on a Deployment: autogen pattern fail / pass messages) and
                              .../test-report-admission-mode (require-owner pass message)
  report_exception_cases.json <- test/conformance/chainsaw/reports/{background,admission}/exception
                              (pattern rule, PolicyException, ConfigMap, skip result + property)
  check_selector.json      <- pkg/utils/match/labels_test.go (TestCheckSelector table:
                              expected LabelSelector.MatchLabels, actual labels, want, wantErr)
  pattern_leaf_cases.json  <- pkg/engine/pattern/pattern_test.go (Validate / validateNilPattern /
                              validateMapPattern / convertNumberToString / validateStringPatterns /
                              compareString tables and the assert one-liners)
  pattern_tree_cases.json  <- pkg/engine/validate/validate_test.go (validateMap /
                              validateResourceElement path+error cases, testValidationPattern
                              calls, MatchPattern status tables)
  cli_cases.json           <- test/cli/test/*/kyverno-test.yaml (policies, resources and expected
                              per-rule results of `kyverno test`; YAML decoded like
                              sigs.k8s.io/yaml: no timestamp resolution, whole floats -> ints;
                              empty namespaces set to "default" as resource.go:56-58 does)
  chart_policies.json      <- charts/kyverno-policies/templates/{baseline,restricted}/*.yaml rendered
                              with the chart defaults (ClusterPolicy, Audit, background, every
                              `if`/`with` false except the file guard, `else` branches taken,
                              backtick-escaped JMESPath kept verbatim)
  image_cases.json         <- pkg/utils/image/infos_test.go (GetImageInfo with the default
                              configuration: docker.io, registry mutation on) and
                              pkg/utils/api/image_test.go Test_extractImageInfo (resource ->
                              images map) for the `images` context
  condition_cases.json     <- pkg/engine/variables/evaluate_test.go TestEvaluate (constant key,
                              operator, value -> Evaluate result; ToJSON literals as JSON)
  match_rd_cases.json      <- pkg/engine/utils/utils_test.go:1828-2460, hand-transcribed below
                              (Go struct literals): MatchesResourceDescription on the nginx
                              Deployment with kinds/name/generateName/selector/exclude blocks

Usage:  python tests/golden/make_golden.py [/root/reference]
"""
import json
import os
import re
import sys

import yaml

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from golit import Reader, Unsupported, table, to_json  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _dump(name, obj):
    with open(os.path.join(OUT, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print(f"wrote {name}: {len(obj) if isinstance(obj, list) else 'obj'}")


def pss_cases():
    rel = "pkg/pss/evaluate_test.go"
    text = open(os.path.join(REF, rel)).read()
    # group variable names, in file order, with their start offsets
    groups = [(m.start(), m.group(1)) for m in re.finditer(r"^var (\w+) = \[\]testCase\{", text, re.M)]
    pat = re.compile(
        r"name:\s*\"(?P<name>[^\"]*)\",\s*"
        r"rawRule:\s*\[\]byte\(`(?P<rule>.*?)`\),\s*"
        r"rawPod:\s*\[\]byte\(`(?P<pod>.*?)`\),\s*"
        r"allowed:\s*(?P<allowed>true|false)",
        re.S,
    )
    cases = []
    for m in pat.finditer(text):
        grp = [g for off, g in groups if off < m.start()][-1]
        line = text.count("\n", 0, m.start()) + 1
        cases.append(
            {
                "name": m.group("name"),
                "group": grp,
                "src": f"{rel}:{line}",
                "rule": json.loads(m.group("rule")),
                "pod": json.loads(m.group("pod")),
                "allowed": m.group("allowed") == "true",
            }
        )
    return cases


def wildcard_cases():
    rel = "ext/wildcard/match_test.go"
    text = open(os.path.join(REF, rel)).read()
    pat = re.compile(
        r"pattern:\s*\"(?P<p>(?:[^\"\\]|\\.)*)\",\s*text:\s*\"(?P<t>(?:[^\"\\]|\\.)*)\",\s*matched:\s*(?P<m>true|false)"
    )
    match = []
    for m in pat.finditer(text):
        match.append({"pattern": json.loads('"' + m.group("p") + '"'),
                      "text": json.loads('"' + m.group("t") + '"'),
                      "matched": m.group("m") == "true",
                      "src": f"{rel}:{text.count(chr(10), 0, m.start()) + 1}"})
    rel2 = "ext/wildcard/utils_test.go"
    t2 = open(os.path.join(REF, rel2)).read()
    body = t2[t2.index("func TestCheckPatterns"):t2.index("func Test_MatchPatterns")]
    check = []
    cur = None
    for line in body.splitlines():
        m = re.search(r"patterns = \[\]string\{(.*)\}", line)
        if m:
            cur = [json.loads(x) for x in re.findall(r"\"[^\"]*\"", m.group(1))]
            continue
        m = re.search(r"res = CheckPatterns\(patterns, \"([^\"]*)\"\)", line)
        if m:
            name = m.group(1)
            continue
        m = re.search(r"assert.Equal\(t, (true|false), res\)", line)
        if m:
            check.append({"patterns": cur, "name": name, "want": m.group(1) == "true"})
    # Test_MatchPatterns tc table: (patterns, names) -> (pattern, name, bool)
    mp = []
    body = t2[t2.index("func Test_MatchPatterns"):t2.index("func Test_SeperateWildcards")]
    for m in re.finditer(
        r"inputPatterns:\s*(nil|\[\]string\{[^}]*\}),\s*inputNs:\s*(nil|\[\]string\{[^}]*\}),\s*"
        r"expString1:\s*\"([^\"]*)\",\s*expString2:\s*\"([^\"]*)\",\s*expBool:\s*(true|false)", body):
        def lst(s):
            return [] if s == "nil" else [json.loads(x) for x in re.findall(r"\"[^\"]*\"", s)]
        mp.append({"patterns": lst(m.group(1)), "names": lst(m.group(2)), "pattern": m.group(3),
                   "name": m.group(4), "want": m.group(5) == "true"})
    return {"match": match, "check_patterns": check, "match_patterns": mp}


def _load_yaml_docs(path):
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d]


def chainsaw_psa():
    base = "test/conformance/chainsaw/validate/clusterpolicy/standard/psa"
    out = []
    for d in sorted(os.listdir(os.path.join(REF, base))):
        full = os.path.join(REF, base, d)
        test = _load_yaml_docs(os.path.join(full, "chainsaw-test.yaml"))[0]
        policy = _load_yaml_docs(os.path.join(full, "policy.yaml"))[0]
        for step in test["spec"]["steps"]:
            for op in step.get("try", []):
                ap = op.get("apply")
                if not ap:
                    continue
                fn = ap["file"]
                if fn.startswith("policy"):
                    continue
                expect_err = any(
                    c.get("check", {}).get("($error != null)") is True for c in ap.get("expect", [])
                )
                for doc in _load_yaml_docs(os.path.join(full, fn)):
                    if doc.get("kind") not in ("Pod", "Deployment", "CronJob", "DaemonSet", "Job",
                                               "StatefulSet", "ReplicaSet", "ReplicationController"):
                        continue
                    out.append({
                        "dir": d,
                        "file": f"{base}/{d}/{fn}",
                        "policy": policy,
                        "resource": doc,
                        # Enforce-mode admission: an admission error means the rule failed.
                        "expect": "fail" if expect_err else "pass",
                    })
    return out


def chainsaw_exceptions():
    """PolicyException scenarios: policy.yaml + exception.yaml + resources applied with an
    expected admission error (Enforce policy: some rule failed) or not. Scenarios whose outcome
    depends on the admission request itself (the requesting user, DELETE) are left out: a
    background scan has neither."""
    base = "test/conformance/chainsaw/exceptions"
    admission_only = {"only-for-specific-user", "applies-to-delete", "events-creation", "background-mode"}
    out = []
    for d in sorted(os.listdir(os.path.join(REF, base))):
        full = os.path.join(REF, base, d)
        if d in admission_only or not os.path.exists(os.path.join(full, "exception.yaml")):
            continue
        test = _load_yaml_docs(os.path.join(full, "chainsaw-test.yaml"))[0]
        policy = _load_yaml_docs(os.path.join(full, "policy.yaml"))[0]
        exceptions = _load_yaml_docs(os.path.join(full, "exception.yaml"))
        for step in test["spec"]["steps"]:
            for op in step.get("try", []):
                ap = op.get("apply")
                if not ap or ap["file"].startswith(("policy", "exception", "ns")):
                    continue
                expect_err = any(c.get("check", {}).get("($error != null)") is True for c in ap.get("expect", []))
                for doc in _load_yaml_docs(os.path.join(full, ap["file"])):
                    if doc.get("kind") in ("Namespace", "PolicyException", "ClusterPolicy", "Policy"):
                        continue
                    out.append({"dir": d, "file": f"{base}/{d}/{ap['file']}", "policy": policy,
                                "exceptions": exceptions, "resource": doc,
                                "expect": "rejected" if expect_err else "allowed"})
    return out


def background_report():
    base = "test/conformance/chainsaw/reports/background/test-report-background-mode"
    policy = _load_yaml_docs(os.path.join(REF, base, "policy.yaml"))[0]
    pod = _load_yaml_docs(os.path.join(REF, base, "pod.yaml"))[0]
    rep = _load_yaml_docs(os.path.join(REF, base, "report-assert.yaml"))[0]
    return {"src": base, "policy": policy, "resource": pod, "results": rep["results"], "summary": rep["summary"]}


def report_message_cases():
    """Admission-report fixtures whose results carry messages: policy, resource, expected results
    (the message of a pattern rule's fail on an autogen rule, and a pass message)."""
    out = []
    base = "test/conformance/chainsaw/reports/admission/update"
    policy = _load_yaml_docs(os.path.join(REF, base, "policy.yaml"))[0]
    for res, rep in (("deployment-fail.yaml", "report-fail-assert.yaml"), ("deployment-pass.yaml", "report-pass-assert.yaml")):
        doc = _load_yaml_docs(os.path.join(REF, base, res))[0]
        r = _load_yaml_docs(os.path.join(REF, base, rep))[0]
        out.append({"src": f"{base}/{rep}", "policy": policy, "resource": doc, "results": r["results"],
                    "summary": r.get("summary")})
    base = "test/conformance/chainsaw/reports/admission/test-report-admission-mode"
    policy = _load_yaml_docs(os.path.join(REF, base, "chainsaw-step-01-apply-1.yaml"))[0]
    doc = _load_yaml_docs(os.path.join(REF, base, "chainsaw-step-02-apply-1.yaml"))[0]
    r = _load_yaml_docs(os.path.join(REF, base, "chainsaw-step-03-assert-1.yaml"))[0]
    out.append({"src": f"{base}/chainsaw-step-03-assert-1.yaml", "policy": policy, "resource": doc,
                "results": r["results"], "summary": r.get("summary")})
    return out


def report_exception_cases():
    """reports/{background,admission}/exception: a pattern rule, a PolicyException naming it, the
    excepted ConfigMap and the report's skip result with its `exception` property."""
    out = []
    for mode in ("background", "admission"):
        base = f"test/conformance/chainsaw/reports/{mode}/exception"
        rep = _load_yaml_docs(os.path.join(REF, base, "report-assert.yaml"))[0]
        out.append({"src": f"{base}/report-assert.yaml",
                    "policy": _load_yaml_docs(os.path.join(REF, base, "policy.yaml"))[0],
                    "exception": _load_yaml_docs(os.path.join(REF, base, "exception.yaml"))[0],
                    "resource": _load_yaml_docs(os.path.join(REF, base, "configmap.yaml"))[0],
                    "results": rep["results"], "summary": rep.get("summary")})
    return out


def _go_string_map(body):
    return {k: v for k, v in re.findall(r'"((?:[^"\\]|\\.)*)"\s*:\s*"((?:[^"\\]|\\.)*)"', body)}


def check_selector():
    rel = "pkg/utils/match/labels_test.go"
    text = open(os.path.join(REF, rel)).read()
    table = text[text.index("tests := []struct"):text.index("for _, tt := range tests")]
    out = []
    for i, case in enumerate(re.split(r"\n\t\}, \{", table)):
        if "args: args{" not in case:
            continue
        line = text[:text.index(table)].count("\n") + table[:table.index(case)].count("\n") + 1
        exp = re.search(r"expected: &metav1\.LabelSelector\{(.*?)\n\t\t\t\},?", case, re.S)
        ml = re.search(r"MatchLabels: map\[string\]string\{(.*?)\}", exp.group(1), re.S) if exp else None
        act = re.search(r"actual: +map\[string\]string\{(.*?)\}", case, re.S)
        want = re.search(r"want: +(true|false)", case)
        werr = re.search(r"wantErr: +(true|false)", case)
        out.append({
            "name": f"{rel}:{line}",
            "selector": {"matchLabels": _go_string_map(ml.group(1))} if ml else {},
            "actual": _go_string_map(act.group(1)) if act else {},
            "want": bool(want and want.group(1) == "true"),
            "wantErr": bool(werr and werr.group(1) == "true"),
        })
    return out


def match_rd_cases():
    rel = "pkg/engine/utils/utils_test.go"

    def deploy(meta):
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": meta,
                "spec": {"replicas": 3, "selector": {"matchLabels": {"app": "nginx"}},
                         "template": {"metadata": {"labels": {"app": "nginx"}},
                                      "spec": {"containers": [{"name": "nginx", "image": "nginx:1.7.9",
                                                               "ports": [{"containerPort": 80}]}]}}}}

    named = {"name": "nginx-deployment", "labels": {"app": "nginx"}}
    gen = {"generateName": "nginx-deployment", "labels": {"app": "nginx"}}
    empty_sel = {"matchLabels": None, "matchExpressions": None}
    cases = [
        (1828, named, {"kinds": ["Deployment", "Pods"], "selector": empty_sel}, None, True),
        (2023, named, {"kinds": ["Deployment"], "name": "nginx-deployment", "selector": empty_sel}, None, True),
        (2081, gen, {"kinds": ["Deployment"], "name": "nginx-deployment", "selector": empty_sel}, None, True),
        (2140, named, {"kinds": ["Deployment"], "name": "nginx-*", "selector": empty_sel}, None, True),
        (2198, gen, {"kinds": ["Deployment"], "name": "nginx-*", "selector": empty_sel}, None, True),
        (2257, named, {"kinds": ["Deployment"], "name": "nginx-*", "selector": {
            "matchLabels": None, "matchExpressions": [{"key": "label2", "operator": "NotIn", "values": ["sometest1"]}]}},
         None, True),
        (2324, named, {"kinds": ["Deployment"], "name": "nginx-*", "selector": {
            "matchLabels": None,
            "matchExpressions": [{"key": "app", "operator": "NotIn", "values": ["nginx1", "nginx2"]}]}}, None, True),
        (2392, {"name": "nginx-deployment", "labels": {"app": "nginx", "block": "true"}},
         {"kinds": ["Deployment"], "name": "nginx-*", "selector": {
             "matchLabels": None,
             "matchExpressions": [{"key": "app", "operator": "NotIn", "values": ["nginx1", "nginx2"]}]}},
         {"selector": {"matchLabels": {"block": "true"}}}, False),
    ]
    out = []
    for line, meta, match, exclude, matched in cases:
        out.append({"name": f"{rel}:{line}", "resource": deploy(meta), "match": {"resources": match},
                    "exclude": {"resources": exclude} if exclude else None, "matched": matched})
    return out


_OPS = {"operator.Equal": "", "operator.MoreEqual": ">=", "operator.LessEqual": "<=", "operator.NotEqual": "!",
        "operator.More": ">", "operator.Less": "<", "operator.InRange": "-", "operator.NotInRange": "!-"}


def _line(text, pos):
    return text.count("\n", 0, pos) + 1


def pattern_leaf_cases():
    rel = "pkg/engine/pattern/pattern_test.go"
    text = open(os.path.join(REF, rel)).read()
    out = []

    def add(func, case, **kw):
        kw.update({"fn": func, "name": f"{rel}:{case}"})
        out.append(kw)

    for func, fixed_pattern in (("TestValidate", None), ("Test_validateNilPattern", "null"),
                                ("Test_validateMapPattern", "{}")):
        for n, c in enumerate(table(text, func)):
            a = c[1]["args"][1]
            try:
                v = to_json(a["value"])
                p = fixed_pattern if fixed_pattern else to_json(a["pattern"])
            except Unsupported:
                continue
            add("validate", f"{func}[{n}]", value=v, pattern=p, want=c[1]["want"][1])
    for n, c in enumerate(table(text, "Test_convertNumberToString")):
        a = c[1]["args"][1]
        try:
            v = to_json(a["value"])
        except Unsupported:
            continue
        we = c[1].get("wantErr", ("bool", False))[1]
        add("n2s", f"Test_convertNumberToString[{n}]", value=v, want=c[1].get("want", ("str", ""))[1], wantErr=we)
    for n, c in enumerate(table(text, "Test_validateStringPatterns")):
        a = c[1]["args"][1]
        add("patterns", f"Test_validateStringPatterns[{n}]", value=to_json(a["value"]), pattern=a["pattern"][1],
            want=c[1]["want"][1])
    for n, c in enumerate(table(text, "Test_compareString")):
        a = c[1]["args"][1]
        add("compare", f"Test_compareString[{n}]", value=to_json(a["value"]), pattern=a["pattern"][1],
            op=_OPS[a["operatorVariable"][1]], want=c[1]["want"][1])
    # one-line asserts
    for m in re.finditer(r"assert\.Assert\(t, (!?)(validateFloatPattern|validateStringPattern|validateString)\("
                         r"logr\.Discard\(\), ", text):
        r = Reader(text, m.end())
        v = r.value()
        r.eat(",")
        p = r.value()
        op = None
        if m.group(2) == "validateString":
            r.eat(",")
            op = _OPS[r.value()[1]]
        want = m.group(1) != "!"
        name = f"{rel}:{_line(text, m.start())}"
        if m.group(2) == "validateFloatPattern":
            if p[0] == "int":
                p = ("float", p[1] + ".0")
            out.append({"fn": "validate", "name": name, "value": to_json(v), "pattern": to_json(p), "want": want})
        elif m.group(2) == "validateStringPattern":
            out.append({"fn": "pattern", "name": name, "value": to_json(v), "pattern": p[1], "want": want})
        else:
            out.append({"fn": "string", "name": name, "value": to_json(v), "pattern": p[1], "op": op, "want": want})
    for m in re.finditer(r"assert\.Equal\(t, operator\.GetOperatorFromStringPattern\((\"[^\"]*\")\), "
                         r"(operator\.\w+)\)", text):
        out.append({"fn": "operator", "name": f"{rel}:{_line(text, m.start())}", "pattern": json.loads(m.group(1)),
                    "want": _OPS[m.group(2)]})
    return out


def pattern_tree_cases():
    rel = "pkg/engine/validate/validate_test.go"
    text = open(os.path.join(REF, rel)).read()
    out = []
    funcs = [(m.group(1), m.start()) for m in re.finditer(r"^func (\w+)\(t \*testing\.T\) \{", text, re.M)]
    for idx, (name, start) in enumerate(funcs):
        end = funcs[idx + 1][1] if idx + 1 < len(funcs) else len(text)
        body = text[start:end]
        if "variables." in body:
            continue  # $(...) reference substitution: not part of the restated subset
        mp = re.search(r"rawPattern := \[\]byte\(`(.*?)`\)", body, re.S)
        mr = re.search(r"rawMap := \[\]byte\(`(.*?)`\)", body, re.S)
        mc = re.search(r"path, err := (validateMap|validateResourceElement)\(", body)
        if mp and mr and mc:
            after = body[mc.end():]
            mpath = re.search(r'assert\.Equal\(t, path, "([^"]*)"\)', after)
            nil_err = bool(re.search(r"assert\.NilError\(t, err\)|assert\.Assert\(t, err == nil\)", after))
            out.append({"name": f"{rel}:{name}", "kind": "element", "mode": 1 if mc.group(1) == "validateMap" else 0,
                        "pattern": mp.group(1), "resource": mr.group(1),
                        "path": mpath.group(1) if mpath else None, "nil_err": nil_err})
    # testValidationPattern(t, num, pattern, resource, path, nilErr) with the preceding assignments
    for m in re.finditer(r'pattern :?= \[\]byte\(`(.*?)`\)\s*resource :?= \[\]byte\(`(.*?)`\)\s*'
                         r'testValidationPattern\(t, "(\w+)", pattern, resource, "([^"]*)", (true|false)\)', text, re.S):
        out.append({"name": f"{rel}:TestValidateMapWildcardKeys/{m.group(3)}", "kind": "element", "mode": 0,
                    "pattern": m.group(1), "resource": m.group(2), "path": m.group(4),
                    "nil_err": m.group(5) == "true"})
    st = {"engineapi.RuleStatusPass": "pass", "engineapi.RuleStatusSkip": "skip",
          "engineapi.RuleStatusFail": "fail", "engineapi.RuleStatusError": "error"}
    for func in ("TestConditionalAnchorWithMultiplePatterns", "Test_global_anchor"):
        for c in table(text, func):
            f = c[1]
            out.append({"name": f"{rel}:{func}/{f['name'][1]}", "kind": "match", "pattern": f["pattern"][1],
                        "resource": f["resource"][1], "status": st[f["status"][1]]})
    return out


class _GoYamlLoader(yaml.SafeLoader):
    pass


# go-yaml into interface{} keeps timestamps as strings
_GoYamlLoader.yaml_implicit_resolvers = {
    k: [(tag, rx) for tag, rx in v if tag != "tag:yaml.org,2002:timestamp"]
    for k, v in yaml.SafeLoader.yaml_implicit_resolvers.items()}


def _go_json(v):
    """YAML value -> JSON-compatible value as YAMLToJSON (json.Marshal of float64) emits it."""
    if isinstance(v, dict):
        return {str(k): _go_json(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_go_json(x) for x in v]
    if isinstance(v, float) and v == int(v) and abs(v) < 1e21:
        return int(v)
    return v


def _yaml_docs(path):
    with open(path) as f:
        return [_go_json(d) for d in yaml.load_all(f, Loader=_GoYamlLoader) if d]


def cli_cases():
    base = "test/cli/test"
    out = []
    for d in sorted(os.listdir(os.path.join(REF, base))):
        tf = os.path.join(REF, base, d, "kyverno-test.yaml")
        if not os.path.exists(tf):
            continue
        t = _yaml_docs(tf)[0]
        if t.get("variables") or t.get("userinfo"):
            continue  # values / admission user info: variables are outside the restated subset
        try:
            pols, ress = [], []
            for f in t.get("policies", []):
                pols += [p for p in _yaml_docs(os.path.join(REF, base, d, f)) if p.get("kind") in
                         ("ClusterPolicy", "Policy")]
            for f in t.get("resources", []):
                ress += _yaml_docs(os.path.join(REF, base, d, f))
        except (OSError, yaml.YAMLError):
            continue
        for r in ress:
            md = r.setdefault("metadata", {})
            if not md.get("namespace"):
                md["namespace"] = "default"
        results = []
        for r in t.get("results", []):
            names = r.get("resources") or ([r["resource"]] if r.get("resource") else [])
            results.append({"policy": r.get("policy"), "rule": r.get("rule"), "resources": names,
                            "kind": r.get("kind"), "namespace": r.get("namespace"), "result": r.get("result")})
        out.append({"name": f"{base}/{d}", "policies": pols, "resources": ress, "results": results})
    return out


def engine_validate_cases():
    """pkg/engine/validation_test.go: every test whose policy / resource are raw JSON
    literals and whose expectation is a rule status (testForEach, :3170-3185), the
    success of the whole response (er.IsSuccessful()) or a status table (Flux, :1997-2054)."""
    path = os.path.join(REF, "pkg/engine/validation_test.go")
    src = open(path).read()
    out = []
    funcs = [(m.start(), m.group(1)) for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\)", src, re.M)]
    funcs.append((len(src), None))
    for (a, name), (b, _) in zip(funcs, funcs[1:]):
        body = src[a:b]
        line = src.count("\n", 0, a) + 1
        if "kyvernov1.Create" not in body and "testForEach" not in body:
            continue
        raws = {}
        for m in re.finditer(r"(\w+)\s*:?=\s*\[\]byte\(`(.*?)`\)", body, re.S):
            raws[m.group(1).lower()] = m.group(2)
        def load(txt):
            try:
                return json.loads(txt)
            except ValueError:
                return None
        if "expectedResults" in body and "policyRaw:" in body:  # status table
            for i, m in enumerate(re.finditer(r"policyRaw:\s*\[\]byte\(`(.*?)`\),.*?resourceRaw:\s*\[\]byte\(`(.*?)`\),"
                                              r".*?expectedResults:\s*\[\]engineapi\.RuleStatus\{(.*?)\}", body, re.S)):
                pol, res = load(m.group(1)), load(m.group(2))
                st = [x.strip().replace("engineapi.RuleStatus", "").lower() for x in m.group(3).split(",") if x.strip()]
                if pol and res:
                    out.append({"name": f"{name}[{i}]", "line": line, "policy": pol, "resource": res, "statuses": st})
            continue
        pol, res = load(raws.get("policyraw", "")), load(raws.get("resourceraw", ""))
        if not pol or not res:
            continue
        m = re.search(r"testForEach\(t, policyraw, resourceRaw, \"[^\"]*\", engineapi\.RuleStatus(\w+)", body)
        if m:
            out.append({"name": name, "line": line, "policy": pol, "resource": res, "first": m.group(1).lower()})
        elif "assert.Assert(t, !er.IsSuccessful())" in body:
            out.append({"name": name, "line": line, "policy": pol, "resource": res, "successful": False})
        elif "assert.Assert(t, er.IsSuccessful())" in body:
            out.append({"name": name, "line": line, "policy": pol, "resource": res, "successful": True})
    return out


def engine_message_cases():
    """pkg/engine/validation_test.go: tests whose policy / resource are raw JSON literals and
    that assert RuleResponse messages, either a `msgs := []string{...}` list checked against
    er.PolicyResponse.Rules in order or `er.PolicyResponse.Rules[i].Message()` equalities."""
    path = os.path.join(REF, "pkg/engine/validation_test.go")
    src = open(path).read()
    out = []
    funcs = [(m.start(), m.group(1)) for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\)", src, re.M)]
    funcs.append((len(src), None))
    gostr = r'"((?:[^"\\]|\\.)*)"'
    for (a, name), (b, _) in zip(funcs, funcs[1:]):
        body = src[a:b]
        if "Message()" not in body:
            continue
        raws = {}
        for m in re.finditer(r"(\w+)\s*:?=\s*\[\]byte\(`(.*?)`\)", body, re.S):
            raws[m.group(1).lower()] = m.group(2)
        try:
            pol = json.loads(raws.get("rawpolicy") or raws.get("policyraw") or "")
            res = json.loads(raws.get("rawresource") or raws.get("resourceraw") or "")
        except ValueError:
            continue
        msgs = {}
        m = re.search(r"msgs\s*:=\s*\[\]string\{(.*?)\n\s*\}", body, re.S)
        if m:
            for i, x in enumerate(re.finditer(gostr, m.group(1))):
                msgs[i] = json.loads('"' + x.group(1) + '"')
        for x in re.finditer(r"Rules\[(\d+)\]\.Message\(\),\s*" + gostr, body):
            msgs[int(x.group(1))] = json.loads('"' + x.group(2) + '"')
        if msgs:
            out.append({"name": name, "line": src.count("\n", 0, a) + 1, "policy": pol, "resource": res,
                        "messages": {str(k): v for k, v in sorted(msgs.items())}})
    print(f"engine_message_cases: {len(out)} tests")
    return out


def engine_table_message_cases():
    """pkg/engine/validation_test.go table-driven tests with `policyRaw: []byte(...)`,
    `resourceRaw: []byte(...)`, `expectedResults` and `expectedMessages` fields (one entry per
    table row; e.g. Test_Flux_Kustomization_PathNotPresent, whose first row pins a RuleError
    text: "failed to check deny conditions: failed to substitute variables in condition key: ...")."""
    path = os.path.join(REF, "pkg/engine/validation_test.go")
    src = open(path).read()
    out = []
    funcs = [(m.start(), m.group(1)) for m in re.finditer(r"^func (Test\w+)\(t \*testing\.T\)", src, re.M)]
    funcs.append((len(src), None))
    gostr = r'"((?:[^"\\]|\\.)*)"'
    status = {"RuleStatusPass": "pass", "RuleStatusFail": "fail", "RuleStatusError": "error",
              "RuleStatusSkip": "skip", "RuleStatusWarn": "warn"}
    for (a, name), (b, _) in zip(funcs, funcs[1:]):
        body = src[a:b]
        if "expectedMessages:" not in body:
            continue
        for row in re.finditer(r"\{\s*name:\s*" + gostr + r"(.*?)expectedMessages:\s*\[\]string\{(.*?)\},\s*\n\s*\}",
                               body, re.S):
            fields = row.group(2)
            raws = {m.group(1).lower(): m.group(2) for m in re.finditer(r"(\w+):\s*\[\]byte\(`(.*?)`\)", fields, re.S)}
            try:
                pol = json.loads(raws["policyraw"])
                res = json.loads(raws["resourceraw"])
            except (KeyError, ValueError):
                continue
            rs = re.search(r"expectedResults:\s*\[\]engineapi\.RuleStatus\{(.*?)\}", fields, re.S)
            results = [status[x] for x in re.findall(r"engineapi\.(RuleStatus\w+)", rs.group(1))] if rs else []
            msgs = [json.loads('"' + x.group(1) + '"') for x in re.finditer(gostr, row.group(3))]
            out.append({"name": name, "row": json.loads('"' + row.group(1) + '"'),
                        "line": src.count("\n", 0, a + row.start()) + 1, "policy": pol, "resource": res,
                        "results": results, "messages": msgs})
    print(f"engine_table_message_cases: {len(out)} rows")
    return out


def _render_chart_template(text):
    name = re.search(r'\$name := "([^"]+)"', text).group(1)
    out, stack = [], []  # stack of "branch active" flags
    for line in text.splitlines():
        ctl = re.match(r"\s*\{\{-?\s*(if|with|else|end)\b(.*?)-?\}\}\s*$", line)
        if ctl:
            kw, arg = ctl.group(1), ctl.group(2)
            if kw in ("if", "with"):
                stack.append("include \"kyverno-policies.podSecurity" in arg)  # the file guard only
            elif kw == "else":
                stack[-1] = not stack[-1]
            else:
                stack.pop()
            continue
        if not all(stack):
            continue
        if line.strip().startswith("{{"):
            continue  # `{{- $x := ... }}`, `{{- include ... }}`
        line = line.replace("{{ .Values.policyKind }}", "ClusterPolicy").replace("{{ $name }}", name)
        line = line.replace("{{ .Values.validationFailureAction }}", "Audit")
        line = line.replace("{{ .Values.background }}", "true").replace("{{ .Values.failurePolicy }}", "Fail")
        if "{{" in re.sub(r"\{\{`(.*?)`\}\}", "", line):
            continue  # labels / severity includes: metadata only
        # {{`...`}} is helm's escape for a literal kyverno variable: keep the inside
        line = re.sub(r"\{\{`(.*?)`\}\}", lambda m: m.group(1), line)
        out.append(line)
    return yaml.load("\n".join(out), Loader=_GoYamlLoader)


def chart_policies():
    base = "charts/kyverno-policies/templates"
    out = {}
    for level in ("baseline", "restricted"):
        for f in sorted(os.listdir(os.path.join(REF, base, level))):
            out.setdefault(level, []).append(_go_json(_render_chart_template(open(os.path.join(REF, base, level, f)).read())))
    return out


def best_practices():
    """test/best_practices/*.yaml (the policies commands/apply/command_test.go:17-230 applies;
    C5 uses require_pod_requests_limits.yaml and disallow_latest_tag.yaml), keyed by file name."""
    base = "test/best_practices"
    out = {}
    for f in sorted(os.listdir(os.path.join(REF, base))):
        if f.endswith(".yaml"):
            out[f] = [p for p in _yaml_docs(os.path.join(REF, base, f)) if p.get("kind") in ("ClusterPolicy", "Policy")]
    return out


def _lit_json(v):
    """golit value -> JSON text, with the typed slice / map literals ToJSON accepts."""
    if v[0] == "other":
        body = v[1]
        if body is None:
            return "null"
        if isinstance(body, list):
            return "[" + ",".join(_lit_json(x) for x in body) + "]"
        return "{" + ",".join(json.dumps(k) + ":" + _lit_json(x) for k, x in body.items()) + "}"
    if v[0] == "list":
        return "[" + ",".join(_lit_json(x) for x in v[1]) + "]"
    if v[0] == "map":
        return "{" + ",".join(json.dumps(k) + ":" + _lit_json(x) for k, x in v[1].items()) + "}"
    if v[0] == "struct":  # map[string]string{...} inside []interface{}{...}: an untyped brace body
        return "{" + ",".join(json.dumps(k) + ":" + _lit_json(x) for k, x in v[1].items()) + "}"
    return to_json(v)


def condition_cases():
    """pkg/engine/variables/evaluate_test.go TestEvaluate: one case per line,
    {kyverno.Condition{RawKey: kyverno.ToJSON(K), Operator: kyverno.ConditionOperators["Op"],
    RawValue: kyverno.ToJSON(V)}, result}. Key and value are JSON (ToJSON marshals them; the
    engine decodes numbers as float64)."""
    rel = "pkg/engine/variables/evaluate_test.go"
    src = open(os.path.join(REF, rel)).read()
    a = src.index("func TestEvaluate(")
    b = src.index("\nfunc ", a + 10)
    out, skipped = [], 0
    for m in re.finditer(r"\{kyverno\.Condition\{RawKey: kyverno\.ToJSON\(", src[a:b]):
        pos = a + m.end()
        line = src.count("\n", 0, pos) + 1
        try:
            r = Reader(src, pos)
            key = r.value()
            r.eat(")")
            r.eat(",")
            r.eat("Operator:")
            r.eat("kyverno.ConditionOperators[")
            r.ws()
            op = r.string()
            r.eat("]")
            r.eat(",")
            r.eat("RawValue:")
            r.eat("kyverno.ToJSON(")
            val = r.value()
            r.eat(")")
            r.eat("}")
            r.eat(",")
            res = r.value()
            if res[0] != "bool":
                raise Unsupported("result")
            out.append({"line": line, "key": json.loads(_lit_json(key)), "operator": op,
                        "value": json.loads(_lit_json(val)), "result": res[1]})
        except (Unsupported, ValueError, IndexError):
            skipped += 1
    print(f"condition_cases: {len(out)} cases, {skipped} skipped")
    return out


def image_cases():
    """GetImageInfo / ExtractImagesFromResource expectations (default config only)."""
    src = open(os.path.join(REF, "pkg/utils/image/infos_test.go")).read()
    infos = []
    for m in re.finditer(r'validateImageInfo\(t,\s*"([^"]*)",\s*"([^"]*)",\s*"([^"]*)",\s*"([^"]*)",\s*"([^"]*)",'
                         r'\s*"([^"]*)",\s*"([^"]*)",\s*"([^"]*)",\s*(true|false)\)', src):
        raw, name, path, reg, tag, dig, string, defreg, mut = m.groups()
        if defreg == "docker.io" and mut == "true":
            infos.append({"image": raw, "name": name, "path": path, "registry": reg, "tag": tag, "digest": dig,
                          "string": string})
    refs = []
    for m in re.finditer(r'input:\s*"([^"]*)",\s*expectedReference:\s*"([^"]*)",\s*expectedReferenceWithTag:\s*"([^"]*)"', src):
        refs.append({"image": m.group(1), "reference": m.group(2), "referenceWithTag": m.group(3)})
    errs = re.search(r"func Test_ParseError.*?testCases := \[\]string\{(.*?)\}", src, re.S).group(1)
    errors = re.findall(r'"([^"]*)"', errs)
    src2 = open(os.path.join(REF, "pkg/utils/api/image_test.go")).read()
    body = src2[src2.index("func Test_extractImageInfo"):]
    body = body[:body.index("\nfunc ")] if "\nfunc " in body else body
    extract = []
    parts = body.split("raw: []byte(`")[1:]
    for part in parts:
        raw = part[:part.index("`)")]
        if "extractionConfig" in part[:part.index("`)")]:
            continue
        rest = part[part.index("`)"):]
        # the case ends at the next raw (already split); skip cases with a custom extraction config
        images = {}
        for tm in re.finditer(r'"(initContainers|containers|ephemeralContainers|custom)":\s*\{', rest):
            seg = rest[tm.end():]
            for em in re.finditer(r'"([^"]+)":\s*\{\s*imageutils\.ImageInfo\{(.*?)\},\s*"([^"]*)",\s*\}', seg, re.S):
                # stop at the next container-type section
                nxt = re.search(r'"(initContainers|containers|ephemeralContainers|custom)":\s*\{', seg)
                if nxt and nxt.start() < em.start():
                    break
                fields = dict(re.findall(r'(\w+):\s*"([^"]*)"', em.group(2)))
                images.setdefault(tm.group(1), {})[em.group(1)] = {**fields, "Pointer": em.group(3)}
        if not images or "custom" in images:
            continue  # a case of a custom extraction config (kyvernov1.ImageExtractorConfigs)
        try:
            extract.append({"raw": json.loads(raw), "images": images})
        except ValueError:
            pass
    print(f"image_cases: {len(infos)} infos, {len(refs)} references, {len(errors)} errors, {len(extract)} extractions")
    return {"infos": infos, "references": refs, "errors": errors, "extract": extract}


if __name__ == "__main__":
    _dump("engine_message_cases.json", engine_message_cases())
    _dump("engine_table_message_cases.json", engine_table_message_cases())
    _dump("image_cases.json", image_cases())
    _dump("condition_cases.json", condition_cases())
    _dump("best_practices.json", best_practices())
    _dump("chart_policies.json", chart_policies())
    _dump("engine_validate_cases.json", engine_validate_cases())
    _dump("cli_cases.json", cli_cases())
    _dump("pattern_leaf_cases.json", pattern_leaf_cases())
    _dump("pattern_tree_cases.json", pattern_tree_cases())
    _dump("pss_evaluate_cases.json", pss_cases())
    _dump("wildcard_match.json", wildcard_cases())
    _dump("chainsaw_psa.json", chainsaw_psa())
    _dump("background_report.json", background_report())
    _dump("report_message_cases.json", report_message_cases())
    _dump("report_exception_cases.json", report_exception_cases())
    _dump("chainsaw_exceptions.json", chainsaw_exceptions())
    _dump("check_selector.json", check_selector())
    _dump("match_rd_cases.json", match_rd_cases())
