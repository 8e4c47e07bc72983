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
  check_selector.json      <- pkg/utils/match/labels_test.go (TestCheckSelector table:
                              expected LabelSelector.MatchLabels, actual labels, want, wantErr)
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


def background_report():
    base = "test/conformance/chainsaw/reports/background/test-report-background-mode"
    policy = _load_yaml_docs(os.path.join(REF, base, "policy.yaml"))[0]
    pod = _load_yaml_docs(os.path.join(REF, base, "pod.yaml"))[0]
    rep = _load_yaml_docs(os.path.join(REF, base, "report-assert.yaml"))[0]
    return {"src": base, "policy": policy, "resource": pod, "results": rep["results"], "summary": rep["summary"]}


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


if __name__ == "__main__":
    _dump("pss_evaluate_cases.json", pss_cases())
    _dump("wildcard_match.json", wildcard_cases())
    _dump("chainsaw_psa.json", chainsaw_psa())
    _dump("background_report.json", background_report())
    _dump("check_selector.json", check_selector())
    _dump("match_rd_cases.json", match_rd_cases())
