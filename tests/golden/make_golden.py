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


if __name__ == "__main__":
    _dump("pss_evaluate_cases.json", pss_cases())
    _dump("wildcard_match.json", wildcard_cases())
    _dump("chainsaw_psa.json", chainsaw_psa())
    _dump("background_report.json", background_report())
