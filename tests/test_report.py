"""PolicyReport results (pkg/utils/report/results.go:89-156).

CPU: the oracle restatement (oracle/report.py) is pinned by the chainsaw background-report
fixture; kpe_report_results (host formatting over a verdict row) is checked against it
with oracle verdict rows. GPU: verdicts and versioned check masks from the scan kernel,
formatted by kpe_report_results, equal the oracle's results field for field."""
import copy
import json
import os
import sys

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import parity_policy_set

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle"))
import report as oracle_report  # noqa: E402  (test infrastructure)

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _no_message(results):
    return [{k: v for k, v in r.items() if k not in ("message", "timestamp")} for r in results]


def report_policy_set():
    """parity_policy_set with report annotations: scored=false (fail => warn), category,
    valid and invalid severities."""
    pols = copy.deepcopy(parity_policy_set())
    for i, p in enumerate(pols):
        ann = {}
        if i % 3 == 0:
            ann["policies.kyverno.io/category"] = "Pod Security <Standards> & \"more\""
        if i % 4 == 1:
            ann["policies.kyverno.io/severity"] = ("high", "medium", "low", "critical", "info", "bogus")[i % 6]
        if i % 5 == 2:
            ann["policies.kyverno.io/scored"] = "false"
        if ann:
            p["metadata"]["annotations"] = ann
    return pols


def _no_timestamp(results):
    return [{k: v for k, v in r.items() if k != "timestamp"} for r in results]


def test_oracle_pinned_by_background_report(oracle):
    bg = json.load(open(os.path.join(GOLD, "background_report.json")))
    names = oracle.rule_names([bg["policy"]])
    v = oracle.validate([bg["policy"]], json.dumps(bg["resource"]).encode())
    got = oracle_report.report_results([bg["policy"]], names, v[0], bg["resource"], oracle.failing_checks)
    assert got == _no_message(bg["results"])
    got = oracle_report.report_results([bg["policy"]], names, v[0], bg["resource"], oracle.failing_checks,
                                       oracle.pss_message)
    assert got == _no_timestamp(bg["results"])  # report-assert.yaml, message included


def _oracle_cv_row(oracle, pols, names, row, doc):
    """Versioned failing-check masks of one row from the oracle (the kpe_fetch_cv_masks layout:
    bit v = versioned check v), for the fail cells of podSecurity rules."""
    m = np.zeros(len(names), dtype=np.uint32)
    for r, full in enumerate(names):
        if int(row[r]) != 2:
            continue
        pname, rname = full.split("/", 1)
        pol = next(p for p in pols if p["metadata"]["name"] == pname)
        ps0 = (oracle_report._source_rule(pol, rname).get("validate") or {}).get("podSecurity")
        if ps0:
            m[r] = oracle.failing_cv(ps0.get("level", ""), ps0.get("version", ""), oracle_report.pod_of(doc)) or 0
    return m


def test_host_messages_match_oracle(oracle):
    """kpe_report_results_msg renders podSecurity pass / fail and pattern pass messages from the
    resource JSON and the failing versioned checks; with the oracle's verdicts and checks as
    input it equals the oracle's report (oracle/pss.hpp FormatChecksPrint) on Pods and
    controllers of two synthetic mixes."""
    pols = [p for p in report_policy_set()
            if not any(((r.get("validate") or {}).get("podSecurity") or {}).get("exclude")
                       for r in p["spec"]["rules"])]
    ps = K.PolicySet(pols)
    names = oracle.rule_names(pols)
    nmsg = 0
    for mix, seed in ((0, 0xC2), (2, 31)):
        nd = K.synth_resources(seed, 300, mix=mix)
        docs = [json.loads(x) for x in nd.split(b"\n") if x.strip()]
        v = oracle.validate(pols, nd, nthreads=4)
        for i, doc in enumerate(docs):
            want = oracle_report.report_results(pols, names, v[i], doc, oracle.failing_checks, oracle.pss_message)
            got = K.report_results(ps, v[i], _oracle_cv_row(oracle, pols, names, v[i], doc), resource=doc)
            assert got == want, (i, got, want)
            nmsg += sum(1 for r in got if r.get("result") in ("fail", "warn") and "message" in r)
    assert nmsg > 100


def _deny_message_policies():
    """cond_policy_set with the deny rule messages varied: kept, removed (default message),
    with variables (substituted), a condition message (not rendered) and preconditions."""
    from tests.policies import cond_policy_set
    pols = copy.deepcopy(cond_policy_set())
    rules = pols[0]["spec"]["rules"]
    for i, r in enumerate(rules):
        val = r.get("validate") or {}
        if "deny" not in val:
            continue
        if i % 4 == 1:
            del val["message"]
        elif i % 4 == 2:
            val["message"] = "bad {{ request.object.metadata.name }}"
        elif i % 4 == 3:
            val["message"] = f"rule {i}: <no> & \"quotes\""
    obj = "request.object"
    rules.append({"name": "deny-pre", "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment"]}}]},
                  "preconditions": {"any": [{"key": "{{ " + obj + ".metadata.labels.tier || '' }}",
                                             "operator": "Equals", "value": "frontend"}]},
                  "validate": {"deny": {"conditions": {"all": [
                      {"key": "{{ " + obj + ".metadata.labels.app || '' }}", "operator": "NotEquals",
                       "value": "app-1*"}]}}}})
    rules.append({"name": "deny-cond-msg", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"message": "m", "deny": {"conditions": {"any": [
                      {"key": "{{ " + obj + ".metadata.labels.app || '' }}", "operator": "Equals",
                       "value": "app-1*", "message": "app label"}]}}}})
    # SubstituteAll of the rule message (validate_resource.go:288-299) on rules that always deny:
    # strings, maps (json.Marshal: sorted keys, HTML escapes), numbers, missing members (null),
    # indexes, quoted identifiers, a whole-message non-string, an escaped variable, two variables
    always = {"conditions": {"all": [{"key": "x", "operator": "Equals", "value": "x"}]}}
    for k, m in enumerate([
            "pod {{ request.object.metadata.name }} in {{request.object.metadata.namespace}}",
            "labels={{ request.object.metadata.labels }}",
            "replicas {{ request.object.spec.replicas }}, missing {{ request.object.spec.nope }}",
            "first {{ request.object.spec.containers[0].image }} last {{ request.object.spec.containers[-1].name }}",
            'ann {{ request.object.metadata."annotations" }}',
            "{{ request.object.metadata.labels }}",
            "{{ request.object.metadata.name }}",
            "literal \\{{ request.object.metadata.name }} and {{ request.object.kind }}"]):
        rules.append({"name": f"deny-subst-{k}", "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment"]}}]},
                      "validate": {"message": m, "deny": copy.deepcopy(always)}})
    return pols


def test_host_deny_messages_match_oracle(oracle):
    """kpe_report_results_msg renders deny pass / fail / preconditions-skip messages
    (validate_resource.go:268-300, engine.go:283) like the oracle's report on the
    condition-rule set, with the rule message kept, removed, templated or escaped."""
    pols = _deny_message_policies()
    ps = K.PolicySet(pols)
    names = oracle.rule_names(pols)
    seen = set()
    for mix, seed in ((2, 0x3D), (4, 5)):
        nd = K.synth_resources(seed, 300, mix=mix)
        docs = [json.loads(x) for x in nd.split(b"\n") if x.strip()]
        v = oracle.validate(pols, nd, nthreads=4)
        for i, doc in enumerate(docs):
            want = oracle_report.report_results(pols, names, v[i], doc, oracle.failing_checks, oracle.pss_message,
                                                oracle.substitute)
            got = K.report_results(ps, v[i], _oracle_cv_row(oracle, pols, names, v[i], doc), resource=doc)
            assert got == want, (i, got, want)
            seen.update((r["result"], r.get("message", "")[:20]) for r in got)
    msgs = {m for _, m in seen}
    assert "validation error: ru" in msgs and "preconditions not me" in msgs and "m" in msgs
    assert any(m.startswith("pod ") for m in msgs) and any(m.startswith("labels={") for m in msgs)
    assert any(m.startswith("the produced messag") for m in msgs) and any(m.startswith("literal {{") for m in msgs)
    assert any(m.startswith("rule ") for m in msgs) and any(m.startswith("validation rule") for m in msgs)


def test_host_report_matches_oracle_without_controls(oracle):
    pols = report_policy_set()
    ps = K.PolicySet(pols)
    names = oracle.rule_names(pols)
    assert names == ps.rule_names
    nd = K.synth_resources(7, 400, mix=2)
    docs = [json.loads(x) for x in nd.split(b"\n") if x.strip()]
    v = oracle.validate(pols, nd, nthreads=4)
    seen = set()
    for i, doc in enumerate(docs):
        want = oracle_report.report_results(pols, names, v[i], doc, lambda *a: [])
        got = K.report_results(ps, v[i])
        assert got == want, i
        seen.update(r["result"] for r in got)
    assert {"pass", "fail", "warn", "error"} <= seen


def test_host_report_versioned_controls():
    """A baseline:v1.19 rule runs seccompProfile_baseline at 1.0 (annotations) and 1.19
    (fields); both failing lists the id twice (pkg/pss/evaluate.go:51-66)."""
    pol = {"apiVersion": "kyverno.io/v1", "kind": "Policy",
           "metadata": {"name": "p", "namespace": "team-a"},
           "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                               "validate": {"podSecurity": {"level": "baseline", "version": "v1.19"}}}]}}
    ps = K.PolicySet([pol])
    L = K.load()
    ids = [L.kpe_pss_check_id(L.kpe_pss_cv_check(c)).decode() for c in range(L.kpe_pss_num_cv())]
    bits = [c for c, x in enumerate(ids) if x == "seccompProfile_baseline"]
    hp = ids.index("hostPorts")
    assert len(bits) == 2
    row_v = np.array([2] + [0] * (ps.num_rules - 1), dtype=np.uint8)
    row_m = np.zeros(ps.num_rules, dtype=np.uint32)
    row_m[0] = (1 << bits[0]) | (1 << bits[1]) | (1 << hp)
    got = K.report_results(ps, row_v, row_m)
    assert got == [{"source": "kyverno", "policy": "team-a/p", "rule": "r", "result": "fail", "scored": True,
                    "properties": {"controls": "hostPorts,seccompProfile_baseline,seccompProfile_baseline",
                                   "standard": "baseline", "version": "v1.19"}}]
    # no response => no result; masks ignored for non-fail cells
    assert K.report_results(ps, np.zeros(ps.num_rules, np.uint8), row_m) == []
    row_v[0] = 1
    assert "properties" not in K.report_results(ps, row_v, row_m)[0]


@pytest.mark.gpu
def test_gpu_report_background_fixture():
    bg = json.load(open(os.path.join(GOLD, "background_report.json")))
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet([bg["policy"]])
    c = K.Corpus(json.dumps(bg["resource"]).encode())
    v, _, _ = eng.evaluate(ps, c, check_masks=True)
    m = eng.cv_masks(ps, c)
    assert K.report_results(ps, v[0], m[0]) == _no_message(bg["results"])
    assert K.report_results(ps, v[0], m[0], resource=bg["resource"]) == _no_timestamp(bg["results"])


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 3000, 0xC2), (2, 3000, 21)])
def test_gpu_report_matches_oracle(oracle, mix, n, seed):
    pols = report_policy_set()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(seed, n, mix=mix)
    c = K.Corpus(nd)
    v, masks, _ = eng.evaluate(ps, c, check_masks=True)
    cv = eng.cv_masks(ps, c)
    L = K.load()
    cv_check = [L.kpe_pss_cv_check(b) for b in range(L.kpe_pss_num_cv())]
    folded = np.zeros_like(cv)
    for b, k in enumerate(cv_check):  # the per-id masks are the OR of the versioned ones
        folded |= ((cv >> np.uint32(b)) & np.uint32(1)) << np.uint32(k)
    assert (folded == masks).all()
    names = oracle.rule_names(pols)
    docs = [json.loads(x) for x in nd.split(b"\n") if x.strip()]
    ref = oracle.validate(pols, nd, nthreads=8)
    assert (v == ref).all()
    dup = 0
    for i in range(0, n, 3):
        want = oracle_report.report_results(pols, names, ref[i], docs[i], oracle.failing_checks)
        got = K.report_results(ps, v[i], cv[i])
        assert got == want, (i, got, want)
        # messages: rules with podSecurity.exclude render no fail message on either side
        want = oracle_report.report_results(pols, names, ref[i], docs[i], oracle.failing_checks, oracle.pss_message)
        got = K.report_results(ps, v[i], cv[i], resource=docs[i])
        assert got == want, (i, got, want)
        dup += sum(1 for r in got if "properties" in r and len(set(r["properties"]["controls"].split(","))) <
                   len(r["properties"]["controls"].split(",")))
    assert dup > 0  # some pinned-version rule lists a check id twice


def _counts(v):
    return [{"na": int((v[:, r] == 0).sum()), "pass": int((v[:, r] == 1).sum()), "fail": int((v[:, r] == 2).sum()),
             "warn": int((v[:, r] == 3).sum()), "error": int((v[:, r] == 4).sum()), "skip": int((v[:, r] == 5).sum())}
            for r in range(v.shape[1])]


def test_cli_summary_pinned_by_background_report(oracle):
    bg = json.load(open(os.path.join(GOLD, "background_report.json")))
    names = oracle.rule_names([bg["policy"]])
    v = oracle.validate([bg["policy"]], json.dumps(bg["resource"]).encode())
    assert oracle_report.cli_summary([bg["policy"]], names, v) == bg["summary"]
    assert K.cli_summary(K.PolicySet([bg["policy"]]), _counts(v)) == bg["summary"]


@pytest.mark.parametrize("audit_warn", [False, True])
def test_cli_summary_matches_oracle(oracle, audit_warn):
    pols = report_policy_set()
    enf = copy.deepcopy(pols[1])
    enf["metadata"]["name"] = "enforced"
    enf["spec"]["validationFailureAction"] = "Enforce"
    dup = copy.deepcopy(pols[2])  # two rules with one name: each response counts twice
    dup["metadata"]["name"] = "dup-names"
    dup["spec"]["rules"].append(copy.deepcopy(dup["spec"]["rules"][0]))
    pols += [enf, dup]
    ps = K.PolicySet(pols)
    names = oracle.rule_names(pols)
    nd = K.synth_resources(9, 600, mix=2)
    v = oracle.validate(pols, nd, nthreads=4)
    want = oracle_report.cli_summary(pols, names, v, audit_warn)
    assert K.cli_summary(ps, _counts(v), audit_warn) == want
    assert want["warn"] > 0 and want["fail"] > 0


def test_cli_summary_overrides_with_audit_warn_refused():
    pol = copy.deepcopy(report_policy_set()[1])
    pol["spec"]["validationFailureActionOverrides"] = [{"action": "Enforce", "namespaces": ["prod-*"]}]
    ps = K.PolicySet([pol])
    cnt = [{"na": 0, "pass": 0, "fail": 1, "warn": 0, "error": 0, "skip": 0}] * ps.num_rules
    assert K.cli_summary(ps, cnt)["fail"] + K.cli_summary(ps, cnt)["warn"] == ps.num_rules
    with pytest.raises(K.KpeError):
        K.cli_summary(ps, cnt, audit_warn=True)


@pytest.mark.gpu
def test_gpu_cli_summary_matches_oracle(oracle):
    pols = report_policy_set()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(13, 5000, mix=2)
    _, _, cnt = eng.evaluate(ps, K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    for aw in (False, True):
        assert K.cli_summary(ps, cnt, aw) == oracle_report.cli_summary(pols, oracle.rule_names(pols), ref, aw)


@pytest.mark.gpu
def test_gpu_report_chart_policies(oracle):
    """The rendered kyverno-policies chart (device-supported policies: PSS-style pattern rules
    with their category annotations) on mixed kinds: report results and the CLI
    summary from the device equal the oracle's."""
    from tests.test_gpu_pattern import chart_pattern_policies

    pols = chart_pattern_policies()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(0xC1, 3000, mix=2)
    docs = [json.loads(x) for x in nd.split(b"\n") if x.strip()]
    v, _, cnt = eng.evaluate(ps, K.Corpus(nd), check_masks=True)
    names = oracle.rule_names(pols)
    ref = oracle.validate(pols, nd, nthreads=8)
    assert (v == ref).all()
    seen = set()
    for i in range(0, len(docs), 5):
        want = oracle_report.report_results(pols, names, ref[i], docs[i], oracle.failing_checks)
        got = K.report_results(ps, v[i])  # pattern rules: no PSS controls
        assert got == want, (i, got, want)
        seen.update((r["result"], "category" in r) for r in got)
    assert ("fail", True) in seen and ("pass", True) in seen
    assert K.cli_summary(ps, cnt) == oracle_report.cli_summary(pols, names, ref)


def test_deny_message_substitution_pinned(oracle):
    """getDenyMessage's SubstituteAll (validate_resource.go:288-299) pinned by
    pkg/engine/validation_test.go Test_VariableSubstitutionValidate_VariablesInMessageAreResolved:
    the host report and the oracle's both render "The animal cow is not in the allowed list of
    animals." from the resource."""
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "engine_message_cases.json")))
    case = next(c for c in cases if c["name"] == "Test_VariableSubstitutionValidate_VariablesInMessageAreResolved")
    pols, doc = [case["policy"]], case["resource"]
    v = oracle.validate(pols, json.dumps(doc).encode())
    assert int(v[0][0]) == 2
    names = oracle.rule_names(pols)
    got = K.report_results(K.PolicySet(pols), v[0], None, resource=doc)
    want = oracle_report.report_results(pols, names, v[0], doc, oracle.failing_checks, oracle.pss_message,
                                        oracle.substitute)
    assert got[0]["message"] == case["messages"]["0"] == want[0]["message"]


EXC_REPORTS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "report_exception_cases.json")))


def _exc_case_report(case, verdicts):
    pols = [case["policy"]]
    ps = K.PolicySet(pols, exceptions=[case["exception"]], background="background" in case["src"])
    return K.report_results(ps, verdicts, None, resource=case["resource"])


def _check_exc_report(case, got):
    meta = case["exception"]["metadata"]
    key = f"{meta['namespace']}/{meta['name']}" if meta.get("namespace") else meta["name"]
    assert len(got) == len(case["results"]) == 1
    want = dict(case["results"][0])
    assert {k: got[0].get(k) for k in want} == want, (got, want)
    # the RuleSkip message (validate_resource.go:43-55): the chainsaw assert leaves it out
    assert got[0]["message"] == "rule skipped due to policy exception " + key


@pytest.mark.parametrize("case", EXC_REPORTS, ids=lambda c: c["src"].split("/")[-3])
def test_exception_skip_report_fixture(oracle, case):
    """reports/{background,admission}/exception: the excepted ConfigMap's skip result carries the
    exception's name as a property and the RuleSkip message (oracle verdicts, host report)."""
    nd = json.dumps(case["resource"]).encode()
    v = oracle.validate([case["policy"]], nd, exceptions=[case["exception"]])
    assert int(v[0][0]) == 5
    _check_exc_report(case, _exc_case_report(case, v[0]))


@pytest.mark.gpu
@pytest.mark.parametrize("case", EXC_REPORTS, ids=lambda c: c["src"].split("/")[-3])
def test_exception_skip_report_fixture_device(case):
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet([case["policy"]], exceptions=[case["exception"]], background="background" in case["src"])
    v, _, _ = eng.evaluate(ps, K.Corpus(json.dumps(case["resource"]).encode()))
    assert int(v[0, 0]) == 5
    _check_exc_report(case, _exc_case_report(case, v[0]))
