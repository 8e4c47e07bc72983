"""Condition messages: EvaluateConditions' message (variables/evaluate.go:
31-125: the true / false `any` and `all` messages joined by "; ", the old list form's first false
message or its true ones joined by ";"), used by the preconditions skip ("preconditions not met;
<message>", engine.go:282-284, validate_resource.go:128-131) and getDenyMessage
(validate_resource.go:279-300: SubstituteAll of the rule message joined with the deny block's
message; on a substitution error the condition message as is).

The device records where each block stopped (kpe_cond_kernel's condition traces, schema.h CT_*);
kpe_report_results_ex renders the messages on the host.

CPU: the oracle against pkg/engine/variables/evaluate_test.go Test_Condition_Messages (its four
assertions, as preconditions skips and as deny fails) and validation_test.go's deny message case;
the condition VM compiled for the host (scripts/condvm_check.cpp) writes the traces, and
kpe_report_results_ex's messages equal the oracle's on cond_message_policy_set.
GPU: the same through kpe_evaluate + kpe_fetch_cond_traces, and PolicyException skips after
preconditions that held."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import cond_message_policy_set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
NEEDS = "\x01"

# evaluate_test.go:451-517 Test_Condition_Messages: the resource, then (any, all, held, message)
# per assertion; a condition is (key, value, message) under operator Equal
TCM_RESOURCE = {"metadata": {"name": "temp", "namespace": "n1"}, "spec": {"foo": "bar", "foo2": "bar2"}}
_N, _F = "{{request.object.metadata.name}}", "{{request.object.spec.foo}}"
TCM_CASES = [
    ([(_N, "temp2", "invalid name"), (_F, "bar2", "invalid foo")], [], False, "invalid name; invalid foo"),
    ([(_N, "temp", "invalid name"), (_F, "bar", "invalid foo")], [], True, "invalid name"),
    ([(_N, "temp", "invalid name"), (_F, "bar", "invalid foo")],
     [(_N, "temp", "invalid name"), (_F, "bar2", "invalid foo")], False, "invalid foo"),
    ([(_N, "temp1", "invalid name"), (_F, "bar2", "invalid foo")],
     [(_N, "temp", "invalid name"), (_F, "bar2", "invalid foo2")], False, "invalid name; invalid foo; invalid foo2"),
]


def _block(any_, all_):
    cv = lambda cs: [{"key": k, "operator": "Equal", "value": v, "message": m} for k, v, m in cs]
    b = {"any": cv(any_)}
    if all_:
        b["all"] = cv(all_)
    return b


def _tcm_policy(i):
    """Case i as a rule's preconditions (its skip shows a false block's message) and as a deny
    block (its fail shows a true block's message)."""
    any_, all_, _, _ = TCM_CASES[i]
    m = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    rules = [{"name": "pre", "match": m, "preconditions": _block(any_, all_),
              "validate": {"deny": {"conditions": {"all": [{"key": "a", "operator": "Equals", "value": "a"}]}}}},
             {"name": "deny", "match": m, "validate": {"deny": {"conditions": _block(any_, all_)}}}]
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"tcm{i}"},
            "spec": {"validationFailureAction": "Audit", "rules": rules}}


def _tcm_expected(i):
    _, _, held, msg = TCM_CASES[i]
    if held:
        return {"pre": (2, "validation error: rule pre failed"), "deny": (2, msg)}
    return {"pre": (5, "preconditions not met; " + msg), "deny": (1, "validation rule 'deny' passed.")}


def _pod():
    return dict(TCM_RESOURCE, apiVersion="v1", kind="Pod")


@pytest.mark.parametrize("i", range(len(TCM_CASES)))
def test_oracle_condition_messages_match_reference(oracle, i):
    pol = _tcm_policy(i)
    nd = json.dumps(_pod()).encode()
    st = oracle.validate([pol], nd)[0]
    msgs = oracle.pattern_messages([pol], nd)[0]
    for col, name in enumerate(("pre", "deny")):
        want = _tcm_expected(i).get(name)
        if want is None:
            continue
        assert int(st[col]) == want[0], (name, st)
        assert msgs[col] == want[1], (name, msgs[col], want[1])


def test_oracle_deny_message_case(oracle):
    """validation_test.go Test_VariableSubstitutionValidate_VariablesInMessageAreResolved: a deny
    rule's message substituted (getDenyMessage)."""
    case = [c for c in json.load(open(os.path.join(GOLD, "engine_message_cases.json")))
            if c["name"] == "Test_VariableSubstitutionValidate_VariablesInMessageAreResolved"][0]
    nd = json.dumps(case["resource"]).encode()
    st = oracle.validate([case["policy"]], nd)[0]
    msgs = oracle.pattern_messages([case["policy"]], nd)[0]
    resp = [r for r, s in enumerate(st) if s != 0]
    for i, want in case["messages"].items():
        assert msgs[resp[int(i)]] == want


@pytest.mark.parametrize("i", range(len(TCM_CASES)))
def test_host_report_tcm(oracle, i):
    """kpe_report_results_ex with traces as the device writes them for the reference's cases."""
    pol = _tcm_policy(i)
    ps = K.PolicySet([pol])
    nd = json.dumps(_pod()).encode()
    st = oracle.validate([pol], nd)[0]
    any_, all_, held, _ = TCM_CASES[i]
    # where the block stopped: first true any, first false all
    truth = lambda cs: [(TCM_RESOURCE["metadata"]["name"] if k == _N else TCM_RESOURCE["spec"]["foo"]) == v
                        for k, v, _ in cs]
    ta, tl = truth(any_), truth(all_)
    as_ = ta.index(True) if True in ta else len(ta)
    ls = tl.index(False) if False in tl else len(tl)
    word = as_ | ls << 7 | 0x4000 | (0x8000 if held else 0)
    names = [n.split("/", 1)[1] for n in ps.rule_names]  # with the autogen rules
    ct = np.array([word if n == "pre" else word << 16 if n == "deny" else 0 for n in names], dtype=np.uint32)
    res = K.report_results(ps, st, resource=nd, cond_traces=ct)
    got = {r["rule"]: r.get("message") for r in res}
    for name, (_, msg) in _tcm_expected(i).items():
        assert got[name] == msg, (name, got[name], msg)


def _keep_lines(seed, n):
    keep = {"Pod", "Deployment", "Service", "ConfigMap"}
    return [l for l in K.synth_resources(seed, n, mix=2).split(b"\n") if l and json.loads(l)["kind"] in keep]


def _message_rules(pols):
    """Columns whose messages the restatement renders: deny rules (every verdict) and, for every
    rule, preconditions skips."""
    rules = pols[0]["spec"]["rules"]
    deny = {j for j, r in enumerate(rules) if "deny" in r["validate"]}
    pre = {j for j, r in enumerate(rules) if "preconditions" in r}
    return rules, deny, pre


def _compare(pols, ps, verdicts, traces, lines, om):
    rules, deny, pre = _message_rules(pols)
    checked = {"deny": 0, "pre": 0, "tmpl": 0}
    for i, line in enumerate(lines):
        res = K.report_results(ps, verdicts[i], resource=line, cond_traces=traces[i])
        got = {r["rule"]: r.get("message", "") for r in res}
        for j, r in enumerate(rules):
            v = int(verdicts[i, j])
            if v in (0, 7) or (j not in deny and not (j in pre and v == 5)):
                continue
            want = om[i][j]  # (RuleError texts included: the substitution error chain)
            if want == NEEDS:
                assert got[r["name"]] == "", (i, r["name"], got[r["name"]])
                continue
            assert got[r["name"]] == want, (i, r["name"], got[r["name"]], want)
            checked["pre" if v == 5 else "deny"] += 1
            checked["tmpl"] += "{{" in json.dumps(r["validate"].get("message", ""))
    return checked


@pytest.fixture(scope="module")
def condvm_bin():
    from tests.conftest import build_host_tool

    return build_host_tool("condvm_check")


PRE_ONLY = {"pre-ns", "pre-kind-pss", "msg-pre-pattern"}  # other handlers behind per-resource preconditions


def test_host_vm_messages_equal_oracle(condvm_bin, oracle, tmp_path):
    pols = cond_message_policy_set()
    ps = K.PolicySet(pols)
    rules = pols[0]["spec"]["rules"]
    lines = _keep_lines(0xB7, 1500)
    nd = b"\n".join(lines)
    kinds = [json.loads(l)["kind"] for l in lines]
    ref = oracle.validate(pols, nd, nthreads=8)
    N, R = ref.shape
    seedm = np.zeros((N, R), dtype=np.uint8)
    for j, r in enumerate(rules):
        rk = set(r["match"]["any"][0]["resources"]["kinds"])
        for i, k in enumerate(kinds):
            if k in rk:
                seedm[i, j] = 3 if r["name"] in PRE_ONLY else 6
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(nd)
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([condvm_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"),
                           str(tmp_path / "seed.bin"), str(tmp_path / "out.bin"), str(tmp_path / "ct.bin")])
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    ct = np.frombuffer((tmp_path / "ct.bin").read_bytes(), dtype=np.uint32).reshape(N, R)
    for j, r in enumerate(rules):
        if r["name"] not in PRE_ONLY:
            assert (out[:, j] == ref[:, j]).all(), r["name"]
    om = oracle.pattern_messages(pols, nd)
    checked = _compare(pols, ps, ref, ct, lines, om)
    assert checked["deny"] > 2000 and checked["pre"] > 300 and checked["tmpl"] > 200, checked


def test_folded_preconditions_message(oracle):
    """Preconditions that fold at compile time (request.operation): the skip message is static."""
    m = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    pre = {"any": [{"key": "{{ request.operation }}", "operator": "Equals", "value": "DELETE", "message": "not delete"},
                   {"key": "{{ request.operation }}", "operator": "Equals", "value": "UPDATE", "message": "not update"}],
           "all": [{"key": "{{ request.operation }}", "operator": "NotEquals", "value": "CONNECT", "message": "x"}]}
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "f"},
           "spec": {"rules": [{"name": "r", "match": m, "preconditions": pre,
                               "validate": {"message": "m", "pattern": {"metadata": {"name": "?*"}}}},
                              {"name": "d", "match": m, "validate": {"message": "deny {{ request.object.kind }}",
                                                                     "deny": {"conditions": pre}}}]}}
    nd = json.dumps(_pod()).encode()
    st = oracle.validate([pol], nd)[0]
    om = oracle.pattern_messages([pol], nd)[0]
    ps = K.PolicySet([pol])
    res = K.report_results(ps, st, resource=nd)
    assert [int(x) for x in st[:2]] == [5, 1]
    assert res[0]["message"] == om[0] == "preconditions not met; not delete; not update"
    assert res[1]["message"] == om[1] == "validation rule 'd' passed."


# ---- device ----------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("i", range(len(TCM_CASES)))
def test_device_tcm_messages(i):
    pol = _tcm_policy(i)
    nd = json.dumps(_pod()).encode()
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet([pol]), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    ct = eng.cond_traces(ps, corpus)
    res = K.report_results(ps, v[0], resource=nd, cond_traces=ct[0])
    got = {r["rule"]: (r["result"], r.get("message")) for r in res}
    for name, (st, msg) in _tcm_expected(i).items():
        assert got[name] == ({1: "pass", 2: "fail", 5: "skip"}[st], msg), (name, got[name])


@pytest.mark.gpu
def test_device_condition_messages_equal_oracle(oracle):
    pols = cond_message_policy_set()
    lines = _keep_lines(0xB8, 3000)
    nd = b"\n".join(lines)
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet(pols), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    ref = oracle.validate(pols, nd, nthreads=8)
    assert (v == ref).all()
    ct = eng.cond_traces(ps, corpus)
    assert (eng.cond_traces(ps, corpus, 7, 5) == ct[7:12]).all()
    om = oracle.pattern_messages(pols, nd)
    checked = _compare(pols, ps, v, ct, lines, om)
    assert checked["deny"] > 4000 and checked["pre"] > 600, checked


@pytest.mark.gpu
def test_device_exception_skip_after_preconditions(oracle):
    """A PolicyException on a rule whose preconditions read the resource: a skip is the
    exception's only once the trace shows the preconditions held (engine.go:278-293)."""
    m = {"any": [{"resources": {"kinds": ["Pod"]}}]}
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "x"},
           "spec": {"rules": [{"name": "r", "match": m,
                               "preconditions": {"all": [{"key": "{{ request.object.metadata.namespace }}",
                                                          "operator": "NotEquals", "value": "ns-01*",
                                                          "message": "not ns-01*"}]},
                               "validate": {"deny": {"conditions": {"all": [
                                   {"key": "{{ request.object.metadata.name }}", "operator": "Equals",
                                    "value": "res-*"}]}}}}]}}
    exc = {"apiVersion": "kyverno.io/v2beta1", "kind": "PolicyException", "metadata": {"name": "e", "namespace": "k"},
           "spec": {"exceptions": [{"policyName": "x", "ruleNames": ["r"]}],
                    "match": {"any": [{"resources": {"kinds": ["Pod"], "names": ["res-1*"]}}]}}}
    lines = [l for l in K.synth_resources(0xE1, 600, mix=2).split(b"\n") if l and json.loads(l)["kind"] == "Pod"]
    nd = b"\n".join(lines)
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet([pol], exceptions=[exc]), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    ct = eng.cond_traces(ps, corpus)
    n_pre = n_exc = 0
    for i, line in enumerate(lines):
        if v[i, 0] != 5:
            continue
        res = K.report_results(ps, v[i], resource=line, cond_traces=ct[i])
        ns = json.loads(line)["metadata"].get("namespace")
        if not ns.startswith("ns-01"):  # preconditions held: the exception's skip
            assert res[0]["message"] == "rule skipped due to policy exception k/e", res[0]
            assert res[0]["properties"] == {"exception": "e"}
            n_exc += 1
        else:
            assert res[0]["message"] == "preconditions not met; not ns-01*", res[0]
            assert "properties" not in res[0]
            n_pre += 1
    assert n_pre and n_exc
