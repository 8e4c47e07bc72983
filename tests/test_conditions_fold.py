"""Preconditions and deny conditions folded at compile time (request.operation = CREATE and
letter-only literals; validate_resource.go:121-132, 268-279, variables/evaluate.go).

CPU: which conditions kpe_program_compile folds and which it refuses (KPE_E_UNSUPPORTED).
GPU: the constant verdicts (skip / fail / pass) land in the matrix bit-exact against the
oracle's condition engine (oracle/conditions.hpp) on synthetic corpora."""
import copy

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import pss_policy

OP = "{{ request.operation }}"


def _rule(name, pre=None, validate=None, kinds=("Pod",)):
    r = {"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
         "validate": validate or {"message": "m", "deny": {}}}
    if pre is not None:
        r["preconditions"] = pre
    return r


def _policy(name, rules):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}


PATTERN = {"message": "m", "pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}


def folded_policy_set():
    rules = [
        _rule("deny-empty"),  # deny {} => fail
        _rule("deny-op-true", validate={"deny": {"conditions": {"any": [{"key": OP, "operator": "Equals",
                                                                           "value": "CREATE"}]}}}),
        _rule("deny-op-false", validate={"deny": {"conditions": {"all": [{"key": OP, "operator": "AnyIn",
                                                                           "value": ["DELETE", "CONNECT"]}]}}}),
        _rule("deny-list-form", validate={"deny": {"conditions": [{"key": OP, "operator": "NotEquals",
                                                                    "value": "UPDATE"}]}}),
        _rule("pre-true-pattern", pre={"all": [{"key": OP, "operator": "AllIn", "value": ["CREATE", "UPDATE"]}]},
              validate=PATTERN),
        _rule("pre-false-pattern", pre={"any": [{"key": OP, "operator": "Equals", "value": "DELETE"}]},
              validate=PATTERN),
        _rule("pre-false-deny", pre=[{"key": OP, "operator": "In", "value": ["UPDATE"]}]),
        _rule("pre-empty-any", pre={"any": []}, validate=PATTERN),  # non-nil empty any => false => skip
        _rule("pre-empty-block", pre={}, validate=PATTERN),  # no any / all => true
        _rule("pre-glob-eq", pre={"all": [{"key": OP, "operator": "Equals", "value": "CRE*"}]}),
        _rule("pre-glob-miss", pre={"all": [{"key": OP, "operator": "Equals", "value": "UPD?TE"}]}),
        _rule("deny-glob-in", validate={"deny": {"conditions": {"any": [{"key": OP, "operator": "AnyIn",
                                                                           "value": ["DEL*", "C?EATE"]}]}}}),
        _rule("deny-glob-notin", validate={"deny": {"conditions": {"all": [{"key": OP, "operator": "NotIn",
                                                                             "value": "*"}]}}}),
        _rule("pre-notin", pre={"all": [{"key": OP, "operator": "NotIn", "value": ["DELETE"]}]}),
        _rule("deny-ctrl", kinds=("Deployment", "CronJob"),
              validate={"deny": {"conditions": {"any": [{"key": OP, "operator": "anynotin", "value": ["CREATE"]}]}}}),
        # scalar string values that are not JSON: in.go / notin.go report an invalid type
        # (both false), anyin.go & co. read them as a one-element list
        _rule("pre-notin-scalar", pre={"all": [{"key": OP, "operator": "NotIn", "value": "DELETE"}]}),
        _rule("pre-in-scalar", pre={"all": [{"key": OP, "operator": "In", "value": "DELETE"}]}),
        _rule("pre-anynotin-scalar", pre={"all": [{"key": OP, "operator": "AnyNotIn", "value": "DELETE"}]}),
        _rule("pre-notin-null", pre={"all": [{"key": OP, "operator": "NotIn", "value": "null"}]}),
        _rule("pre-allnotin-true", pre={"all": [{"key": OP, "operator": "AllNotIn", "value": "true"}]}),
        # a validate block with no handler still skips on false preconditions (validation.go:52)
        _rule("pre-false-message-only", pre={"all": [{"key": OP, "operator": "Equals", "value": "DELETE"}]},
              validate={"message": "m"}),
    ]
    pols = [_policy("folded", rules)]
    p = pss_policy("pre-pss", "restricted", "latest", kinds=("Pod",))
    p["spec"]["rules"][0]["preconditions"] = {"all": [{"key": OP, "operator": "Equals", "value": "DELETE"}]}
    pols.append(p)
    p = pss_policy("pre-pss-true", "baseline", "v1.24", kinds=("Pod", "Deployment"))
    p["spec"]["rules"][0]["preconditions"] = {"any": [{"key": OP, "operator": "Equals", "value": "CREATE"}]}
    pols.append(p)
    # autogen: a Pod rule with folded preconditions expands to Deployment/CronJob rules
    pols.append(_policy("autogen", [_rule("deny-pod", pre={"all": [{"key": OP, "operator": "Equals",
                                                                       "value": "CREATE"}]})]))
    return pols


def test_fold_compiles():
    ps = K.PolicySet(folded_policy_set())
    assert ps.num_rules >= 14
    assert any(n.startswith("autogen/autogen-") for n in ps.rule_names)


# Expected verdicts restated from the reference operators on key "CREATE" (CPU, oracle only):
# in.go:60-92 keyExistsInArray, notin.go:45-53, anyin.go:61-101, allnotin.go:43-50.
# 1 = pass (deny false), 2 = fail (deny true), 5 = skip (preconditions false).
@pytest.mark.parametrize("op,value,want", [
    ("NotIn", "DELETE", 5),          # not JSON => invalid type => NotIn false => preconditions skip
    ("In", "DELETE", 5),
    ("AnyNotIn", "DELETE", 2),       # json.Valid fails => ["DELETE"] => CREATE not in => true
    ("NotIn", "null", 2),            # null decodes to an empty list => NotIn true
    ("AllNotIn", "true", 5),         # valid JSON, not a []string => invalid => false
    ("NotIn", ["DELETE"], 2),
    ("In", ["CRE*"], 2),
    ("In", ["*EATE", "x"], 2),
])
def test_oracle_in_notin_semantics(oracle, op, value, want):
    pol = _policy("p", [_rule("r", pre={"all": [{"key": OP, "operator": op, "value": value}]})])
    nd = b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"a","namespace":"d"},"spec":{}}'
    assert int(oracle.validate([pol], nd)[0, 0]) == want


def test_oracle_in_list_key_semantics(oracle):
    """in.go:35-40 / setExistsInArray :108-140: a one-element key list equal to a string value
    reports keyExists, so NotIn is true there (notin.go:55-63); list values match exactly."""
    def deny(op, key, value):
        return _rule("r", validate={"deny": {"conditions": {"all": [{"key": key, "operator": op, "value": value}]}}})
    nd = b'{"apiVersion":"v1","kind":"Pod","metadata":{"name":"web","namespace":"d"},"spec":{}}'
    name = "{{ request.object.metadata.name }}"
    cases = [("NotIn", [name], "web", 2), ("In", [name], "web", 2), ("In", [name], ["we*"], 1),
             ("NotIn", [name], ["we*"], 2), ("In", [name], ["web", "x"], 2), ("NotIn", [name], "[1]", 1)]
    for op, key, value, want in cases:
        assert int(oracle.validate([_policy("p", [deny(op, key, value)])], nd)[0, 0]) == want, (op, key, value)


@pytest.mark.parametrize("cond", [
    {"all": [{"key": OP, "operator": "Equals", "value": "$(./x)"}]},  # a $(...) reference
])
def test_unfoldable_refused(cond):
    for pol in (_policy("p", [_rule("r", pre=cond, validate=PATTERN)]),
                _policy("p", [_rule("r", validate={"deny": {"conditions": cond}})])):
        with pytest.raises(K.KpeError):
            K.PolicySet([pol])


@pytest.mark.parametrize("cond", [
    {"all": [{"key": "{{ request.object.metadata.name }}", "operator": "Equals", "value": "x"}]},
    {"all": [{"key": "CRE*", "operator": "Equals", "value": OP}]},          # glob key
    {"all": [{"key": OP, "operator": "AnyIn", "value": ["a-b"]}]},          # range text inside a list
    {"all": [{"key": "1Gi", "operator": "Equals", "value": "1024Mi"}]},       # quantities
    {"all": [{"key": "{{ request.operation || 'BACKGROUND' }}", "operator": "NotEquals", "value": "DELETE"}]},
])
def test_unfoldable_compiled_per_resource(cond):
    """Not folded at compile time: evaluated per resource by kpe_cond_kernel instead."""
    for pol in (_policy("p", [_rule("r", pre=cond, validate=PATTERN)]),
                _policy("p", [_rule("r", validate={"deny": {"conditions": cond}})])):
        K.PolicySet([pol])


RES_COND = {"any": [{"key": "{{ request.object.spec.hostNetwork || `false` }}", "operator": "Equals",
                     "value": True}]}


def apply_one_policy_set():
    """applyRules: One policies whose rules mix every handler the device has: constant (folded)
    conditions, PSS with and without exclusions, patterns, resource-reading preconditions and
    deny (validation.go:75-77 stops after the first pass / fail response)."""
    one = []
    one.append(_policy("one-folded", [_rule("a"), _rule("b", validate=PATTERN)]))
    one.append(_policy("one-pattern-first", [
        _rule("img", validate=PATTERN),
        _rule("pss", validate={"podSecurity": {"level": "restricted", "version": "latest"}}),
        _rule("deny", validate={"deny": {"conditions": RES_COND}})]))
    one.append(_policy("one-cond-first", [
        _rule("hostnet", pre=RES_COND, validate=PATTERN),
        _rule("deny-hostnet", validate={"deny": {"conditions": RES_COND}}),
        _rule("pss", validate={"podSecurity": {"level": "baseline", "version": "latest"}})]))
    one.append(_policy("one-pssx", [
        _rule("pss-excl", validate={"podSecurity": {"level": "baseline", "version": "latest", "exclude": [
            {"controlName": "Host Namespaces"}, {"controlName": "Host Ports", "images": ["*nginx*"]}]}}),
        _rule("img", validate=PATTERN),
        _rule("pre-false", pre={"any": [{"key": OP, "operator": "Equals", "value": "DELETE"}]}, validate=PATTERN)]))
    one.append(_policy("one-kinds", [
        _rule("deploy-only", kinds=("Deployment",), validate=PATTERN),
        _rule("pods", kinds=("Pod", "Deployment"), validate={"podSecurity": {"level": "restricted", "version": "v1.24"}}),
        _rule("last", validate={"deny": {}})]))
    for p in one:
        p["spec"]["applyRules"] = "One"
    return one


def test_apply_one_compiles():
    K.PolicySet(apply_one_policy_set())


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 6000, 0xA1), (2, 6000, 0xA2)])
def test_apply_one_bit_exact(oracle, mix, n, seed):
    pols = apply_one_policy_set()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, cnt = eng.evaluate(ps, K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} {v[tuple(bad[0])]} {ref[tuple(bad[0])]}"
    # ApplyOne really cut rules: some row has a later rule without response after an applied one
    assert ((v[:, 0] == 2) & (v[:, 1] == 0)).any() or ((v[:, 0] == 1) & (v[:, 1] == 0)).any()
    for r in range(v.shape[1]):
        assert cnt[r]["na"] == int((v[:, r] == 0).sum())


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 4000, 0xC2), (2, 4000, 31)])
def test_folded_conditions_bit_exact(oracle, mix, n, seed):
    pols = folded_policy_set()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, cnt = eng.evaluate(ps, K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} {v[tuple(bad[0])]} {ref[tuple(bad[0])]}"
    assert {1, 2, 5} <= set(np.unique(v).tolist())  # pass, fail and skip all occur
    for r in range(v.shape[1]):
        assert cnt[r]["skip"] == int((v[:, r] == 5).sum())


@pytest.mark.gpu
def test_folded_with_wide_program(oracle):
    """Many distinct match terms push the program off the narrow / truth-table paths."""
    pols = folded_policy_set()
    for i in range(40):
        p = copy.deepcopy(pols[0])
        p["metadata"]["name"] = f"folded-{i}"
        for r in p["spec"]["rules"]:
            r["match"]["any"][0]["resources"]["names"] = [f"res-{i}*"]
        pols.append(p)
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = K.synth_resources(5, 3000, mix=2)
    v, _, _ = eng.evaluate(ps, K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
