"""PolicyExceptions (kyverno.io/v2beta1; pkg/engine/exceptions.go:12-35, engine.go:286-293,
pkg/engine/utils/exceptions.go:14-47 MatchesException, pkg/utils/match/match.go:26-193).

CPU: the oracle against the chainsaw exception scenarios (tests/golden/chainsaw_exceptions.json:
an Enforce policy + exception, resources expected to be admitted or rejected), and what
kpe_program_compile_ex accepts or refuses.
GPU: the device against the same scenarios and bit-exact against the oracle on synthetic corpora
with exceptions of every supported shape."""
import copy
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import pss_policy

GOLD = os.path.join(os.path.dirname(__file__), "golden", "chainsaw_exceptions.json")
FAIL, SKIP = 2, 5


def _cases():
    with open(GOLD) as f:
        return json.load(f)


def _pss_exc(c):
    return any((x.get("spec") or {}).get("podSecurity") for x in c["exceptions"])


def test_oracle_chainsaw_exceptions(oracle):
    """Admitted <=> no rule fails, podSecurity exceptions (ApplyPodSecurityExclusion after
    convertChecks, validate_pss.go:88-104) included."""
    n = npss = 0
    for c in _cases():
        v = oracle.validate([c["policy"]], json.dumps(c["resource"]).encode(), exceptions=c["exceptions"])[0]
        assert 7 not in v.tolist(), c["file"]
        rejected = FAIL in v.tolist()
        assert rejected == (c["expect"] == "rejected"), (c["file"], v.tolist())
        n += 1
        npss += _pss_exc(c)
    assert n >= 8 and npss >= 4


NS_POL = "ns-0001"


def _cpol(name, rules, kind="ClusterPolicy", ns=None):
    meta = {"name": name}
    if ns:
        meta["namespace"] = ns
    return {"apiVersion": "kyverno.io/v1", "kind": kind, "metadata": meta,
            "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}


def _rule(name, kinds=("Pod",), validate=None, pre=None):
    r = {"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
         "validate": validate or {"message": "m", "pattern": {"metadata": {"labels": {"team": "?*"}}}}}
    if pre is not None:
        r["preconditions"] = pre
    return r


def _exc(name, refs, match=None, ns=None, **spec):
    meta = {"name": name}
    if ns:
        meta["namespace"] = ns
    sp = {"exceptions": [{"policyName": p, "ruleNames": list(r)} for p, r in refs]}
    if match is not None:
        sp["match"] = match
    sp.update(spec)
    return {"apiVersion": "kyverno.io/v2beta1", "kind": "PolicyException", "metadata": meta, "spec": sp}


def _any(*rds):
    return {"any": [{"resources": rd} for rd in rds]}


def exception_set():
    """Policies (PSS, pattern, deny, folded conditions, autogen) and exceptions of every shape the
    device evaluates: names / namespaces / selector / namespaceSelector / annotations filters,
    `all` blocks, an empty match (always), userInfo (never in a scan), several exceptions on one
    rule, wildcard and autogen rule names, a namespaced Policy key, background: false."""
    restricted = pss_policy("restricted", "restricted", "latest", kinds=("Pod", "Deployment"))
    baseline = pss_policy("baseline", "baseline", "latest")
    pols = [
        restricted,
        baseline,
        _cpol("labels", [_rule("require-team", kinds=("Pod", "ConfigMap", "Deployment")),
                         _rule("deny-cm", kinds=("ConfigMap",), validate={"deny": {}}),
                         _rule("app-pods", validate={"message": "m", "pattern": {
                             "metadata": {"labels": {"app": "app-1*"}}}})]),
        _cpol("folded", [_rule("pre-op", pre={"all": [{"key": "{{ request.operation }}", "operator": "Equals",
                                                        "value": "CREATE"}]},
                               validate={"message": "m", "deny": {}})]),
        _cpol("nsd", [_rule("ns-rule", kinds=("Pod",))], kind="Policy", ns=NS_POL),
        # deny / foreach-deny rules whose conditions read the resource (kpe_cond_kernel): an
        # exception's RuleSkip must survive the condition pass (validate_resource.go:44-56)
        _cpol("dyn-deny", [
            _rule("deny-name", kinds=("Pod", "ConfigMap"), validate={"message": "m", "deny": {"conditions": {"any": [
                {"key": "{{ request.object.metadata.name }}", "operator": "Equals", "value": "res-*"}]}}}),
            _rule("fe-deny", kinds=("Pod",), validate={"message": "m", "foreach": [{
                "list": "request.object.spec.containers",
                "deny": {"conditions": {"any": [{"key": "{{ element.name }}", "operator": "NotEquals",
                                                 "value": "zz-*"}]}}}]})]),
    ]
    rname = restricted["spec"]["rules"][0]["name"]
    bname = baseline["spec"]["rules"][0]["name"]
    rpol, bpol = restricted["metadata"]["name"], baseline["metadata"]["name"]
    excs = [
        _exc("by-name", [(rpol, [rname, "autogen-" + rname])],
             _any({"kinds": ["Pod", "Deployment"], "names": ["res-1*", "res-2?"]})),
        _exc("by-ns", [(bpol, ["*"])], _any({"namespaces": ["ns-00*"]}, {"namespaces": ["ns-1?3"]})),
        _exc("by-sel", [("labels", ["require-*"])], _any({"kinds": ["ConfigMap"], "selector": {
            "matchLabels": {"tier": "front*"}}})),
        _exc("by-ann-all", [("labels", ["app-pods"])],
             {"all": [{"resources": {"kinds": ["Pod"]}}, {"resources": {"annotations": {"owner": "team-1*"}}}]}),
        _exc("always", [("labels", ["deny-cm"])]),  # no match block: every resource
        _exc("users-only", [("folded", ["pre-op"])], {"any": [{"resources": {"kinds": ["Pod"]},
                                                              "subjects": [{"kind": "User", "name": "x"}]}]}),
        _exc("nssel", [("folded", ["pre-op"])], _any({"kinds": ["*"], "namespaceSelector": {
            "matchExpressions": [{"key": "env", "operator": "In", "values": ["prod"]}]}})),
        _exc("ns-key", [(NS_POL + "/nsd", ["ns-rule"])], _any({"kinds": ["Pod"], "names": ["res-*3"]}), ns=NS_POL),
        _exc("wrong-key", [("nsd", ["ns-rule"])], _any({"kinds": ["Pod"]})),  # the key is ns/name
        _exc("no-bg", [(rpol, [rname])], _any({"kinds": ["Pod"], "names": ["res-3*"]}), background=False),
        _exc("folded-cond", [(bpol, ["autogen-" + bname])], _any({"names": ["res-4*"]}),
             conditions={"all": [{"key": "{{ request.operation }}", "operator": "Equals", "value": "CREATE"}]}),
        _exc("dyn-deny-x", [("dyn-deny", ["deny-name", "fe-*"])], _any({"namespaces": ["ns-0*"]})),
    ]
    # exceptions whose conditions read the resource (CheckAnyAllConditions after the match,
    # exceptions.go:33-41: error or false => no exception) and rules whose preconditions read it
    # (preconditions first, engine.go:278-293): kpe_cond_kernel applies them (XE_DEFER)
    pols += [
        pss_policy("cond-pss", "baseline", "latest", kinds=("Pod", "Deployment")),
        _cpol("cond-rules", [
            _rule("team-label", kinds=("Pod", "ConfigMap", "Deployment")),
            _rule("deny-many", kinds=("Pod",), validate={"message": "m", "deny": {"conditions": {"any": [
                {"key": "{{ request.object.spec.containers[] | length(@) }}", "operator": "GreaterThan",
                 "value": "1"}]}}}),
            _rule("pre-dyn", kinds=("Pod", "ConfigMap"), pre={"any": [
                {"key": "{{ request.object.metadata.labels.tier || '' }}", "operator": "NotEquals", "value": ""}]},
                validate={"message": "m", "pattern": {"metadata": {"labels": {"app": "?*"}}}}),
            _rule("pre-dyn-deny", kinds=("Pod",), pre={"all": [
                {"key": "{{ length(request.object.metadata.name) }}", "operator": "GreaterThan", "value": 5}]},
                validate={"message": "m", "deny": {"conditions": {"any": [
                    {"key": "{{ request.object.metadata.namespace }}", "operator": "Equals", "value": "ns-00*"}]}}}),
        ]),
    ]
    excs += [
        _exc("cond-pss-x", [("pol-cond-pss", ["*"])], _any({"kinds": ["Pod", "Deployment"]}), conditions={"any": [
            {"key": "{{ request.object.metadata.labels.tier || '' }}", "operator": "Equals", "value": "front*"}]}),
        _exc("cond-team", [("cond-rules", ["team-label", "autogen-team-label"])], _any({"kinds": ["*"]}),
             conditions={"all": [{"key": "{{ request.object.metadata.name }}", "operator": "Equals", "value": "res-*1"}],
                         "any": []}),
        _exc("cond-many", [("cond-rules", ["deny-many"])], None, conditions={"any": [
            {"key": "{{ request.object.spec.containers[0].image }}", "operator": "Equals", "value": "*:latest"},
            {"key": "{{ request.object.spec.nope.deeper }}", "operator": "Equals", "value": "x"}]}),
        _exc("pre-dyn-x", [("cond-rules", ["pre-dyn", "pre-dyn-deny"])], _any({"namespaces": ["ns-0*"]})),
    ]
    return pols, excs


def test_compile_accepts_and_refuses():
    pols, excs = exception_set()
    K.PolicySet(pols, excs)
    K.PolicySet(pols, excs, background=True)
    pss = _exc("pss", [("pol-baseline", ["*"])], _any({"kinds": ["Pod"]}),
               podSecurity=[{"controlName": "Host Ports"}])
    K.PolicySet(pols, [pss])
    with pytest.raises(K.KpeError):  # several exceptions on one PSS rule, one with podSecurity
        K.PolicySet(pols, [pss, _exc("pss2", [("pol-baseline", ["*"])], _any({"kinds": ["Pod"]}))])
    cond = _exc("cond", [("pol-baseline", ["*"])], _any({"kinds": ["Pod"]}), conditions={"any": [
        {"key": "{{ request.object.metadata.labels.color || '' }}", "operator": "Equals", "value": "blue"}]})
    K.PolicySet(pols, [cond])  # resource-reading conditions: deferred to kpe_cond_kernel
    with pytest.raises(K.KpeError):  # several exceptions on a rule, one with conditions: the first decides
        K.PolicySet(pols, [cond, _exc("plain", [("pol-baseline", ["*"])], _any({"kinds": ["Pod"]}))])
    dyn = _cpol("dyn", [_rule("r", pre={"all": [{"key": "{{ request.object.metadata.name }}", "operator": "Equals",
                                                 "value": "x"}]})])
    K.PolicySet(pols + [dyn], [_exc("d", [("dyn", ["r"])], _any({"kinds": ["Pod"]}))])
    with pytest.raises(K.KpeError):  # a pipe other than `| length(@)`
        K.PolicySet(pols, [_exc("p", [("pol-baseline", ["*"])], _any({"kinds": ["Pod"]}), conditions={"any": [
            {"key": "{{ request.object.spec.containers | [0] }}", "operator": "Equals", "value": "x"}]})])
    # an exception that names no compiled rule changes nothing and compiles
    K.PolicySet(pols, [_exc("none", [("missing", ["*"])], _any({"kinds": ["Pod"]}))])


def test_oracle_exception_set_has_skips(oracle):
    pols, excs = exception_set()
    nd = K.synth_resources(7, 3000, mix=2)
    nsl = K.synth_ns_labels(7, 1000, mix=2)
    ref = oracle.validate(pols, nd, ns_labels=nsl, nthreads=8, exceptions=excs)
    base = oracle.validate(pols, nd, ns_labels=nsl, nthreads=8)
    changed = ref != base
    assert changed.any()
    assert set(np.unique(ref[changed]).tolist()) == {SKIP}  # an exception only ever skips
    bg = oracle.validate(pols, nd, ns_labels=nsl, nthreads=8, exceptions=excs, background=True)
    assert (bg != ref).any()  # the background: false exception is dropped


@pytest.mark.gpu
def test_gpu_chainsaw_exceptions(oracle):
    eng = K.Engine(ordinal=0)
    n = 0
    for c in _cases():  # every scenario compiles, conditions included
        ps = K.PolicySet([c["policy"]], c["exceptions"])
        v, _, _ = eng.evaluate(ps, K.Corpus(json.dumps(c["resource"]).encode()))
        assert (FAIL in v[0].tolist()) == (c["expect"] == "rejected"), (c["file"], v[0].tolist())
        n += 1
    assert n == len(_cases()) and n >= 10


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed,background", [(0, 8000, 0xE1, False), (2, 8000, 0xE2, False),
                                                   (2, 8000, 0xE3, True)])
def test_gpu_exceptions_bit_exact(oracle, mix, n, seed, background):
    pols, excs = exception_set()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols, excs, background=background)
    nd = K.synth_resources(seed, n, mix=mix)
    nsl = K.synth_ns_labels(seed, 1000, mix=mix)
    v, _, _ = eng.evaluate(ps, K.Corpus(nd, nsl))
    ref = oracle.validate(pols, nd, ns_labels=nsl, nthreads=8, exceptions=excs, background=background)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} {v[tuple(bad[0])]} {ref[tuple(bad[0])]}"
    assert (v == SKIP).any()


@pytest.mark.gpu
def test_gpu_exceptions_wide_program(oracle):
    """Many distinct terms: the WIDE (transposed) rule path evaluates the exception blocks."""
    pols, excs = exception_set()
    for i in range(30):
        p = copy.deepcopy(pols[2])
        p["metadata"]["name"] = f"labels-{i}"
        for r in p["spec"]["rules"]:
            r["match"]["any"][0]["resources"]["names"] = [f"res-{i}*"]
        pols.append(p)
        excs.append(_exc(f"x-{i}", [(f"labels-{i}", ["*"])], _any({"namespaces": [f"ns-0{i % 10}*"]})))
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols, excs)
    nd = K.synth_resources(11, 4000, mix=2)
    v, _, _ = eng.evaluate(ps, K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8, exceptions=excs)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} {v[tuple(bad[0])]} {ref[tuple(bad[0])]}"
