"""Preconditions, deny and foreach-deny conditions that read the resource, evaluated per
resource on the device (kpe_cond_kernel over the compiled condition program; SURVEY.md 8(a)
A14-A17, V1, V2, V4).

CPU: what kpe_program_compile accepts / refuses (KPE_E_UNSUPPORTED).
GPU: bit-exact verdict matrices against the oracle's condition engine (oracle/conditions.hpp,
pinned by the reference's validation_test.go deny / foreach tests and test/cli/test scenarios)
on synthetic corpora; every chart policy (including the deny / foreach ones) on the C1 mix."""
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import cond_policy_set

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CHART = json.load(open(os.path.join(GOLD, "chart_policies.json")))


def _pol(rule):
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "p"},
            "spec": {"validationFailureAction": "Audit", "rules": [rule]}}


def _deny(cond):
    return _pol({"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                 "validate": {"deny": {"conditions": {"all": [cond]}}}})


def test_chart_policies_all_compile():
    pols = CHART["baseline"] + CHART["restricted"]
    ps = K.PolicySet(pols)
    assert ps.num_rules >= 19 * 3 - 6


def test_condition_set_compiles(oracle):
    pols = cond_policy_set()
    assert K.PolicySet(pols).rule_names == oracle.rule_names(pols)


@pytest.mark.parametrize("cond", [
    {"key": "{{ request.object.metadata.labels | keys(@) }}", "operator": "Equals", "value": []},  # pipe
    {"key": "{{ request.userInfo.username }}", "operator": "AnyIn", "value": ["x"]},          # context value
    {"key": "{{ request.object.spec.containers[*].* }}", "operator": "AnyIn", "value": ["x"]},  # nested `.*`
    {"key": "{{ request.object.spec.containers[?name == 'a'] }}", "operator": "Equals", "value": []},  # filter
    {"key": "{{ to_upper(request.object.metadata.name) }}", "operator": "Equals", "value": "A"},  # function
    {"key": "{{ request.object.spec.containers | [0] }}", "operator": "Equals", "value": "a"},  # pipe
    {"key": "{{ request.object.spec.containers | length(@) || `0` }}", "operator": "Equals", "value": 1},
    {"key": "$(./name)", "operator": "Equals", "value": "a"},                                  # reference
    {"key": "{{ divide('{{ request.object.spec.replicas }}', '2') }}", "operator": "Equals", "value": 1},  # nested
    {"key": "{{ request.object.metadata }}", "operator": "Equals", "value": {"a": 1}},        # object value
])
def test_outside_subset_refused(cond):
    with pytest.raises(K.KpeError) as e:
        K.PolicySet([_deny(cond)])
    assert e.value.status == 2


def test_foreach_context_entries_refused():
    r = {"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
         "validate": {"foreach": [{"list": "request.object.spec.containers", "context": [{"name": "x", "variable": {
             "value": 1}}], "pattern": {"name": "*"}}]}}
    with pytest.raises(K.KpeError):
        K.PolicySet([_pol(r)])


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 20000, 0xA1), (1, 20000, 0xA2), (2, 20000, 0xA3)])
def test_conditions_bit_exact(oracle, mix, n, seed):
    pols = cond_policy_set()
    eng = K.Engine(ordinal=0)
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, cnt = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    assert (v == 7).sum() == 0, "no cell of these corpora is beyond the device's limits"
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} " \
                          f"gpu={[int(v[i, j]) for i, j in bad[:5]]} ref={[int(ref[i, j]) for i, j in bad[:5]]}"
    assert (v == 6).sum() == 0
    for r in range(v.shape[1]):
        col = v[:, r]
        assert cnt[r]["fail"] == int((col == 2).sum()) and cnt[r]["error"] == int((col == 4).sum())
        assert cnt[r]["skip"] == int((col == 5).sum()) and cnt[r]["undecided"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 20000, 0xC1), (2, 20000, 0xC7)])
def test_full_chart_bit_exact(oracle, mix, n, seed):
    """All 17 chart policies (19 rules + autogen), deny / foreach ones included."""
    pols = CHART["baseline"] + CHART["restricted"]
    eng = K.Engine(ordinal=0)
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} " \
                          f"gpu={[int(v[i, j]) for i, j in bad[:5]]} ref={[int(ref[i, j]) for i, j in bad[:5]]}"
    assert (v == 7).sum() == 0 and (v == 6).sum() == 0


@pytest.mark.gpu
def test_condition_list_overflow_is_undecided(oracle):
    """A foreach list longer than the VM's list capacity gives KPE_UNDECIDED cells for that
    row only; the other rows stay bit-exact."""
    pol = _pol({"name": "r", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                "validate": {"foreach": [{"list": "request.object.spec.containers[].name",
                                          "deny": {"conditions": {"all": [{"key": "{{ element }}",
                                                                           "operator": "Equals", "value": "x"}]}}}]}})
    big = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "big", "namespace": "d"},
           "spec": {"containers": [{"name": f"c{i}", "image": "a"} for i in range(100)]}}
    small = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "s", "namespace": "d"},
             "spec": {"containers": [{"name": "x", "image": "a"}]}}
    nd = "\n".join(json.dumps(d) for d in (small, big, small)).encode()
    v, _, cnt = K.Engine(ordinal=0).evaluate(K.PolicySet([pol]), K.Corpus(nd))
    ref = oracle.validate([pol], nd)
    assert v[1, 0] == 7 and cnt[0]["undecided"] == 1
    assert v[0, 0] == ref[0, 0] and v[2, 0] == ref[2, 0]
