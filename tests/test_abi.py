"""CPU-only checks of the C-ABI library: it loads, exports every symbol the
headers declare, and its host half (policy compiler, flattener, generator)
behaves; evaluation without a GPU must fail loudly (no CPU fallback)."""
import json
import os
import re

import numpy as np
import pytest

import kyverno_amd as K
from kyverno_amd._lib import KpeError, load
from tests.policies import parity_policy_set, pss_policy, restricted_latest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(kpe_[a-z0-9_]+)\s*\(", txt)))


@pytest.mark.parametrize("header", ["kpe.h", "kpe_synth.h"])
def test_library_exports_every_declared_symbol(header):
    L = load()
    names = _declared(header)
    assert names
    for n in names:
        assert hasattr(L, n), n


def test_version_and_check_ids():
    L = load()
    assert b"gfx950" in L.kpe_version()
    ids = [L.kpe_pss_check_id(k).decode() for k in range(L.kpe_pss_num_checks())]
    assert ids[0] == "allowPrivilegeEscalation" and ids[-1] == "windowsHostProcess" and len(ids) == 17


def test_compile_autogen_rule_layout():
    ps = K.PolicySet([restricted_latest()])
    assert ps.rule_names == ["podsecurity-subrule-restricted/restricted",
                             "podsecurity-subrule-restricted/autogen-restricted",
                             "podsecurity-subrule-restricted/autogen-cronjob-restricted"]
    assert all(ps.is_pss)


def test_compile_matches_oracle_rule_names(oracle):
    pols = parity_policy_set()
    ps = K.PolicySet(pols)
    assert ps.rule_names == oracle.rule_names(pols)


def test_compile_unsupported_is_loud():
    pol = pss_policy("x", "baseline")
    # a condition outside the device's JMESPath subset (a function call) is refused
    pol["spec"]["rules"][0]["validate"] = {"deny": {"conditions": {"any": [{"key": "{{ to_upper(request.object.kind) }}",
                                                                            "operator": "Equals", "value": "a"}]}}}
    with pytest.raises(KpeError) as e:
        K.PolicySet([pol])
    assert e.value.status == 2  # KPE_E_UNSUPPORTED
    # pattern variables whose query is outside the subset: refused too
    pol["spec"]["rules"][0]["validate"] = {"pattern": {"metadata": {"name": "{{ to_upper(request.object.kind) }}"}}}
    with pytest.raises(KpeError) as e:
        K.PolicySet([pol])
    assert e.value.status == 2
    # plain patterns compile (H_PATTERN)
    pol["spec"]["rules"][0]["validate"] = {"pattern": {"spec": {"containers": [{"image": "!*:latest"}]}}}
    assert K.PolicySet([pol]).num_rules == 3


def test_compile_selectors():
    from tests.policies import c4_policy_set, selector_policy

    ps = K.PolicySet(c4_policy_set())
    assert ps.num_rules == len(c4_policy_set())  # selectors disable autogen
    # two wildcard keys can resolve to one label key: Go map order decides => refused
    with pytest.raises(KpeError) as e:
        K.PolicySet([selector_policy("c", selector={"matchLabels": {"a*": "x", "ab": "y"}})])
    assert e.value.status == 2
    with pytest.raises(KpeError) as e:
        K.PolicySet([selector_policy("c", selector={"matchLabels": {"a*": "x", "b*": "y"}})])
    assert e.value.status == 2
    with pytest.raises(KpeError) as e:  # malformed (not an object)
        K.PolicySet([selector_policy("c", selector="app=x")])
    assert e.value.status == 1


def test_flatten_synth_counts():
    nd = K.synth_resources(1, 5000, mix=2)
    assert nd.count(b"\n") == 5000
    c = K.Corpus(nd)
    assert c.n == 5000 and c.nbytes > 0
    # deterministic and shardable: rows depend only on (seed, index)
    a = K.synth_resources(1, 10, mix=2, first_index=100).split(b"\n")
    b = K.synth_resources(1, 110, mix=2).split(b"\n")[100:110]
    assert a[:10] == b


def test_flatten_rejects_malformed():
    with pytest.raises(KpeError) as e:
        K.Corpus(b'{"kind": "Pod", "metadata": ')
    assert e.value.status == 1


def test_cap_dictionary_limit_is_per_row():
    """A pod past the 64-name capability dictionary is kept (its cells come back undecided,
    tests/test_limits.py); the batch is not refused."""
    res = [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"},
            "spec": {"containers": [{"name": "c", "image": "x",
                                     "securityContext": {"capabilities": {"add": [f"CAP{i}" for i in range(70)]}}}]}}]
    assert K.Corpus(res).n == 1


def test_no_gpu_means_loud_device_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(KpeError) as e:
        K.Device(0)
    assert e.value.status == 3  # KPE_E_DEVICE
