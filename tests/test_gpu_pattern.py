"""GPU parity for pattern / anyPattern rules: kpe_pattern_kernel through
the C-ABI against the CPU oracle (itself pinned by pattern_test.go, validate_test.go and the
test/cli/test scenarios in test_oracle_golden.py). Bit-exact verdict cells required."""
import json
import os

import numpy as np
import pytest

import kyverno_amd as K

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CHART = json.load(open(os.path.join(GOLD, "chart_policies.json")))
PTREE = json.load(open(os.path.join(GOLD, "pattern_tree_cases.json")))
CLI = json.load(open(os.path.join(GOLD, "cli_cases.json")))


def device_policies(pols):
    """The subset of `pols` the device program accepts (deny / foreach / variables are
    reported as KPE_E_UNSUPPORTED by kpe_program_compile)."""
    out = []
    for p in pols:
        try:
            K.PolicySet([p])
        except K.KpeError as e:
            assert e.status == 2, e  # KPE_E_UNSUPPORTED only
            continue
        out.append(p)
    return out


def chart_pattern_policies():
    return device_policies(CHART["baseline"] + CHART["restricted"])


def _policy_for(name, pattern, any_pattern=False):
    v = {"anyPattern": pattern} if any_pattern else {"pattern": pattern}
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
            "spec": {"rules": [{"name": "r", "match": {"any": [{"resources": {"kinds": ["*"]}}]}, "validate": v}]}}


def test_chart_patterns_compile_like_oracle(oracle):
    """CPU: every chart pattern policy compiles; rule columns equal the oracle's autogen order."""
    pols = chart_pattern_policies()
    names = {p["metadata"]["name"] for p in pols}
    assert {"disallow-host-namespaces", "disallow-host-ports", "restrict-apparmor-profiles", "restrict-sysctls",
            "require-run-as-nonroot", "restrict-seccomp-strict"} <= names
    ps = K.PolicySet(pols)
    assert ps.rule_names == oracle.rule_names(pols)


def test_docs_required_for_pattern_rules():
    """CPU-side contract: a corpus flattened without document tapes cannot serve pattern
    rules (checked when the program is bound, on the device)."""
    c = K.Corpus([{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "a"}}], docs=False)
    assert c.n == 1


@pytest.mark.gpu
@pytest.mark.parametrize("mix,n,seed", [(0, 20000, 0xC1), (1, 20000, 21), (2, 20000, 22)])
def test_chart_patterns_bit_exact(oracle, mix, n, seed):
    eng = K.Engine(ordinal=0)
    pols = chart_pattern_policies()
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, cnt = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} " \
                          f"gpu={[int(v[i, j]) for i, j in bad[:5]]} ref={[int(ref[i, j]) for i, j in bad[:5]]}"
    assert (v == 6).sum() == 0  # no pending cell survives
    for r in range(v.shape[1]):
        col = v[:, r]
        assert cnt[r]["pass"] == int((col == 1).sum()) and cnt[r]["fail"] == int((col == 2).sum())
        assert cnt[r]["skip"] == int((col == 5).sum()) and cnt[r]["error"] == int((col == 4).sum())


@pytest.mark.gpu
def test_pattern_tree_golden_on_device(oracle):
    """validate_test.go trees (MatchPattern tables + validateMap/validateResourceElement
    cases) as single-rule policies over a resource of kind *; the oracle is the reference."""
    eng = K.Engine(ordinal=0)
    pols, docs = [], []
    cases = [c for c in PTREE if isinstance(json.loads(c["resource"]), dict)]  # a resource is an object
    for i, c in enumerate(cases):
        pols.append(_policy_for(f"t{i}", json.loads(c["pattern"])))
        docs.append(json.loads(c["resource"]))
    pols = device_policies(pols)
    assert len(cases) >= len(PTREE) - 4
    nd = "\n".join(json.dumps(d) for d in docs).encode()
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
    assert len(pols) >= len(cases) - 4  # all but the $(...) reference-substitution trees


@pytest.mark.gpu
@pytest.mark.parametrize("case", CLI, ids=[c["name"] for c in CLI])
def test_cli_scenarios_on_device(oracle, case):
    pols = device_policies(case["policies"])
    if not pols or not case["resources"]:
        pytest.skip("no device-supported policy in this scenario")
    nd = "\n".join(json.dumps(r) for r in case["resources"]).encode()
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"


def edge_case_inputs(n=3000, seed=5):
    """Leaf typing and anchor edge cases: numbers as strings / floats, quantities, durations,
    nulls, arrays in leaf positions, existence / negation / global anchors, empty arrays."""
    pats = [
        {"spec": {"containers": [{"resources": {"limits": {"memory": "<=1Gi", "cpu": "100m-2"}}}]}},
        {"spec": {"=(replicas)": ">=2 & <10", "=(ttl)": "<1h"}},
        {"spec": {"^(containers)": [{"name": "sidecar-*"}], "X(hostNetwork)": "null"}},
        {"spec": {"<(priority)": 5, "containers": [{"(image)": "*:latest", "imagePullPolicy": "Always"}]}},
        {"metadata": {"labels": {"app*": "?*", "=(tier)": "front* | back*"}}},
        # anchored glob keys, expanded per resource (wildcards.go:145-162)
        {"metadata": {"labels": {"(app.kubernetes.io/*)": "web-* | 3", "tier": "?*"}}},
        {"metadata": {"labels": {"X(team*)": "null", "=(ti?r)": "front* | 1*"}}},
        {"metadata": {"annotations": {"<(owner*)": "team-*"}, "labels": {"=(app*)": "x | 2"}}},
        {"spec": {"values": [1.5], "flags": [True], "empty": [], "pos": [[1], [2]]}},
        {"spec": {"n": None, "z": 0, "s": "", "f": 0.0}},
    ]
    pols = [_policy_for(f"e{i}", p) for i, p in enumerate(pats)]
    pols.append(_policy_for("any", [{"spec": {"replicas": 3}}, {"spec": {"replicas": "3"}}], any_pattern=True))
    rng = np.random.default_rng(seed)
    vals = [None, 0, 1, 2, 3, 5, 12, "3", "3.0", "1e3", 1.5, 3.0, -1, "100m", "2", "1Gi", "2048Mi", "30m", "2h",
            "0", True, False, "", "x", [], [1], [1.5, 2.5], {}, {"a": 1}, "sidecar-1", "nginx:latest", "Always"]
    docs = []
    for i in range(n):
        def pick():
            return vals[int(rng.integers(len(vals)))]
        spec = {k: pick() for k in ("replicas", "ttl", "priority", "hostNetwork", "values", "flags", "empty",
                                    "pos", "n", "z", "s", "f") if rng.random() < 0.7}
        ctrs = []
        for _ in range(int(rng.integers(0, 3))):
            c = {"name": rng.choice(["sidecar-a", "app", "x"]), "image": rng.choice(["nginx:latest", "nginx:1"])}
            if rng.random() < 0.7:
                c["imagePullPolicy"] = pick()
            if rng.random() < 0.6:
                c["resources"] = {"limits": {"memory": pick(), "cpu": pick()}}
            ctrs.append(c)
        if rng.random() < 0.8:
            spec["containers"] = ctrs
        labels = {k: str(pick()) for k in rng.choice(["app", "app.kubernetes.io/name", "tier", "x", "team-a"], 2)}
        meta = {"name": f"d{i}", "labels": labels}
        if rng.random() < 0.5:
            meta["annotations"] = {rng.choice(["owner", "owner-b", "y"]): rng.choice(["team-a", "x", ""])}
        docs.append({"apiVersion": "v1", "kind": "Thing", "metadata": meta, "spec": spec})
    return pols, "\n".join(json.dumps(d) for d in docs).encode()


@pytest.mark.gpu
def test_pattern_edge_documents(oracle):
    pols, nd = edge_case_inputs()
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} " \
                          f"gpu={[int(v[i, j]) for i, j in bad[:5]]} ref={[int(ref[i, j]) for i, j in bad[:5]]}"


def test_anchored_glob_metadata_keys_compile():
    """Anchored glob keys in labels / annotations compile (ExpandInMetadata, wildcards.go:145-162)
    unless another anchor-phase key starts with the glob's literal prefix: the anchors then run in
    the sorted order of the per-resource expansions, which the compile-time order may not be."""
    ok = [{"metadata": {"labels": {"(app.kubernetes.io/*)": "web-*", "tier": "?*"}}},
          {"metadata": {"labels": {"X(team*)": "null", "=(tier)": "a"}}},
          {"metadata": {"annotations": {"<(owner*)": "team-*"}}}]
    for p in ok:
        K.PolicySet([_policy_for("ok", p)])
    bad = {"metadata": {"labels": {"(app*)": "x", "(app.kubernetes.io/name)": "y"}}}
    with pytest.raises(K.KpeError):
        K.PolicySet([_policy_for("bad", bad)])
    with pytest.raises(K.KpeError):  # glob keys under an array pattern: the reference rewrites the shared pattern
        K.PolicySet([_policy_for("arr", {"items": [{"metadata": {"labels": {"app*": "x"}}}]})])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,sites", [("c5", False), ("c5", True), ("c3", True)])
def test_pattern_kernel_fanout_bit_exact(oracle, monkeypatch, cfg, sites):
    """The lane-per-row kernel (LDS frame stacks, deep walks retried on the private stack) gives
    the oracle's matrix on the C5 fan-out corpus (1-64 containers, Pods and Deployments: the
    Deployments' walks are deeper than the LDS stack) with the C5 pattern set, and with the
    array sites on (KPE_SITES=1: kpe_site_kernel validates the elements of arrays of maps one lane
    per element and the walk takes the row's result) on C5 and C3."""
    from tests.policies import c3_policy_set, c5_policy_set

    if sites:
        monkeypatch.setenv("KPE_SITES", "1")
    pols = c5_policy_set() if cfg == "c5" else c3_policy_set()
    nd = (K.synth_resources(0xC5, 6000, mix=K.SYNTH_FANOUT) if cfg == "c5"
          else K.synth_resources(0xC3 + 5, 20000, mix=K.SYNTH_C3))
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
    assert (v == 6).sum() == 0
