"""GPU parity: the HIP path (libkpe through the C-ABI) against the CPU oracle
and the reference's golden vectors. Bit-exact verdict cells required."""
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import parity_policy_set, pss_policy, restricted_latest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def engine():
    return K.Engine(ordinal=0)


def _gpu(engine, policies, nd, nsl=None, masks=False):
    ps = K.PolicySet(policies)
    c = K.Corpus(nd, nsl)
    return engine.evaluate(ps, c, check_masks=masks)


def test_pss_golden_all_cases(engine):
    """Every pkg/pss/evaluate_test.go case (222 of 227 with exclusions: kpe_pssx_kernel)."""
    cases = json.load(open(os.path.join(GOLD, "pss_evaluate_cases.json")))
    assert len(cases) == 227
    for c in cases:
        pol = pss_policy("golden", c["rule"]["level"], c["rule"].get("version", "latest"), exclude=c["rule"].get("exclude"))
        v, _, _ = _gpu(engine, [pol], json.dumps(c["pod"]).encode())
        assert v[0, 0] == (1 if c["allowed"] else 2), c["name"]


def test_background_report_restricted_latest(engine):
    bg = json.load(open(os.path.join(GOLD, "background_report.json")))
    v, m, cnt = _gpu(engine, [bg["policy"]], json.dumps(bg["resource"]).encode(), masks=True)
    assert list(v[0]) == [2, 0, 0]
    assert m[0, 0] == 1 << 3  # capabilities_restricted only
    assert cnt[0]["fail"] == 1 and cnt[1]["na"] == 1


def test_chainsaw_all(engine):
    """Every chainsaw psa admission; test-exclusion-procmount/good-pod.yaml's expectation depends on
    the API server's ProcMountType gate (tests/test_oracle_golden.py): the engine verdict is fail."""
    for c in json.load(open(os.path.join(GOLD, "chainsaw_psa.json"))):
        if c["file"].endswith("test-exclusion-procmount/good-pod.yaml"):
            continue
        v, _, _ = _gpu(engine, [c["policy"]], json.dumps(c["resource"]).encode())
        applied = [x for x in v[0] if x]
        assert len(applied) == 1 and {1: "pass", 2: "fail"}[applied[0]] == c["expect"], c["file"]


@pytest.mark.parametrize("mix,n,seed", [(0, 20000, 0xC2), (1, 20000, 11), (2, 20000, 12)])
def test_synthetic_matrix_bit_exact(engine, oracle, mix, n, seed):
    pols = parity_policy_set()
    nd = K.synth_resources(seed, n, mix=mix)
    v, _, cnt = _gpu(engine, pols, nd)
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
    # counters agree with the matrix
    for r in range(v.shape[1]):
        col = v[:, r]
        assert cnt[r]["pass"] == int((col == 1).sum()) and cnt[r]["fail"] == int((col == 2).sum())
        assert cnt[r]["error"] == int((col == 4).sum()) and cnt[r]["na"] == int((col == 0).sum())


def test_check_masks_match_oracle(engine, oracle):
    nd = K.synth_resources(99, 3000, mix=2)
    lines = nd.split(b"\n")
    for lvl, ver in (("restricted", "latest"), ("baseline", "v1.0"), ("restricted", "v1.24")):
        pol = pss_policy("m", lvl, ver, kinds=("Pod",))
        v, m, _ = _gpu(engine, [pol], nd, masks=True)
        ids = [K._lib.load().kpe_pss_check_id(k).decode() for k in range(17)]
        for i in range(0, 3000, 7):
            doc = json.loads(lines[i])
            if doc["kind"] != "Pod" or v[i, 0] not in (1, 2):
                continue
            want = set(oracle.failing_checks(lvl, ver, doc))
            got = {ids[k] for k in range(17) if (int(m[i, 0]) >> k) & 1}
            assert got == want, (i, lvl, ver)


def test_c2_scale_properties(engine, oracle):
    """1M Pods x restricted:latest (the headline config): counts are consistent, evaluation is
    idempotent and shard-position independent, and the whole matrix matches the oracle."""
    n = 1_000_000
    nd = K.synth_resources(0xC2, n, mix=0)
    ps = K.PolicySet([restricted_latest()])
    c = K.Corpus(nd)
    v, _, cnt = engine.evaluate(ps, c)
    assert v.shape == (n, 3)
    assert (v[:, 1:] == 0).all()  # autogen twins never match Pods
    assert cnt[0]["pass"] + cnt[0]["fail"] + cnt[0]["error"] == n
    frac_fail = cnt[0]["fail"] / n
    assert 0.3 < frac_fail < 0.9
    # idempotence: a second evaluation gives the identical matrix
    v2, _, _ = engine.evaluate(ps, c)
    assert np.array_equal(v, v2)
    # batch-position independence: a separately flattened shard gives the same rows
    first = 500_000
    shard = K.Corpus(K.synth_resources(0xC2, 1000, mix=0, first_index=first))
    vs, _, _ = engine.evaluate(ps, shard)
    assert np.array_equal(vs, v[first:first + 1000])
    # the whole 1M x 3 matrix against the oracle
    ref = oracle.validate([restricted_latest()], nd, nthreads=16)
    assert np.array_equal(v, ref)


def test_selector_golden(engine):
    """pkg/utils/match/labels_test.go and utils_test.go selector/name cases through the GPU."""
    from tests.test_oracle_golden import MRD, SEL, match_rd_inputs, selector_case_inputs

    for case in SEL:
        pol, pod = selector_case_inputs(case)
        v, _, _ = _gpu(engine, [pol], json.dumps(pod).encode())
        assert (v[0, 0] != 0) == (case["want"] and not case["wantErr"]), case["name"]
    for case in MRD:
        pol, res = match_rd_inputs(case)
        v, _, _ = _gpu(engine, [pol], json.dumps(res).encode())
        assert (v[0, 0] != 0) == case["matched"], case["name"]


@pytest.mark.parametrize("n,seed", [(20000, 0xC4), (50000, 41), (625_000, 0xC4), (5_000_000, 0xC4)])  # 5M: C4 on one GPU
def test_c4_selectors_bit_exact(engine, oracle, n, seed):
    from tests.policies import c4_policy_set

    pols = c4_policy_set()
    nd = K.synth_resources(seed, n, mix=3)
    nsl = K.synth_ns_labels(seed, 10000, mix=3)
    v, _, cnt = _gpu(engine, pols, nd, nsl)
    ref = oracle.validate(pols, nd, ns_labels=nsl, nthreads=16)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
    for r in range(v.shape[1]):
        assert cnt[r]["pass"] == int((v[:, r] == 1).sum()) and cnt[r]["na"] == int((v[:, r] == 0).sum())


@pytest.mark.parametrize("psum", ["1", "0"])
def test_general_scan_both_pss_forms_bit_exact(oracle, psum):
    """The general scan of a podSecurity program in both forms (KPE_PSUM, read at device open):
    walking each pod's lists itself (the default) and reading kpe_psum_kernel's per-pod records;
    verdicts and check masks equal the oracle's on the C4 mix and the C1 mixes."""
    from tests.policies import c4_policy_set

    old = os.environ.get("KPE_PSUM")
    os.environ["KPE_PSUM"] = psum
    try:
        eng = K.Engine(ordinal=0)
        for pols, mix, seed in ((c4_policy_set(), 3, 0x41), (parity_policy_set(), 2, 0x42)):
            nd = K.synth_resources(seed, 20000, mix=mix)
            nsl = K.synth_ns_labels(seed, 10000, mix=3) if mix == 3 else None
            v, _, _ = _gpu(eng, pols, nd, nsl)
            ref = oracle.validate(pols, nd, ns_labels=nsl, nthreads=16)
            bad = np.argwhere(v != ref)
            assert bad.size == 0, f"KPE_PSUM={psum}: {len(bad)} mismatching cells, first {bad[:5].tolist()}"
    finally:
        if old is None:
            os.environ.pop("KPE_PSUM", None)
        else:
            os.environ["KPE_PSUM"] = old


@pytest.mark.parametrize("copies", [1, 4, 8, 9])
def test_selector_requirement_masks_and_fallback(engine, oracle, copies):
    """Selector terms decided from the per-binding requirement masks (<= 64 requirements per
    space: label selectors, namespaceSelectors) and, past 64, by the per-requirement label walk:
    C4's policy set (19 label-selector and 8 namespaceSelector requirements that build) repeated
    `copies` times: 1 both spaces masked; 4 label selectors past 64; 8 namespaceSelectors at
    exactly 64 bits; 9 both past 64. Bit-exact against the oracle."""
    import copy as _copy
    from tests.policies import c4_policy_set

    pols = []
    for k in range(copies):
        for p in c4_policy_set():
            q = _copy.deepcopy(p)
            q["metadata"]["name"] += f"-{k}"
            pols.append(q)
    nd = K.synth_resources(0x5E1 + copies, 30000, mix=3)
    nsl = K.synth_ns_labels(0x5E1, 10000, mix=3)
    v, _, _ = _gpu(engine, pols, nd, nsl)
    ref = oracle.validate(pols, nd, ns_labels=nsl, nthreads=16)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
