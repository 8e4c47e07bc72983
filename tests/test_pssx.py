"""podSecurity.exclude on the device (kpe_pssx_kernel, kyverno_amd/csrc/pssx.inl) against the
oracle's restatement of pkg/pss/evaluate.go:72-317, which the reference's own cases pin
(pkg/pss/evaluate_test.go: 222 cases with exclusions; chainsaw psa exclusion fixtures).

CPU: the exclusion pass compiled for the host under ASan/UBSan (scripts/pssx_check.cpp),
seeded with the plain PSS verdicts. GPU: the whole device path through the C-ABI."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from oracle.report import pod_of
from tests.policies import pss_policy
from tests.pss_fuzz import exception_case, fuzz_case, strip_exclusions, strip_pss, xfail_seed

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
BIN = os.path.join(ROOT, "scripts", "build", "pssx_check")


def golden_cases():
    cases = [c for c in json.load(open(os.path.join(GOLD, "pss_evaluate_cases.json"))) if c["rule"].get("exclude")]
    pols = [pss_policy(f"g{i}", c["rule"]["level"], c["rule"].get("version", "latest"), exclude=c["rule"]["exclude"])
            for i, c in enumerate(cases)]
    return cases, pols


def chainsaw_cases():
    """Chainsaw admissions with exclusions, minus test-exclusion-procmount/good-pod.yaml: its
    expectation depends on the API server's ProcMountType gate (tests/test_oracle_golden.py);
    the engine-level verdict is fail."""
    cs = [c for c in json.load(open(os.path.join(GOLD, "chainsaw_psa.json")))
          if c["policy"]["spec"]["rules"][0]["validate"]["podSecurity"].get("exclude")
          and not c["file"].endswith("test-exclusion-procmount/good-pod.yaml")]
    return cs


@pytest.fixture(scope="module")
def pssx_bin():
    from tests.conftest import build_host_tool

    build_host_tool("pssx_check")
    return BIN


def _host(pssx_bin, tmp_path, pols, nd, seed, excs=None):
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(nd)
    (tmp_path / "seed.bin").write_bytes(np.ascontiguousarray(seed, dtype=np.uint8).tobytes())
    extra = []
    if excs is not None:
        (tmp_path / "x.json").write_text(json.dumps(excs))
        extra = [str(tmp_path / "x.json")]
    subprocess.check_call([pssx_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"),
                           str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")] + extra, stdout=subprocess.DEVNULL)
    return np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(seed.shape)


def test_compile_exclusions():
    cases, pols = golden_cases()
    ps = K.PolicySet(pols)
    assert ps.num_rules == 3 * len(pols)  # + the two autogen rules of each
    bad = pss_policy("b", "baseline", exclude={"controlName": "x"})
    with pytest.raises(K.KpeError):
        K.PolicySet([bad])


def test_golden_evaluate_cases_host(pssx_bin, oracle, tmp_path):
    """Every evaluate_test.go case with exclusions: one rule per case, all pods against all rules."""
    cases, pols = golden_cases()
    nd = "\n".join(json.dumps(c["pod"]) for c in cases).encode()
    ref = oracle.validate(pols, nd, nthreads=8)
    # the reference's own expectations sit on the diagonal (rule g<i> is column 3i)
    assert [int(ref[i, 3 * i]) for i in range(len(cases))] == [1 if c["allowed"] else 2 for c in cases]
    seed = oracle.validate(strip_exclusions(pols), nd, nthreads=8)
    out = _host(pssx_bin, tmp_path, pols, nd, seed)
    bad = np.argwhere(out != ref)
    assert bad.size == 0, [(cases[j // 3]["name"], i, int(out[i, j]), int(ref[i, j])) for i, j in bad[:5]]


def test_chainsaw_exclusions_host(pssx_bin, oracle, tmp_path):
    cs = chainsaw_cases()
    assert len(cs) >= 40
    for c in cs:
        nd = json.dumps(c["resource"]).encode()
        ref = oracle.validate([c["policy"]], nd)
        seed = oracle.validate(strip_exclusions([c["policy"]]), nd)
        out = _host(pssx_bin, tmp_path, [c["policy"]], nd, seed)
        assert (out == ref).all(), c["file"]
        applied = [x for x in out[0] if x]
        assert len(applied) == 1 and {1: "pass", 2: "fail"}[int(applied[0])] == c["expect"], c["file"]


@pytest.mark.parametrize("seed", [1, 2, 3, 4, 5, 6])
def test_fuzz_exclusions_host(pssx_bin, oracle, tmp_path, seed):
    pols, nd = fuzz_case(seed)
    ref = oracle.validate(pols, nd, nthreads=8)
    base = oracle.validate(strip_exclusions(pols), nd, nthreads=8)
    out = _host(pssx_bin, tmp_path, pols, nd, base)
    assert (out == 7).sum() == 0
    bad = np.argwhere(out != ref)
    assert bad.size == 0, [(int(i), int(j), int(out[i, j]), int(ref[i, j])) for i, j in bad[:8]]
    # the exclusions change verdicts (the test exercises them)
    assert ((base == 2) & (ref == 1)).sum() > 20


def _exception_oracle(oracle, pols, excs, nd):
    ref = oracle.validate(pols, nd, nthreads=8, exceptions=excs)
    base = oracle.validate(strip_exclusions(pols), nd, nthreads=8)
    skipped = oracle.validate(strip_exclusions(pols), nd, nthreads=8, exceptions=strip_pss(excs))
    return ref, base, skipped


@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_pss_exceptions_host(pssx_bin, oracle, tmp_path, seed):
    """PolicyException podSecurity controls (validate_pss.go:45-110): the exclusion pass over the
    cells the scan marks KPE_XFAIL_, after the rule's own exclusions, on Pods, Deployments and
    CronJobs, with invalid entries in either list."""
    pols, excs, nd = exception_case(seed)
    ref, base, skipped = _exception_oracle(oracle, pols, excs, nd)
    assert (ref == 7).sum() == 0
    out = _host(pssx_bin, tmp_path, pols, nd, xfail_seed(pols, excs, base, skipped), excs)
    bad = np.argwhere(out != ref)
    assert bad.size == 0, [(int(i), int(j), int(out[i, j]), int(ref[i, j])) for i, j in bad[:8]]
    # the exceptions both clear failing pods (skip) and leave others failing
    xfail = xfail_seed(pols, excs, base, skipped) == 8
    assert (xfail & (ref == 5)).sum() > 10 and (xfail & (ref == 2)).sum() > 10


def test_pss_exception_compile():
    pols, excs, _ = exception_case(21)
    K.PolicySet(pols, excs)
    first = next(x for x in excs if x["spec"].get("podSecurity"))
    two = json.loads(json.dumps(first))
    two["metadata"]["name"] = "second"
    with pytest.raises(K.KpeError):  # the first matching exception decides: not restated
        K.PolicySet(pols, excs + [two])
    bad = json.loads(json.dumps(first))
    bad["spec"]["podSecurity"] = {"controlName": "Capabilities"}
    with pytest.raises(K.KpeError):
        K.PolicySet(pols, [bad])


# ---- GPU: the device path through the C-ABI ------------------------------------------------
@pytest.mark.gpu
def test_golden_evaluate_cases_gpu(oracle):
    cases, pols = golden_cases()
    nd = "\n".join(json.dumps(c["pod"]) for c in cases).encode()
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, [(cases[j // 3]["name"], i, int(v[i, j]), int(ref[i, j])) for i, j in bad[:5]]
    assert [int(v[i, 3 * i]) for i in range(len(cases))] == [1 if c["allowed"] else 2 for c in cases]


@pytest.mark.gpu
def test_chainsaw_exclusions_gpu():
    eng = K.Engine(ordinal=0)
    for c in chainsaw_cases():
        v, _, _ = eng.evaluate(K.PolicySet([c["policy"]]), K.Corpus(json.dumps(c["resource"]).encode()))
        applied = [x for x in v[0] if x]
        assert len(applied) == 1 and {1: "pass", 2: "fail"}[int(applied[0])] == c["expect"], c["file"]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_fuzz_exclusions_gpu(oracle, seed):
    pols, nd = fuzz_case(seed, npods=4000, nrules=32)
    eng = K.Engine(ordinal=0)
    v, masks, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd), check_masks=True)
    ref = oracle.validate(pols, nd, nthreads=8)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, [(int(i), int(j), int(v[i, j]), int(ref[i, j])) for i, j in bad[:8]]
    assert (masks[v != 2] == 0).all()  # masks: the checks still failing after the exclusions


@pytest.mark.gpu
@pytest.mark.parametrize("seed,nrules", [(31, 24), (32, 8)])  # 72 rules: the WIDE scan; 24: NARROW
def test_pss_exceptions_gpu(oracle, seed, nrules):
    pols, excs, nd = exception_case(seed, npods=3000, nrules=nrules)
    eng = K.Engine(ordinal=0)
    v, masks, _ = eng.evaluate(K.PolicySet(pols, excs), K.Corpus(nd), check_masks=True)
    ref = oracle.validate(pols, nd, nthreads=8, exceptions=excs)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, [(int(i), int(j), int(v[i, j]), int(ref[i, j])) for i, j in bad[:8]]
    assert (masks[v != 2] == 0).all()
    assert (v == 5).any()


# ---- messages: FormatChecksPrint after the exclusions (validate_pss.go:76-110) -----------------
def _excl_messages(oracle, pols, nd, excs=None, xmatch=None):
    """(device-side message, oracle message) of every FAIL cell of the podSecurity rules: the host
    report (kpe_report_results_msg) given the oracle's verdict row and, for PolicyException rules,
    whether the exception matched (KPE_CVM_XMATCH); the oracle's EvaluatePod / convertChecks /
    ApplyPodSecurityExclusion restatement."""
    ps = K.PolicySet(pols, excs) if excs else K.PolicySet(pols)
    names = ps.rule_names
    ref = oracle.validate(pols, nd, nthreads=8, exceptions=excs) if excs else oracle.validate(pols, nd, nthreads=8)
    by_name = {p["metadata"]["name"]: p for p in pols}
    xby = {x["spec"]["exceptions"][0]["policyName"]: x["spec"].get("podSecurity") for x in (excs or [])}
    docs = [json.loads(l) for l in nd.split(b"\n") if l.strip()]
    pairs = []
    for i, doc in enumerate(docs):
        row = ref[i]
        cv = np.zeros(len(names), dtype=np.uint32)
        for j, full in enumerate(names):
            if row[j] == 2:  # the failing versioned checks (they render the rules without exclusions)
                ps0 = by_name[full.split("/", 1)[0]]["spec"]["rules"][0]["validate"]["podSecurity"]
                f = max(oracle.failing_cv(ps0["level"], ps0.get("version", "latest"), pod_of(doc)), 0)
                cv[j] = (f or 1) | ((1 << 31) if xmatch is not None and xmatch[i, j] else 0)
        got = {r["rule"]: r.get("message") for r in K.report_results(ps, row, cv, resource=doc)}
        for j, full in enumerate(names):
            if row[j] != 2:
                continue
            pname, rname = full.split("/", 1)
            ps0 = by_name[pname]["spec"]["rules"][0]["validate"]["podSecurity"]
            if not ps0.get("exclude") and not xby.get(pname):
                continue  # no exclusions: the plain message (tests/test_report.py)
            xex = xby.get(pname) if xmatch is not None and xmatch[i, j] else None
            st, want = oracle.pss_message_ex(rname, ps0["level"], ps0.get("version", "latest"), doc,
                                             ps0.get("exclude"), xex)
            assert st == 0, (full, st)
            pairs.append((full, i, got.get(rname), want))
    return pairs


def test_exclusion_messages_golden_host(oracle):
    """The 222 evaluate_test.go exclusion cases: every FAIL cell's message."""
    cases, pols = golden_cases()
    nd = "\n".join(json.dumps(c["pod"]) for c in cases).encode()
    pairs = _excl_messages(oracle, pols, nd)
    bad = [p for p in pairs if p[2] != p[3]]
    assert pairs and not bad, bad[:3]


@pytest.mark.parametrize("seed", [11, 12])
def test_exclusion_messages_fuzz_host(oracle, seed):
    """Random pods x random exclusion lists (pod-level and image entries on one control, values):
    where at most one check id survives the exclusions the reference's order is fixed and the
    message must match exactly; with several, the reference lists them in Go map order, so only
    the set of per-check texts is compared."""
    pols, nd = fuzz_case(seed, npods=300, nrules=16)
    pairs = _excl_messages(oracle, pols, nd)
    assert len(pairs) > 100
    for full, i, got, want in pairs:
        assert got is not None, (full, i)
        head, sep, rest = want.partition('": ')
        ghead, gsep, grest = got.partition('": ')
        assert ghead == head
        if rest.count("\n(Forbidden reason") <= 1:
            assert got == want, (full, i)
        else:
            assert sorted(grest.split("\n")) == sorted(rest.split("\n")), (full, i)


@pytest.mark.parametrize("seed", [21, 22])
def test_exception_messages_host(oracle, seed):
    """PolicyException podSecurity controls: the fail message after the exception's exclusions
    when it matched (KPE_CVM_XMATCH; the scan's KPE_XFAIL_ cells), after the rule's own otherwise."""
    pols, excs, nd = exception_case(seed, npods=300)
    base = oracle.validate(strip_exclusions(pols), nd, nthreads=8)
    skipped = oracle.validate(strip_exclusions(pols), nd, nthreads=8, exceptions=strip_pss(excs))
    xmatch = xfail_seed(pols, excs, base, skipped) == 8
    pairs = _excl_messages(oracle, pols, nd, excs, xmatch)
    assert len(pairs) > 50
    for full, i, got, want in pairs:
        assert got is not None, (full, i)
        rest, grest = want.partition('": ')[2], got.partition('": ')[2]
        if rest.count("\n(Forbidden reason") <= 1:
            assert got == want, (full, i)
        else:
            assert sorted(grest.split("\n")) == sorted(rest.split("\n")), (full, i)


@pytest.mark.gpu
def test_exception_messages_gpu(oracle):
    """End to end: the device's check masks carry KPE_CVM_XMATCH exactly on the FAIL cells whose
    podSecurity PolicyException matched, and the messages rendered from them equal the oracle's."""
    pols, excs, nd = exception_case(41, npods=400)
    eng = K.Engine(ordinal=0)
    ps, c = K.PolicySet(pols, excs), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, c, check_masks=True)
    ref = oracle.validate(pols, nd, nthreads=8, exceptions=excs)
    assert np.array_equal(v, ref)
    cvm = eng.cv_masks(ps, c, raw=True)
    base = oracle.validate(strip_exclusions(pols), nd, nthreads=8)
    skipped = oracle.validate(strip_exclusions(pols), nd, nthreads=8, exceptions=strip_pss(excs))
    xm = xfail_seed(pols, excs, base, skipped) == 8
    fail = v == 2
    assert np.array_equal(((cvm >> 31) & 1).astype(bool) & fail, xm & fail)
    assert (xm & fail).sum() > 10
    by_name = {p["metadata"]["name"]: p for p in pols}
    xby = {x["spec"]["exceptions"][0]["policyName"]: x["spec"].get("podSecurity") for x in excs}
    docs = [json.loads(l) for l in nd.split(b"\n") if l.strip()]
    n = 0
    for i, doc in enumerate(docs):
        got = {r["rule"]: r.get("message") for r in K.report_results(ps, v[i], cvm[i], resource=doc)}
        for j, full in enumerate(ps.rule_names):
            pname, rname = full.split("/", 1)
            ps0 = by_name[pname]["spec"]["rules"][0]["validate"]["podSecurity"]
            if v[i, j] != 2 or not (ps0.get("exclude") or xby.get(pname)):
                continue
            st, want = oracle.pss_message_ex(rname, ps0["level"], ps0.get("version", "latest"), doc,
                                             ps0.get("exclude"), xby.get(pname) if xm[i, j] else None)
            rest, grest = want.partition('": ')[2], got[rname].partition('": ')[2]
            if rest.count("\n(Forbidden reason") <= 1:
                assert got[rname] == want, (full, i)
            else:
                assert sorted(grest.split("\n")) == sorted(rest.split("\n")), (full, i)
            n += 1
    assert n > 50
