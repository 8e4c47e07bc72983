"""RuleResponse messages of validate.foreach rules and the RuleError texts (SURVEY.md 8(f1);
validate_resource.go:121-254,268-300,347-350,456-476; engine.go:279-281).

- foreach: pass "rule passed" (:203); fail / last-element error "validation failure: <element
  response>" once per nesting level (:239-247), where the element response is getDenyMessage over
  the element's context, buildErrorMessage / buildAnyPatternErrorMessage of the entry's pattern on
  the element, or a RuleError text; AddElementToContext's elementScope error unwrapped at its level.
- RuleError texts: "failed to evaluate preconditions: <err>", "failed to check deny conditions:
  <err>", "variable substitution failed: <err>", "failed to deserialize anyPattern, expected type
  array: <err>", with <err> the substitution error chain (variables/evaluate.go:14-27, vars.go:
  311-389, context/evaluate.go:27-31).

Pins: the oracle against validation_test.go's Test_Flux_Kustomization_PathNotPresent rows (a
RuleError text asserted verbatim, tests/golden/engine_table_message_cases.json) and the
`Unknown key "name1" in path` containment assertions; the host renderer against the same text from
a device-shaped trace. No reference vector asserts a foreach message (every testForEach call passes
msg ""): those follow the restatement (parity pinned by the oracle only).
CPU: the condition VM compiled for the host (scripts/condvm_check.cpp) writes the traces and the
host renders every foreach / error message of tests.policies.foreach_message_policy_set like the
oracle. GPU: kpe_fetch_cond_traces_ex + kpe_pattern_traces + kpe_report_results_ex against the
oracle on the chart's restricted set and the foreach sets at 20k rows."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import VAR_UNDECIDED_OK, foreach_message_policy_set, var_policy_set

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TABLE = json.load(open(os.path.join(GOLD, "engine_table_message_cases.json")))
CASES = json.load(open(os.path.join(GOLD, "engine_message_cases.json")))
NEEDS = "\x01"
STATUS = {"pass": 1, "fail": 2, "warn": 3, "error": 4, "skip": 5}
CONTAINS = {"Test_VariableSubstitutionPathNotExistInPattern",
            "Test_VariableSubstitutionPathNotExistInAnyPattern_OnePatternStatisfiesButSubstitutionFails",
            "Test_VariableSubstitutionPathNotExistInAnyPattern_AllPathNotPresent"}


def test_table_fixture_extracted():
    rows = {(c["name"], c["row"]) for c in TABLE}
    assert ("Test_Flux_Kustomization_PathNotPresent", "path-not-present") in rows
    c = [c for c in TABLE if c["row"] == "path-not-present"][0]
    assert c["results"] == ["pass", "error"] and c["messages"][1].startswith("failed to check deny conditions: ")


@pytest.mark.parametrize("case", TABLE, ids=lambda c: c["row"])
def test_oracle_table_messages_match_reference(oracle, case):
    nd = json.dumps(case["resource"]).encode()
    pols = [case["policy"]]
    st = oracle.validate(pols, nd)[0]
    msgs = oracle.pattern_messages(pols, nd)[0]
    assert [int(x) for x in st] == [STATUS[r] for r in case["results"]]
    assert msgs == case["messages"]


@pytest.mark.parametrize("case", [c for c in CASES if c["name"] in CONTAINS], ids=lambda c: c["name"])
def test_oracle_substitution_errors_contain_reference_text(oracle, case):
    """validation_test.go:1588,1674,1812 assert strings.Contains(message, `Unknown key "name1" in
    path`): the oracle's RuleError text is "variable substitution failed: failed to resolve
    request.object.metadata.name1 at path <pattern path>: JMESPath query failed: Unknown key ..."."""
    nd = json.dumps(case["resource"]).encode()
    pols = [case["policy"]]
    st = oracle.validate(pols, nd)[0]
    msgs = oracle.pattern_messages(pols, nd)[0]
    r = [i for i, s in enumerate(st) if s != 0][0]
    assert int(st[r]) == 4
    assert case["messages"]["0"] in msgs[r]
    assert msgs[r].startswith("variable substitution failed: failed to resolve request.object.metadata.name1 at path /")


def test_host_renders_reference_deny_error_text():
    """The host renderer gives the reference's RuleError text from a device-shaped trace: the deny
    block's first condition raised the error on its key (KPE_CT_ERR | condition 0 | side 0)."""
    case = [c for c in TABLE if c["row"] == "path-not-present"][0]
    ps = K.PolicySet([case["policy"]])
    v = np.array([STATUS[r] for r in case["results"]], dtype=np.uint8)
    ct = np.array([0, 0x8000 << 16], dtype=np.uint32)
    res = K.report_results(ps, v, resource=case["resource"], cond_traces=ct)
    assert [r.get("message") for r in res] == case["messages"]


@pytest.fixture(scope="module")
def condvm_bin():
    from tests.conftest import build_host_tool

    return build_host_tool("condvm_check")


# rules whose failing cells are decided by a pattern walk: their paths come from kpe_pattern_traces
# (the device's trace kernel), which the host VM run does not produce
def _pattern_leaf(msg):
    return "failed at path" in msg


def _host_vm_traces(condvm_bin, pols, lines, ref, tmp_path):
    nd = b"\n".join(lines)
    seedm = np.where(ref != 0, 6, 0).astype(np.uint8)  # matched cells, pending (KPE_PENDING_)
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes(nd)
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([condvm_bin, str(tmp_path / "p.json"), str(tmp_path / "r.ndjson"), str(tmp_path / "seed.bin"),
                           str(tmp_path / "out.bin"), str(tmp_path / "ct.bin"), str(tmp_path / "cx.bin")])
    N, R = ref.shape
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(N, R)
    cx = np.frombuffer((tmp_path / "cx.bin").read_bytes(), dtype=np.uint32).reshape(N, R, 4)
    return out, cx


def test_host_vm_foreach_messages_equal_oracle(condvm_bin, oracle, tmp_path):
    pols = foreach_message_policy_set()
    ps = K.PolicySet(pols)
    lines = [l for l in K.synth_resources(0xF1, 1500, mix=2).split(b"\n") if l]
    ref = oracle.validate(pols, b"\n".join(lines), nthreads=8)
    out, cx = _host_vm_traces(condvm_bin, pols, lines, ref, tmp_path)
    assert (out == ref).all()
    om = oracle.pattern_messages(pols, b"\n".join(lines))
    corpus = K.Corpus(b"\n".join(lines))  # the element documents (same tape as the tool's flatten)
    names = ps.rule_names
    checked = {}
    for i, line in enumerate(lines):
        res = K.report_results(ps, ref[i], resource=line, cond_traces=cx[i], corpus=corpus)
        got = {r["rule"]: r.get("message", "") for r in res}
        for r in range(ps.num_rules):
            if ref[i, r] in (0, 7):
                continue
            want, name = om[i][r], names[r].split("/", 1)[1]
            if want == NEEDS:
                assert got[name] == "", (i, name, got[name])
                continue
            if _pattern_leaf(want):
                continue
            assert got[name] == want, (i, name, got[name], want)
            key = "wrapped" if want.startswith("validation failure: ") else "error" if ref[i, r] == 4 else "other"
            checked[key] = checked.get(key, 0) + 1
    assert checked.get("wrapped", 0) > 3000 and checked.get("error", 0) > 1500, checked


def _gpu_messages(eng, ps, corpus, v, lines, rows):
    out = {}
    R = ps.num_rules
    cx = eng.cond_traces(ps, corpus, ex=True)
    for i in rows:
        if not (v[i] != 0).any():
            continue
        tr = eng.row_traces(ps, corpus, i)
        res = K.report_results(ps, v[i], resource=lines[i], traces=tr, corpus=corpus, cond_traces=cx[i])
        k = 0
        for r in range(R):
            if v[i, r] in (0, 7):
                continue
            out[(i, r)] = res[k].get("message", "")
            k += 1
    return out


def _check_gpu(oracle, pols, lines, rows, chart_rules=None, undecided_ok=()):
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    nd = b"\n".join(lines)
    c = K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, c)
    ref = oracle.validate(pols, nd, nthreads=8)
    # columns whose cells the device may leave undecided (a documented device limit)
    und = np.array([n.split("/", 1)[1].replace("autogen-cronjob-", "").replace("autogen-", "") in undecided_ok
                    for n in ps.rule_names])
    assert ((v == ref) | ((v == 7) & und[None, :])).all()
    om = oracle.pattern_messages(pols, b"\n".join(lines[i] for i in rows))
    got = _gpu_messages(eng, ps, c, v, lines, rows)
    names = ps.rule_names
    n = {"wrapped": 0, "error": 0, "pass": 0}
    for k, i in enumerate(rows):
        for r in range(ps.num_rules):
            if v[i, r] in (0, 7):
                continue
            want = om[k][r]
            if chart_rules is not None and names[r] not in chart_rules:
                continue
            g = got[(i, r)]
            if want == NEEDS:
                assert g == "", (i, names[r], g)
                continue
            assert g == want, (i, names[r], g, want)
            n["wrapped" if want.startswith("validation failure: ") else "error" if v[i, r] == 4 else "pass"] += 1
    return n


@pytest.mark.gpu
def test_gpu_foreach_messages_equal_oracle(oracle):
    pols = foreach_message_policy_set()
    lines = [l for l in K.synth_resources(0xF2, 20000, mix=2).split(b"\n") if l]
    rows = list(range(0, len(lines), 7))  # every seventh row (the oracle's messages are one-thread)
    n = _check_gpu(oracle, pols, lines, rows)
    assert n["wrapped"] > 5000 and n["error"] > 2000, n


@pytest.mark.gpu
def test_gpu_var_policy_foreach_messages_equal_oracle(oracle):
    """The foreach pattern / anyPattern / nested entries of var_policy_set: element walks traced
    by kpe_pattern_traces, variables of the element substituted into the messages."""
    pols = var_policy_set()
    lines = [l for l in K.synth_resources(0x5A, 6000, mix=0).split(b"\n") if l]
    n = _check_gpu(oracle, pols, lines, list(range(0, len(lines), 3)),
                   chart_rules={x for x in K.PolicySet(pols).rule_names if "/fe-" in x or "/autogen-fe-" in x
                                or "/autogen-cronjob-fe-" in x}, undecided_ok=VAR_UNDECIDED_OK)
    assert n["wrapped"] > 1000, n


@pytest.mark.gpu
def test_gpu_chart_restricted_messages_equal_oracle(oracle):
    """SURVEY 8(f1) done-criterion: the chart's restricted set, both disallow-capabilities-strict
    foreach rules included, at 20k rows: every validate rule's message equals the oracle's."""
    from tests.test_gpu_pattern import chart_pattern_policies

    pols = chart_pattern_policies()
    assert "disallow-capabilities-strict" in {p["metadata"]["name"] for p in pols}
    lines = [l for l in K.synth_resources(0xC1, 20000, mix=2).split(b"\n") if l]
    names = set(K.PolicySet(pols).rule_names)
    n = _check_gpu(oracle, pols, lines, list(range(0, len(lines), 5)), chart_rules=names)
    assert n["wrapped"] > 100, n
