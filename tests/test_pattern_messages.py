"""Pattern / anyPattern RuleResponse messages (validate_resource.go:316-454
validatePatterns, buildErrorMessage, buildAnyPatternErrorMessage; validate.go PatternError.Path).

CPU: the oracle's messages equal every message pkg/engine/validation_test.go asserts for a
pattern / anyPattern rule (tests/golden/engine_message_cases.json, extracted by make_golden.py).
GPU: the device records each failure's path while re-walking the cell (kpe_pattern_traces) and
kpe_report_results_msg_tr renders the message; it must equal the reference's assertion and the
oracle's message on the chart pattern policies, the C5 pattern set and the validate_test.go trees.
A message whose reference text embeds a Go error string (skips, empty-path failures) is not
rendered by either side and must be absent from the device's result."""
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import c5_policy_set
from tests.test_gpu_pattern import PTREE, _policy_for, chart_pattern_policies, device_policies

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = json.load(open(os.path.join(GOLD, "engine_message_cases.json")))
NEEDS = "\x01"

# validation_test.go message assertions that are not pattern messages the restatement renders:
# variable substitution errors of patterns (`Unknown key "name1" in path`), deny / foreach
# messages with substituted variables, a context (API call) rule
NOT_PATTERN = {"Test_VariableSubstitutionPathNotExistInPattern",
               "Test_VariableSubstitutionPathNotExistInAnyPattern_OnePatternStatisfiesButSubstitutionFails",
               "Test_VariableSubstitutionPathNotExistInAnyPattern_AllPathNotPresent",
               "Test_VariableSubstitutionValidate_VariablesInMessageAreResolved",
               "TestValidate_context_variable_substitution_CLI", "TestValidate_foreach_zero_reported_asskip"}


def _responses(statuses):
    return [r for r, s in enumerate(statuses) if s != 0]


def test_message_fixtures_extracted():
    names = {c["name"] for c in CASES}
    assert {"TestValidate_image_tag_fail", "TestValidate_Fail_anyPattern", "TestValidate_host_network_port",
            "TestValidate_anchor_arraymap_fail", "TestValidate_anchor_map_found_invalid",
            "TestValidate_negationAnchor_deny", "Test_VariableSubstitution_NotOperatorWithStringVariable",
            "Test_VariableSubstitutionPathNotExistInAnyPattern_AllPathPresent_NonePatternSatisfy"} <= names


@pytest.mark.parametrize("case", [c for c in CASES if c["name"] not in NOT_PATTERN], ids=lambda c: c["name"])
def test_oracle_messages_match_reference(oracle, case):
    nd = json.dumps(case["resource"]).encode()
    pols = [case["policy"]]
    st = oracle.validate(pols, nd)[0]
    msgs = oracle.pattern_messages(pols, nd)[0]
    resp = _responses(st)
    for i, want in case["messages"].items():
        r = resp[int(i)]
        assert msgs[r] == want, (case["name"], i, msgs[r], want)


def _device_messages(eng, ps, corpus, v, nd_lines, rows=None):
    """{(row, rule): message} from kpe_report_results_msg_tr with the row's traces."""
    out = {}
    R = ps.num_rules
    for i in (range(v.shape[0]) if rows is None else rows):
        if not (v[i] != 0).any():
            continue
        tr = eng.row_traces(ps, corpus, i)
        res = K.report_results(ps, v[i], resource=nd_lines[i], traces=tr, corpus=corpus)
        names = [n.split("/", 1)[1] for n in ps.rule_names]
        k = 0
        for r in range(R):
            if v[i, r] in (0, 7):
                continue
            assert res[k]["rule"] == names[r]
            out[(i, r)] = res[k].get("message", "")
            k += 1
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in CASES if c["name"] not in NOT_PATTERN], ids=lambda c: c["name"])
def test_device_messages_match_reference(case):
    pols = device_policies([case["policy"]])
    if not pols:
        pytest.skip("policy not compiled for the device")
    nd = json.dumps(case["resource"]).encode()
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet(pols), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    if (v == 7).any():  # a `!` / `|` formed by a substituted variable: undecided on the device
        pytest.skip("cell beyond the device's documented limits (KPE_UNDECIDED)")
    dm = _device_messages(eng, ps, corpus, v, [nd])
    resp = _responses(v[0])
    for i, want in case["messages"].items():
        assert dm[(0, resp[int(i)])] == want, (case["name"], i)


def pattern_rule_names(pols):
    """'<policy>/<rule>' of the validate.pattern / anyPattern rules, with their autogen forms."""
    out = set()
    for p in pols:
        for r in p["spec"]["rules"]:
            v = r.get("validate") or {}
            if v.get("pattern") is not None or v.get("anyPattern") is not None:
                for pre in ("", "autogen-", "autogen-cronjob-"):
                    out.add(p["metadata"]["name"] + "/" + (pre + r["name"])[:63])
    return out


def _compare_with_oracle(oracle, pols, nd, max_rows=None):
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet(pols), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    lines = nd.split(b"\n")
    rows = range(v.shape[0]) if max_rows is None else range(min(max_rows, v.shape[0]))
    om = oracle.pattern_messages(pols, b"\n".join(lines[: rows.stop]))
    dm = _device_messages(eng, ps, corpus, v, lines, rows)
    names = pattern_rule_names(pols)
    pat_cols = {r for r in range(ps.num_rules) if ps.rule_names[r] in names}
    checked = rendered = 0
    for (i, r), got in dm.items():
        if r not in pat_cols:
            continue
        want = om[i][r]
        if want == "" and got == "":
            continue
        checked += 1
        if want == NEEDS:
            assert got == "", (i, ps.rule_names[r], got)
        else:
            assert got == want, (i, ps.rule_names[r], got, want)
            rendered += 1
    assert pat_cols
    return checked, rendered


@pytest.mark.gpu
@pytest.mark.parametrize("mix", [0, 2])
def test_chart_pattern_messages_equal_oracle(oracle, mix):
    pols = chart_pattern_policies()
    nd = K.synth_resources(0xC1 + mix, 600, mix=mix)
    checked, rendered = _compare_with_oracle(oracle, pols, nd)
    assert rendered > 100


@pytest.mark.gpu
def test_c5_pattern_messages_equal_oracle(oracle):
    nd = K.synth_resources(0xC5, 400, mix=K.SYNTH_FANOUT)
    checked, rendered = _compare_with_oracle(oracle, c5_policy_set(), nd)
    assert rendered > 100


@pytest.mark.gpu
def test_tree_pattern_messages_equal_oracle(oracle):
    cases = [c for c in PTREE if isinstance(json.loads(c["resource"]), dict)]
    pols = device_policies([_policy_for(f"t{i}", json.loads(c["pattern"])) for i, c in enumerate(cases)])
    nd = "\n".join(json.dumps(json.loads(c["resource"])) for c in cases).encode()
    checked, rendered = _compare_with_oracle(oracle, pols, nd)
    assert rendered > 0


REPORTS = json.load(open(os.path.join(GOLD, "report_message_cases.json")))


def _expected(case, names):
    """{rule column: message} of the report case's results (rule names as the program lists them)."""
    out = {}
    for res in case["results"]:
        cols = [r for r, n in enumerate(names) if n.split("/", 1)[1] == res["rule"]]
        assert len(cols) == 1, res["rule"]
        out[cols[0]] = (res["result"], res["message"])
    return out


@pytest.mark.parametrize("case", REPORTS, ids=lambda c: c["src"].split("/")[-2] + "/" + c["src"].split("/")[-1])
def test_report_fixture_messages_oracle(oracle, case):
    """Admission-report fixtures (reports/admission/update/report-*-assert.yaml: an autogen rule's
    failure path with its trailing '/'; test-report-admission-mode: a pass message): the oracle's
    RuleResponse messages equal the report's."""
    pols = [case["policy"]]
    nd = json.dumps(case["resource"]).encode()
    names = K.PolicySet(pols).rule_names
    st = oracle.validate(pols, nd)[0]
    msgs = oracle.pattern_messages(pols, nd)[0]
    for col, (result, msg) in _expected(case, names).items():
        assert {1: "pass", 2: "fail"}.get(int(st[col])) == result, (case["src"], col)
        assert msgs[col] == msg, (case["src"], msgs[col], msg)


@pytest.mark.gpu
@pytest.mark.parametrize("case", REPORTS, ids=lambda c: c["src"].split("/")[-2] + "/" + c["src"].split("/")[-1])
def test_report_fixture_messages_device(case):
    """The same report fixtures through the device: verdicts, traces and kpe_report_results_msg_tr."""
    pols = [case["policy"]]
    nd = json.dumps(case["resource"]).encode()
    eng = K.Engine(ordinal=0)
    ps, corpus = K.PolicySet(pols), K.Corpus(nd)
    v, _, _ = eng.evaluate(ps, corpus)
    dm = _device_messages(eng, ps, corpus, v, [nd])
    for col, (result, msg) in _expected(case, ps.rule_names).items():
        assert {1: "pass", 2: "fail"}.get(int(v[0, col])) == result, (case["src"], col)
        assert dm[(0, col)] == msg, (case["src"], dm[(0, col)], msg)


@pytest.mark.gpu
def test_substituted_pattern_messages_equal_oracle(oracle):
    """buildErrorMessage's SubstituteAll of the rule message (validate_resource.go:428-433): the C5
    pattern policies with their messages templated on the resource (names, labels as JSON, a
    missing member: a substitution error, so no message), device against the oracle."""
    import copy as _copy

    pols = _copy.deepcopy(c5_policy_set())
    tmpl = ["{{ request.object.metadata.name }} breaks it", "labels {{ request.object.metadata.labels }}",
            "kind {{request.object.kind}}", "missing {{ request.object.metadata.nope }}"]
    k = 0
    for p in pols:
        for r in p["spec"]["rules"]:
            v = r.get("validate") or {}
            if v.get("pattern") is not None:
                v["message"] = tmpl[k % len(tmpl)]
                k += 1
    nd = K.synth_resources(0xC5 + 1, 300, mix=K.SYNTH_FANOUT)
    checked, rendered = _compare_with_oracle(oracle, pols, nd)
    assert rendered > 50
