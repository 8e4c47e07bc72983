"""Oracle (TEST INFRASTRUCTURE ONLY — imported by tests/, never by the product path):
PolicyReport results of one resource, a pure-Python restatement of
EngineResponseToReportResults (pkg/utils/report/results.go:89-156) over the oracle's
verdict cells and its failing PSA check list (oracle/pss.hpp evaluate_pss, which keeps one
entry per failing versioned check, pkg/pss/evaluate.go:24-70).

Restated:
  - policy key: cache.MetaNamespaceKeyFunc -> "<ns>/<name>" or "<name>" (results.go:93)
  - scored: annotation policies.kyverno.io/scored != "false"; category / severity from
    policies.kyverno.io/{category,severity}, SeverityFromString (results.go:73-87, 96-107)
  - toPolicyResult (results.go:56-71); unscored fail => warn (results.go:131-133)
  - properties {standard, version, controls}: failing check ids sorted and comma-joined,
    only when at least one check failed (results.go:114-129); PodSecurityChecks.Level /
    Version are the rule's raw podSecurity strings (validate_pss.go:79-82)
  - JSON omitempty of PolicyReportResult (api/policyreport/v1alpha2/common.go:93-137)
message (when a `pss_message` callable is given): podSecurity pass "Validation rule '<rule>'
passed." (validate_pss.go:85), podSecurity fail without exclusions through the C++ oracle's
FormatChecksPrint (validate_pss.go:108, oracle/pss.hpp format_checks_print), validate.pattern
pass "validation rule '<rule>' passed." (validate_resource.go:339), validate.deny rules: pass
"validation rule '<rule>' passed." (validate_resource.go:275) and, when their conditions (fail) or
preconditions (skip) carry no `message` (so the condition message is empty,
variables/evaluate.go:14-28), fail getDenyMessage (validate_resource.go:279-300: the rule message,
or "validation error: rule <rule> failed" when it is empty; with variables, SubstituteAll through
the oracle's JMESPath when a `substitute` callable is given), preconditions skip "preconditions
not met" (engine.go:283); other messages are not restated (condition messages need the device's
condition traces: tests/test_cond_messages.py checks them against the C++ oracle). Not restated: timestamp, exception
and ValidatingAdmissionPolicy branches (out of the path's scope).
Autogen rules are mapped back to their source rule by the "autogen-" / "autogen-cronjob-"
prefix (pkg/autogen/autogen.go:213-222); names truncated to 63 characters are not mapped
(the fixtures used have short names).
"""
from typing import Callable, Dict, List, Optional

RESULT = {1: "pass", 2: "fail", 3: "warn", 4: "error", 5: "skip"}
SEVERITIES = ("critical", "high", "medium", "low", "info")
_POD_PATH = {  # validate_pss.go:137-188 getSpec
    "Pod": (),
    "CronJob": ("spec", "jobTemplate", "spec", "template"),
}
_TEMPLATE_KINDS = ("DaemonSet", "Deployment", "Job", "StatefulSet", "ReplicaSet", "ReplicationController")


def pod_of(resource: dict) -> Optional[dict]:
    """The Pod (metadata + spec) a podSecurity rule evaluates for this resource."""
    kind = resource.get("kind")
    path = _POD_PATH.get(kind, ("spec", "template") if kind in _TEMPLATE_KINDS else None)
    if path is None:
        return None
    node = resource
    for k in path:
        node = (node or {}).get(k)
    node = node or {}
    return {"kind": "Pod", "metadata": node.get("metadata") or {}, "spec": node.get("spec") or {}}


def _source_rule(policy: dict, rule_name: str) -> dict:
    rules = {r.get("name"): r for r in (policy.get("spec") or {}).get("rules") or []}
    for prefix in ("autogen-cronjob-", "autogen-", ""):
        if rule_name.startswith(prefix) and rule_name[len(prefix):] in rules:
            return rules[rule_name[len(prefix):]]
    return {}


def _cond_messages(block) -> bool:
    """True when a condition in a conditions block (list, or any / all lists) has a message."""
    if isinstance(block, list):
        return any(_cond_messages(c) for c in block)
    if not isinstance(block, dict):
        return False
    if "key" in block or "operator" in block:
        return bool(block.get("message"))
    return _cond_messages(block.get("any")) or _cond_messages(block.get("all"))


def report_results(policies: List[dict], rule_names: List[str], verdict_row, resource: dict,
                   failing_checks: Callable[[str, str, dict], List[str]],
                   pss_message: Optional[Callable[[str, str, str, dict], Optional[str]]] = None,
                   substitute: Optional[Callable[[str, dict], tuple]] = None) -> List[Dict]:
    """[]PolicyReportResult for one resource over all policies (rules in rule_names order).
    substitute: variables.SubstituteAll of a message over the resource (the oracle's), for deny
    rule messages with variables; without it such messages are not restated."""
    by_name = {p["metadata"]["name"]: p for p in policies}
    out = []
    for r, full in enumerate(rule_names):
        cell = int(verdict_row[r])
        if cell not in RESULT:
            continue  # no RuleResponse
        pname, rname = full.split("/", 1)
        pol = by_name[pname]
        meta = pol.get("metadata") or {}
        ann = meta.get("annotations") or {}
        ns = meta.get("namespace") or ""
        scored = ann.get("policies.kyverno.io/scored") != "false"
        res = RESULT[cell]
        if res == "fail" and not scored:
            res = "warn"
        item = {"source": "kyverno", "policy": f"{ns}/{pname}" if ns else pname}
        val = _source_rule(pol, rname).get("validate") or {}
        ps0 = val.get("podSecurity")
        if pss_message is not None:
            msg = None
            if ps0 and cell == 1:
                msg = f"Validation rule '{rname}' passed."
            elif ps0 and cell == 2 and not ps0.get("exclude"):
                msg = pss_message(rname, ps0.get("level", ""), ps0.get("version", ""), resource)
            elif not ps0 and val.get("pattern") is not None and cell == 1:
                msg = f"validation rule '{rname}' passed."
            elif not ps0 and isinstance(val.get("deny"), dict):
                m = val.get("message") if isinstance(val.get("message"), str) else ""
                cond_msgs = _cond_messages(val["deny"].get("conditions"))
                pre_msgs = _cond_messages(_source_rule(pol, rname).get("preconditions"))
                if cell == 1:
                    msg = f"validation rule '{rname}' passed."
                elif (cell == 2 and cond_msgs) or (cell == 5 and pre_msgs):
                    msg = None  # the condition message depends on where the block stopped (traces)
                elif cell == 2 and not m:
                    msg = f"validation error: rule {rname} failed"
                elif cell == 2 and "{{" not in m and "$(" not in m:
                    msg = m
                elif cell == 2 and substitute is not None and "$(" not in m:
                    # getDenyMessage (validate_resource.go:288-299): SubstituteAll; an error gives the
                    # (empty) condition message, a non-string value a fixed text
                    k, text = substitute(m, resource)
                    if k == 0:
                        msg = text
                    elif k == 1:
                        msg = "the produced message didn't resolve to a string, check your policy definition."
                elif cell == 5 and _source_rule(pol, rname).get("preconditions") is not None:
                    msg = "preconditions not met"
            elif (not ps0 and val.get("pattern") is None and val.get("anyPattern") is None
                  and isinstance(val.get("foreach"), list) and val["foreach"] and cell == 1):
                msg = "rule passed"  # validateForEach (validate_resource.go:203)
            if msg:
                item["message"] = msg
        if rname:
            item["rule"] = rname
        item["result"] = res
        if scored:
            item["scored"] = True
        ps = ((_source_rule(pol, rname).get("validate") or {}).get("podSecurity"))
        if ps and cell == 2:
            controls = sorted(failing_checks(ps.get("level", ""), ps.get("version", ""), pod_of(resource)))
            if controls:
                item["properties"] = {"controls": ",".join(controls), "standard": ps.get("level", ""),
                                      "version": ps.get("version", "")}
        if ann.get("policies.kyverno.io/category"):
            item["category"] = ann["policies.kyverno.io/category"]
        sev = ann.get("policies.kyverno.io/severity", "")
        if sev in SEVERITIES:
            item["severity"] = sev
        out.append(item)
    return out


def cli_summary(policies: List[dict], rule_names: List[str], verdicts, audit_warn: bool = False) -> Dict[str, int]:
    """`kyverno apply` totals, ResultCounts.addEngineResponse
    (cmd/cli/kubectl-kyverno/processor/result.go:34-68), over an N x R verdict matrix:
    per resource and policy, every computed validate rule is matched by name against the
    response rules (so duplicate names count twice); unscored fail => warn; with
    --audit-warn a fail of an Audit policy (spec_types.go:31-37) => warn."""
    by_name = {p["metadata"]["name"]: p for p in policies}
    cols: Dict[str, List[int]] = {}
    for r, full in enumerate(rule_names):
        cols.setdefault(full.split("/", 1)[0], []).append(r)
    tot = {"pass": 0, "fail": 0, "warn": 0, "error": 0, "skip": 0}
    for row in verdicts:
        for pname, rs in cols.items():
            pol = by_name[pname]
            responses = [(rule_names[r].split("/", 1)[1], int(row[r])) for r in rs if int(row[r]) in RESULT]
            if not responses:
                continue  # response.IsEmpty()
            ann = (pol.get("metadata") or {}).get("annotations") or {}
            scored = ann.get("policies.kyverno.io/scored") != "false"
            action = (pol.get("spec") or {}).get("validationFailureAction", "")
            audit = action not in ("Enforce", "enforce")
            for r in rs:
                rname = rule_names[r].split("/", 1)[1]
                if not (_source_rule(pol, rname).get("validate")):
                    continue  # rule.HasValidate()
                for name, cell in responses:
                    if name != rname:
                        continue
                    st = RESULT[cell]
                    if st == "fail" and (not scored or (audit_warn and audit)):
                        st = "warn"
                    tot[st] += 1
    return tot
