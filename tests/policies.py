"""Policy builders shared by the parity tests and bench.py (kyverno.io/v1 schema)."""


def pss_policy(name, level, version="latest", kinds=("Pod",), any_block=True, exclude=None, apply_one=False,
               namespaced_in=None, extra_match=None):
    ps = {"level": level, "version": version}
    if exclude:
        ps["exclude"] = exclude
    res = {"kinds": list(kinds)}
    if extra_match:
        res.update(extra_match)
    match = {"any": [{"resources": res}]} if any_block else {"resources": res}
    spec = {"background": True, "validationFailureAction": "Audit",
            "rules": [{"name": name, "match": match, "validate": {"podSecurity": ps}}]}
    if apply_one:
        spec["applyRules"] = "One"
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"pol-{name}"},
           "spec": spec}
    if namespaced_in:
        pol["kind"] = "Policy"
        pol["metadata"]["namespace"] = namespaced_in
    return pol


def restricted_latest():
    """The C2 policy: chainsaw reports/background/test-report-background-mode/policy.yaml shape."""
    return {
        "apiVersion": "kyverno.io/v1",
        "kind": "ClusterPolicy",
        "metadata": {"name": "podsecurity-subrule-restricted"},
        "spec": {"background": True, "validationFailureAction": "Audit",
                 "rules": [{"name": "restricted", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                            "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}}]},
    }


def parity_policy_set():
    """A mix exercising levels, versions, autogen, kind globs, names/namespaces and exclude blocks."""
    pols = [restricted_latest()]
    for lvl in ("baseline", "restricted", "privileged"):
        for ver in ("latest", "v1.0", "v1.19", "v1.22", "v1.24", "v1.25", "v1.27", "v1.29"):
            pols.append(pss_policy(f"{lvl}-{ver.replace('.', '-')}", lvl, ver))
    pols.append(pss_policy("bad-version", "baseline", "v2.0"))
    pols.append(pss_policy("glob-kinds", "baseline", "latest", kinds=("Pod*", "apps/v1/Deploy*")))
    pols.append(pss_policy("all-kinds", "restricted", "latest", kinds=("*",)))  # matches Service/ConfigMap => error
    pols.append(pss_policy("names", "restricted", "v1.24", extra_match={"names": ["res-1*", "res-2?"]}))
    pols.append(pss_policy("nss", "baseline", "v1.24", extra_match={"namespaces": ["ns-00*", "ns-1?3"]}))
    p = pss_policy("excl", "restricted", "latest")
    p["spec"]["rules"][0]["exclude"] = {"any": [{"resources": {"namespaces": ["ns-05*"]}}]}
    pols.append(p)
    p = pss_policy("one", "baseline", "latest", apply_one=True)
    p["spec"]["rules"].append({"name": "second", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                               "validate": {"podSecurity": {"level": "restricted", "version": "latest"}}})
    pols.append(p)
    pols.append(pss_policy("nsd", "restricted", "latest", namespaced_in="ns-0001"))
    p = pss_policy("legacy", "baseline", "latest", any_block=False)
    pols.append(p)
    p = pss_policy("ann", "restricted", "latest", extra_match={"annotations": {"owner": "team-1*"}})
    pols.append(p)
    pols.append(pss_policy("sel", "baseline", "latest", kinds=("Pod", "Deployment"),
                           extra_match={"selector": {"matchLabels": {"tier": "front*"},
                                                     "matchExpressions": [{"key": "team", "operator": "Exists"}]}}))
    pols.append(pss_policy("nssel", "baseline", "latest", kinds=("*",),
                           extra_match={"namespaceSelector": {"matchExpressions": [
                               {"key": "env", "operator": "NotIn", "values": ["prod"]}]}}))
    return pols


def selector_policy(name, level="baseline", kinds=("Deployment",), selector=None, ns_selector=None, exclude=None,
                    any_filters=None, all_filters=None):
    """A podSecurity rule whose match block uses label selectors (C4 shape)."""
    if any_filters is not None:
        match = {"any": any_filters}
    elif all_filters is not None:
        match = {"all": all_filters}
    else:
        res = {"kinds": list(kinds)}
        if selector is not None:
            res["selector"] = selector
        if ns_selector is not None:
            res["namespaceSelector"] = ns_selector
        match = {"any": [{"resources": res}]}
    rule = {"name": name, "match": match, "validate": {"podSecurity": {"level": level, "version": "latest"}}}
    if exclude is not None:
        rule["exclude"] = exclude
    return {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"sel-{name}"},
            "spec": {"background": True, "validationFailureAction": "Audit", "rules": [rule]}}


def c4_policy_set():
    """C4: matchLabels incl. wildcard keys/values, matchExpressions
    In/NotIn/Exists/DoesNotExist, namespaceSelector over the namespace label table,
    selector excludes, invalid selectors, any/all blocks."""
    P = selector_policy
    return [
        P("eq", selector={"matchLabels": {"k12": "v1"}}),
        P("eq-prefixed", selector={"matchLabels": {"app.kubernetes.io/k13": "v3", "k16": "v0"}}),
        P("wild-value", selector={"matchLabels": {"example.com/k14": "v1*"}}),
        P("wild-key", selector={"matchLabels": {"team.io/*": "v?"}}),
        P("wild-both", selector={"matchLabels": {"*": "*"}}),
        P("wild-miss", selector={"matchLabels": {"nope/*": "*"}}),
        P("in", selector={"matchExpressions": [{"key": "k20", "operator": "In", "values": ["v1", "v2", "v3"]}]}),
        P("notin", selector={"matchExpressions": [{"key": "k24", "operator": "NotIn", "values": ["v0", "v5"]}]}),
        P("exists", selector={"matchExpressions": [{"key": "example.com/k30", "operator": "Exists"}]}),
        P("notexist", selector={"matchExpressions": [{"key": "k32", "operator": "DoesNotExist"}]}),
        P("mixed", kinds=("Deployment", "Service"), selector={
            "matchLabels": {"k36": "v*"},
            "matchExpressions": [{"key": "app.kubernetes.io/k37", "operator": "NotIn", "values": ["v1"]},
                                 {"key": "k40", "operator": "Exists"}]}),
        P("empty-sel", selector={}),
        P("bad-op", selector={"matchExpressions": [{"key": "k1", "operator": "Foo"}]}),
        P("bad-in", selector={"matchExpressions": [{"key": "k1", "operator": "In", "values": []}]}),
        P("bad-key", selector={"matchLabels": {"Bad_/key/x": "v1"}}),
        P("ns-env", ns_selector={"matchLabels": {"env": "prod"}}),
        P("ns-pss", level="restricted", ns_selector={"matchExpressions": [
            {"key": "pss", "operator": "In", "values": ["restricted"]}]}),
        P("ns-wild", kinds=("*",), ns_selector={"matchLabels": {"team": "team-1*"}}),
        P("ns-notexist", kinds=("Service",), ns_selector={"matchExpressions": [
            {"key": "region", "operator": "DoesNotExist"}]}),
        P("ns-bad", ns_selector={"matchExpressions": [{"key": "env", "operator": "Exists", "values": ["x"]}]}),
        P("sel-and-ns", selector={"matchLabels": {"k8": "v2"}}, ns_selector={"matchLabels": {"env": "dev"}}),
        P("excl", selector={"matchLabels": {"k4": "*"}},
          exclude={"any": [{"resources": {"selector": {"matchLabels": {"app.kubernetes.io/k5": "v1"}}}},
                           {"resources": {"namespaceSelector": {"matchLabels": {"env": "staging"}}}}]}),
        P("any-two", any_filters=[{"resources": {"kinds": ["Deployment"], "selector": {"matchLabels": {"example.com/k2": "v0"}}}},
                                  {"resources": {"kinds": ["Deployment"],
                                                 "namespaceSelector": {"matchLabels": {"team": "team-7"}}}}]),
        P("all-two", all_filters=[{"resources": {"kinds": ["Deployment"], "selector": {"matchLabels": {"team.io/k3": "v*"}}}},
                                  {"resources": {"namespaceSelector": {"matchExpressions": [
                                      {"key": "env", "operator": "NotIn", "values": ["dev"]}]}}}]),
    ]


def _golden(name):
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", name)))


def _pattern_policy(name, pattern=None, any_pattern=None, kinds=("Pod",), annotations=None):
    v = {"message": f"{name} failed"}
    if pattern is not None:
        v["pattern"] = pattern
    else:
        v["anyPattern"] = any_pattern
    pol = {"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": name},
           "spec": {"background": True, "validationFailureAction": "Audit",
                    "rules": [{"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]},
                               "validate": v}]}}
    if annotations:
        pol["metadata"]["annotations"] = dict(annotations)
    return pol


def c5_policy_set():
    """C5: test/best_practices/require_pod_requests_limits.yaml and
    disallow_latest_tag.yaml, chart baseline disallow-host-ports (nested =() arrays), and
    conditional / existence / negation / equality-anchor variants shaped like the
    pkg/engine/validation_test.go patterns (:111 conditional image, :1227 ^(containers),
    :1375 X(hostPath)) and pkg/engine/validate/validate_test.go:1368 (`|` with `!`)."""
    bp = _golden("best_practices.json")
    chart = _golden("chart_policies.json")
    pols = list(bp["require_pod_requests_limits.yaml"]) + list(bp["disallow_latest_tag.yaml"])
    pols += [p for p in chart["baseline"] if p["metadata"]["name"] == "disallow-host-ports"]
    pols.append(_pattern_policy("latest-needs-always", {"spec": {"containers": [
        {"(image)": "*:latest", "imagePullPolicy": "Always"}]}}))
    pols.append(_pattern_policy("untagged-not-always", {"spec": {"containers": [
        {"name": "*", "(image)": "*:latest | !*:*", "imagePullPolicy": "!Always"}]}}))
    pols.append(_pattern_policy("has-nginx", {"spec": {"^(containers)": [{"image": "nginx*"}]}}))
    pols.append(_pattern_policy("no-hostpath", {"spec": {"=(volumes)": [{"name": "*", "X(hostPath)": "null"}]}}))
    pols.append(_pattern_policy("memory-cap", {"spec": {"=(initContainers)": [
        {"=(resources)": {"=(limits)": {"=(memory)": "<=1Gi"}}}], "containers": [
        {"=(resources)": {"=(limits)": {"=(memory)": "<=512Mi", "=(cpu)": "<=2"}}}]}}))
    pols.append(_pattern_policy("pinned-image", any_pattern=[
        {"spec": {"containers": [{"image": "*@sha256:*"}]}},
        {"spec": {"containers": [{"image": "*:?*.*"}]}}]))
    return pols


def c3_policy_set(n=200, seed=0xC3):
    """C3: `n` ClusterPolicies whose match / exclude blocks use wildcard kinds
    (`*`, `Deploy*`, `apps/v1/*`, `batch/v1/*`, `*Job`), names (`app-*-?`, `web-*`, `*-db-*`) and
    namespaces (`team-*`, `*-prod`, `team-?-prod`) in any / all / legacy form, with
    podSecurity (Pod-like kinds) or pattern handlers. Deterministic in `seed`."""
    import random
    rng = random.Random(seed)
    kinds_pool = [["*"], ["Deploy*"], ["apps/v1/*"], ["Pod"], ["Pod", "Deployment"], ["batch/v1/*"], ["Service"],
                  ["ConfigMap"], ["StatefulSet", "DaemonSet"], ["*Job"], ["v1/Pod"], ["Pod", "Deploy*"],
                  ["Service", "ConfigMap"], ["apps/*/Deployment"], ["*/*"]]
    podlike = {"Pod", "Deploy*", "apps/v1/*", "v1/Pod", "StatefulSet", "DaemonSet", "Deployment", "*Job",
               "batch/v1/*", "apps/*/Deployment"}
    names_pool = [None, None, ["app-*-?"], ["app-*"], ["web-*"], ["*-db-*"], ["app-api-?", "web-ui-*"]]
    ns_pool = [None, None, ["team-*"], ["*-prod"], ["team-?-prod"], ["team-1*", "shop-*"], ["default"]]
    excl_pool = [None, None, None, {"namespaces": ["kube-*"]}, {"names": ["*-canary"]}, {"kinds": ["ConfigMap"]},
                 {"namespaces": ["*-dev"], "names": ["app-*"]}]
    patterns = [
        {"metadata": {"labels": {"app": "?*"}}},
        {"metadata": {"labels": {"tier": "front* | back*"}}},
        {"metadata": {"=(annotations)": {"=(owner)": "team-*"}}},
        {"metadata": {"name": "!*-canary"}},
        {"spec": {"=(replicas)": "<5"}},
    ]
    pod_patterns = [
        {"spec": {"containers": [{"image": "!*:latest"}]}},
        {"spec": {"=(hostNetwork)": False}},
        {"spec": {"containers": [{"=(securityContext)": {"=(privileged)": False}}]}},
    ]
    pols = []
    for i in range(n):
        def resdesc():
            rd = {"kinds": list(rng.choice(kinds_pool))}
            nm = rng.choice(names_pool)
            if nm:
                rd["names"] = list(nm)
            ns = rng.choice(ns_pool)
            if ns:
                rd["namespaces"] = list(ns)
            return rd
        rd = resdesc()
        mode = rng.random()
        if mode < 0.6:
            match = {"any": [{"resources": rd}] + ([{"resources": resdesc()}] if rng.random() < 0.3 else [])}
        elif mode < 0.8:
            match = {"all": [{"resources": rd}, {"resources": {"namespaces": list(rng.choice(ns_pool[2:]))}}]}
        else:
            match = {"resources": rd}
        rule = {"name": f"r{i}", "match": match}
        ex = rng.choice(excl_pool)
        if ex:
            rule["exclude"] = {"any": [{"resources": dict(ex)}]}
        is_pod = all(k in podlike for k in rd["kinds"])
        h = rng.random()
        if is_pod and h < 0.45:
            rule["validate"] = {"podSecurity": {"level": rng.choice(["baseline", "restricted"]),
                                                "version": rng.choice(["latest", "v1.24", "v1.29"])}}
        elif is_pod and h < 0.75:
            rule["validate"] = {"message": "m", "pattern": rng.choice(pod_patterns)}
        else:
            rule["validate"] = {"message": "m", "pattern": rng.choice(patterns)}
        pols.append({"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": f"c3-{i:03d}"},
                     "spec": {"background": True, "validationFailureAction": "Audit", "rules": [rule]}})
    return pols


def cond_policy_set():
    """Preconditions / deny / foreach-deny rules whose conditions read the resource (evaluated
    per resource by kpe_cond_kernel): every operator family (variables/operator/*.go) over
    strings, numbers, lists and missing values, the JMESPath forms the device restates
    (fields, [n], [], [*], multi-select, keys(@), `||` defaults) and foreach with element
    preconditions, elementScope and elementIndex (validate_resource.go:186-254)."""
    def rule(name, validate, pre=None, kinds=("Pod", "Deployment", "Service", "ConfigMap")):
        r = {"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]}, "validate": validate}
        if pre is not None:
            r["preconditions"] = pre
        return r

    def deny(*conds, any_block=False):
        return {"message": "m", "deny": {"conditions": {("any" if any_block else "all"): list(conds)}}}

    def c(key, op, value):
        return {"key": key, "operator": op, "value": value}

    obj = "request.object"
    spec_ctrs = "{{ " + obj + ".spec.[initContainers, containers][] }}"
    rules = [
        rule("app-anyin", deny(c("{{ " + obj + ".metadata.labels.app }}", "AnyIn", ["app-1*", "app-2?"]))),
        rule("team-strict", deny(c("{{ " + obj + ".metadata.labels.team }}", "Equals", "team-1"))),  # missing => error
        rule("team-default", deny(c("{{ " + obj + ".metadata.labels.team || 'none' }}", "NotEquals", "none"))),
        rule("tier-notin", deny(c("{{ " + obj + ".metadata.labels.tier }}", "NotIn", ["frontend"]))),
        rule("tier-in-scalar", deny(c("{{ " + obj + ".metadata.labels.tier }}", "In", "back*"))),
        rule("images-allnotin", deny(c("{{ " + obj + ".spec.containers[].image }}", "AllNotIn", ["*:latest"]))),
        rule("images-anyin", deny(c("{{ " + obj + ".spec.[initContainers, containers][].image }}", "AnyIn",
                                    ["nginx:*", "redis:*"]))),
        rule("names-any-or", deny(c("{{ " + obj + ".spec.[initContainers, containers][].name }}", "AnyIn",
                                    ["init-*"]),
                                  c("{{ " + obj + ".metadata.name }}", "Equals", "res-1?"), any_block=True)),
        rule("replicas-eq", deny(c("{{ " + obj + ".spec.replicas || `1` }}", "Equals", 3)), kinds=("Deployment",)),
        rule("replicas-anyin", deny(c("{{ " + obj + ".spec.replicas }}", "AnyIn", ["2", "4"])), kinds=("Deployment",)),
        rule("ports-first", deny(c("{{ " + obj + ".spec.containers[0].ports[0].containerPort || `0` }}", "Equals",
                                   "8080"))),
        rule("ns-list-key", deny(c(["{{ " + obj + ".metadata.namespace }}"], "NotIn", ["ns-0001", "ns-0002"]))),
        # a string with a variable inside it as one element of a list (value side, then key side)
        rule("list-tmpl-value", deny(c("{{ " + obj + ".metadata.name }}", "AnyIn",
                                       ["{{ " + obj + ".metadata.namespace }}-x", "res-1*", "web"]))),
        rule("list-tmpl-key", deny(c(["{{ " + obj + ".metadata.namespace }}/{{ " + obj + ".metadata.name }}",
                                      "{{ " + obj + ".kind }}"], "AnyIn", ["ns-000?/res-2*", "Service"]))),
        # several partial-string elements, one after another in the side's lane text slot
        rule("list-tmpl-two", deny(c(["{{ " + obj + ".metadata.namespace }}/{{ " + obj + ".metadata.name }}",
                                      "k-{{ " + obj + ".kind }}", "{{ " + obj + ".metadata.name }}"], "AnyIn",
                                     ["ns-000?/res-2*", "k-Service", "x-{{ " + obj + ".metadata.namespace }}",
                                      "{{ " + obj + ".kind }}-{{ " + obj + ".metadata.name }}"]))),
        rule("vol-keys", deny(c("{{ " + obj + ".spec.volumes[].keys(@)[] || '' }}", "AnyNotIn",
                                ["name", "configMap", "emptyDir", ""]))),
        rule("caps-add", deny(c("{{ " + obj + ".spec.[ephemeralContainers, initContainers, containers][]."
                                "securityContext.capabilities.add[] }}", "AnyNotIn", ["CHOWN", "NET_BIND_SERVICE"]))),
        rule("star-proj", deny(c("{{ " + obj + ".spec.containers[*].name }}", "AllIn", ["c-*", "init-*"]))),
        rule("missing-default", deny(c("{{ " + obj + ".spec.nothing || `[]` }}", "Equals", []))),
        rule("pre-ns", {"message": "m", "pattern": {"metadata": {"name": "res-*"}}},
             pre={"all": [c("{{ " + obj + ".metadata.namespace }}", "NotEquals", "ns-00*")]}),
        rule("pre-kind-pss", {"podSecurity": {"level": "baseline", "version": "latest"}},
             pre={"any": [c("{{ " + obj + ".metadata.labels.tier }}", "Equals", "frontend")]}, kinds=("Pod",)),
        rule("pre-only", {"message": "m"}, pre=[c("{{ " + obj + ".kind }}", "Equals", "Service")]),
        rule("foreach-image", {"message": "m", "foreach": [{
            "list": obj + ".spec.containers",
            "preconditions": {"all": [c("{{ element.name }}", "NotEquals", "c-0")]},
            "deny": {"conditions": {"any": [c("{{ element.image }}", "Equals", "*:latest")]}}}]}),
        rule("foreach-strings", {"message": "m", "foreach": [{
            "list": obj + ".spec.containers[].image",
            "deny": {"conditions": {"all": [c("{{ element }}", "NotEquals", "nginx*")]}}}]}),
        rule("foreach-scope", {"message": "m", "foreach": [{
            "list": obj + ".spec.containers[].image", "elementScope": True,
            "deny": {"conditions": {"all": [c("{{ element }}", "Equals", "x")]}}}]}),
        rule("foreach-index", {"message": "m", "foreach": [{
            "list": obj + ".spec.[initContainers, containers][]",
            "deny": {"conditions": {"all": [c("{{ elementIndex }}", "Equals", 2),
                                            c("{{ element.securityContext.privileged || `false` }}", "Equals",
                                              False)]}}}]}),
        rule("foreach-drop-all", {"message": "m", "foreach": [{
            "list": obj + ".spec.[ephemeralContainers, initContainers, containers][]",
            "deny": {"conditions": {"all": [c("ALL", "AnyNotIn",
                                              "{{ element.securityContext.capabilities.drop[] || `[]` }}")]}}}]}),
        rule("foreach-none", {"message": "m", "foreach": [{
            "list": obj + ".spec.missing[]",
            "deny": {"conditions": {"all": [c("{{ element }}", "Equals", "x")]}}}]}),
        rule("spec-ctrs-count", deny(c(spec_ctrs, "Equals", []))),
        # length() (go-jmespath functions.go jpfLength) as a function and after a pipe
        rule("len-pipe", deny(c("{{ " + obj + ".spec.containers[] | length(@) }}", "GreaterThan", "2"))),
        rule("len-name", deny(c("{{ length(" + obj + ".metadata.name) }}", "LessThanOrEquals", 5))),
        rule("len-labels", deny(c("{{ length(" + obj + ".metadata.labels) }}", "Equals", 2))),
        rule("len-missing", deny(c("{{ length(" + obj + ".spec.nothing) }}", "Equals", 0))),  # null => error
        rule("len-vols", deny(c("{{ length(" + obj + ".spec.volumes[]) }}", "AnyIn", ["1", "3"]))),
        rule("len-proj", deny(c("{{ " + obj + ".spec.containers[*].ports[] | length(@) }}", "GreaterThanOrEquals",
                                1))),
        # variables inside strings (substituteVariablesIfAny, vars.go:311-389): strings as is, other
        # values json.Marshal-ed
        rule("tmpl-ns-name", deny(c("{{ " + obj + ".metadata.namespace }}/{{ " + obj + ".metadata.name }}",
                                    "Equals", "ns-000*/res-1*"))),
        rule("tmpl-value", deny(c("{{ " + obj + ".metadata.name }}", "NotEquals",
                                  "res-{{ " + obj + ".metadata.labels.tier || 'x' }}*"))),
        rule("tmpl-number", deny(c("n={{ " + obj + ".spec.replicas || `1` }}", "AnyIn", ["n=3", "n=1"]))),
        rule("tmpl-bool-null", deny(c("{{ " + obj + ".spec.hostNetwork || `false` }}:{{ " + obj +
                                      ".spec.nothing || `null` }}", "Equals", "false:null"))),
        rule("tmpl-len", deny(c("{{ length(" + obj + ".metadata.name) }}-{{ " + obj + ".kind }}", "In",
                                ["5-Pod", "6-Pod", "7-Service"]))),
        rule("tmpl-missing", deny(c("x-{{ " + obj + ".metadata.labels.team }}", "Equals", "x-team-1"))),  # error
        rule("foreach-tmpl", {"message": "m", "foreach": [{
            "list": obj + ".spec.containers",
            "deny": {"conditions": {"any": [c("{{ element.name }}@{{ element.image }}", "Equals", "c-0@*:latest"),
                                            c("{{ elementIndex }}:{{ element.name }}", "Equals", "1:c-?")]}}}]}),
    ]
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "cond"},
             "spec": {"background": True, "validationFailureAction": "Audit", "rules": rules}}]


def cond_message_policy_set():
    """cond_policy_set with a `message` on every condition of its preconditions and deny blocks
    (kyvernov1.Condition.Message) and rule messages that vary: none, plain text, a substituted
    resource field, a non-string value and a missing member (getDenyMessage,
    validate_resource.go:279-300), plus old-style and any + all blocks with messages, some empty,
    some with variables (substituted only after the join). EvaluateConditions' message
    (variables/evaluate.go:31-125) depends on where each block stopped."""
    import copy

    pols = copy.deepcopy(cond_policy_set())
    obj = "request.object"
    rmsgs = ["", "m", "{{ " + obj + ".metadata.name }} is denied", "{{ " + obj + ".metadata.labels }}",
             "x {{ " + obj + ".metadata.nope }}", "kind {{ " + obj + ".kind }}."]

    def tag(block, prefix):
        if isinstance(block, list):
            for k, cnd in enumerate(block):
                cnd["message"] = f"{prefix}{k}" if k % 3 != 2 else ""
            return
        for part in ("any", "all"):
            for k, cnd in enumerate(block.get(part) or []):
                cnd["message"] = f"{prefix}{part}{k}" + (" {{ " + obj + ".kind }}" if k == 1 else "")

    rules = pols[0]["spec"]["rules"]
    for i, r in enumerate(rules):
        v = r["validate"]
        if "preconditions" in r:
            tag(r["preconditions"], f"p{i}.")
        if "deny" in v:
            tag(v["deny"]["conditions"], f"d{i}.")
            m = rmsgs[i % len(rmsgs)]
            if m:
                v["message"] = m
            else:
                v.pop("message", None)

    def c(key, op, value, msg):
        return {"key": key, "operator": op, "value": value, "message": msg}

    name = "{{ " + obj + ".metadata.name }}"
    ns = "{{ " + obj + ".metadata.namespace }}"
    k_ = ("Pod", "Deployment", "Service", "ConfigMap")

    def rule(rn, validate, pre=None):
        r = {"name": rn, "match": {"any": [{"resources": {"kinds": list(k_)}}]}, "validate": validate}
        if pre is not None:
            r["preconditions"] = pre
        return r

    rules += [
        # any + all: the true `any` message and every `all` message, or the false ones
        rule("msg-any-all", {"message": "deny {{ " + obj + ".kind }}", "deny": {"conditions": {
            "any": [c(name, "Equals", "res-1*", "name-1"), c(ns, "Equals", "ns-0001", "ns-1")],
            "all": [c("{{ " + obj + ".kind }}", "NotEquals", "Service", "not-svc"),
                    c(name, "NotEquals", "res-19*", "")]}}}),
        # old-style deny list: the first false message, else the true ones joined by ";"
        rule("msg-old-deny", {"deny": {"conditions": [c(name, "Equals", "res-*", "a"), c(ns, "NotEquals", "ns-0003", "b"),
                                                      c(name, "Equals", "res-2*", "")]}}),
        # preconditions with messages on a pattern rule (its skip) and an old-style list
        rule("msg-pre-pattern", {"message": "m", "pattern": {"metadata": {"name": "res-*"}}},
             pre={"any": [c(ns, "Equals", "ns-0001", "in ns-1"), c(name, "Equals", "res-3*", "name res-3")],
                  "all": [c("{{ " + obj + ".kind }}", "Equals", "Pod", "a pod")]}),
        rule("msg-pre-old", {"message": "m", "deny": {"conditions": {"all": [c(name, "Equals", "res-1*", "res-1 {{ " + obj + ".kind }}")]}}},
             pre=[c("{{ " + obj + ".kind }}", "NotEquals", "ConfigMap", "not a cm"), c(ns, "NotEquals", "ns-0002", "")]),
        # a deny block whose messages are all empty, and one holding only a variable message
        rule("msg-empty", {"deny": {"conditions": {"any": [c(name, "Equals", "res-1*", ""), c(ns, "Equals", "ns-0002", "")]}}}),
        rule("msg-var-only", {"deny": {"conditions": {"all": [c(ns, "Equals", "ns-000*", "{{ " + obj + ".metadata.namespace }}")]}}}),
        rule("msg-var-missing", {"message": "r", "deny": {"conditions": {"all": [c(ns, "Equals", "ns-000*",
                                                                                   "{{ " + obj + ".metadata.zzz }}")]}}}),
    ]
    return pols


def var_policy_set():
    """Pattern rules with {{ }} variables (substitutePatterns, validate_resource.go:456-476) and
    foreach entries with pattern / anyPattern / nested foreach bodies (validate_resource.go:
    186-254), over the synth_resources mixes (kinds Pod, autogen controllers)."""
    def rule(name, validate, pre=None):
        r = {"name": name, "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
             "validate": dict(validate, message="m")}
        if pre is not None:
            r["preconditions"] = pre
        return r
    ctr = "request.object.spec.containers"
    rules = [
        # whole-string variables keep the JSON type: strings, numbers, a missing key (error)
        rule("v-same-tier", {"pattern": {"metadata": {"labels": {"tier": "{{request.object.metadata.labels.tier}}"}}}}),
        rule("v-app-owner", {"pattern": {"metadata": {"labels": {"app": "{{request.object.metadata.annotations.owner}}"}}}}),
        rule("v-default", {"pattern": {"metadata": {"labels": {"tier": "{{request.object.metadata.labels.zone || 'backend'}}"}}}}),
        rule("v-star", {"pattern": {"spec": {"volumes": "{{request.object.metadata.labels.star || '*'}}"}}}),
        rule("v-number", {"pattern": {"spec": {"containers": [{"name": "c-{{request.object.spec.containers[0].ports[0].containerPort || `0`}}*"}]}}}),
        rule("v-idx", {"pattern": {"spec": {"containers": [{"image": "*{{request.object.metadata.labels.tier}}*"}]}}}),
        rule("v-tmpl-name", {"pattern": {"metadata": {"name": "res-{{request.object.spec.containers[0].name}}"}}}),
        rule("v-anchor", {"pattern": {"metadata": {"=(labels)": {"=(tier)": "{{request.object.metadata.labels.tier}}"},
                                                   "name": "{{request.object.metadata.name}}"}}}),
        rule("v-any", {"anyPattern": [{"metadata": {"labels": {"app": "{{request.object.metadata.labels.tier}}"}}},
                                      {"metadata": {"namespace": "{{request.object.metadata.namespace}}"}}]}),
        rule("v-pre", {"pattern": {"spec": {"containers": [{"name": "{{request.object.spec.containers[0].name}}"}]}}},
             pre={"all": [{"key": "{{request.object.metadata.labels.tier}}", "operator": "Equals", "value": "backend"}]}),
        rule("v-map", {"pattern": {"spec": {"securityContext": "{{request.object.spec.securityContext}}"}}}),
        rule("v-len", {"pattern": {"spec": {"containers": [{"ports": [{"containerPort": "{{ length(request.object.spec.containers) }}"}]}]}}}),
        rule("v-len-pipe", {"pattern": {"metadata": {"labels": "{{ request.object.metadata.labels | length(@) }}"}}}),
        # variables in map keys (jsonutils/traverse.go:90-117: keys are substituted and renamed)
        rule("vk-default", {"pattern": {"metadata": {"labels": {"{{request.object.metadata.labels.kind || 'team'}}": "team-?"}}}}),
        rule("vk-tmpl", {"pattern": {"metadata": {"labels": {"ti{{request.object.metadata.labels.zone || 'er'}}": "back*"}}}}),
        rule("vk-own", {"pattern": {"metadata": {"labels": {"{{request.object.metadata.labels.tier}}": "*"}}}}),
        rule("vk-order", {"pattern": {"metadata": {"labels": {"app": "?*", "{{request.object.metadata.labels.tier}}": "*",
                                                              "zzz": "!x"}}}}),
        rule("vk-collide", {"pattern": {"metadata": {"labels": {"app": "?*", "{{request.object.metadata.labels.kind || 'app'}}": "x"}}}}),
        rule("vk-number", {"pattern": {"spec": {"{{request.object.spec.containers[0].ports[0].containerPort}}": "x"}}}),
        rule("vk-spec", {"pattern": {"spec": {"{{request.object.metadata.labels.field || 'containers'}}": [{"name": "c-*"}]}}}),
        # several whole-string key variables in one map; equal substituted keys collide (undecided)
        rule("vk-two", {"pattern": {"metadata": {"labels": {"{{request.object.metadata.labels.zone || 'tier'}}": "back*",
                                                            "{{request.object.metadata.annotations.owner || 'app'}}": "?*"}}}}),
        # anchored keys with variables: renamed first (traverse.go:90-117), then parsed as anchors
        rule("vk-anchor-eq", {"pattern": {"metadata": {"labels": {"=({{request.object.metadata.labels.zone || 'tier'}})": "back*"}}}}),
        rule("vk-anchor-cond", {"pattern": {"metadata": {"labels": {
            "({{request.object.metadata.annotations.owner || 'tier'}})": "front*", "app": "app-1*"}}}}),
        rule("vk-anchor-neg", {"pattern": {"metadata": {"labels": {"X({{request.object.metadata.annotations.owner || 'tier'}})": "null"}}}}),
        rule("vk-anchor-order", {"pattern": {"metadata": {"labels": {"=(c)": "x",
                                                                     "=({{request.object.metadata.labels.tier}})": "x*"}}}}),
        rule("vk-two-collide", {"pattern": {"metadata": {"labels": {"{{request.object.metadata.annotations.owner || 'x1'}}": "?*",
                                                                    "{{request.object.metadata.annotations.owner || 'x2'}}": "?*"}}}}),
        # foreach entries
        rule("fe-pat", {"foreach": [{"list": ctr, "pattern": {"securityContext": {"=(privileged)": False}}}]}),
        rule("fe-pat-var", {"foreach": [{"list": ctr, "pattern": {"name": "c-{{elementIndex}}"}}]}),
        rule("fe-pat-el", {"foreach": [{"list": ctr, "pattern": {"image": "{{element.name}}*"}}]}),
        rule("fe-any", {"foreach": [{"list": ctr, "anyPattern": [{"image": "*:latest"}, {"name": "init-*"}]}]}),
        rule("fe-pre", {"foreach": [{"list": ctr, "preconditions": {"any": [{"key": "{{element.image}}", "operator": "Equals",
                                                                             "value": "*:latest"}]},
                                      "pattern": {"securityContext": {"runAsNonRoot": True}}}]}),
        rule("fe-nested", {"foreach": [{"list": ctr, "foreach": [{"list": "element.ports",
                                                                   "pattern": {"containerPort": "<9000"}}]}]}),
        rule("fe-nested-el0", {"foreach": [{"list": ctr, "foreach": [{"list": "element.securityContext.capabilities.drop",
                                                                       "deny": {"conditions": {"any": [
                                                                           {"key": "{{element0.name}}", "operator": "Equals",
                                                                            "value": "c-0"}]}}}]}]}),
        rule("fe-unscoped", {"foreach": [{"list": "request.object.metadata.labels.tier", "elementScope": False,
                                          "pattern": {"metadata": {"labels": {"tier": "{{element}}"}}}}]}),
        rule("fe-scope-bad", {"foreach": [{"list": "request.object.metadata.labels.app", "elementScope": True,
                                           "pattern": {"x": "y"}}]}),
        rule("fe-two", {"foreach": [{"list": "request.object.spec.initContainers", "pattern": {"image": "*:1.*"}},
                                    {"list": ctr, "pattern": {"image": "!*:latest"}}]}),
        rule("fe-none", {"foreach": [{"list": ctr}]}),
    ]
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "vars"},
             "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}]


# rules of var_policy_set whose cells the device may leave KPE_UNDECIDED (a variable resolving
# to a map is a pattern subtree; documented device limit)
# vk-*collide: a key renamed onto another key; vk-anchor-order: an anchor key that sorts elsewhere
VAR_UNDECIDED_OK = {"v-map", "vk-collide", "vk-two-collide", "vk-anchor-order"}


def foreach_message_policy_set():
    """validate.foreach rules and RuleError texts for the message renderers (validate_resource.go:
    121-254: foreach pass "rule passed", "validation failure: <element message>" once per nesting
    level, and the RuleError texts of preconditions / deny / pattern substitution errors, engine.go
    :279-281). The chart's restricted disallow-capabilities-strict rules first (charts/kyverno-
    policies/templates/restricted/disallow-capabilities-strict.yaml, rendered with the default
    values)."""
    obj = "request.object"
    ctrs = obj + ".spec.[ephemeralContainers, initContainers, containers][]"
    not_delete = {"all": [{"key": "{{ request.operation || 'BACKGROUND' }}", "operator": "NotEquals", "value": "DELETE"}]}

    def rule(name, validate, pre=None, kinds=("Pod",)):
        r = {"name": name, "match": {"any": [{"resources": {"kinds": list(kinds)}}]}, "validate": validate}
        if pre is not None:
            r["preconditions"] = pre
        return r

    def c(key, op, value, message=None):
        x = {"key": key, "operator": op, "value": value}
        if message is not None:
            x["message"] = message
        return x

    rules = [
        rule("require-drop-all", {"message": "Containers must drop `ALL` capabilities.", "foreach": [
            {"list": ctrs, "deny": {"conditions": {"all": [
                c("ALL", "AnyNotIn", "{{ element.securityContext.capabilities.drop[] || `[]` }}")]}}}]}, pre=not_delete),
        rule("adding-capabilities-strict", {
            "message": "Any capabilities added other than NET_BIND_SERVICE are disallowed.", "foreach": [
                {"list": ctrs, "deny": {"conditions": {"all": [
                    c("{{ element.securityContext.capabilities.add[] || `[]` }}", "AnyNotIn",
                      ["NET_BIND_SERVICE", ""])]}}}]}, pre=not_delete),
        # condition messages, element variables in the rule message
        rule("fe-cond-msg", {"message": "container {{ element.name }} ({{ elementIndex }}) of {{ request.object.metadata.name }}",
                             "foreach": [{"list": obj + ".spec.containers", "deny": {"conditions": {"any": [
                                 c("{{ element.image }}", "Equals", "*:latest", "latest tag"),
                                 c("{{ element.securityContext.privileged || `false` }}", "Equals", True, "privileged")]}}}]}),
        rule("fe-no-msg", {"foreach": [{"list": obj + ".spec.containers[].image", "deny": {"conditions": {"all": [
            c("{{ element }}", "NotEquals", "nginx*")]}}}]}),
        rule("fe-all-msgs", {"message": "m.", "foreach": [{"list": obj + ".spec.containers", "deny": {"conditions": {"all": [
            c("{{ element.name }}", "Equals", "c-*", "named c-"),
            c("{{ element.image }}", "NotEquals", "redis:*", "not redis")]}}}]}),
        # nested foreach: wrapped twice
        rule("fe-nested-deny", {"message": "port {{ element.containerPort }} at {{ elementIndex1 }}", "foreach": [
            {"list": obj + ".spec.containers", "foreach": [{"list": "element.ports", "deny": {"conditions": {"all": [
                c("{{ element.containerPort }}", "GreaterThan", 8000)]}}}]}]}),
        # errors raised by an element: preconditions / deny substitutions (NotFound), elementScope
        rule("fe-pre-err", {"message": "m", "foreach": [{"list": obj + ".spec.containers", "preconditions": {"all": [
            c("{{ element.securityContext.runAsUser }}", "Equals", 0)]},
            "deny": {"conditions": {"all": [c("a", "Equals", "a")]}}}]}),
        rule("fe-deny-err", {"message": "m", "foreach": [{"list": obj + ".spec.containers", "deny": {"conditions": {"any": [
            c("x", "Equals", ["{{ element.name }}", "{{ element.resources.limits.memory }}"])]}}}]}),
        rule("fe-scope-err", {"message": "m", "foreach": [{"list": obj + ".spec.containers[].name", "elementScope": True,
                                                          "deny": {"conditions": {"all": [c("a", "Equals", "a")]}}}]}),
        # pattern entries on the element
        rule("fe-pattern", {"message": "image of {{ element.name }} must be pinned",
                            "foreach": [{"list": obj + ".spec.containers", "pattern": {"image": "!*:latest"}}]}),
        rule("fe-pattern-nomsg", {"foreach": [{"list": ctrs, "pattern": {"securityContext": {"runAsNonRoot": True}}}]}),
        rule("fe-any", {"message": "pinned or init", "foreach": [{"list": obj + ".spec.containers", "anyPattern": [
            {"image": "*:1.*"}, {"name": "init-*"}]}]}),
        rule("fe-pvar-err", {"foreach": [{"list": obj + ".spec.containers", "pattern": {
            "image": "{{ element.imagePullPolicy }}*"}}]}),
        rule("fe-any-bad", {"foreach": [{"list": obj + ".spec.containers", "anyPattern": {"image": "x"}}]}),
        rule("fe-nested-pat", {"foreach": [{"list": obj + ".spec.containers", "foreach": [
            {"list": "element.ports", "pattern": {"containerPort": "<8000"}}]}]}),
        # rule-level RuleErrors
        rule("pre-err", {"message": "m", "pattern": {"metadata": {"name": "?*"}}},
             pre={"all": [c("{{ " + obj + ".metadata.labels.team }}", "Equals", "x")]}),
        rule("pre-nil-query", {"message": "m", "deny": {"conditions": {"all": [c("{{ " + obj + ".kind }}", "Equals", "Pod")]}}},
             pre={"any": [c("{{ }}", "Equals", "x")]}),
        rule("deny-err-value", {"message": "m", "deny": {"conditions": [
            c("{{ " + obj + ".kind }}", "In", ["Pod", "{{ " + obj + ".metadata.labels.team }}"])]}}),
        rule("deny-bad-op", {"message": "m", "deny": {"conditions": {"all": [c("{{ " + obj + ".kind }}", "Bogus", "Pod")]}}}),
        rule("pat-var-err", {"message": "m", "pattern": {"metadata": {"labels": {"app": "{{ " + obj + ".metadata.labels.team }}"}}}}),
        rule("any-bad", {"message": "m", "anyPattern": {"metadata": {"name": "x"}}}),
    ]
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "femsg"},
             "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}]
