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
