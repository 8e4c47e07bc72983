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
    return pols
