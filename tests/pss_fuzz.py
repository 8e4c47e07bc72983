"""Random pods and podSecurity exclusion lists for the exclusion parity tests: every field a
PSA check reads, in legal and bad states, container names that repeat and carry digits (the
field-path normalisation), image globs, and exclusions that mix pod-level and image entries
on the same control (the swap-remove order of exemptExclusions matters there)."""
import json
import random

CTR_TYPES = ("initContainers", "containers", "ephemeralContainers")
IMAGES = ["nginx", "nginx:1.25", "busybox", "registry.k8s.io/pause:3.9", "app1:v2", "app2:v2"]
NAMES = ["app", "app1", "app2", "sidecar", "nginx", "init0", "fake", "x"]
CAPS = ["NET_BIND_SERVICE", "CHOWN", "SYS_ADMIN", "NET_RAW", "ALL", "KILL", "SETUID"]
SECCOMP = ["RuntimeDefault", "Localhost", "Unconfined", "", "bogus"]
SYSCTLS = ["kernel.shm_rmid_forced", "net.ipv4.ip_local_reserved_ports", "net.ipv4.tcp_keepalive_time",
           "kernel.msgmax", "net.ipv4.ip_unprivileged_port_start", ""]
ANN_VALUES = ["runtime/default", "localhost/prof", "unconfined", "docker/default", ""]
VOLUMES = [{"emptyDir": {}}, {"hostPath": {"path": "/x"}}, {"nfs": {"server": "s", "path": "/"}},
           {"configMap": {"name": "c"}}, {"gcePersistentDisk": {"pdName": "p"}}, {"cephfs": {"monitors": ["m"]}},
           {"secret": {"secretName": "s"}}, {"hostPath": {"path": "/y"}, "nfs": {"server": "s", "path": "/"}}]
CONTROLS = ["Capabilities", "Seccomp", "Privileged Containers", "Host Ports", "/proc Mount Type", "HostProcess",
            "SELinux", "Host Namespaces", "HostPath Volumes", "Sysctls", "AppArmor", "Privilege Escalation",
            "Running as Non-root", "Running as Non-root user", "Volume Types", "Unknown Control"]
CTR_FIELDS = ["securityContext.allowPrivilegeEscalation", "securityContext.capabilities.add",
              "securityContext.capabilities.drop", "ports[*].hostPort", "securityContext.privileged",
              "securityContext.procMount", "securityContext.runAsNonRoot", "securityContext.runAsUser",
              "securityContext.seLinuxOptions.type", "securityContext.seLinuxOptions.user",
              "securityContext.seLinuxOptions.role", "securityContext.seccompProfile.type",
              "securityContext.windowsOptions.hostProcess"]
POD_FIELDS = ["spec.hostNetwork", "spec.hostPID", "spec.hostIPC", "spec.securityContext.runAsNonRoot",
              "spec.securityContext.runAsUser", "spec.securityContext.seLinuxOptions.type",
              "spec.securityContext.seLinuxOptions.user", "spec.securityContext.seccompProfile.type",
              "spec.securityContext.sysctls[*].name", "spec.securityContext.windowsOptions.hostProcess",
              "spec.volumes[*].hostPath", "spec.volumes[*].nfs", "spec.volumes[*].gcePersistentDisk",
              "spec.volumes[*].unknown", "spec.containers[0].securityContext.privileged",
              "metadata.annotations[container.apparmor.security.beta.kubernetes.io/app*]",
              "metadata.annotations[container.apparmor.security.beta.kubernetes.io/nginx]",
              "metadata.annotations[seccomp.security.alpha.kubernetes.io/pod]",
              "metadata.annotations[container.seccomp.security.alpha.kubernetes.io/app*]",
              "metadata.annotations[container.seccomp.security.alpha.kubernetes.io/fake]"]
VALUES = ["true", "false", "0", "*", "SYS_ADMIN", "NET_*", "CHOWN", "Unconfined", "bogus", "", "unconfined",
          "kernel.*", "net.ipv4.tcp_keepalive_time", "8080", "80*", "Masked", "spc_t", "user*", "role1",
          "localhost/*", "runtime/default"]


def _good_ctr(rng):
    return {"name": rng.choice(NAMES), "image": rng.choice(IMAGES),
            "securityContext": {"allowPrivilegeEscalation": False, "runAsNonRoot": True,
                                "seccompProfile": {"type": "RuntimeDefault"},
                                "capabilities": {"drop": ["ALL"]}}}


def _violate_ctr(rng, c):
    sc = c.setdefault("securityContext", {})
    k = rng.randrange(12)
    if k == 0:
        sc["allowPrivilegeEscalation"] = rng.choice([True, None])
    elif k == 1:
        sc["capabilities"] = {"drop": rng.choice([["ALL"], [], ["NET_RAW"]]),
                              "add": rng.sample(CAPS, rng.randint(1, 2))}
    elif k == 2:
        sc["privileged"] = True
    elif k == 3:
        sc["runAsNonRoot"] = rng.choice([False, None])
    elif k == 4:
        sc["runAsUser"] = 0
    elif k == 5:
        sc["seccompProfile"] = rng.choice([{"type": "Unconfined"}, {"type": "bogus"}, {"type": ""}, None])
    elif k == 6:
        sc["seLinuxOptions"] = rng.choice([{"type": "spc_t"}, {"user": "user1"}, {"role": "role1", "type": "x"}])
    elif k == 7:
        sc["procMount"] = rng.choice(["Unmasked", ""])
    elif k == 8:
        sc["windowsOptions"] = {"hostProcess": True}
    elif k == 9:
        c["ports"] = [{"containerPort": 80, "hostPort": rng.choice([8080, 80, 9090])} for _ in range(rng.randint(1, 2))]
    elif k == 10:
        del c["securityContext"]
    else:
        sc.pop("capabilities", None)
    for f in [f for f, v in sc.items() if v is None]:
        del sc[f]


def random_pod(rng, i):
    """A restricted-compliant pod with a few violations (so exclusions can flip verdicts)."""
    ann = {}
    spec = {}
    ctrs = []
    for ct in CTR_TYPES:
        n = rng.choice([1, 1, 2, 3]) if ct == "containers" else rng.choice([0, 0, 0, 1, 2])
        if n:
            spec[ct] = [_good_ctr(rng) for _ in range(n)]
            ctrs += spec[ct]
    psc = {}
    if rng.random() < 0.3:
        psc["runAsNonRoot"] = rng.choice([True, False])
    if rng.random() < 0.3:
        psc["seccompProfile"] = {"type": rng.choice(SECCOMP)}
    for _ in range(rng.choice([0, 1, 1, 2, 3])):
        r = rng.random()
        if r < 0.6:
            _violate_ctr(rng, rng.choice(ctrs))
        elif r < 0.68:
            spec[rng.choice(["hostNetwork", "hostPID", "hostIPC"])] = True
        elif r < 0.76:
            spec["volumes"] = [dict(name=f"v{j}", **rng.choice(VOLUMES)) for j in range(rng.randint(1, 3))]
        elif r < 0.82:
            psc["sysctls"] = [{"name": rng.choice(SYSCTLS), "value": "1"} for _ in range(rng.randint(1, 3))]
        elif r < 0.86:
            psc["runAsUser"] = 0
        elif r < 0.9:
            psc["seLinuxOptions"] = {"type": "spc_t", "user": "u"}
        elif r < 0.93:
            psc["windowsOptions"] = {"hostProcess": True}
        elif r < 0.97:
            for c in rng.sample(ctrs, min(len(ctrs), 2)):
                ann["container.apparmor.security.beta.kubernetes.io/" + c["name"]] = rng.choice(ANN_VALUES)
        else:
            key = rng.choice(["seccomp.security.alpha.kubernetes.io/pod",
                              "container.seccomp.security.alpha.kubernetes.io/" + rng.choice(NAMES)])
            ann[key] = rng.choice(ANN_VALUES)
    if psc:
        spec["securityContext"] = psc
    if rng.random() < 0.08:
        spec["os"] = {"name": rng.choice(["windows", "linux"])}
    meta = {"name": f"p{i}", "namespace": "default"}
    if ann:
        meta["annotations"] = ann
    return {"apiVersion": "v1", "kind": "Pod", "metadata": meta, "spec": spec}


def random_exclusions(rng):
    out = []
    n = rng.randint(1, 4)
    ctl = rng.choice(CONTROLS)
    for _ in range(n):
        e = {"controlName": ctl if rng.random() < 0.6 else rng.choice(CONTROLS)}
        if rng.random() < 0.5:
            e["images"] = rng.sample(IMAGES + ["nginx*", "app?:v2", "*"], rng.randint(1, 2))
        r = rng.random()
        if r < 0.35:
            pass  # whole control
        elif r < 0.95:
            ct = rng.choice(CTR_TYPES)
            e["restrictedField"] = (f"spec.{ct}[*]." + rng.choice(CTR_FIELDS)) if rng.random() < 0.6 else \
                rng.choice(POD_FIELDS)
            e["values"] = rng.sample(VALUES, rng.randint(1, 3))
        elif rng.random() < 0.5:
            e["restrictedField"] = "spec.hostNetwork"  # invalid: no values
        else:
            e["values"] = ["true"]  # invalid: no restrictedField
        out.append(e)
    return out


def fuzz_case(seed, npods=600, nrules=24):
    """(policies, ndjson bytes): one single-rule Pod policy per exclusion list."""
    from tests.policies import pss_policy

    rng = random.Random(seed)
    pols = []
    for k in range(nrules):
        level = rng.choice(["baseline", "restricted", "restricted"])
        version = rng.choice(["latest", "latest", "v1.24", "v1.19", "v1.29", "v1.26", "v1.0"])
        pols.append(pss_policy(f"x{k}", level, version, exclude=random_exclusions(rng)))
    pods = [random_pod(rng, i) for i in range(npods)]
    return pols, "\n".join(json.dumps(p) for p in pods).encode()


def strip_exclusions(pols):
    out = json.loads(json.dumps(pols))
    for p in out:
        for r in p["spec"]["rules"]:
            r["validate"]["podSecurity"].pop("exclude", None)
    return out


def _wrap(rng, pod):
    """The pod itself, or as the template of a Deployment or a CronJob (whose converted check
    fields no PolicyException podSecurity entry can match, validate_pss.go:114-135)."""
    r = rng.random()
    if r < 0.65:
        return pod
    meta = {"name": pod["metadata"]["name"], "namespace": "default"}
    tmpl = {"metadata": {k: v for k, v in pod["metadata"].items() if k == "annotations"}, "spec": pod["spec"]}
    if r < 0.85:
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": meta, "spec": {"template": tmpl}}
    return {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": meta,
            "spec": {"schedule": "* * * * *", "jobTemplate": {"spec": {"template": tmpl}}}}


def exception_case(seed, npods=600, nrules=16):
    """(policies, exceptions, ndjson bytes): single-rule Pod policies (and their autogen rules),
    some with their own exclusion lists, each with at most one PolicyException, most of them
    with podSecurity controls (validate_pss.go:88-104), some plain (RuleSkip)."""
    from tests.policies import pss_policy

    rng = random.Random(seed)
    pols, excs = [], []
    for k in range(nrules):
        level = rng.choice(["baseline", "restricted", "restricted"])
        version = rng.choice(["latest", "latest", "v1.24", "v1.19", "v1.29"])
        excl = random_exclusions(rng) if rng.random() < 0.35 else None
        pols.append(pss_policy(f"e{k}", level, version, exclude=excl))
        if rng.random() < 0.1:
            continue
        spec = {"exceptions": [{"policyName": f"pol-e{k}", "ruleNames": [f"e{k}", "autogen-*"]}],
                "match": {"any": [{"resources": {"kinds": ["Pod", "Deployment", "CronJob"],
                                                 "names": rng.sample(["p*", "p1*", "p?", "*3", "*7*"], 2)}}]}}
        if rng.random() < 0.85:
            x = random_exclusions(rng)
            if rng.random() < 0.6:  # whole controls too, so that some failing pods clear entirely
                x += [{"controlName": c} for c in rng.sample(CONTROLS[:-1], rng.randint(4, 12))]
                rng.shuffle(x)
            spec["podSecurity"] = x
        excs.append({"apiVersion": "kyverno.io/v2beta1", "kind": "PolicyException",
                     "metadata": {"name": f"x{k}", "namespace": "kyverno"}, "spec": spec})
    docs = [_wrap(rng, random_pod(rng, i)) for i in range(npods)]
    return pols, excs, "\n".join(json.dumps(d) for d in docs).encode()


def xfail_seed(pols, excs, base, skipped):
    """The scan kernel's verdicts for exception_case: `base` (no exclusions, no exceptions) with
    the cells an exception matched (`skipped`: SKIP under the exceptions stripped of podSecurity)
    set to RuleSkip, or to KPE_XFAIL_ (8) when that exception has podSecurity controls."""
    seed = base.copy()
    pss = {x["spec"]["exceptions"][0]["policyName"] for x in excs if x["spec"].get("podSecurity")}
    col_pss = [pols[j // 3]["metadata"]["name"] in pss for j in range(base.shape[1])]
    for j, p in enumerate(col_pss):
        hit = (skipped[:, j] == 5) & ((base[:, j] == 1) | (base[:, j] == 2))
        seed[hit, j] = 8 if p else 5
    return seed


def strip_pss(excs):
    out = json.loads(json.dumps(excs))
    for x in out:
        x["spec"].pop("podSecurity", None)
    return out
