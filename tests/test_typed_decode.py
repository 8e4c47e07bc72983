"""Typed decode of getSpec (validate_pss.go:137-188): encoding/json into corev1.Pod /
appsv1.Deployment / batchv1.CronJob fails on a type mismatch at ANY depth, and the PSS rule is a
RuleError. The product flattener (kpe_corpus_row_flags) and the oracle (verdict KPE_ERROR) must
agree with each other AND with the expectation this file states per injection: the injection
table below is hand-written from the k8s.io/api v0.29.1 field types, independent of the schema
tables both sides use (kyverno_amd/csrc/k8s_schema.hpp, oracle/k8s_schema.hpp).

No reference test holds these cases; the expected answers follow from the Go types (parity
pinned by the Go type declarations, not by a reference vector)."""
import copy
import json
import random

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import restricted_latest

# (path inside a PodSpec, value, decode fails?)
SPEC_INJECTIONS = [
    ("containers.0.readinessProbe.periodSeconds", "3", True),
    ("containers.0.readinessProbe.periodSeconds", 3, False),
    ("containers.0.readinessProbe.periodSeconds", 3.5, True),
    ("containers.0.readinessProbe.periodSeconds", 2 ** 31, True),
    ("containers.0.livenessProbe.httpGet.port", True, True),
    ("containers.0.livenessProbe.httpGet.port", "http", False),
    ("containers.0.livenessProbe.httpGet.port", 8080, False),
    ("containers.0.livenessProbe.httpGet.port", 1.5, True),
    ("containers.0.livenessProbe.grpc.port", "9090", True),
    ("containers.0.startupProbe.exec.command", "ls", True),
    ("containers.0.startupProbe.exec.command", ["ls", "-l"], False),
    ("containers.0.resources.limits.cpu", True, True),
    ("containers.0.resources.limits.cpu", "500m", False),
    ("containers.0.resources.limits.cpu", "5xx", True),
    ("containers.0.resources.limits.cpu", 2, False),
    ("containers.0.resources.requests.memory", " 64Mi ", False),
    ("containers.0.resources.requests", [], True),
    ("containers.0.resources.claims.0.name", 1, True),
    ("containers.0.env", {}, True),
    ("containers.0.env", [], False),
    ("containers.0.env.0.valueFrom.fieldRef.fieldPath", 3, True),
    ("containers.0.env.0.valueFrom.resourceFieldRef.divisor", "1m", False),
    ("containers.0.env.0.valueFrom.resourceFieldRef.divisor", "1q", True),
    ("containers.0.envFrom.0.configMapRef.optional", "yes", True),
    ("containers.0.volumeMounts.0.readOnly", "true", True),
    ("containers.0.volumeMounts.0.mountPath", "/data", False),
    ("containers.0.lifecycle.preStop.sleep.seconds", "x", True),
    ("containers.0.lifecycle.postStart.httpGet.httpHeaders.0.value", 5, True),
    ("containers.0.resizePolicy.0.resourceName", ["cpu"], True),
    ("containers.0.securityContext.appArmorProfile", 3, False),  # not a member in v0.29.1
    ("containers.0.unknownMember", {"x": [1, "y"]}, False),
    ("containers.0.ReadinessProbe", {"periodSeconds": "x"}, True),  # case-insensitive member
    ("containers.0.tty", "true", True),
    ("initContainers.0.restartPolicy", 1, True),
    ("ephemeralContainers.0.targetContainerName", 2, True),
    ("ephemeralContainers.0.targetContainerName", "c", False),
    ("terminationGracePeriodSeconds", "30", True),
    ("terminationGracePeriodSeconds", 30, False),
    ("terminationGracePeriodSeconds", 30.5, True),
    ("affinity.nodeAffinity.requiredDuringSchedulingIgnoredDuringExecution.nodeSelectorTerms", {}, True),
    ("affinity.podAntiAffinity.preferredDuringSchedulingIgnoredDuringExecution.0.weight", "1", True),
    ("affinity.podAffinity.requiredDuringSchedulingIgnoredDuringExecution.0.matchLabelKeys", ["a"], False),
    ("tolerations.0.tolerationSeconds", "x", True),
    ("tolerations.0.tolerationSeconds", 300, False),
    ("volumes.0.projected.sources.0.serviceAccountToken.expirationSeconds", "3600", True),
    ("volumes.0.emptyDir.sizeLimit", "1Gi", False),
    ("volumes.0.emptyDir.sizeLimit", "1Gx", True),
    ("volumes.0.configMap.items.0.mode", "0644", True),
    ("volumes.0.ephemeral.volumeClaimTemplate.spec.resources.requests.storage", "1Gi", False),
    ("volumes.0.ephemeral.volumeClaimTemplate.spec.resources.requests.storage", {}, True),
    ("volumes.0.csi.volumeAttributes.a", 1, True),
    ("dnsConfig.options.0.value", 1, True),
    ("topologySpreadConstraints.0.maxSkew", "1", True),
    ("topologySpreadConstraints.0.labelSelector.matchExpressions.0.values", "a", True),
    ("overhead.cpu", [], True),
    ("readinessGates", "x", True),
    ("hostAliases.0.hostnames", ["a", 1], True),
    ("nodeSelector.zone", "a", False),
    ("nodeSelector.zone", 1, True),
    ("securityContext.supplementalGroups", ["1"], True),
    ("securityContext.fsGroupChangePolicy", "Always", False),
    ("schedulingGates.0.name", False, True),
    ("resourceClaims.0.source.resourceClaimName", "x", False),
    ("priority", 1e3, False),
    ("fooBar", {"anything": True}, False),
]
META_INJECTIONS = [
    ("ownerReferences.0.controller", "true", True),
    ("ownerReferences.0.controller", True, False),
    ("managedFields.0.fieldsV1", {"f:x": {}}, False),
    ("managedFields.0.fieldsV1", 3, False),
    ("managedFields.0.time", "2024-01-01", True),
    ("creationTimestamp", "2024-01-01", True),
    ("creationTimestamp", "2024-01-01T00:00:00Z", False),
    ("deletionGracePeriodSeconds", "30", True),
    ("finalizers", [1], True),
]
POD_STATUS_INJECTIONS = [
    ("containerStatuses.0.restartCount", "1", True),
    ("containerStatuses.0.state.terminated.exitCode", 1, False),
    ("containerStatuses.0.allocatedResources.cpu", "x1", True),
    ("startTime", 5, True),
    ("phase", "Running", False),
    ("podIPs.0.ip", 1, True),
]
DEPLOY_INJECTIONS = [
    ("strategy.rollingUpdate.maxSurge", True, True),
    ("strategy.rollingUpdate.maxSurge", "25%", False),
    ("replicas", "3", True),
    ("paused", "no", True),
]
DEPLOY_STATUS_INJECTIONS = [
    ("conditions.0.lastUpdateTime", "yesterday", True),
    ("readyReplicas", "1", True),
    ("currentNumberScheduled", "x", False),  # DaemonSet status member, unknown to DeploymentStatus
]
CRON_INJECTIONS = [
    ("jobTemplate.spec.podFailurePolicy.rules.0.onExitCodes.values", ["1"], True),
    ("jobTemplate.spec.podFailurePolicy.rules.0.onExitCodes.values", [1, 2], False),
    ("jobTemplate.spec.backoffLimitPerIndex", "2", True),
    ("jobTemplate.metadata.labels.a", 1, True),
    ("startingDeadlineSeconds", "10", True),
]
CRON_STATUS_INJECTIONS = [("active.0.name", 1, True), ("lastScheduleTime", "now", True)]


last_path = [None]


def _set(root, path, value):
    last_path[0] = path
    keys = path.split(".")
    cur = root
    for i, k in enumerate(keys):
        last = i == len(keys) - 1
        nxt = None if last else keys[i + 1]
        if isinstance(cur, list):
            k = int(k)
            while len(cur) <= k:
                cur.append([] if (nxt is not None and nxt.isdigit()) else {})
            if last:
                cur[k] = value
            else:
                if not isinstance(cur[k], (dict, list)):
                    cur[k] = [] if nxt.isdigit() else {}
                cur = cur[k]
        else:
            if last:
                cur[k] = value
            else:
                if not isinstance(cur.get(k), (dict, list)):
                    cur[k] = [] if nxt.isdigit() else {}
                cur = cur[k]


def _pod_spec():
    return {"containers": [{"name": "c", "image": "nginx:1.25"}]}


def _base(kind, name):
    meta = {"name": name, "namespace": "default"}
    if kind == "Pod":
        return {"apiVersion": "v1", "kind": "Pod", "metadata": meta, "spec": _pod_spec()}
    if kind == "Deployment":
        return {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": meta,
                "spec": {"selector": {"matchLabels": {"a": "b"}},
                         "template": {"metadata": {"labels": {"a": "b"}}, "spec": _pod_spec()}}}
    return {"apiVersion": "batch/v1", "kind": "CronJob", "metadata": meta,
            "spec": {"schedule": "* * * * *",
                     "jobTemplate": {"spec": {"template": {"spec": _pod_spec()}}}}}


def _spec_root(kind):
    return {"Pod": "spec", "Deployment": "spec.template.spec",
            "CronJob": "spec.jobTemplate.spec.template.spec"}[kind]


def cases(seed=11, n=900):
    """(resource, expected decode failure); one or two injections per resource."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        kind = ("Pod", "Deployment", "CronJob")[i % 3]
        r = _base(kind, f"r{i}")
        exp = {}  # full path -> fails (a later injection at the same path replaces the value)
        for _ in range(rnd.choice((1, 1, 2))):
            where = rnd.random()
            if where < 0.6:
                p, v, bad = rnd.choice(SPEC_INJECTIONS)
                _set(r, _spec_root(kind) + "." + p, copy.deepcopy(v))
            elif where < 0.72:
                p, v, bad = rnd.choice(META_INJECTIONS)
                _set(r, "metadata." + p, copy.deepcopy(v))
            elif where < 0.82:
                tbl = {"Pod": POD_STATUS_INJECTIONS, "Deployment": DEPLOY_STATUS_INJECTIONS,
                       "CronJob": CRON_STATUS_INJECTIONS}[kind]
                p, v, bad = rnd.choice(tbl)
                _set(r, "status." + p, copy.deepcopy(v))
            elif kind == "Deployment":
                p, v, bad = rnd.choice(DEPLOY_INJECTIONS)
                _set(r, "spec." + p, copy.deepcopy(v))
            elif kind == "CronJob":
                p, v, bad = rnd.choice(CRON_INJECTIONS)
                _set(r, "spec." + p, copy.deepcopy(v))
            else:
                p, v, bad = rnd.choice(SPEC_INJECTIONS)
                _set(r, "spec." + p, copy.deepcopy(v))
            exp[last_path[0]] = bad
        out.append((r, any(exp.values())))
    return out


def _expect():
    cs = cases()
    rows = [r for r, _ in cs]
    exp = np.array([e for _, e in cs])
    nd = "\n".join(json.dumps(r) for r in rows).encode()
    return rows, exp, nd


def _context_error(r):
    """NewPolicyContext fails before any rule runs (policy_context.go:230 AddImageInfos): the
    standard image extractors (pkg/utils/api/image.go:54-180) need every non-null entry of
    initContainers / containers / ephemeralContainers to be a map with a string `name`."""
    spec = r
    for k in _spec_root(r["kind"]).split("."):
        spec = spec.get(k) if isinstance(spec, dict) else None
    if not isinstance(spec, dict):
        return False
    for tag in ("initContainers", "containers", "ephemeralContainers"):
        lst = spec.get(tag)
        for c in (lst if isinstance(lst, list) else []):
            if c is not None and (not isinstance(c, dict) or not isinstance(c.get("name"), str)):
                return True
    return False


def test_injection_table_has_both_outcomes():
    _, exp, _ = _expect()
    assert 0.3 < exp.mean() < 0.8


def test_flattener_decode_flag_matches_go_types():
    rows, exp, nd = _expect()
    flags = K.Corpus(nd).row_flags()
    got = (flags & 1).astype(bool)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, [(int(i), json.dumps(rows[i])[:300], bool(exp[i])) for i in bad[:5]]


def test_oracle_decode_error_matches_go_types(oracle):
    rows, exp, nd = _expect()
    ctx = np.array([_context_error(r) for r in rows])
    assert 0 < ctx.sum() < len(rows) // 4
    v = oracle.validate([restricted_latest()], nd, nthreads=4)
    assert (v[ctx] == 7).all()  # no response at all
    got = (v == 4).any(axis=1)
    bad = np.nonzero(got != (exp & ~ctx))[0]
    assert bad.size == 0, [(int(i), json.dumps(rows[i])[:300], bool(exp[i])) for i in bad[:5]]


def test_flattener_context_error_flag(oracle):
    rows, exp, nd = _expect()
    ctx = np.array([_context_error(r) for r in rows])
    flags = K.Corpus(nd).row_flags()
    assert np.array_equal((flags & 8).astype(bool), ctx)


@pytest.mark.gpu
def test_gpu_typed_decode_parity(oracle):
    rows, exp, nd = _expect()
    pols = [restricted_latest()]
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert np.array_equal(v, ref)
    ctx = np.array([_context_error(r) for r in rows])
    assert (v[ctx] == 7).all()
    assert np.array_equal((v == 4).any(axis=1), exp & ~ctx)
