"""The `images` JSON context: NewPolicyContext's AddImageInfos
(pkg/engine/context/context.go:293-348, pkg/utils/api/image.go:17-229,
pkg/utils/image/infos.go:48-100, distribution/reference v0.5.0 Parse).

The flattener builds each Pod-like resource's images map as a subtree of its document tape
(rows whose images fail to extract get KPE_ROW_CONTEXT_ERROR: the reference gives no response);
the condition program's QO_IMG root reads it.

CPU: the oracle and the product flattener against the reference's image tests
(tests/golden/image_cases.json: infos_test.go, image_test.go); the condition VM on the host.
GPU: the CLI `restrict-something` scenario and bit-exact matrices with images queries and
invalid images over synthetic mixes."""
import json
import os
import subprocess

import numpy as np
import pytest

import kyverno_amd as K

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "image_cases.json")))
FIELDS = {"Registry": "registry", "Name": "name", "Path": "path", "Tag": "tag", "Digest": "digest",
          "Reference": "reference", "ReferenceWithTag": "referenceWithTag", "Pointer": "jsonPointer"}
PASS, FAIL, UNDECIDED = 1, 2, 7


def test_oracle_image_info_golden(oracle):
    for c in GOLD["infos"]:
        got = oracle.image_info(c["image"])
        for k in ("name", "path", "registry", "tag", "digest"):
            assert got[k] == c[k], (c, got)
        assert got["reference"] == c["string"]
    for c in GOLD["references"]:
        got = oracle.image_info(c["image"])
        assert (got["reference"], got["referenceWithTag"]) == (c["reference"], c["referenceWithTag"])
    for e in GOLD["errors"]:
        assert oracle.image_info(e) is None


def _expected_map(images):
    return {t: {n: {FIELDS[k]: v for k, v in info.items() if v != "" or k in ("Name", "Path", "Pointer")}
                for n, info in per.items()} for t, per in images.items()}


def test_oracle_extract_golden(oracle):
    assert len(GOLD["extract"]) >= 3
    for c in GOLD["extract"]:
        assert oracle.images_context(c["raw"]) == _expected_map(c["images"])


# image references beyond the reference's tests (grammar edges; parity unpinned beyond the
# restated grammar): valid and invalid
EDGE = ["nginx", "Nginx", "nginx:1.25", "nginx:", "nginx@sha256:" + "a" * 64, "nginx@sha256:" + "A" * 64,
        "nginx@sha512:" + "0" * 128, "nginx@md5:" + "0" * 32, "ghcr.io/org/app:v1@sha256:" + "b" * 64,
        "localhost:5000/a/b", "[::1]:5000/x", "a_b/c", "a__b/c", "a___b/c", "a-b--c/d", "a./b", "UP/x", "x/UP",
        "registry.example.com:443/team/app:1.2-rc.1", "r/a:" + "t" * 128, "r/a:" + "t" * 129, "a:b:c", "a@b",
        "docker.io/library/busybox:latest", "my.registry/ns/img:tag_with.dots-1", "q/" + "a" * 300, " nginx"]


def test_flattener_context_error_rows(oracle):
    """A Pod per edge image: KPE_ROW_CONTEXT_ERROR exactly where GetImageInfo fails (both with and
    without document tapes), plus the structural errors of extract()."""
    pods = [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"p{i}", "namespace": "d"},
             "spec": {"containers": [{"name": "c", "image": im}]}} for i, im in enumerate(EDGE)]
    pods += [
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "noname"}, "spec": {"containers": [{"image": "x"}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "numname"}, "spec": {"containers": [{"name": 1}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "strctr"}, "spec": {"containers": ["x"]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "scalarlist"}, "spec": {"containers": 3}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "specstr"}, "spec": "x"},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "noimage"}, "spec": {"containers": [{"name": "c"}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "blank"}, "spec": {"containers": [{"name": "c", "image": "  "}]}},
        {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm"}, "spec": {"containers": [{"image": "BAD"}]}},
    ]
    nd = "\n".join(json.dumps(p) for p in pods).encode()
    want = np.array([oracle.images_context(p) == "error" for p in pods])
    assert want[:len(EDGE)].any() and not want[:len(EDGE)].all()
    flags = K.Corpus(nd).row_flags()
    assert np.array_equal((flags & 8).astype(bool), want), [p["metadata"]["name"] for p, w, f in
                                                            zip(pods, want, flags) if bool(f & 8) != w]
    # without tapes only the typed container images are checked (structural errors are not)
    flags = K.Corpus(nd, docs=False).row_flags()
    assert np.array_equal((flags[:len(EDGE)] & 8).astype(bool), want[:len(EDGE)])


def field_policy():
    """One deny rule per (extraction case, container type, container, field): fails when the
    device's images context differs from the reference's expectation."""
    rules = []
    for i, c in enumerate(GOLD["extract"]):
        for t, per in c["images"].items():
            for n, info in per.items():
                for k, v in info.items():
                    rules.append({"name": f"c{i}-{t}-{n}-{k}",
                                  "match": {"any": [{"resources": {"kinds": [c["raw"]["kind"]],
                                                                   "names": [c["raw"]["metadata"]["name"]]}}]},
                                  "validate": {"deny": {"conditions": {"any": [{
                                      "key": f"{{{{ images.{t}.{n}.{FIELDS[k]} || '' }}}}", "operator": "NotEquals",
                                      "value": v}]}}}})
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy",
             "metadata": {"name": "img", "annotations": {"pod-policies.kyverno.io/autogen-controllers": "none"}},
             "spec": {"validationFailureAction": "Audit", "background": True, "rules": rules}}]


def _corpus_rows():
    rows = []
    for i, c in enumerate(GOLD["extract"]):
        r = json.loads(json.dumps(c["raw"]))
        r["metadata"]["name"] = r["metadata"]["name"]
        rows.append(r)
    return rows


def test_condvm_host_images_golden(tmp_path):
    from tests.conftest import build_host_tool

    build_host_tool("condvm_check")
    pols = field_policy()
    rows = _corpus_rows()
    ps = K.PolicySet(pols)
    names = [n.split("/", 1)[1] for n in ps.rule_names]
    seedm = np.zeros((len(rows), len(names)), dtype=np.uint8)
    for j, n in enumerate(names):
        seedm[int(n.split("-")[0][1:]), j] = 6
    (tmp_path / "p.json").write_text(json.dumps(pols))
    (tmp_path / "r.ndjson").write_bytes("\n".join(json.dumps(r) for r in rows).encode())
    (tmp_path / "seed.bin").write_bytes(seedm.tobytes())
    subprocess.check_call([os.path.join(ROOT, "scripts", "build", "condvm_check"), str(tmp_path / "p.json"),
                           str(tmp_path / "r.ndjson"), str(tmp_path / "seed.bin"), str(tmp_path / "out.bin")],
                          stdout=subprocess.DEVNULL)
    out = np.frombuffer((tmp_path / "out.bin").read_bytes(), dtype=np.uint8).reshape(seedm.shape)
    bad = [(names[j], int(out[i, j])) for i, j in zip(*np.nonzero(seedm)) if out[i, j] != PASS]
    assert not bad, bad[:10]


def image_policy_set():
    ctr = "request.object.spec.containers"
    return [{"apiVersion": "kyverno.io/v1", "kind": "ClusterPolicy", "metadata": {"name": "imgs"},
             "spec": {"validationFailureAction": "Audit", "background": True, "rules": [
                 {"name": "no-latest", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"deny": {"conditions": {"any": [{"key": "{{ images.containers.*.tag }}",
                                                                 "operator": "AnyIn", "value": ["latest"]}]}}}},
                 {"name": "registries", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"deny": {"conditions": {"all": [{"key": "{{ images.containers.*.registry }}", "operator": "AnyNotIn",
                                                                 "value": ["docker.io", "ghcr.io"]}]}}}},
                 {"name": "strict", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"deny": {"conditions": {"any": [{"key": "{{ images.initContainers.\"init-0\".name }}",
                                                                 "operator": "Equals", "value": "gitlab"}]}}}},
                 {"name": "fe-tag", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"foreach": [{"list": "images.containers.*", "deny": {"conditions": {"any": [
                      {"key": "{{ element.tag || '' }}", "operator": "Equals", "value": "latest"}]}}}]}},
                 {"name": "pat-path", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"pattern": {"spec": {"containers": [{"image": "*{{ images.initContainers.\"init-0\".path || 'x' }}*"}]}}}},
                 {"name": "pss", "match": {"any": [{"resources": {"kinds": ["Pod"]}}]},
                  "validate": {"podSecurity": {"level": "baseline", "version": "latest"}}},
             ]}}]


def _with_bad_images(nd, every=37):
    lines = nd.split(b"\n")
    out = []
    for i, l in enumerate(lines):
        if i % every == 5 and b'"image":"' in l:
            l = l.replace(b'"image":"', b'"image":"x/Bad', 1)
        out.append(l)
    return b"\n".join(out)


def test_image_policy_set_compiles(oracle):
    pols = image_policy_set()
    names = oracle.rule_names(pols)
    assert K.PolicySet(pols[:1]).num_rules >= 1
    assert len(names) >= 6


@pytest.mark.gpu
def test_gpu_images_golden():
    pols = field_policy()
    rows = _corpus_rows()
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    v, _, _ = eng.evaluate(ps, K.Corpus("\n".join(json.dumps(r) for r in rows).encode()))
    names = [n.split("/", 1)[1] for n in ps.rule_names]
    bad = [names[j] for j, n in enumerate(names) if v[int(n.split("-")[0][1:]), j] != PASS]
    assert not bad, bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("mix,seed", [(0, 0x1A), (2, 0x1B)])
def test_gpu_images_bit_exact(oracle, mix, seed):
    pols = image_policy_set()
    nd = _with_bad_images(K.synth_resources(seed, 12000, mix=mix))
    eng = K.Engine(ordinal=0)
    v, _, _ = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=16)
    bad = np.argwhere(v != ref)
    assert bad.size == 0, [(int(i), int(j), int(v[i, j]), int(ref[i, j])) for i, j in bad[:8]]
    assert (v == UNDECIDED).all(axis=1).any()  # context-error rows
    assert {1, 2} <= set(np.unique(v).tolist())
