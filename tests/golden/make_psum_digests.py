#!/usr/bin/env python3
"""Digests of the per-pod PSA summary (kyverno_amd/csrc/lean.inl kpe_psum_kernel) over seeded
synthetic corpora and the reference's PSS fixtures, from the host restatement
scripts/psum_check.cpp (the summary the flattener built until round 3, moved, plus the container
seccomp-annotation bit the v1.0 seccomp check reads, so that every level / version is LEAN). The
GPU test (tests/test_psum.py) holds the device summary to these digests; the CPU test holds
the host restatement to them."""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import kyverno_amd as K  # noqa: E402

CORPORA = [  # (name, mix, seed, rows)
    ("pods", K.SYNTH_PODS, 0xC2, 20000),
    ("mixed", K.SYNTH_MIXED, 0x71, 20000),
    ("edge", K.SYNTH_EDGE, 0xE1, 20000),
    ("fanout", K.SYNTH_FANOUT, 0xC5, 4000),
]


def seccomp_ndjson(n=400):
    """Pods with container / pod seccomp annotations (check_seccompProfile v1.0 reads them) and
    AppArmor annotations, allowed and forbidden values, deterministic."""
    vals = ["runtime/default", "docker/default", "localhost/prof", "unconfined", "", "runtime/x"]
    aa = ["runtime/default", "localhost/a", "unconfined", "x"]
    out = []
    for i in range(n):
        ctrs = [{"name": f"c-{k}", "image": "nginx:1.0"} for k in range(1 + i % 3)]
        ann = {}
        for k, c in enumerate(ctrs):
            if (i >> k) % 3:
                ann[f"container.seccomp.security.alpha.kubernetes.io/{c['name']}"] = vals[(i + k) % len(vals)]
            if (i >> (k + 2)) % 4 == 1:
                ann[f"container.apparmor.security.beta.kubernetes.io/{c['name']}"] = aa[(i + k) % len(aa)]
        if i % 5 == 0:
            ann["container.seccomp.security.alpha.kubernetes.io/other"] = "unconfined"  # no such container
        if i % 7 == 0:
            ann["seccomp.security.alpha.kubernetes.io/pod"] = vals[i % len(vals)]
        out.append({"apiVersion": "v1", "kind": "Pod",
                    "metadata": {"name": f"sc-{i}", "namespace": "default", "annotations": ann},
                    "spec": {"containers": ctrs}})
    return "\n".join(json.dumps(o, separators=(",", ":")) for o in out).encode()


def fixture_ndjson():
    cases = json.load(open(os.path.join(ROOT, "tests", "golden", "pss_evaluate_cases.json")))
    return "\n".join(json.dumps(c["pod"], separators=(",", ":")) for c in cases).encode()


def corpus_ndjson(name):
    if name == "fixtures":
        return fixture_ndjson()
    if name == "seccomp":
        return seccomp_ndjson()
    mix, seed, n = next((m, s, n) for nm, m, s, n in CORPORA if nm == name)
    return K.synth_resources(seed, n, mix=mix)


def names():
    return [c[0] for c in CORPORA] + ["fixtures", "seccomp"]


def digest(words_bytes: bytes) -> str:
    return hashlib.sha256(words_bytes).hexdigest()[:32]


def host_summary(tool, nd: bytes) -> bytes:
    with tempfile.TemporaryDirectory() as d:
        p, o = os.path.join(d, "r.ndjson"), os.path.join(d, "o.bin")
        open(p, "wb").write(nd)
        subprocess.check_call([tool, p, o])
        return open(o, "rb").read()


def main():
    from tests.conftest import build_host_tool

    tool = build_host_tool("psum_check")
    out = {n: digest(host_summary(tool, corpus_ndjson(n))) for n in names()}
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "psum_digests.json"), "w"), indent=1)
    print(out)


if __name__ == "__main__":
    main()
