"""Per-resource encoding limits (> 255 containers / volumes / sysctls / annotations, a 65th
capability name, a 2049th capability set, a 4097th kind, documents nested deeper than 256):
the row is kept with every cell KPE_UNDECIDED (the caller evaluates it on the Go engine), the
rest of the batch is evaluated as usual."""
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import parity_policy_set


def _pod(name, **spec):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
            "spec": {"containers": [{"name": "c", "image": "nginx"}], **spec}}


def _deep(d):
    x = {"leaf": 1}
    for _ in range(d):
        x = {"n": x}
    return x


def limited_batch():
    rows = []
    limited = []
    for i in range(40):
        rows.append(_pod(f"ok{i}"))
        if i % 10 == 3:
            limited.append(len(rows))
            rows.append(_pod(f"many{i}", containers=[{"name": f"c{j}", "image": "x"} for j in range(300)]))
        if i % 10 == 5:
            limited.append(len(rows))
            rows.append(_pod(f"caps{i}", containers=[{"name": "c", "image": "x", "securityContext": {
                "capabilities": {"add": [f"CAP{i}_{j}" for j in range(70)]}}}]))
        if i % 10 == 7:
            limited.append(len(rows))
            p = _pod(f"deep{i}")
            p["spec"]["extra"] = _deep(300)
            rows.append(p)
    return rows, limited


def test_limited_rows_flatten():
    rows, limited = limited_batch()
    c = K.Corpus(rows)
    assert c.n == len(rows)


def test_limited_rows_parallel_flatten_matches_sequential():
    rows, _ = limited_batch()
    # big enough for several chunks: the 65th capability name is crossed only by the merge
    nd = K.synth_resources(5, 30000, mix=0) + b"\n" + "\n".join(json.dumps(r) for r in rows).encode()
    out = []
    for t in (1, 8):
        os.environ["KPE_FLATTEN_THREADS"] = str(t)
        try:
            c = K.Corpus(nd)
            out.append((c.n, c.digest()))
        finally:
            os.environ.pop("KPE_FLATTEN_THREADS")
    assert out[0] == out[1]


@pytest.mark.gpu
def test_limited_rows_undecided(oracle):
    rows, limited = limited_batch()
    pols = parity_policy_set()
    nd = "\n".join(json.dumps(r) for r in rows).encode()
    eng = K.Engine(ordinal=0)
    v, _, cnt = eng.evaluate(K.PolicySet(pols), K.Corpus(nd))
    assert (v[limited] == 7).all()
    keep = np.setdiff1d(np.arange(len(rows)), limited)
    ref = oracle.validate(pols, nd, nthreads=8)
    assert (v[keep] == ref[keep]).all()
    assert sum(c["undecided"] for c in cnt) == len(limited) * v.shape[1]
