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


def test_lean6_column_guard():
    """kpe_lean6_kernel addresses every column it reads with 32-bit byte offsets: a corpus whose
    pod annotation pairs (or volume / sysctl / container annotation items) pass the limit must take
    the 64-bit template scan, not only one whose pod or container records do."""
    L = K._lib.load()
    many_ann = [{"apiVersion": "v1", "kind": "Pod",
                 "metadata": {"name": f"p{i}", "namespace": "default",
                              "annotations": {f"a{j}": "v" for j in range(20)}},
                 "spec": {"containers": [{"name": "c", "image": "nginx"}]}} for i in range(64)]
    c = K.Corpus(many_ann, docs=False)
    assert L.kpe_debug_lean_kind(c.h, 0) == 7  # far below 4 GiB
    # pods: 64 x 16 B; containers 64 x 8 B; annotation pairs 64 x 20 x 8 B = 10240 B
    assert L.kpe_debug_lean_kind(c.h, 4096 + 64 * 20 * 8 - 1) == 2
    assert L.kpe_debug_lean_kind(c.h, 4096 + 64 * 20 * 8 + 1) == 7
    vols = [{"apiVersion": "v1", "kind": "Pod", "metadata": {"name": f"v{i}", "namespace": "default"},
             "spec": {"containers": [{"name": "c", "image": "nginx"}],
                      "volumes": [{"name": f"x{j}", "emptyDir": {}} for j in range(100)]}} for i in range(8)]
    c2 = K.Corpus(vols, docs=False)
    assert L.kpe_debug_lean_kind(c2.h, 4096 + 8 * 100 * 4 - 1) == 2
    assert L.kpe_debug_lean_kind(c2.h, 4096 + 8 * 100 * 4 + 1) == 7
