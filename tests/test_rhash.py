"""Resource hashes (CalculateResourceHash, pkg/utils/report/metadata.go:137-155) and incremental
background scans keyed by them (kyverno_amd/scan.py, after
pkg/controllers/report/background/controller.go:247-297 needsReconcile).

The reference has no hash vectors, so the C++ hash (kpe_resource_hash) is checked against an
independent Python restatement of the same steps written here from the Go sources: the
unstructured decode (int64 when strconv.ParseInt accepts the literal, else float64), Go 1.21
encoding/json (sorted keys, HTML and U+2028/9 escapes, \\n \\r \\t short escapes, strconv 'f' /
'e' shortest floats) and md5. Parity against the Go runtime itself is unpinned."""
import copy
import decimal
import hashlib
import json

import numpy as np
import pytest

import kyverno_amd as K

INT64 = (-(1 << 63), (1 << 63) - 1)


def _go_float(f):
    a = abs(f)
    sign, digits, exp = decimal.Decimal(repr(f)).as_tuple()
    ds = "".join(map(str, digits)).lstrip("0") or "0"
    # value = 0.ds * 10^(point) with point = len(all digits) + exp, leading zeros removed
    point = len(digits) + exp - (len(digits) - len("".join(map(str, digits)).lstrip("0") or "0"))
    ds = ds.rstrip("0") or "0"
    neg = "-" if sign else ""
    if a != 0 and (a < 1e-6 or a >= 1e21):
        e = point - 1
        m = ds[0] + ("." + ds[1:] if len(ds) > 1 else "")
        es = f"{abs(e):02d}"
        s = f"{neg}{m}e{'-' if e < 0 else '+'}{es}"
        if s[-4] == "e" and s[-3] == "-" and s[-2] == "0":  # Go's e-09 -> e-9 cleanup
            s = s[:-2] + s[-1]
        return s
    if ds == "0":
        return neg + "0"
    if point <= 0:
        return f"{neg}0.{'0' * -point}{ds}"
    if point >= len(ds):
        return neg + ds + "0" * (point - len(ds))
    return f"{neg}{ds[:point]}.{ds[point:]}"


def _go_str(s):
    out = ['"']
    for ch in s:
        c = ord(ch)
        if ch in '"\\':
            out.append("\\" + ch)
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif c < 0x20 or ch in "<>&" or c in (0x2028, 0x2029):
            out.append(f"\\u{c:04x}")
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _go_marshal(v):
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v) if INT64[0] <= v <= INT64[1] else _go_float(float(v))
    if isinstance(v, float):
        return _go_float(v)
    if isinstance(v, str):
        return _go_str(v)
    if isinstance(v, list):
        return "[" + ",".join(_go_marshal(x) for x in v) + "]"
    items = sorted(v.items(), key=lambda kv: kv[0].encode())
    return "{" + ",".join(_go_str(k) + ":" + _go_marshal(x) for k, x in items) + "}"


def ref_hash(obj):
    obj = copy.deepcopy(obj)
    meta = obj.get("metadata") if isinstance(obj.get("metadata"), dict) else None

    def string_map(f):
        m = meta.get(f) if meta else None
        return m if isinstance(m, dict) and all(isinstance(x, str) for x in m.values()) else None

    labels, annotations = string_map("labels"), string_map("annotations")
    for k in ("metadata", "status", "scale"):
        obj.pop(k, None)
    if isinstance(obj.get("spec"), dict):
        obj["spec"].pop("nodeName", None)
    return hashlib.md5(_go_marshal([labels, annotations, obj]).encode()).hexdigest()


EDGE = [
    {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "a", "labels": {"b": "1", "a": "2"}},
     "spec": {"nodeName": "n1", "containers": [{"name": "c", "image": "<x>&y"}]}, "status": {"phase": "Running"}},
    {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "a", "labels": {"a": "2", "b": "1"}},
     "spec": {"nodeName": "n2", "containers": [{"name": "c", "image": "<x>&y"}]}, "status": {"phase": "Pending"}},
    {"kind": "ConfigMap", "metadata": {"name": "x", "labels": {"n": 1}, "annotations": {}},
     "data": {"k": "line\nnext\ttab\r\u0001\u007f   é 日本"}},
    {"kind": "X", "metadata": "not-a-map", "spec": [1, 2.5, -0.0, 1e-7, 1e21, 1e20, 0.000001, 123.456, 5e-324,
                                                     1.7976931348623157e308, 99999999999999999999, -(1 << 63)]},
    {"kind": "Y", "scale": {"replicas": 3}, "spec": {"nodeName": None, "x": {"z": True, "y": False, "a": None}}},
    {"kind": "Z", "metadata": {"annotations": {"a": "b"}}, "spec": "string spec"},
]


def test_hash_edge_documents():
    for d in EDGE:
        assert K.resource_hash(d) == ref_hash(d), d
    # status and spec.nodeName do not count; label order does not either
    assert K.resource_hash(EDGE[0]) == K.resource_hash(EDGE[1])


def test_hash_duplicate_keys_and_text_forms():
    txt = b'{"kind":"A","spec":{"x":1,"x":2.0,"y":1.50,"z":1e2}}'
    assert K.resource_hash(txt) == ref_hash(json.loads(txt))
    with pytest.raises(K.KpeError):
        K.resource_hash(b"[1,2]")


@pytest.mark.parametrize("mix", [0, 2, 4, 5])
def test_hash_synthetic_rows(mix):
    nd = K.synth_resources(0x4A + mix, 400, mix=mix)
    hs = K.resource_hashes(nd)
    rows = [json.loads(x) for x in nd.decode().splitlines() if x.strip()]
    assert len(hs) == len(rows)
    assert hs == [ref_hash(r) for r in rows]


@pytest.mark.gpu
def test_incremental_scan_matches_full(oracle):
    from tests.policies import parity_policy_set
    pols = parity_policy_set()
    ps = K.PolicySet(pols)
    eng = K.Engine(ordinal=0)
    sc = K.BackgroundScanner(eng)
    nd = K.synth_resources(0x1C, 5000, mix=2)
    v0 = sc.scan(ps, nd)
    assert sc.last_stats["rescanned"] == 5000
    rows = [json.loads(x) for x in nd.decode().splitlines()]
    rng = np.random.default_rng(5)
    changed = sorted(rng.choice(len(rows), 300, replace=False).tolist())
    for i in changed:  # spec changes: rescanned
        spec = rows[i].setdefault("spec", {})
        if isinstance(spec, dict):
            spec["hostNetwork"] = True
        else:
            rows[i]["spec"] = {"hostNetwork": True}
    for i in range(0, len(rows), 7):  # status / nodeName only: the hash ignores them
        if i not in changed:
            rows[i]["status"] = {"phase": "Running"}
    nd2 = "\n".join(json.dumps(r) for r in rows).encode()
    moved = sum(a != b for a, b in zip(K.resource_hashes(nd), K.resource_hashes(nd2)))
    assert 0.9 * len(changed) <= moved <= len(changed)  # a spec that already had hostNetwork: true stays
    v1 = sc.scan(ps, nd2)
    assert sc.last_stats["rescanned"] == moved and not sc.last_stats["full"]
    full, _, _ = eng.evaluate(ps, K.Corpus(nd2))
    assert (v1 == full).all()
    assert (v1 != v0).any()
    assert (v1 == oracle.validate(pols, nd2, nthreads=8)).all()
    v2 = sc.scan(ps, nd2, force=True)
    assert sc.last_stats["full"] and (v2 == full).all()


def test_batch_hash_rows_that_are_not_objects():
    """kpe_resource_hashes keeps going past a row that is not a JSON object (the flattener keeps
    such rows with KPE_ROW_DECODE_ERROR): that row has no hash and the others are unchanged."""
    from kyverno_amd.scan import NO_HASH

    good = K.synth_resources(7, 3, mix=0).decode().splitlines()
    nd = "\n".join([good[0], "[1,2]", good[1], "7", good[2]]).encode()
    hs = K.resource_hashes(nd)
    assert hs[1] == NO_HASH and hs[3] == NO_HASH
    assert [hs[0], hs[2], hs[4]] == K.resource_hashes("\n".join(good).encode())
