"""Incremental background scans keyed by the resource hash.

The background controller (pkg/controllers/report/background/controller.go:247-297,
needsReconcile) rescans a resource when its CalculateResourceHash
(pkg/utils/report/metadata.go:137-155) differs from the hash recorded on its report, when a
policy or exception resourceVersion changed, or when the last scan is older than the forced
rescan interval. BackgroundScanner keeps the last verdict row of every resource: a scan
re-flattens and re-evaluates only the rows that are new or whose hash changed, and every row
when the policy set, the namespace labels or `force` say so. The hash is computed by
kpe_resource_hashes (C++, 16 threads); the evaluation is the device path (kpe_evaluate).
"""
import ctypes
import json

import numpy as np

from ._lib import KpeError, load
from .engine import Corpus


def resource_hash(resource) -> str:
    """CalculateResourceHash of one resource (a dict or its JSON text)."""
    raw = resource if isinstance(resource, bytes) else (
        resource.encode() if isinstance(resource, str) else json.dumps(resource).encode())
    out = ctypes.create_string_buffer(33)
    st = load().kpe_resource_hash(raw, len(raw), out)
    if st != 0:
        raise KpeError(st, "resource is not a JSON object")
    return out.value.decode()


NO_HASH = "-" * 32  # kpe_resource_hashes' mark of a row that is not a JSON object


def resource_hashes(ndjson: bytes):
    """CalculateResourceHash of every NDJSON row (the rows kpe_corpus_flatten makes); NO_HASH
    for a row that is not a JSON object."""
    L = load()
    n = L.kpe_resource_hashes(ndjson, len(ndjson), None, 0)
    buf = ctypes.create_string_buffer(max(n, 1) * 32)
    m = L.kpe_resource_hashes(ndjson, len(ndjson), buf, n)
    if m < 0:
        raise KpeError(-m, "resource hash buffer")
    raw = buf.raw
    return [raw[32 * i:32 * i + 32].decode() for i in range(m)]


def ndjson_rows(ndjson: bytes):
    """The non-blank NDJSON lines, trimmed as the flattener trims them (flatten.cpp flatten_range)."""
    rows = []
    for line in ndjson.split(b"\n"):
        t = line.strip(b" \t\r")
        if t:
            rows.append(t)
    return rows


def _key(row: bytes, i: int):
    """Report identity of a resource: its UID when set, else (apiVersion, kind, namespace, name);
    a row that is not a JSON object is keyed by its position (it is re-evaluated every scan)."""
    try:
        d = json.loads(row)
    except ValueError:
        d = None
    if not isinstance(d, dict):
        return ("row", i)
    meta = d.get("metadata") if isinstance(d.get("metadata"), dict) else {}
    uid = meta.get("uid")
    if isinstance(uid, str) and uid:
        return ("uid", uid)
    return (d.get("apiVersion"), d.get("kind"), meta.get("namespace"), meta.get("name"))


class BackgroundScanner:
    """Verdict rows of the last scan per resource; `scan` evaluates what changed."""

    def __init__(self, engine):
        self.engine = engine
        self._rows = {}  # key -> (hash, verdict row)
        self._policy_token = None
        self._policies = None  # the PolicySet of the last scan (held: identity is the default token)
        self._nrules = None
        self._ns_labels = None
        self.last_stats = {}

    def scan(self, policies, ndjson: bytes, ns_labels=None, policy_version=None, force=False):
        """Verdict matrix (N x R) of the corpus in row order. `policy_version` stands for the
        policies' and exceptions' resourceVersions (any change rescans every row); by default
        the PolicySet object itself."""
        rows = ndjson_rows(ndjson)
        hashes = resource_hashes(b"\n".join(rows))
        keys = [_key(r, i) for i, r in enumerate(rows)]
        R = policies.num_rules
        if policy_version is not None:
            same_policies = policy_version == self._policy_token
        else:  # the PolicySet itself: compared by identity while this scanner holds it
            same_policies = self._policy_token is None and policies is self._policies
        full = force or not same_policies or R != self._nrules or ns_labels != self._ns_labels
        dirty = [i for i, (k, h) in enumerate(zip(keys, hashes))
                 if full or h == NO_HASH or k not in self._rows or self._rows[k][0] != h]
        out = np.zeros((len(rows), R), dtype=np.uint8)
        if dirty:
            delta = b"\n".join(rows[i] for i in dirty)
            nsl = json.dumps(ns_labels).encode() if isinstance(ns_labels, dict) else ns_labels
            v, _, _ = self.engine.evaluate(policies, Corpus(delta, nsl))
            out[dirty] = v
        fresh = set(dirty)
        rows_next = {}
        for i, (k, h) in enumerate(zip(keys, hashes)):
            if i not in fresh:
                out[i] = self._rows[k][1]
            rows_next[k] = (h, out[i].copy())
        self._rows = rows_next  # resources absent from this scan are forgotten (deleted)
        self._policy_token, self._ns_labels = policy_version, ns_labels
        self._policies, self._nrules = policies, R
        self.last_stats = {"rows": len(rows), "rescanned": len(dirty), "full": bool(full)}
        return out
