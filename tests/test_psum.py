"""The per-pod PSA summary (kyverno_amd/csrc/lean.inl: kpe_psa_codes_kernel's dictionary codes, then
kpe_psum_kernel's per-pod pass, the same OR-reduction kpe_lean6_kernel runs inside every LEAN
evaluation) over each pod's container / volume / sysctl / annotation lists. Every PSA v0.29 check is "some item of the pod is in state s" for
fixed sets s (pss_fixed.hpp), so the summary is the OR of the items' codes.

Pinned two ways: digests of the summary over seeded corpora and the reference's PSS fixtures
(tests/golden/psum_digests.json, from the host restatement scripts/psum_check.cpp, which is the
flattener's round-3 summary moved verbatim), and, semantically, by the LEAN full-matrix tests in
tests/test_gpu_parity.py (every versioned check's failure reaches the check masks)."""
import hashlib
import json
import os

import numpy as np
import pytest

import kyverno_amd as K
from tests.golden.make_psum_digests import corpus_ndjson, host_summary, names

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIGESTS = json.load(open(os.path.join(ROOT, "tests", "golden", "psum_digests.json")))


def _digest(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()[:32]


@pytest.fixture(scope="module")
def psum_tool():
    from tests.conftest import build_host_tool

    return build_host_tool("psum_check")


@pytest.mark.parametrize("name", names())
def test_host_summary_digest(psum_tool, name):
    assert _digest(host_summary(psum_tool, corpus_ndjson(name))) == DIGESTS[name]


@pytest.mark.gpu
@pytest.mark.parametrize("name", names())
def test_device_summary_digest(name):
    dev = K.Device(0)
    c = K.Corpus(corpus_ndjson(name), docs=False).upload(dev)
    ps = c.psa_summary()
    assert ps.shape == (c.n, 2)
    assert _digest(np.ascontiguousarray(ps).tobytes()) == DIGESTS[name]


@pytest.mark.gpu
def test_device_summary_cold_rebuild_is_identical():
    """A cold evaluation rebuilds the summaries (KPE_EVAL_COLD); the result is unchanged."""
    from tests.policies import restricted_latest

    eng = K.Engine(ordinal=0)
    ps = K.PolicySet([restricted_latest()])
    c = K.Corpus(corpus_ndjson("edge"), docs=False).upload(eng.device)
    v0, _, _ = eng.evaluate(ps, c)
    s0 = c.psa_summary().copy()
    eng.evaluate_async(ps, c, cold=True)
    eng.device.sync()
    assert np.array_equal(c.psa_summary(), s0)
    v1, _, _ = eng.evaluate(ps, c)
    assert np.array_equal(v0, v1)
