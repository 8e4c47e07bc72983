"""kpe_lean5_kernel (the headline C2 scan) over full matrices at every PSS level and version.

Every kind-only podSecurity policy (baseline / restricted / privileged x latest and each version
a PSA check changes at) is forced through the LEAN5 instantiation, asserted by the kernel stats,
over 20k-row synthetic mixes with Deployments, CronJobs, nulls, type errors and windows pods.
Compared with the oracle: the whole verdict matrix, and with masks the whole versioned-check
matrix (kpe_fetch_cv_masks: a FAIL cell holds the failing versioned checks of its level /
version, evaluate.go:24-70; every other cell 0). That pins the per-pod PSA summary
(tests/test_psum.py) semantically: each versioned check's failure reaches the masks."""
import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import pss_policy

pytestmark = pytest.mark.gpu

LEVELS = ("baseline", "restricted", "privileged")
VERSIONS = ("latest", "v1.0", "v1.8", "v1.19", "v1.22", "v1.23", "v1.24", "v1.25", "v1.27", "v1.29")
LEAN5 = 7  # kpe_kernel_stats.scan_kernel of kpe_lean5_kernel


@pytest.fixture(scope="module")
def engine():
    return K.Engine(ordinal=0)


@pytest.fixture(scope="module", params=[(1, 20000, 0x51), (2, 20000, 0x52), (-1, 400, 0)], ids=["mixed", "edge", "seccomp"])
def corpus(request, engine):
    mix, n, seed = request.param
    if mix < 0:  # container / pod seccomp and AppArmor annotations (the v1.0 checks)
        from tests.golden.make_psum_digests import seccomp_ndjson
        nd = seccomp_ndjson(n)
    else:
        nd = K.synth_resources(seed, n, mix=mix)
    return nd, K.Corpus(nd, docs=False).upload(engine.device)


@pytest.mark.parametrize("level", LEVELS)
def test_lean5_full_matrix_every_version(engine, oracle, corpus, level):
    nd, c = corpus
    for ver in VERSIONS:
        pol = pss_policy(f"{level}-{ver.replace('.', '-')}", level, ver)
        ps = K.PolicySet([pol])
        assert ps.num_rules == 3  # Pod + the autogen controller and CronJob rules
        ref = oracle.validate([pol], nd, nthreads=8)
        # verdicts, no masks: the LEAN5 instantiation must be the one that ran
        engine.device.set_timing(True)
        engine.device.kernel_stats(reset=True)
        engine.evaluate_async(ps, c)
        st = engine.device.kernel_stats(reset=True)
        engine.device.set_timing(False)
        assert st.launches == 1 and st.scan_kernel == LEAN5, (level, ver, st.scan_kernel)
        v, _, _ = engine.evaluate(ps, c)
        bad = np.argwhere(v != ref)
        assert bad.size == 0, (level, ver, len(bad), bad[:5].tolist())
        # with masks: the same verdicts and the whole versioned-check matrix
        vm, _, _ = engine.evaluate(ps, c, check_masks=True)
        assert np.array_equal(vm, ref), (level, ver)
        cv = engine.cv_masks(ps, c)
        want_row = oracle.failing_cv_batch(level, ver, nd)
        assert want_row.shape[0] == c.n
        fail = vm == 2
        want = np.where(fail, np.maximum(want_row, 0)[:, None], 0).astype(np.int64)
        assert (want_row[fail.any(axis=1)] >= 0).all()  # a FAIL row always decodes
        got = cv.astype(np.int64)
        bad = np.argwhere(got != want)
        assert bad.size == 0, (level, ver, len(bad), bad[:5].tolist())
        if level != "privileged":
            assert fail.sum() > 0 and (got[fail] != 0).all()
