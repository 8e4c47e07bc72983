"""GPU parity for the C3 and C5 benchmark configurations through the C-ABI.

C3: mixed kinds (kpe_synth KPE_SYNTH_C3) x 200 ClusterPolicies with wildcard kind / name /
    namespace match and exclude blocks (tests/policies.c3_policy_set), resource-sharded
    over 8 GPUs: one GPU holds a 1/8 shard of the 10M-row corpus (1.25M rows).
C5: Pods / Deployments with 1-64 containers (KPE_SYNTH_FANOUT) x require-pod-requests-limits,
    disallow-latest-tag, chart disallow-host-ports and anchor variants (c5_policy_set).

Bit-exact verdict matrices against the oracle at 50k rows; at full size the size-independent
properties (counts == histogram, idempotence, shard-position independence) plus a strided
row sample against the oracle."""
import numpy as np
import pytest

import kyverno_amd as K
from tests.policies import c3_policy_set, c5_policy_set

pytestmark = pytest.mark.gpu

CONFIGS = {"c3": (c3_policy_set, K.SYNTH_C3, 0xC3), "c5": (c5_policy_set, K.SYNTH_FANOUT, 0xC5)}


@pytest.fixture(scope="module")
def engine():
    return K.Engine(ordinal=0)


def _check_counts(v, cnt):
    for r in range(v.shape[1]):
        col = v[:, r]
        for code, key in ((0, "na"), (1, "pass"), (2, "fail"), (4, "error"), (5, "skip")):
            assert cnt[r][key] == int((col == code).sum()), (r, key)


@pytest.mark.parametrize("cfg,n,seed_off", [("c3", 50000, 0), ("c3", 20000, 7), ("c5", 50000, 0), ("c5", 20000, 9)])
def test_config_bit_exact(engine, oracle, cfg, n, seed_off):
    make, mix, seed = CONFIGS[cfg]
    pols = make()
    nd = K.synth_resources(seed + seed_off, n, mix=mix)
    v, _, cnt = engine.evaluate(K.PolicySet(pols), K.Corpus(nd))
    ref = oracle.validate(pols, nd, nthreads=8)
    assert v.shape == ref.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()} " \
                          f"gpu={[int(v[i, j]) for i, j in bad[:5]]} ref={[int(ref[i, j]) for i, j in bad[:5]]}"
    assert (v == 6).sum() == 0
    _check_counts(v, cnt)
    assert {1, 2} <= set(np.unique(v).tolist())


@pytest.mark.parametrize("cfg,n", [("c3", 1_250_000), ("c5", 1_000_000)])
def test_config_full_size_bit_exact(engine, oracle, cfg, n):
    make, mix, seed = CONFIGS[cfg]
    pols = make()
    ps = K.PolicySet(pols)
    nd = K.synth_resources(seed, n, mix=mix)
    c = K.Corpus(nd)
    v, _, cnt = engine.evaluate(ps, c)
    assert v.shape == (n, ps.num_rules)
    _check_counts(v, cnt)
    v2, _, _ = engine.evaluate(ps, c)
    assert np.array_equal(v, v2)  # idempotence
    first = n // 2 + 13
    shard = K.Corpus(K.synth_resources(seed, 2000, mix=mix, first_index=first))
    vs, _, _ = engine.evaluate(ps, shard)
    assert np.array_equal(vs, v[first:first + 2000])  # shard-position independence
    # the whole matrix against the oracle (16 host threads: about a minute for C3's 1.25M x 604)
    ref = oracle.validate(pols, nd, nthreads=16)
    assert ref.shape == v.shape
    bad = np.argwhere(v != ref)
    assert bad.size == 0, f"{len(bad)} mismatching cells, first {bad[:5].tolist()}"
