"""bench.py's algorithmic-byte accounting: the bytes of the timed scan launches
are summed, not taken from the last launch, so one step's bytes are the same at any K even though
kpe_evaluate_batch_async deals the K steps into launches of unequal size (ceil(K / 24) launches)."""
import importlib.util
import math
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


SHARD = 40.75e6  # one C2 shard's algorithmic bytes (record, header, list items, verdicts)


def _launches(K, per=24):
    """The shard counts of the launches the batch path makes for K steps: ceil(K / per) launches
    over near-equal shares (as launch_lean_run deals them)."""
    L = math.ceil(K / per)
    base, extra = divmod(K, L)
    return [base + (1 if i < extra else 0) for i in range(L)]


@pytest.mark.parametrize("K", [1, 20, 23, 24, 25, 200, 1000])
def test_bytes_per_step_is_one_shard_at_any_K(K):
    b = _bench()
    shards = _launches(K)
    assert sum(shards) == K
    bytes_sum = sum(s * SHARD for s in shards)
    kernel_ms_sum = sum(0.0095 * s + 0.002 for s in shards)  # 9.5 us per shard + 2 us fixed
    a = b.scan_accounting(len(shards), kernel_ms_sum, bytes_sum, K, 0.0110, replicas=15)
    assert a["alg_bytes_per_step"] == pytest.approx(SHARD)
    assert a["alg_bytes_per_launch"] == pytest.approx(SHARD * K / len(shards))
    assert a["rotated_scan_bytes"] == pytest.approx(15 * SHARD)
    # achieved = summed bytes over summed kernel time, never the last launch's bytes / mean time
    assert a["achieved_gbs"] == pytest.approx(bytes_sum / (kernel_ms_sum * 1e-3) / 1e9)
    assert a["achieved_per_step_gbs"] == pytest.approx(SHARD / 11e-6 / 1e9)


def test_unequal_launches_not_scaled_from_the_last():
    b = _bench()
    # 200 steps: the round-5 accounting multiplied the last launch's bytes (23 shards) by the
    # launch count, overstating the step by 23 / 22.2
    shards = [23] * 2 + [22] * 7
    assert sum(shards) == 200
    a = b.scan_accounting(len(shards), 2.0, sum(s * SHARD for s in shards), 200, 0.011, replicas=15)
    assert a["alg_bytes_per_step"] == pytest.approx(SHARD)
    assert shards[0] * SHARD * len(shards) / 200 != pytest.approx(SHARD)  # the old formula


def test_zero_launches_do_not_divide_by_zero():
    b = _bench()
    a = b.scan_accounting(0, 0.0, 0.0, 5, 0.0, replicas=1)
    assert a["achieved_gbs"] == 0.0 and a["alg_bytes_per_step"] == 0.0
