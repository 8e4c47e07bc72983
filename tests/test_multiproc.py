"""N>1 path on CPU: world_size-2 gloo ranks shard one logical corpus by rows
(kyverno_amd/shard.py), evaluate their shards and all-reduce the per-rule
totals, as bench.py does over RCCL. The shard evaluation here is the oracle
(this is a test of sharding + the exchange, not of the kernels, which
tests/test_gpu_parity.py covers)."""
import json
import os
import sys
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kyverno_amd import shard

TOTAL = 3001  # odd: ranks get unequal shards


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _counts(verdicts):
    names = {0: "na", 1: "pass", 2: "fail", 3: "warn", 4: "error", 5: "skip"}
    out = []
    for r in range(verdicts.shape[1]):
        c = dict.fromkeys(shard.COUNT_FIELDS, 0)
        vals, n = np.unique(verdicts[:, r], return_counts=True)
        for v, k in zip(vals, n):
            c[names[int(v)]] += int(k)
        out.append(c)
    return out


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    import kyverno_amd as K
    from tests.oracle_lib import load as load_oracle
    from tests.policies import parity_policy_set

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard.shard_range(TOTAL, rank, world)
    nd = K.synth_resources(0xC3, n, mix=2, first_index=first)
    v = load_oracle().validate(parity_policy_set(), nd, nthreads=2)
    local = _counts(v)
    total = shard.allreduce_counts(local)
    slowest = shard.max_over_ranks(float(rank + 1))
    if rank == 0:
        np.save(os.path.join(outdir, "counts.npy"), np.array(shard.counts_to_rows(total), dtype=np.int64))
        np.save(os.path.join(outdir, "slowest.npy"), np.array([slowest]))
        # `kyverno apply` summary of the whole job from the all-reduced per-rule counts
        summ = K.cli_summary(K.PolicySet(parity_policy_set()), total)
        with open(os.path.join(outdir, "summary.json"), "w") as f:
            json.dump(summ, f)
    np.save(os.path.join(outdir, f"verdicts{rank}.npy"), v)
    full = shard.gather_rows(v, TOTAL, dst=0)  # grouped point-to-point gather to rank 0
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), full)
    else:
        assert full is None
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_partitions():
    for total in (0, 1, 7, 64, 1000, 3001):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                first, n = shard.shard_range(total, r, world)
                rows.extend(range(first, first + n))
            assert rows == list(range(total))
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_synth_shards_concatenate():
    import kyverno_amd as K

    full = K.synth_resources(0xC3, 300, mix=2)
    a = K.synth_resources(0xC3, 137, mix=2, first_index=0)
    b = K.synth_resources(0xC3, 163, mix=2, first_index=137)
    assert a + b == full


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_counts_and_gather(tmp_path, world):
    from tests.oracle_lib import load as load_oracle
    from tests.policies import parity_policy_set

    import kyverno_amd as K

    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(tmp_path / "counts.npy")
    full = K.synth_resources(0xC3, TOTAL, mix=2)
    ref_v = load_oracle().validate(parity_policy_set(), full, nthreads=4)
    want = np.array(shard.counts_to_rows(_counts(ref_v)), dtype=np.int64)
    assert np.array_equal(got, want)
    # verdict rows stay on their rank; stacked in rank order they are the full matrix
    stacked = np.concatenate([np.load(tmp_path / f"verdicts{r}.npy") for r in range(world)])
    assert np.array_equal(stacked, ref_v)
    # ... and the gathered matrix on rank 0 is the oracle's matrix of the whole corpus
    assert np.array_equal(np.load(tmp_path / "gathered.npy"), ref_v)
    assert float(np.load(tmp_path / "slowest.npy")[0]) == float(world)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import report as oracle_report

    pols = parity_policy_set()
    want_summary = oracle_report.cli_summary(pols, load_oracle().rule_names(pols), ref_v)
    assert json.load(open(tmp_path / "summary.json")) == want_summary
