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


def test_unpack_matches_numpy_packing():
    """kpe_unpack_verdicts inverts the 3-bit packing kpe_pack_verdicts writes on the device
    (cell i in bits 3*(i % 10) of word i / 10), restated here in numpy."""
    import kyverno_amd as K

    rng = np.random.default_rng(3)
    for n, r in ((0, 3), (1, 1), (7, 3), (1001, 17)):
        v = rng.integers(0, 8, size=(n, r), dtype=np.uint8)
        flat = v.reshape(-1).astype(np.uint32)
        words = K.packed_words(n * r)
        pad = np.zeros(words * 10, dtype=np.uint32)
        pad[:flat.size] = flat
        packed = (pad.reshape(-1, 10) << (3 * np.arange(10, dtype=np.uint32))).sum(axis=1, dtype=np.uint64).astype(np.uint32)
        assert np.array_equal(K.unpack_verdicts(packed, n, r), v)


def _gpu_worker(rank, world, port, outdir):
    """A rank of the GPU N>1 path on one device: HIP evaluation of its shard, the verdict
    matrix packed on the device (kpe_pack_verdicts) and gathered over gloo (RCCL refuses two
    ranks on one GPU; bench.py runs the same gather over RCCL, one rank per GPU)."""
    import torch.distributed as dist

    import kyverno_amd as K
    from tests.policies import parity_policy_set

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard.shard_range(TOTAL, rank, world)
    nd = K.synth_resources(0xC3, n, mix=2, first_index=first)
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(parity_policy_set())
    c = K.Corpus(nd)
    _, _, cnt = eng.evaluate(ps, c)
    total = shard.allreduce_counts(cnt)
    full = shard.gather_packed(eng, ps, c, TOTAL, dst=0, device="cpu")
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), full)
        np.save(os.path.join(outdir, "counts.npy"), np.array(shard.counts_to_rows(total), dtype=np.int64))
    else:
        assert full is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_gpu_ranks_packed_gather(tmp_path, world):
    from tests.oracle_lib import load as load_oracle
    from tests.policies import parity_policy_set

    import kyverno_amd as K

    mp.start_processes(_gpu_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    full = K.synth_resources(0xC3, TOTAL, mix=2)
    ref_v = load_oracle().validate(parity_policy_set(), full, nthreads=4)
    assert np.array_equal(np.load(tmp_path / "gathered.npy"), ref_v)
    want = _counts(ref_v)
    got = shard.rows_to_counts(np.load(tmp_path / "counts.npy"))
    assert [{k: v for k, v in g.items() if k != "undecided"} for g in got] == \
        [{k: v for k, v in w.items() if k != "undecided"} for w in want]


@pytest.mark.gpu
def test_gpu_sharded_single_process(oracle):
    """kpe_evaluate_sharded over the devices of this process (one here), and the device
    verdict address / packed form against the byte matrix."""
    import torch

    import kyverno_amd as K
    from tests.policies import parity_policy_set

    pols = parity_policy_set()
    nd = K.synth_resources(0xC3, TOTAL, mix=2)
    eng = K.Engine(ordinal=0)
    ps = K.PolicySet(pols)
    c = K.Corpus(nd)
    v, cnt = K.evaluate_sharded([eng], ps, [c])
    assert np.array_equal(v, oracle.validate(pols, nd, nthreads=4))
    v1, _, cnt1 = eng.evaluate(ps, c)
    assert cnt == cnt1
    ptr, nbytes = eng.device_verdicts(ps, c)
    assert ptr and nbytes == v.size
    words = K.packed_words(v.size)
    buf = torch.zeros(words, dtype=torch.int32, device="cuda:0")
    eng.pack_verdicts(ps, c, buf.data_ptr(), words)
    assert np.array_equal(K.unpack_verdicts(buf.cpu().numpy().view(np.uint32), *v.shape), v)
    with pytest.raises(K.KpeError):  # one shard per device
        K.evaluate_sharded([eng, eng], ps, [c, K.Corpus(nd)])


def _small_worker(rank, world, port, outdir, total):
    """total < world: some ranks hold no rows and still join the gather group."""
    import torch.distributed as dist

    import kyverno_amd as K
    from tests.oracle_lib import load as load_oracle
    from tests.policies import parity_policy_set

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard.shard_range(total, rank, world)
    pols = parity_policy_set()
    R = K.PolicySet(pols).num_rules
    v = load_oracle().validate(pols, K.synth_resources(0xC3, n, mix=2, first_index=first)) if n else \
        np.zeros((0, R), dtype=np.uint8)
    full = shard.gather_rows(v, total, dst=0)
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), full)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_gather_with_empty_shards(tmp_path):
    from tests.oracle_lib import load as load_oracle
    from tests.policies import parity_policy_set

    import kyverno_amd as K

    total, world = 2, 3
    mp.start_processes(_small_worker, args=(world, _free_port(), str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    ref = load_oracle().validate(parity_policy_set(), K.synth_resources(0xC3, total, mix=2))
    assert np.array_equal(np.load(tmp_path / "gathered.npy"), ref)
