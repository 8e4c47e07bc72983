"""Resource sharding across the GPUs of one node.

Every (resource, rule) cell is independent given the replicated program and
namespace-label table (MatchesResourceDescription reads only the resource, its
namespace labels and the rule: pkg/engine/utils/match.go:168), so ranks take
contiguous row ranges of one logical corpus and evaluate them with no data-path
collective. The only exchange is the per-rule totals (kpe_counts, R x 6 u64)
that `kyverno apply` prints (cmd/cli/kubectl-kyverno/processor/result.go:34-68),
summed with one all-reduce; PolicyReports are per resource, so verdict bytes
stay on the rank that produced them.
"""
from typing import Dict, List, Sequence, Tuple

COUNT_FIELDS = ("na", "pass", "fail", "warn", "error", "skip", "undecided")


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [first, first+n) rows of a `total`-row corpus owned by `rank`.
    The first `total % world` ranks take one extra row."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def counts_to_rows(counts: Sequence[Dict[str, int]]) -> List[List[int]]:
    return [[int(c[f]) for f in COUNT_FIELDS] for c in counts]


def rows_to_counts(rows) -> List[Dict[str, int]]:
    return [dict(zip(COUNT_FIELDS, (int(x) for x in r))) for r in rows]


def allreduce_counts(counts: Sequence[Dict[str, int]], device=None) -> List[Dict[str, int]]:
    """Sum per-rule counters over the default process group (RCCL on GPU ranks,
    gloo on CPU). One R x 6 int64 tensor; identity when not initialised."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [dict(c) for c in counts]
    t = torch.tensor(counts_to_rows(counts), dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return rows_to_counts(t.cpu().tolist())


def max_over_ranks(seconds: float, device=None) -> float:
    """The job's time is the slowest rank's (bench.py contract)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
