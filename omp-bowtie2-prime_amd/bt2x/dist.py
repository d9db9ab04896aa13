"""Read sharding across GPUs: one process per GPU, the index replicated
in every GPU's HBM, reads partitioned, no collective on the data path.

Every read is independent and its RNG stream is derived from its own content
(pat.cpp:45-88), so any read-to-rank assignment gives the same per-read results; the
only cross-rank step is the final sum of the additive counters (ReportingMetrics,
aln_sink.h:148) and, for the benchmark, the max of the ranks' wall times.
"""
from __future__ import annotations

import os


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_bounds(n: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n reads for `rank` (sizes differ by <= 1)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} of {world_size}")
    q, r = divmod(n, world_size)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def rank_seed(base_seed: int, rank: int) -> int:
    """Per-rank seed of the synthetic read batch (weak scaling: every rank its own batch)."""
    return base_seed + 7919 * rank


def sum_counters(counters: dict, dist=None, device=None) -> dict:
    """Sum integer counters over ranks (the one reduction the path needs)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(counters)
    import torch
    keys = sorted(counters)
    t = torch.tensor([int(counters[k]) for k in keys], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return {k: int(v) for k, v in zip(keys, t.tolist())}


def max_over_ranks(x: float, dist=None, device=None) -> float:
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
