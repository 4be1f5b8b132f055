"""Camera-stream sharding across GPUs: one process per GPU,
stream block [rank*S, (rank+1)*S) on rank `rank`, no data-path collective.

Every stream's frames, detections and SORT state live on the one rank that
owns it (SORT needs a stream's frames in order, sort_tracker.py:212-278), so
ranks never exchange data; the only cross-rank traffic is the bench's
barrier and a max over ranks of the timed region (weak scaling).
"""
from __future__ import annotations

from typing import List

import torch


def rank_streams(streams_per_rank: int, rank: int) -> range:
    """Global stream ids owned by `rank` (contiguous block)."""
    if streams_per_rank < 0 or rank < 0:
        raise ValueError("streams_per_rank and rank must be >= 0")
    return range(rank * streams_per_rank, (rank + 1) * streams_per_rank)


def partition(total_streams: int, world: int) -> List[range]:
    """Config 4 layout: total_streams split evenly over `world` ranks
    (256 streams over 8 GPUs -> 32 per GPU)."""
    if world < 1 or total_streams % world:
        raise ValueError(f"{total_streams} streams do not split evenly over {world} ranks")
    return [rank_streams(total_streams // world, r) for r in range(world)]


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (the timed region) over the process group;
    the identity without one."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def job_throughput(frames_per_rank: int, world: int, elapsed_max_s: float) -> float:
    """Whole-job frames/s: every rank's frames over the slowest rank's time."""
    return frames_per_rank * world / elapsed_max_s
