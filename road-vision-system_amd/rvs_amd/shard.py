"""Camera-stream sharding across GPUs: one process per GPU,
stream block [rank*S, (rank+1)*S) on rank `rank`, no data-path collective.

Every stream's frames, detections and SORT state live on the one rank that
owns it (SORT needs a stream's frames in order, sort_tracker.py:212-278), so
ranks never exchange data; the only cross-rank traffic is the bench's
barrier and a max over ranks of the timed region (weak scaling).
"""
from __future__ import annotations

import os
import time
from typing import Callable, List, Optional, Tuple

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


def gather_over_ranks(value: float, device=None) -> List[float]:
    """Every rank's value of a per-rank scalar, in rank order ([value]
    without a process group)."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return [float(value)]
    n = torch.distributed.get_world_size()
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(n)]
    torch.distributed.all_gather(out, t)
    return [float(x.item()) for x in out]


def device_identity(device) -> str:
    """Identity of this rank's device for the bench line: the GPU's PCI bus
    id from hipDeviceGetPCIBusId (libamdhip64), so a multi-GPU line shows
    that every rank ran on its own card; a CPU rank (gloo rehearsal) is
    named host:pid."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return f"cpu:{os.uname().nodename}:{os.getpid()}"
    import ctypes
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    try:
        hip = ctypes.CDLL("libamdhip64.so")
        buf = ctypes.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(buf, 64, int(idx)) == 0:
            return buf.value.decode()
    except OSError:
        pass
    return f"cuda:{idx}"


def gather_strings(value: str) -> List[str]:
    """Every rank's string, in rank order ([value] without a process group)."""
    if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
        return [str(value)]
    out: List[Optional[str]] = [None] * torch.distributed.get_world_size()
    torch.distributed.all_gather_object(out, str(value))
    return [str(x) for x in out]


def job_throughput(frames_per_rank: int, world: int, elapsed_max_s: float) -> float:
    """Whole-job frames/s: every rank's frames over the slowest rank's time."""
    return frames_per_rank * world / elapsed_max_s


def init_from_env(backend: str = "nccl") -> Tuple[int, int, int]:
    """(rank, world, local_rank) from the torchrun environment; joins the
    process group when world > 1 (nccl = RCCL on ROCm, bound to the local
    GPU; gloo for CPU rehearsals).  No group for a single process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not torch.distributed.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            torch.distributed.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    return rank, world, local


def _barrier() -> None:
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.barrier()


def timed_job(run: Callable[[], None], sync: Callable[[], None], units_per_rank: int,
              device=None) -> dict:
    """The timed region every rank runs: barrier + device sync, `run()` (the
    K steps), device sync, barrier; the elapsed time is reduced with a MAX
    over ranks and the whole-job rate is all ranks' units over that time.
    Returns {"local_s", "per_rank_s" (every rank's local_s, rank order),
    "elapsed_s" (max over ranks), "value"}."""
    world = torch.distributed.get_world_size() if (
        torch.distributed.is_available() and torch.distributed.is_initialized()) else 1
    _barrier()
    sync()
    t0 = time.perf_counter()
    run()
    sync()
    local = time.perf_counter() - t0
    _barrier()
    elapsed = max_over_ranks(local, device)
    per_rank = gather_over_ranks(local, device)
    return {"local_s": local, "per_rank_s": per_rank, "elapsed_s": elapsed,
            "value": job_throughput(units_per_rank, world, elapsed)}
