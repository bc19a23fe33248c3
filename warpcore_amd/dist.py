"""Multi-GPU sharding of a checksum batch: one process per GPU.

The path has no exchange step -- packets are independent -- so a batch is
split into even contiguous packet ranges, one per rank (SURVEY.md 8(e):
rank r gets [r*N/G, (r+1)*N/G)), and every rank checksums its range on its own
GPU with no collective on the data path.  Collectives appear only around the
timed region (barrier, max of the per-rank times) and, when the caller wants
every result in one place, in an all-gather of the 2-byte results after it.
With the "nccl" backend (RCCL on ROCm) those go over xGMI; the same code runs
on "gloo" for the CPU tests.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Even contiguous split: rank r gets packets [r*n//w, (r+1)*n//w)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    return n * rank // world, n * (rank + 1) // world


def shard_ragged(offsets, lengths, rank: int, world: int):
    """Shard a ragged batch by packet count; returns the rank's (offsets,
    lengths, first packet index).  Offsets stay relative to the same base."""
    lo, hi = shard_range(len(offsets), rank, world)
    return offsets[lo:hi], lengths[lo:hi], lo


def _pg_active() -> bool:
    return dist.is_available() and dist.is_initialized()


def world() -> Tuple[int, int]:
    if _pg_active():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def barrier(device: Optional[torch.device] = None) -> None:
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)
    if _pg_active():
        dist.barrier()
    if device is not None and device.type == "cuda":
        torch.cuda.synchronize(device)


def max_over_ranks(x: float, device: Optional[torch.device] = None) -> float:
    if not _pg_active():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: int, device: Optional[torch.device] = None) -> int:
    if not _pg_active():
        return x
    t = torch.tensor([x], dtype=torch.int64, device=device or "cpu")
    dist.all_reduce(t)
    return int(t.item())


def gather_results(local: torch.Tensor, n: int) -> torch.Tensor:
    """All-gather each rank's 2-byte results (shard order) into one length-n
    tensor on every rank.  Shards differ by at most one packet, so they are
    padded to the largest shard for the collective."""
    rank, w = world()
    if w == 1:
        return local
    counts = [shard_range(n, r, w) for r in range(w)]
    width = max(hi - lo for lo, hi in counts)
    # Pairs of 2-byte results travel as int32 words (gloo has no int16).
    words = (width + 1) // 2
    pad = torch.zeros(2 * words, dtype=torch.int16, device=local.device)
    pad[: local.numel()] = local.view(torch.int16)
    parts = [torch.empty(words, dtype=torch.int32, device=local.device) for _ in range(w)]
    dist.all_gather(parts, pad.view(torch.int32))
    out = torch.empty(n, dtype=torch.int16, device=local.device)
    for (lo, hi), part in zip(counts, parts):
        out[lo:hi] = part.view(torch.int16)[: hi - lo]
    return out


def run_sharded(n: int, compute: Callable[[int, int], torch.Tensor],
                gather: bool = True) -> torch.Tensor:
    """Checksum packets [0, n) across the process group: `compute(lo, hi)`
    returns this rank's results for packets [lo, hi) (on its own GPU).  No
    collective runs until every rank is done; with gather=True the results
    are then all-gathered in packet order."""
    rank, w = world()
    lo, hi = shard_range(n, rank, w)
    local = compute(lo, hi)
    if local.numel() != hi - lo:
        raise RuntimeError("compute returned the wrong number of results")
    return gather_results(local, n) if gather else local
