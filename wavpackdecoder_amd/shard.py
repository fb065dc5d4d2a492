"""Multi-GPU decode: files partition across ranks, no data-path collective.

WavPack blocks (and so files) are independent, so N GPUs
decode N disjoint file sets: one process per GPU, each with its own HIP
context, batch and output region.  The only cross-rank traffic is host-side
bookkeeping after the fact (frame/CRC-error totals, the max of the timings)
over a CPU process group (gloo); nothing goes over xGMI.
"""
from __future__ import annotations

import heapq
from typing import Callable, Sequence


def partition(sizes: Sequence[int], world: int) -> list[list[int]]:
    """Greedy longest-processing-time split of file indices by size (bytes or frames)."""
    parts: list[list[int]] = [[] for _ in range(world)]
    heap = [(0, r) for r in range(world)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(sizes[i]), r))
    for p in parts:
        p.sort()
    return parts


def reduce_totals(pg, frames: int, crc_errors: int, seconds: float) -> tuple[int, int, float]:
    """Sum frames / CRC errors and take the max time over ranks (host process group)."""
    if pg is None:
        return frames, crc_errors, seconds
    import torch
    t = torch.tensor([float(frames), float(crc_errors)], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    m = torch.tensor([seconds], dtype=torch.float64)
    pg.all_reduce(m, op=pg.ReduceOp.MAX)
    return int(t[0].item()), int(t[1].item()), float(m.item())


def run_rank(files: Sequence[bytes], rank: int, world: int,
             decode: Callable[[list[bytes]], tuple[int, int, float]], pg=None) -> tuple[int, int, float]:
    """Decode this rank's share of `files`; return the job totals (frames, crc_errors, max seconds).

    `decode(list_of_files) -> (frames, crc_errors, seconds)` runs on this rank's
    device (DecodeBatch in bench.py); the partition is deterministic, so every
    rank computes the same split without communicating.
    """
    mine = partition([len(f) for f in files], world)[rank]
    frames, crc, sec = decode([files[i] for i in mine]) if mine else (0, 0, 0.0)
    if pg is not None:
        pg.barrier()
    return reduce_totals(pg, frames, crc, sec)
