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


# Relative device cost per decoded frame of each block kind (one serial chain per block,
# lanes of 64 blocks): the inverse of the kinds' in-flight rates on the lane kernels,
# normalised to 16-bit stereo (C2 56,000 Mframes/s, C3-shaped 16-term
# 24-bit ~37,000 at C5's block sizes, DSD mode 0 212,000, mode 1 7,350, mode 3 9,330;
# mono about half of stereo).  The partition balances the ranks' summed cost; with
# several batches in flight per rank (bench.py --c5-copies) a rank's time is its summed
# cost, not its longest chain, which every rank shares (DSD mode 3's 22,050-frame blocks).
KIND_COST = {"stereo16": 1.0, "mono16": 0.5, "stereo24": 1.5, "mono24": 0.75,
             "dsd0": 0.3, "dsd1": 7.6, "dsd3": 6.0, "dsd0m": 0.15, "dsd1m": 3.8, "dsd3m": 3.0}


def file_kind(data: bytes) -> tuple[str, int]:
    """(kind, frames) of a .wv file from its first block header (WavPackUtils.cs:600-671)
    and, for DSD, the mode byte of its ID_DSD_BLOCK (DsdUtils.cs:17-54)."""
    if len(data) < 32 or data[:4] != b"wvpk":
        return "stereo16", 0
    ck = int.from_bytes(data[4:8], "little")
    total = int.from_bytes(data[12:16], "little") | (data[11] << 32)
    flags = int.from_bytes(data[24:28], "little")
    mono = bool(flags & 4)
    if flags & 0x80000000:
        mode = 0
        p, end = 32, min(len(data), ck + 8)
        while p + 2 <= end:
            mid = data[p]
            if mid & 0x80:
                if p + 4 > end:
                    break
                size, hdr = (data[p + 1] | data[p + 2] << 8 | data[p + 3] << 16) * 2, 4
            else:
                size, hdr = data[p + 1] * 2, 2
            if mid & 0x3F == 0x0E and size >= 2 and p + hdr + 2 <= end:
                mode = data[p + hdr + 1]
                break
            p += hdr + size
        return "dsd%d%s" % (mode if mode in (0, 1, 3) else 1, "m" if mono else ""), total
    bps = (flags & 3) + 1
    return ("mono" if mono else "stereo") + ("16" if bps <= 2 else "24"), total


def file_cost(data: bytes) -> float:
    kind, frames = file_kind(data)
    return KIND_COST[kind] * max(frames, 1)


def partition(sizes: Sequence[float], world: int) -> list[list[int]]:
    """Greedy longest-processing-time split of file indices by cost (file_cost, or bytes)."""
    parts: list[list[int]] = [[] for _ in range(world)]
    heap = [(0, r) for r in range(world)]
    for i in sorted(range(len(sizes)), key=lambda k: (-sizes[k], k)):
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
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
             decode: Callable[[list[bytes]], tuple[int, int, float]], pg=None,
             cost: Callable[[bytes], float] = file_cost) -> tuple[int, int, float]:
    """Decode this rank's share of `files`; return the job totals (frames, crc_errors, max seconds).

    `decode(list_of_files) -> (frames, crc_errors, seconds)` runs on this rank's
    device (DecodeBatch in bench.py); the partition is deterministic, so every
    rank computes the same split without communicating.  `cost` is the same per-file
    device cost bench.py's C5 split uses (file_cost; corpora.c5_cost restates it from
    the corpus' file parameters).
    """
    mine = partition([cost(f) for f in files], world)[rank]
    frames, crc, sec = decode([files[i] for i in mine]) if mine else (0, 0, 0.0)
    if pg is not None:
        pg.barrier()
    return reduce_totals(pg, frames, crc, sec)
