#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X.

metric : Msamples/sec decoded (node) + HBM GB/s, batched 44.1 kHz/16-bit stereo blocks
step   : one decode of the config-2 batch (1,024 independent WavPack blocks x
         22,050 frames, 16-bit stereo, fast terms {17,17}) already resident in
         HBM -> int32 PCM in HBM (the WavpackUnpackSamples output contract)
N GPUs : one process per GPU (torch.distributed.run); each rank decodes its
         own C2-sized shard of blocks (weak scaling, per-GPU file partition);
         no data-path collective -- only a CPU (gloo) barrier and a max-reduce
         of the timings.
value  : frames decoded by all ranks / max-over-ranks wall time of the K steps.

Also printed in the same JSON line:
  roofline     : algorithmic bytes per launch (compressed bytes in + int32
                 out) / mean device time per launch measured
                 with hipEvents on the decode stream, vs 8 TB/s HBM peak.
  cpu_baseline : the oracle (C restatement of the reference algorithm,
                 kind "port") decoding the same C2 file split across host
                 threads, on rank 0 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=ws)  # CPU barrier + timing reduce only
        pg = dist
    return ws, rank, local, pg


def _barrier(pg):
    if pg is not None:
        pg.barrier()


def _max(pg, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def _sum(pg, v: float) -> float:
    if pg is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def split_blocks(data: bytes, parts: int):
    """Split a multi-block .wv file at block boundaries into `parts` files."""
    offs = []
    i = 0
    n = len(data)
    while i + 32 <= n:
        if data[i:i + 4] != b"wvpk":
            break
        ck = int.from_bytes(data[i + 4:i + 8], "little")
        offs.append(i)
        i += ck + 8
    offs.append(n)
    nb = len(offs) - 1
    per = (nb + parts - 1) // parts
    return [data[offs[k]:offs[min(k + per, nb)]] for k in range(0, nb, per)]


def algorithmic_bytes(data: bytes, nch: int = 2) -> int:
    """sum(ckSize + 8) + sum(block_samples * nch * 4)."""
    i, tot = 0, 0
    while i + 32 <= len(data) and data[i:i + 4] == b"wvpk":
        ck = int.from_bytes(data[i + 4:i + 8], "little")
        bs = int.from_bytes(data[i + 20:i + 24], "little")
        tot += ck + 8 + bs * nch * 4
        i += ck + 8
    return tot


def pmc_traffic(kernel_substr: str = "wv_pcm_2wave<17, 17>"):
    """Per-launch HBM bytes of the bench kernel from the newest profiles/<tag>_pmc.json
    (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, scripts/profile.sh + scripts/pmc_to_profile.py)."""
    import glob
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json"))):
        with open(path) as f:
            d = json.load(f)
        if kernel_substr in d.get("kernel", ""):
            best = (path, d)
    if best is None:
        return None, None
    return float(best[1]["traffic_bytes_per_launch"]), os.path.relpath(best[0], ROOT)


def cpu_baseline(data: bytes, threads: int, reps: int):
    """Oracle (C port of the reference path) on host threads; ctypes drops the GIL."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    parts = split_blocks(data, threads)
    frames = 0
    times = []
    with ThreadPoolExecutor(max_workers=threads) as ex:
        for _ in range(reps):
            t0 = time.perf_counter()
            res = list(ex.map(lambda p: O.decode_file(p, chunk=4096, max_frames=len(p) * 2), parts))
            times.append(time.perf_counter() - t0)
            frames = sum(r.frames for r in res)
            assert all(r.crc_errors == 0 for r in res)
    t = float(np.median(times))
    return frames / t / 1e6, t, frames


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=1024)
    ap.add_argument("--block-frames", type=int, default=22050)
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("WV_CPU_THREADS", "16")))
    ap.add_argument("--cpu-reps", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--check", action="store_true", help="verify the decoded PCM against the generator's")
    args = ap.parse_args()

    ws, rank, local, pg = _dist()

    from synth import corpora
    from wavpackdecoder_amd import _lib
    from wavpackdecoder_amd.api import DecodeBatch

    # each rank: its own C2-sized shard (rank 0 = the canonical C2 batch)
    pcm, data = corpora.c2(nblocks=args.blocks, block=args.block_frames, return_pcm=True) if rank == 0 else (None, None)
    if rank != 0:
        data = corpora.c2_shard(rank, nblocks=args.blocks, block=args.block_frames)

    L = _lib.lib()
    import wavpackdecoder_amd.api as api
    api._ctx = L.wvg_open(local)
    if not api._ctx:
        raise SystemExit("no GPU")

    b = DecodeBatch(4096)
    fi = b.add_file(data)
    assert fi == 0
    b.upload()
    frames_rank = b.frames
    alg_bytes = algorithmic_bytes(data)

    for _ in range(args.warmup):
        b.decode()
    b.sync()
    if args.check:
        out = b.download()
        if pcm is not None:
            assert np.array_equal(out, pcm.reshape(-1)), "decoded PCM differs from the generator's"
        r = b.result(0)
        assert r.crc_errors == 0

    # device time per launch (hipEvents on the decode stream)
    kernel_ms = b.time(max(args.steps, 1))

    _barrier(pg)
    b.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        b.decode()
    b.sync()
    t1 = time.perf_counter()
    _barrier(pg)
    dt = _max(pg, t1 - t0)
    frames_total = _sum(pg, float(frames_rank))
    value = frames_total * args.steps / dt / 1e6

    # PCIe-inclusive rate (host bytes in -> host int32 out), reported beside `value`, never as it
    host_out = np.empty(max(b.out_ints, 1), dtype=np.int32)
    t_e2e = time.perf_counter()
    b.upload()
    b.decode()
    b.sync()
    b._check(b._L.wvg_batch_download(b._b, host_out.ctypes.data, host_out.size))
    t_e2e = time.perf_counter() - t_e2e
    e2e = frames_rank / t_e2e / 1e6

    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    traffic, traffic_src = pmc_traffic()
    line = None
    if rank == 0:
        cpu = None
        if not args.no_cpu:
            v, t, fr = cpu_baseline(data, args.cpu_threads, args.cpu_reps)
            cpu = {"value": round(v, 2), "unit": "Msamples/s", "cores": args.cpu_threads, "kind": "port",
                   "sample": f"oracle (C restatement of the C# path) decoding the full C2 file ({fr} frames) split "
                             f"at block boundaries over {args.cpu_threads} threads, 4096-frame calls, median of "
                             f"{args.cpu_reps} runs"}
        line = {
            "metric": "Msamples/sec decoded (node) + HBM GB/s, batched 44.1kHz/16-bit stereo blocks",
            "value": round(value, 2),
            "unit": "Msamples/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (repo encoder, seeds 0xC2+block)",
            "config": {"workload": "C2: 1024-block batch, 16-bit stereo 'fast' {17,17}, joint stereo, 44.1 kHz",
                       "blocks_per_gpu": args.blocks, "block_frames": args.block_frames, "chunk_frames": 4096,
                       "frames_per_gpu": int(frames_rank), "compressed_bytes_per_gpu": len(data),
                       "parallelism": f"file-shard x{ws}, no collectives"},
            "hbm_gbs": round(achieved, 2),
            "pcie_inclusive": {"value": round(e2e, 2), "unit": "Msamples/s", "ms": round(t_e2e * 1e3, 3),
                               "what": "upload of the compressed batch + decode + download of int32 PCM, rank 0"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 6),
                         "traffic": None if traffic is None else int(traffic),
                         "traffic_unit": "bytes/launch (PMC FETCH_SIZE + WRITE_SIZE, scale calibrated in the profile)", "traffic_source": traffic_src,
                         "kernel_ms": round(kernel_ms, 4), "alg_bytes_per_launch": alg_bytes,
                         "binding_limit": "serial entropy decode per block (scalar issue of one wave), not HBM"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    b.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
